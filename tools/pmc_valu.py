"""Fold a tools/gpu_pmc.sh run into profiles/pmc_valu.json: per-launch VALU / SALU instruction
counts and lane utilisation of rt_render_kernel for one config (bench.py's issue roofline).

    python tools/pmc_valu.py gpurun_out/<tag> <config> <round>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out, config, rnd = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vals = defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "rt_render_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
need = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES"]
missing = [k for k in need if k not in m]
if missing:
    sys.exit(f"missing counters {missing} under {out}")
path = os.path.join(root, "profiles", "pmc_valu.json")
d = json.load(open(path)) if os.path.exists(path) else {}
d[config] = {"kernel": "rt_render_kernel", "valu_insts_per_launch": m["SQ_INSTS_VALU"],
             "salu_insts_per_launch": m["SQ_INSTS_SALU"],
             "lane_utilisation": m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]),
             "gpu_cycles_per_launch": m["GRBM_GUI_ACTIVE"] / 8, "waves": m["SQ_WAVES"],
             "method": "rocprofv3 --pmc (tools/gpu_pmc.sh, one counter group per pass, --kernel-trace); "
                       "wave-level instruction counts; GRBM_GUI_ACTIVE summed over 8 XCDs",
             "round": rnd}
json.dump(d, open(path, "w"), indent=1)
print(config, d[config])
