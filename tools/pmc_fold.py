"""Fold a tools/pmc_run.sh directory into profiles/pmc_valu.json under "<config>/<precision>":
per-launch VALU instruction counts (total and by class), lane utilisation, GPU cycles and the
HBM traffic (FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note, WRITE_SIZE as is) of
rt_render_kernel — what bench.py's `roofline` reads.

    python tools/pmc_fold.py <outdir> <config> <precision> <round>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out, config, prec, rnd = sys.argv[1:5]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vals = defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "rt_render_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
need = ["SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES"]
missing = [k for k in need if k not in m]
if missing:
    sys.exit(f"missing counters {missing} under {out}")
mix = {k[len("SQ_INSTS_VALU_"):].lower(): m[k] for k in m if k.startswith("SQ_INSTS_VALU_")}
rec = {"kernel": "rt_render_kernel", "valu_insts_per_launch": m["SQ_INSTS_VALU"], "valu_mix_per_launch": mix,
       "salu_insts_per_launch": m.get("SQ_INSTS_SALU"),
       "lane_utilisation": m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]),
       "gpu_cycles_per_launch": m["GRBM_GUI_ACTIVE"] / 8, "waves": m["SQ_WAVES"],
       "wait_any_frac": m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in m else None,
       "wait_inst_any_frac": m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in m else None,
       "method": "rocprofv3 --pmc (tools/pmc_run.sh: one counter group per pass, --kernel-trace only, one "
                 "stream); counts per dispatch of rt_render_kernel, GRBM_GUI_ACTIVE summed over 8 XCDs",
       "round": rnd}
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    fetch, write = 2 * m["FETCH_SIZE"] * 1024, m["WRITE_SIZE"] * 1024
    rec.update(hbm_bytes_per_launch=int(round(fetch + write)), fetch_bytes_corrected=int(round(fetch)),
               write_bytes=int(round(write)))
path = os.path.join(root, "profiles", "pmc_valu.json")
d = json.load(open(path)) if os.path.exists(path) else {}
d = {k: v for k, v in d.items() if "/" in k}  # round-1 entries (f32 only, unkeyed precision) are superseded
d[f"{config}/{prec}"] = rec
json.dump(d, open(path, "w"), indent=1)
print(config, prec, json.dumps({k: rec[k] for k in ("valu_insts_per_launch", "lane_utilisation")}))
