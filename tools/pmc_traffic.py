"""Fold the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_round.sh (step `pmc`) into
profiles/pmc_traffic.json: HBM-side bytes per launch of rt_render_kernel for one config.

    python tools/pmc_traffic.py gpurun_out/<tag> <config> <round>

FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM section: gfx950 reports half the bytes of wide
reads); WRITE_SIZE is taken as is.  Both are KiB per dispatch."""
import csv
import glob
import json
import os
import sys

out, config, rnd = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
raw = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = []
    for f in glob.glob(os.path.join(out, f"pmc_{c}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "rt_render_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        sys.exit(f"no {c} samples under {out}")
    raw[c] = {"launches": len(vals), "mean_kib": sum(vals) / len(vals), "values_kib": vals}
fetch = 2 * raw["FETCH_SIZE"]["mean_kib"] * 1024
write = raw["WRITE_SIZE"]["mean_kib"] * 1024
path = os.path.join(root, "profiles", "pmc_traffic.json")
d = json.load(open(path)) if os.path.exists(path) else {}
d[config] = {"kernel": "rt_render_kernel", "hbm_bytes_per_launch": int(round(fetch + write)),
             "fetch_bytes_corrected": int(round(fetch)), "write_bytes": int(round(write)), "raw": raw,
             "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, --kernel-trace; "
                       "FETCH_SIZE (KiB) x2 per MI355X_MICROARCH.md HBM section, WRITE_SIZE (KiB) as is",
             "round": rnd}
json.dump(d, open(path, "w"), indent=1)
print(config, d[config]["hbm_bytes_per_launch"], "bytes per launch")
