"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of rt_render_kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
vals = defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "rt_render_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(m):
    print(f"{k:32s} {m[k]:.6g}  (n={len(vals[k])})")
if "SQ_WAVE_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m:
    print("VALU active / wave cycles:", m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"])
if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
    print("wait_any / wave cycles:", m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"])
    print("wait_inst_any / wave cycles:", m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"])
if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
    print("lane utilisation (thread cycles / (64 x active valu)):", m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]))
if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
    print("VALU insts per wave:", m["SQ_INSTS_VALU"] / m["SQ_WAVES"])
