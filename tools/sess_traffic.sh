#!/bin/bash
# HBM traffic of the render kernel (FETCH_SIZE, WRITE_SIZE passes of their own, one stream) for
# configs x precisions, with the in-tree build and with each exp lib:
#   bash tools/sess_traffic.sh <tag> "<config>:<prec> ..."
set -o pipefail
export TMPDIR=/tmp
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
for cp in $2; do
  c=${cp%%:*}; p=${cp#*:}
  for lib in "" ${LIBS:-raytrace_amd/_lib/exp/*.so}; do
    if [ -n "$lib" ]; then [ -e "$lib" ] || continue; export RT_AMD_LIB=$PWD/$lib; nm=$(basename $lib .so); else unset RT_AMD_LIB; nm=intree; fi
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${c}_${p}_${nm}_$ctr -o run -- \
        python3 bench.py --config $c --precision $p --no-f32 --steps 3 --warmup 1 --warmup-s 0 --no-cpu-baseline --streams 1 \
        > $O/${c}_${p}_${nm}_$ctr.json 2> $O/${c}_${p}_${nm}_$ctr.err || { echo "pass $c $p $nm $ctr failed"; tail -3 $O/${c}_${p}_${nm}_$ctr.err; exit 1; }
      python3 - "$O/${c}_${p}_${nm}_$ctr" "$c $p $nm $ctr" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if "rt_render_kernel" in r["Kernel_Name"]]
print(sys.argv[2], "per launch (KB as reported):", sum(v) / max(1, len(v)), "launches", len(v))
PY
    done
  done
done
