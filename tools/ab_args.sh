#!/bin/bash
# A/B of bench.py argument sets: bash tools/ab_args.sh <tag> "name1:--args ..." "name2:--args ..." ...
# Prints kernel ms, Msamples/s and ms per step for each.
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for spec in "$@"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > $OUT/$n.json 2>>$OUT/err.log || { echo "$n failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', d['roofline']['kernel_ms'], d['value'], d['ms_per_step'], d['check'])"
done
