#!/bin/bash
# A/B of environment settings: bash tools/ab_env.sh <tag> "name1:VAR=1 VAR2=2" "name2:" ...
# (ARGS env = bench.py arguments).  Prints kernel ms and Msamples/s per setting.
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
ARGS=${ARGS:-"--no-cpu-baseline --steps 5 --warmup 1"}
for spec in "$@"; do
  n=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py $ARGS > $OUT/$n.json 2>>$OUT/err.log || { echo "$n failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', d['roofline']['kernel_ms'], d['value'], d['check'])"
done
