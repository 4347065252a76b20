#!/bin/bash
# Sweep env tuning knobs (RT_AMD_*) for one config and precision, 2 repetitions each:
#   bash tools/sweep_env.sh <tag> <config> <f64|f32> "<K=V,K2=V2> <K=V> ..." [steps]
# ("base" as an entry = no knob).  Prints kernel ms per frame for every setting.
export RT_AMD_EXPERIMENTS=1  # the library reads RT_AMD_* knobs / RT_AMD_LIB only with this set
TAG=$1; CFG=$2; PREC=$3; SETS=$4; STEPS=${5:-5}  # EXTRA: more bench.py arguments (e.g. --streams 1)
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
for set in $SETS; do
  envs=""; [ "$set" != base ] && envs=$(echo $set | tr ',' ' ')
  f=$OUT/${CFG}_${PREC}_$(echo $set | tr ',=' '_-')_r$rep.json
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 --precision $PREC --config $CFG --steps $STEPS \
    --warmup-s 0.3 ${EXTRA} > $f 2>>$OUT/err.log || { echo "fail $set"; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('$CFG $PREC $set rep $rep', d['roofline']['kernel_ms'])"
done; done
