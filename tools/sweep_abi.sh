#!/bin/bash
# Like sweep_env.sh, but reports the line's kernel ms AND its one-call C-ABI record (ms per call,
# library ms, lone-launch kernel ms): bash tools/sweep_abi.sh <tag> <config> <f64|f32> "<K=V,...> ..." [steps]
export RT_AMD_EXPERIMENTS=1
TAG=$1; CFG=$2; PREC=$3; SETS=$4; STEPS=${5:-10}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
for set in $SETS; do
  envs=""; [ "$set" != base ] && envs=$(echo $set | tr ',' ' ')
  f=$OUT/${CFG}_${PREC}_$(echo $set | tr ',=' '_-')_r$rep.json
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 --precision $PREC --config $CFG --steps $STEPS \
    --warmup-s 0.3 > $f 2>>$OUT/err.log || { echo "fail $set"; exit 1; }
  python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);a=d.get('abi_device_list') or {}
print('$CFG $PREC $set rep $rep line', d['roofline']['kernel_ms'], 'abi', a.get('ms_per_frame'), a.get('library_ms_per_call'), a.get('kernel_ms_max_device'))"
done; done
