#!/bin/bash
# A/B of experiment libraries (raytrace_amd/_lib/exp/*.so) against the in-tree build over bench
# configs: bash tools/ab_libs.sh <tag> "<config>:<sim-shards> ..." [steps]
# REPS=k repeats the base / experiment pair k times in ABAB order (run-to-run noise is ~1 %)
export RT_AMD_EXPERIMENTS=1  # the library reads RT_AMD_* knobs / RT_AMD_LIB only with this set
TAG=$1; CFGS=$2; STEPS=${3:-20}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for cfg in $CFGS; do
  n=${cfg%%:*}; sh=${cfg#*:}
  for rep in $(seq 1 ${REPS:-1}); do
  for lib in base ${LIBS:-raytrace_amd/_lib/exp/*.so}; do
    nm=$(basename $lib .so); [ ${REPS:-1} -gt 1 ] && nm=${nm}_r$rep
    if [ "$lib" = base ]; then unset RT_AMD_LIB; else export RT_AMD_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-f32 --precision ${PREC:-f64} --config $n --steps $STEPS --sim-shards $sh > $OUT/${n}_${sh}_$nm.json 2>>$OUT/err.log || { echo "$nm failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${n}_${sh}_$nm.json'));print('$n shards $sh $nm', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['sha16'])"
  done
  done
done
