#!/bin/bash
# A/B of the in-tree build against raytrace_amd/_lib/exp/*.so on one and two streams (kernel ms per
# frame, ms per step, frame hash): POOL_TAG=<out dir> POOL_CPS="<config>:<prec> ..." bash tools/streams_ab.sh
export RT_AMD_EXPERIMENTS=1
OUT=gpurun_out/${POOL_TAG:-r5_pool}; mkdir -p $OUT
for rep in 1 2; do
for lib in base raytrace_amd/_lib/exp/*.so; do
  nm=$(basename $lib .so); if [ $lib = base ]; then unset RT_AMD_LIB; else export RT_AMD_LIB=$PWD/$lib; fi
  for cfg in ${POOL_CPS:-cornell:f64 cornell:f32 bunny_cornell:f64 pawn_fog:f32}; do
    c=${cfg%%:*}; p=${cfg#*:}
    for st in 1 2; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps 10 --streams $st > $OUT/${c}_${p}_s${st}_${nm}_$rep.json 2>>$OUT/err.log || { echo "fail $nm $cfg"; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/${c}_${p}_s${st}_${nm}_$rep.json'));print('$c $p streams $st $nm rep $rep', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['sha16'])"
    done
  done
done
done
