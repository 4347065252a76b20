#!/bin/bash
# Frames on 1 vs 2 HIP streams for the BVH configs (bench.py --streams), at one GPU and at one
# rank's share of 8 GPUs: bash tools/streams_ab.sh <tag>   (ABAB order, binary64 line + FP32 record)
O=gpurun_out/${1:-streams_ab}; mkdir -p $O
for c in ${CFGS:-bunny_cornell:1 demo1:1 bunny_cornell:8 pawn_fog:1}; do
  n=${c%%:*}; sh=${c#*:}
  for rep in 1 2; do
    for st in 1 2; do
      timeout -k 10 300 python bench.py --config $n --sim-shards $sh --streams $st --steps 5 --no-cpu-baseline --no-abi-devices \
        > $O/${n}_${sh}_s${st}_r$rep.json 2>> $O/err.log || { echo "$n $sh $st failed"; exit 1; }
      python3 -c "import json;d=json.load(open('$O/${n}_${sh}_s${st}_r$rep.json'));print('$n', '$sh', 'streams $st', d['roofline']['kernel_ms'], d['ms_per_step'], 'f32', d['f32_fast_path']['roofline']['kernel_ms'], d['check']['sha16'])"
    done
  done
done
