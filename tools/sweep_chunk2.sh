#!/bin/bash
# Flat-kernel item sizes (RT_AMD_CHUNK: small items, RT_AMD_BIG_CHUNK: big items) on the Cornell box
# at one GPU and at one rank's share of 8, binary64 and FP32, two repetitions:
#   bash tools/sweep_chunk2.sh <tag>
export RT_AMD_EXPERIMENTS=1
O=gpurun_out/${1:-chunk2}; mkdir -p $O
for rep in 1 2; do
  for sh in 1 8; do
    for set in base RT_AMD_CHUNK=3 RT_AMD_CHUNK=6 RT_AMD_BIG_CHUNK=8 RT_AMD_BIG_CHUNK=32; do
      envs=""; [ "$set" != base ] && envs=$set
      f=$O/cornell_${sh}_$(echo $set | tr '=' '-')_r$rep.json
      env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-abi-devices --sim-shards $sh --steps 20 > $f 2>> $O/err.log || { echo "fail $set"; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));print('cornell $sh $set rep $rep', d['roofline']['kernel_ms'], 'f32', d['f32_fast_path']['roofline']['kernel_ms'])"
    done
  done
done
