#!/bin/bash
# Small-item size 3 vs 4 on README and Cornell, 1 GPU and one rank's share of 8, two repetitions
export RT_AMD_EXPERIMENTS=1
O=gpurun_out/${1:-chunk3}; mkdir -p $O
for rep in 1 2; do
  for cfg in readme cornell; do
    for sh in 1 8; do
      for set in base RT_AMD_CHUNK=3; do
        envs=""; [ "$set" != base ] && envs=$set
        f=$O/${cfg}_${sh}_$(echo $set | tr '=' '-')_r$rep.json
        env $envs timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-abi-devices --sim-shards $sh --steps 40 > $f 2>> $O/err.log || { echo "fail $set"; exit 1; }
        python3 -c "import json;d=json.load(open('$f'));print('$cfg $sh $set rep $rep', d['roofline']['kernel_ms'], 'f32', d['f32_fast_path']['roofline']['kernel_ms'])"
      done
    done
  done
done
