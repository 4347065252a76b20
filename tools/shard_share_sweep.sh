#!/bin/bash
# One rank's share of an N-GPU frame (bench.py --sim-shards N, one process) for N = 1, 2, 4, 8 on
# the Cornell box, and N = 8 for bunny-Cornell and pawn+fog: bash tools/shard_share_sweep.sh
O=gpurun_out/${1:-shards}; mkdir -p $O
for s in 1 2 4 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --sim-shards $s > $O/sim_shards_$s.json 2>>$O/err.log || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 --sim-shards 8 --config bunny_cornell > $O/bunny_sim_shards_8.json 2>>$O/err.log || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --sim-shards 8 --config pawn_fog > $O/pawn_fog_sim_shards_8.json 2>>$O/err.log || exit 1
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['roofline']['kernel_ms'], d['ms_per_step'], d['value'])"; done
