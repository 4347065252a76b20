#!/bin/bash
# Round-2 late session: bit-identity of the FP32 node test against the binary64 one, refreshed
# binary64 PMC passes (the kernels changed), then the bench lines and the headline's rocprofv3 stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/g33; mkdir -p $O
timeout -k 10 400 python tools/image_ab.py raytrace_amd/_lib/exp/librt_amd_node_f64.so $O/image_ab_node.json > $O/image_ab.log 2>&1 || { echo "image_ab failed"; tail -20 $O/image_ab.log; exit 1; }
cat $O/image_ab.log
for c in cornell demo1 bunny_cornell pawn_fog; do
  bash tools/pmc_run.sh $O/pmc_${c}_f64 $c f64 || exit 1
  python3 tools/pmc_fold.py $O/pmc_${c}_f64 $c f64 r2 || exit 1
done
cp profiles/pmc_valu.json $O/pmc_valu.json
bash tools/gpu_round.sh g33r tests bench benchall prof
