#!/bin/bash
# Round-2 final refresh: binary64 PMC passes of the BVH configs after the FP32 node reciprocal,
# then GPU tests, every config's bench line and the headline's rocprofv3 stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/g35; mkdir -p $O
for c in demo1 bunny_cornell pawn_fog; do
  bash tools/pmc_run.sh $O/pmc_${c}_f64 $c f64 || exit 1
  python3 tools/pmc_fold.py $O/pmc_${c}_f64 $c f64 r2 || exit 1
done
cp profiles/pmc_valu.json $O/pmc_valu.json
bash tools/gpu_round.sh g35r tests bench benchall prof
