#!/bin/bash
# Copy a measurement session (tools/gpu_round.sh <tag> tests bench benchall prof pmc, plus the
# bunny prof/pmc and tools/gpu_pmc.sh runs) into profiles/<round>/ and fold the PMC summaries.
# usage: tools/save_profiles.sh <tag> <round>   (expects gpurun_out/<tag>, <tag>_bunny,
#        pmc_<tag>c, pmc_<tag>b)
set -e
TAG=$1; RND=${2:-r1}
G=gpurun_out; D=profiles/$RND
mkdir -p $D
cp $G/$TAG/bench.json $D/bench_cornell.json
cp $G/$TAG/prof/run_kernel_stats.csv $D/cornell_kernel_stats.csv
cp $G/$TAG/prof_bench.json $D/prof_bench_cornell.json
for c in readme demo1 bunny_cornell pawn_fog; do cp $G/$TAG/bench_$c.json $D/bench_$c.json; done
cp $G/${TAG}_bunny/prof/run_kernel_stats.csv $D/bunny_cornell_kernel_stats.csv
tail -3 $G/$TAG/pytest_gpu.log > $D/pytest_gpu_tail.txt
python3 tools/pmc_traffic.py $G/$TAG cornell $RND
python3 tools/pmc_traffic.py $G/${TAG}_bunny bunny_cornell $RND
cp $G/pmc_${TAG}c/summary.txt $D/pmc_counters_cornell.txt
cp $G/pmc_${TAG}b/summary.txt $D/pmc_counters_bunny.txt
python3 tools/pmc_valu.py $G/pmc_${TAG}c cornell $RND
python3 tools/pmc_valu.py $G/pmc_${TAG}b bunny_cornell $RND
