set -o pipefail
O=gpurun_out/g2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 tools/microbench/valu_rates > $O/valu_rates.json 2> $O/valu_rates.err &&
bash tools/pmc_run.sh $O/pmc_cornell_f64 cornell f64 &&
bash tools/pmc_run.sh $O/pmc_cornell_f32 cornell f32 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --steps 10 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
echo exit $?
