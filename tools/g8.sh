set -o pipefail
O=gpurun_out/g8; mkdir -p $O; export TMPDIR=/tmp
bash tools/pmc_run.sh $O/pmc_readme_f64 readme f64 &&
timeout -k 10 400 python3 bench.py > $O/bench_cornell.json 2> $O/bench_cornell.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err &&
for c in readme demo1 demo1_1200x800 bunny_cornell pawn_fog; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --steps 5 > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
echo exit $?
