# Round-2 final measurements: PMC refresh (Cornell both precisions, bunny f32), every config's
# bench line, rocprofv3 kernel stats with one stream (durations comparable with bench kernel_ms)
# and with the bench default (two streams for flat scenes).
set -o pipefail
O=gpurun_out/g19; mkdir -p $O; export TMPDIR=/tmp
bash tools/pmc_run.sh $O/pmc_cornell_f64 cornell f64 || exit 1
bash tools/pmc_run.sh $O/pmc_cornell_f32 cornell f32 || exit 1
bash tools/pmc_run.sh $O/pmc_bunny_cornell_f32 bunny_cornell f32 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench_cornell.json 2> $O/bench_cornell.err || { echo bench failed; exit 1; }
for c in readme demo1 demo1_1200x800 bunny_cornell pawn_fog; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --steps 5 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 bench.py --no-cpu-baseline --streams 1 > $O/prof1_bench.json 2> $O/prof1.err || { echo prof1 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --no-cpu-baseline > $O/prof2_bench.json 2> $O/prof2.err || { echo prof2 failed; exit 1; }
echo done
