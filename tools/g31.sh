set -o pipefail
# Round-2 final counters: GPU tests, math accuracy, PMC passes of every config in both precisions
# (bench.py's roofline reads them once folded), rocprofv3 kernel stats of the headline, binary64
# shard shares.
O=gpurun_out/g31; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 60 tools/microbench/f64_math_check > $O/f64_math_check.json || { echo "math failed"; exit 1; }
for prec in f64 f32; do
  for p in cornell bunny_cornell demo1 readme pawn_fog; do
    timeout -k 10 600 bash tools/pmc_run.sh $O/pmc_${p}_$prec $p $prec || { echo "pmc $p $prec failed"; exit 1; }
    echo "pmc $p $prec done"
  done
done
for s in 2 4 8; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --config cornell --steps 20 --sim-shards $s > $O/shards_$s.json 2>> $O/bench.err || { echo "shards $s failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/shards_$s.json'));print('shards $s', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- \
  python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --streams 1 > $O/prof_bench_cornell_1stream.json 2> $O/prof1.err || { echo "rocprof 1 failed"; tail -5 $O/prof1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- \
  python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/prof_bench_cornell.json 2> $O/prof2.err || { echo "rocprof 2 failed"; tail -5 $O/prof2.err; exit 1; }
echo prof done
