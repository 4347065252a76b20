set -o pipefail
O=gpurun_out/g20; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "chunk or emulator or variants" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 bench.py > $O/bench_cornell.json 2> $O/bench_cornell.err || { echo bench failed; exit 1; }
for c in readme pawn_fog; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --steps 5 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 bench.py --no-cpu-baseline --streams 1 > $O/prof1_bench.json 2> $O/prof1.err || { echo prof1 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --no-cpu-baseline > $O/prof2_bench.json 2> $O/prof2.err || { echo prof2 failed; exit 1; }
echo done
