#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace + PMC traffic passes.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh <tag> [tests|bench|prof|pmc ...]
set -o pipefail
TAG=${1:-r1}
shift
STEPS=${STEPS:-"tests bench prof pmc"}
[ $# -gt 0 ] && STEPS="$*"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu.log" ;;
    bench)
      timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    benchall)
      for c in readme demo1 bunny_cornell pawn_fog; do
        timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_$c.json" 2>> "$OUT/bench.err" || { echo "bench $c failed"; exit 1; }
        cat "$OUT/bench_$c.json"
      done ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps ${PROF_STEPS:-20} --warmup 2 --no-cpu-baseline ${CONFIG:+--config $CONFIG} > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 1; }
      find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc_$c" -o run -- \
          python3 bench.py --steps 5 --warmup 1 --warmup-s 0 --no-cpu-baseline ${CONFIG:+--config $CONFIG} > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err" || { echo "pmc $c failed"; tail -20 "$OUT/pmc_$c.err"; exit 1; }
      done
      echo pmc done ;;
  esac
done
