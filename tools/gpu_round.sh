#!/bin/bash
# One GPU session: the parameterised replacement of the round-2 one-off lease scripts.
# Usage (from the repo root, on the GPU box):
#   bash tools/gpu_round.sh <tag> [tests|bench|benchall|prof|pmc|pmcvalu|microbench|rehearse ...]
# Env: CONFIG (bench/prof/pmc config), CONFIGS + PRECS (pmcvalu), PROF_STEPS, PYTEST_K (-k filter).
# Each GPU step runs under its own timeout and the script stops at the first failing step.
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
      timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
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
    pmcvalu)  # instruction-mix / wave-state / traffic passes folded into profiles/pmc_valu.json
      for c in ${CONFIGS:-cornell}; do
        for p in ${PRECS:-f64 f32}; do
          bash tools/pmc_run.sh "$OUT/pmc_${c}_$p" $c $p || exit 1
          python3 tools/pmc_fold.py "$OUT/pmc_${c}_$p" $c $p ${ROUND:-r3} || exit 1
        done
      done
      cp profiles/pmc_valu.json "$OUT/pmc_valu.json" ;;
    microbench)  # built from source here, never a committed binary
      make -C tools/microbench all > "$OUT/microbench_build.log" 2>&1 || { echo "microbench build failed"; exit 1; }
      timeout -k 10 120 tools/microbench/valu_rates > "$OUT/valu_rates.json" || exit 1
      timeout -k 10 120 tools/microbench/f64_math_check > "$OUT/f64_math_check.json" || exit 1 ;;
    rehearse)
      bash tools/rehearse_dist.sh "$TAG/rehearse" || exit 1 ;;
  esac
done
