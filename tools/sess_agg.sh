#!/bin/bash
# Commit-aggregation session (round 3): GPU tests, image bit-identity against the previous kernel
# build (raytrace_amd/_lib/exp/*.so), then kernel ms per config and precision for the in-tree
# build with aggregation (agg), without it (RT_AMD_AGG=0: pixel-major ids only) and each exp lib;
# VARIANTS="name:ENV=v ..." replaces the two in-tree settings (one name:ENV pair per word).
#   bash tools/sess_agg.sh <tag> ["<config> ..."] [precisions]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-agg}; CFGS=${2:-"cornell bunny_cornell pawn_fog readme demo1"}; PRECS=${3:-"f64 f32"}
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
for lib in raytrace_amd/_lib/exp/*.so; do
  [ -e "$lib" ] && [ -z "$NO_IMAGE" ] || continue
  nm=$(basename $lib .so)
  timeout -k 10 400 python3 tools/image_ab.py $lib $O/image_ab_$nm.json > $O/image_ab_$nm.log 2>&1 || { echo "image_ab $nm failed"; tail -20 $O/image_ab_$nm.log; exit 1; }
  echo "$nm: $(grep -c "'bit_identical': True" $O/image_ab_$nm.log) bit-identical of $(grep -c bit_identical $O/image_ab_$nm.log)"
done
run() {  # name lib-or-empty env...
  local nm=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export RT_AMD_LIB=$PWD/$lib; else unset RT_AMD_LIB; fi
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps ${STEPS:-10} > $O/${c}_${p}_$nm.json 2>>$O/err.log || { echo "$nm failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${c}_${p}_$nm.json'));print('$c $p $nm', d['roofline']['kernel_ms'], d['ms_per_step'], d['check'].get('sha16'))"
}
for rep in $(seq 1 ${REPS:-1}); do
for p in $PRECS; do
  for c in $CFGS; do
    for v in ${VARIANTS:-"agg:RT_AMD_AGG=1" "noagg:RT_AMD_AGG=0"}; do run ${v%%:*}_r$rep "" ${v#*:}; done
    for lib in raytrace_amd/_lib/exp/*.so; do [ -e "$lib" ] && run $(basename $lib .so)_r$rep $lib RT_AMD_AGG=1; done
  done
done
done
