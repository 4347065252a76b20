#!/bin/bash
# A/B session for experiment libraries (raytrace_amd/_lib/exp/*.so) against the in-tree build:
# bit-identity of the images on every test config, then kernel time per config in both precisions.
#   bash tools/ab_session.sh <tag> "<config>:<shards> ..." [precisions]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-ab}; CFGS=${2:-"cornell:1 bunny_cornell:1 demo1:1 pawn_fog:1 readme:1"}; PRECS=${3:-"f64 f32"}
O=gpurun_out/$TAG; mkdir -p $O
for lib in raytrace_amd/_lib/exp/*.so; do
  nm=$(basename $lib .so)
  timeout -k 10 400 python3 tools/image_ab.py $lib $O/image_ab_$nm.json > $O/image_ab_$nm.log 2>&1 || { echo "image_ab $nm failed"; tail -20 $O/image_ab_$nm.log; exit 1; }
  echo "$nm: $(grep -c "'bit_identical': True" $O/image_ab_$nm.log) bit-identical of $(grep -c bit_identical $O/image_ab_$nm.log)"
done
for p in $PRECS; do PREC=$p timeout -k 10 1200 bash tools/ab_libs.sh $TAG/ab_$p "$CFGS" ${STEPS:-5} || exit 1; done
