#!/bin/bash
# Round-4 experiment: the workgroup ray-queue BVH kernel (RT_VAR_BVH_WG, rt_trace.h lane_loop_wg)
# against the decoupled kernel (RT_VAR_BVH), same library, knob RT_AMD_VARIANT = 3 / 2.
#   1. small renders of every BVH config, both variants and precisions: images bit-identical
#   2. kernel ms per frame at full size, ABAB (REPS) on bench.py (binary64 line + the FP32 record)
# usage: bash tools/wg_experiment.sh <tag> [configs]
export RT_AMD_EXPERIMENTS=1
set -o pipefail
OUT=gpurun_out/${1:-wg}; mkdir -p $OUT
CFGS=${2:-"bunny_cornell pawn_fog demo1"}
export TMPDIR=/tmp
timeout -k 10 120 python3 - $CFGS <<'PY' > $OUT/identity.log 2>&1 || { echo "identity step failed"; tail -20 $OUT/identity.log; exit 1; }
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import raytrace_amd as R
from raytrace_amd import scenes
ok = True
for n in sys.argv[1:]:
    cs, w, g = scenes.CONFIGS[n](width=96, spp=16)
    for prec in ("f64", "f32"):
        os.environ["RT_AMD_VARIANT"] = "2"
        a = R.raytrace(cs, w, g, precision=prec)
        os.environ["RT_AMD_VARIANT"] = "3"
        b = R.raytrace(cs, w, g, precision=prec)
        same = np.array_equal(a, b, equal_nan=True)
        ok = ok and same
        print(n, prec, "bit-identical" if same else f"DIFFERENT max {np.abs(a - b).max()}", flush=True)
sys.exit(0 if ok else 1)
PY
cat $OUT/identity.log
for c in $CFGS; do
  for rep in $(seq 1 ${REPS:-2}); do
    for v in 2 3; do
      RT_AMD_VARIANT=$v timeout -k 10 300 python3 bench.py --config $c --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-abi-devices \
        > $OUT/${c}_v${v}_r$rep.json 2>> $OUT/bench.err || { echo "bench $c v$v failed"; tail -5 $OUT/bench.err; exit 1; }
      python3 -c "import json;d=json.loads(open('$OUT/${c}_v${v}_r$rep.json').read().strip().splitlines()[-1]);f=d['f32_fast_path'];print('$c v$v r$rep f64', d['roofline']['kernel_ms'], d['check']['sha16'], 'f32', f['roofline']['kernel_ms'], f['check']['sha16'])"
    done
  done
done
