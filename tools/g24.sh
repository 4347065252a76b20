set -o pipefail
# one-Newton-step binary64 reciprocal / reciprocal square root: accuracy, A/B, parity tests
O=gpurun_out/g24; mkdir -p $O; export TMPDIR=/tmp
for v in "" _rcp1 _rsq1; do
  timeout -k 10 60 tools/microbench/f64_math_check$v > $O/math$v.json || { echo "math$v failed"; exit 1; }
  echo "math$v"; cat $O/math$v.json
done
E=$PWD/raytrace_amd/_lib/exp
for c in cornell bunny_cornell pawn_fog; do
  for lib in base rcp1 rcp1rsq1; do
    if [ $lib = base ]; then unset RT_AMD_LIB; else export RT_AMD_LIB=$E/librt_amd_$lib.so; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision f64 --config $c --steps ${STEPS:-10} > $O/${c}_$lib.json 2>>$O/err.log || { echo "$c $lib failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${c}_$lib.json'));print('$c $lib', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['mean_rgb'])"
  done
done
unset RT_AMD_LIB
RT_AMD_LIB=$E/librt_amd_rcp1rsq1.so timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_rcp1rsq1.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_rcp1rsq1.log; exit 1; }
tail -3 $O/pytest_rcp1rsq1.log
