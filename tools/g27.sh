set -o pipefail
# table-based binary64 sin / cos of 2 pi u: accuracy, A/B against the quadrant polynomial, GPU tests
O=gpurun_out/g27; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 60 tools/microbench/f64_math_check > $O/math_tab.json || { echo "math failed"; exit 1; }
cat $O/math_tab.json
E=$PWD/raytrace_amd/_lib/exp
for c in cornell bunny_cornell demo1 readme; do
  for lib in base poly base poly; do
    if [ $lib = base ]; then unset RT_AMD_LIB; else export RT_AMD_LIB=$E/librt_amd_$lib.so; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision f64 --config $c --steps ${STEPS:-10} > $O/${c}_$lib.json 2>>$O/err.log || { echo "$c $lib failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${c}_$lib.json'));print('$c $lib', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['mean_rgb'])"
  done
done
unset RT_AMD_LIB
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
