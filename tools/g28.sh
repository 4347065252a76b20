set -o pipefail
# world-aligned box axes from the shared reciprocal direction (binary64): A/B, GPU tests
O=gpurun_out/g28; mkdir -p $O; export TMPDIR=/tmp
E=$PWD/raytrace_amd/_lib/exp
for c in cornell bunny_cornell; do
  for lib in base noalign base noalign; do
    if [ $lib = base ]; then unset RT_AMD_LIB; else export RT_AMD_LIB=$E/librt_amd_$lib.so; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision f64 --config $c --steps ${STEPS:-10} > $O/${c}_$lib.json 2>>$O/err.log || { echo "$c $lib failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${c}_$lib.json'));print('$c $lib', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['mean_rgb'])"
  done
done
unset RT_AMD_LIB
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
