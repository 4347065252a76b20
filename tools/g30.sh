set -o pipefail
# guard-free reciprocal in plane / target tests and 5 waves for the light binary64 flat kernel: A/B, GPU tests
O=gpurun_out/g30; mkdir -p $O; export TMPDIR=/tmp
E=$PWD/raytrace_amd/_lib/exp
for p in f64; do
  for c in cornell bunny_cornell; do
    for lib in base prev w5 base prev w5; do
      if [ $lib = base ]; then unset RT_AMD_LIB; else export RT_AMD_LIB=$E/librt_amd_$lib.so; fi
      f=$O/${c}_${p}_$lib.json
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps ${STEPS:-10} > $f 2>>$O/err.log || { echo "$c $p $lib failed"; exit 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['mean_rgb'])" $f "$c $p $lib"
    done
  done
done
unset RT_AMD_LIB
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
