set -o pipefail
O=gpurun_out/g4; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 tools/microbench/f64_math_check > $O/f64_math_check.json 2> $O/f64_math_check.err &&
timeout -k 10 300 python3 tools/gpu_quick.py > $O/quick.log 2>&1 &&
bash tools/ab_libs.sh g4/ab "cornell:1 bunny_cornell:1" 10
echo exit $?
