set -o pipefail
export TMPDIR=/tmp
bash tools/sweep_env.sh iso cornell f64 "base RT_AMD_GRID_RESERVE=0 RT_AMD_BIG_CHUNK=16 RT_AMD_GRID_RESERVE=0,RT_AMD_BIG_CHUNK=16 RT_AMD_BIG_CHUNK=24" 20 || exit 1
mkdir -p gpurun_out/iso
for r in 0 8; do
  RT_AMD_GRID_RESERVE=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iso/prof32_res$r -o run -- python3 bench.py --no-cpu-baseline --precision f32 --no-f32 --steps 20 > gpurun_out/iso/prof32_res$r.json 2> gpurun_out/iso/prof32_res$r.err || { echo "prof $r failed"; exit 1; }
  grep -h "resolve" gpurun_out/iso/prof32_res$r/*kernel_stats.csv | cut -c1-160
done
