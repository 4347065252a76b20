set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/bvh4; mkdir -p $O
timeout -k 10 400 python3 tools/image_ab.py raytrace_amd/_lib/exp/librt_amd_bvh4.so $O/image_ab.json > $O/image_ab.log 2>&1 || { echo image_ab failed; tail -20 $O/image_ab.log; exit 1; }
cat $O/image_ab.log
for p in f32 f64; do PREC=$p timeout -k 10 900 bash tools/ab_libs.sh bvh4/ab_$p "bunny_cornell:1 pawn_fog:1 demo1:1" 5 || exit 1; done
timeout -k 10 900 bash tools/sweep_items.sh items "cornell:1 cornell:8 readme:1" "16:16 32:16 64:16 16:4 32:4 64:4 64:8" || exit 1
for r in 0 8; do
  RT_AMD_GRID_RESERVE=$r RT_AMD_LIB=$PWD/raytrace_amd/_lib/exp/librt_amd_bvh4r.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_res$r -o run -- python3 bench.py --no-cpu-baseline --no-f32 --steps 20 > $O/prof_res$r.json 2> $O/prof_res$r.err || { echo "prof $r failed"; exit 1; }
  grep -h "resolve\|render" $O/prof_res$r/*kernel_stats.csv | cut -c1-200
done
