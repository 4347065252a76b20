set -o pipefail
O=gpurun_out/g23; mkdir -p $O; export TMPDIR=/tmp
run() {  # tag config prec [env...]
  local tag=$1 c=$2 p=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps 5 > $O/$tag.json 2>>$O/err.log || { echo "$tag failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['mean_rgb'] if 'check' in d else '')"
}
E=$PWD/raytrace_amd/_lib/exp
for c in bunny_cornell demo1 pawn_fog; do
  run ${c}_base $c f32 X=1
  run ${c}_selpark $c f32 RT_AMD_LIB=$E/librt_amd_selpark.so
done
run bunny64_base bunny_cornell f64 X=1
run bunny64_selpark bunny_cornell f64 RT_AMD_LIB=$E/librt_amd_selpark.so
echo done
