set -o pipefail
O=gpurun_out/g11; mkdir -p $O; export TMPDIR=/tmp
run() {  # tag config prec [env...]
  local tag=$1 c=$2 p=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps 5 > $O/$tag.json 2>>$O/err.log || { echo "$tag failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['mean_rgb'] if 'check' in d else '')"
}
NC=RT_AMD_LIB=$PWD/raytrace_amd/_lib/exp/librt_amd_nocull.so
for c in bunny_cornell demo1; do
  run ${c}_nocull $c f32 $NC
  run ${c}_cull $c f32 X=1
  for t in 25 35 65 80; do run ${c}_cull_t$t $c f32 RT_AMD_TRAV_PCT=$t; done
done
run bunny64_nocull bunny_cornell f64 $NC
run bunny64_cull bunny_cornell f64 X=1
echo done
