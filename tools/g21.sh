set -o pipefail
O=gpurun_out/g21; mkdir -p $O; export TMPDIR=/tmp
run() {  # tag config prec [env...]
  local tag=$1 c=$2 p=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps 20 > $O/$tag.json 2>>$O/err.log || { echo "$tag failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['roofline']['kernel_ms'], d['ms_per_step'])"
}
E=$PWD/raytrace_amd/_lib/exp
run c64_base cornell f64 X=1
run c64_w3 cornell f64 RT_AMD_LIB=$E/librt_amd_w3.so
run c64_w5 cornell f64 RT_AMD_LIB=$E/librt_amd_w5.so
run c64_base2 cornell f64 X=1
echo done
run c32_flat cornell f32 X=1
run c32_bvh cornell f32 RT_AMD_VARIANT=2
run c32_bvhlock cornell f32 RT_AMD_VARIANT=1
run c32_bvh_nobox cornell f32 RT_AMD_VARIANT=2 RT_AMD_NO_BOX=1
echo done2
