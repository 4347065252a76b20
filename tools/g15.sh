set -o pipefail
O=gpurun_out/g15; mkdir -p $O; export TMPDIR=/tmp
run() {  # tag config prec steps [env...]
  local tag=$1 c=$2 p=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps $st > $O/$tag.json 2>>$O/err.log || { echo "$tag failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['roofline']['kernel_ms'], d['ms_per_step'])"
}
E=$PWD/raytrace_amd/_lib/exp
run cornell64_base cornell f64 20 X=1
run cornell64_nocommit cornell f64 20 RT_AMD_LIB=$E/librt_amd_nocommit.so
for c in 6 8 12 16; do run cornell64_c$c cornell f64 20 RT_AMD_CHUNK=$c; done
run readme64_base readme f64 40 X=1
run readme64_nocommit readme f64 40 RT_AMD_LIB=$E/librt_amd_nocommit.so
for c in 6 8 10 13 25; do run readme64_c$c readme f64 40 RT_AMD_CHUNK=$c; done
run cornell32_nocommit cornell f32 20 RT_AMD_LIB=$E/librt_amd_nocommit.so
run cornell32_base cornell f32 20 X=1
run cornell64_base2 cornell f64 20 X=1
echo done
