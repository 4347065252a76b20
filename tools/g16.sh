set -o pipefail
O=gpurun_out/g16; mkdir -p $O; export TMPDIR=/tmp
run() {  # tag config prec steps shards [env...]
  local tag=$1 c=$2 p=$3 st=$4 sh=$5; shift 5
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-f32 --precision $p --config $c --steps $st --sim-shards $sh > $O/$tag.json 2>>$O/err.log || { echo "$tag failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['roofline']['kernel_ms'], d['ms_per_step'], d['check']['mean_rgb'] if 'check' in d else '')"
}
for p in f64 f32; do
  run cornell_${p}_t0 cornell $p 20 1 X=1
  for t in 8 16 32 64; do run cornell_${p}_t$t cornell $p 20 1 RT_AMD_TAIL_ITEMS=$t; done
  run cornell_${p}_t16_b8 cornell $p 20 1 RT_AMD_TAIL_ITEMS=16 RT_AMD_BIG_CHUNK=8
  run cornell_${p}_sh8_t0 cornell $p 40 8 X=1
  run cornell_${p}_sh8_t16 cornell $p 40 8 RT_AMD_TAIL_ITEMS=16
  run cornell_${p}_sh8_t32 cornell $p 40 8 RT_AMD_TAIL_ITEMS=32
done
echo done
