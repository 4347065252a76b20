export RT_AMD_EXPERIMENTS=1
set -o pipefail
OUT=gpurun_out/wg2; mkdir -p $OUT
export TMPDIR=/tmp
for pct in 25 90; do
  for v in 3; do
    RT_AMD_TRAV_PCT=$pct RT_AMD_VARIANT=$v timeout -k 10 300 python3 bench.py --config bunny_cornell --steps 3 --warmup 1 --no-cpu-baseline --no-abi-devices > $OUT/bunny_v${v}_p$pct.json 2>> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/bunny_v${v}_p$pct.json').read().strip().splitlines()[-1]);f=d['f32_fast_path'];print('bunny v$v pct $pct f64', d['roofline']['kernel_ms'], 'f32', f['roofline']['kernel_ms'])"
  done
done
for v in 2 3; do
  RT_AMD_VARIANT=$v bash tools/pmc_run.sh $OUT/pmc_bunny_f64_v$v bunny_cornell f64 || exit 1
  grep -E "lane util|wait_any /|VALU insts per wave|SQ_INSTS_SALU|SQ_INSTS_LDS|SQ_INSTS_VALU  |SQ_WAVES" $OUT/pmc_bunny_f64_v$v/summary.txt
done
