set -o pipefail
# Round-2 final bench lines (after the PMC fold of g31): the default headline run with the CPU
# baseline, then every other config (binary64 line + FP32 record).
O=gpurun_out/g32; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $O/bench_cornell.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench_cornell.json
for c in readme demo1 demo1_1200x800 bunny_cornell pawn_fog; do
  timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || { echo "bench $c failed"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('mix_frac'), d['f32_fast_path']['value'], d['f32_fast_path']['ms_per_step'])" $O/bench_$c.json $c
done
