#!/bin/bash
# Round-3 validation + measurement session: every GPU test, every config's bench line, rocprofv3
# kernel stats of the headline (default two streams and one stream).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_cornell.json 2> $O/bench_cornell.err || { echo "bench failed"; tail -5 $O/bench_cornell.err; exit 1; }
for c in readme demo1 demo1_1200x800 bunny_cornell pawn_fog; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench_other.err || { echo "bench $c failed"; exit 1; }
done
for c in cornell readme demo1 demo1_1200x800 bunny_cornell pawn_fog; do python3 -c "
import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); f=d.get('f32_fast_path',{})
print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], 'f32', f.get('value'), f.get('ms_per_step'))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams 1 > $O/prof1_bench.json 2> $O/prof1.err || { echo "rocprof 1-stream failed"; exit 1; }
for d in prof prof1; do echo $d; grep -h "render_kernel\|resolve" $O/$d/*kernel_stats.csv | cut -c1-160; done
