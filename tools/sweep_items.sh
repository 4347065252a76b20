#!/bin/bash
# Two-size item sweep: big item samples (RT_AMD_BIG_CHUNK) x tail items per resident lane
# (RT_AMD_TAIL_ITEMS) over bench configs and --sim-shards values, binary64 unless PREC is set:
#   bash tools/sweep_items.sh <tag> "<config>:<shards> ..." "<big>:<tail> ..."
export RT_AMD_EXPERIMENTS=1  # the library reads RT_AMD_* knobs / RT_AMD_LIB only with this set
OUT=gpurun_out/$1; mkdir -p $OUT
for rep in 1 2; do
for cfg in $2; do
for bt in $3; do
  n=${cfg%%:*}; sh=${cfg#*:}; big=${bt%%:*}; tail=${bt#*:}
  f=$OUT/${n}_s${sh}_b${big}_t${tail}_r$rep.json
  RT_AMD_BIG_CHUNK=$big RT_AMD_TAIL_ITEMS=$tail timeout -k 10 120 python bench.py --no-cpu-baseline --no-f32 \
    --precision ${PREC:-f64} --config $n --steps 20 --sim-shards $sh > $f 2>>$OUT/err.log || { echo "fail $bt"; exit 1; }
  python3 -c "import json;d=json.load(open('$f'));print('$n shards $sh big $big tail $tail rep $rep', d['roofline']['kernel_ms'], d['ms_per_step'])"
done; done; done
