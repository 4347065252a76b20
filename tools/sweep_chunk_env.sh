#!/bin/bash
# Item chunk sweep (RT_AMD_CHUNK) over bench configs and --sim-shards values:
#   bash tools/sweep_chunk_env.sh "<config>:<shards> ..." "<chunk> ..."
export RT_AMD_EXPERIMENTS=1  # the library reads RT_AMD_* knobs / RT_AMD_LIB only with this set
OUT=gpurun_out/chunk; mkdir -p $OUT
for rep in 1 2; do
for cfg in $1; do
for c in $2; do
  n=${cfg%%:*}; sh=${cfg#*:}
  RT_AMD_CHUNK=$c timeout -k 10 120 python bench.py --no-cpu-baseline --config $n --steps 20 --sim-shards $sh > $OUT/${n}_c${c}_s${sh}_r$rep.json 2>>$OUT/err.log || { echo fail $c; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/${n}_c${c}_s${sh}_r$rep.json'));print('$n chunk $c shards $sh rep $rep', d['roofline']['kernel_ms'], d['ms_per_step'])"
done; done; done
