#!/bin/bash
# run bench.py against each experiment build in raytrace_amd/_lib/exp and print kernel ms
export RT_AMD_EXPERIMENTS=1  # the library reads RT_AMD_* knobs / RT_AMD_LIB only with this set
OUT=gpurun_out/${1:-ablate}; mkdir -p $OUT
ARGS=${ARGS:-"--no-cpu-baseline --steps 5 --warmup 1"}
timeout -k 10 120 python bench.py $ARGS > $OUT/base.json 2>>$OUT/err.log && python3 -c "import json;d=json.load(open('$OUT/base.json'));print('base', d['roofline']['kernel_ms'], d['value'], d['check'])"
for f in raytrace_amd/_lib/exp/*.so; do
  n=$(basename $f .so)
  RT_AMD_LIB=$PWD/$f timeout -k 10 120 python bench.py $ARGS > $OUT/$n.json 2>>$OUT/err.log || { echo "$n failed"; continue; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', d['roofline']['kernel_ms'], d['value'], d['check'])"
done
