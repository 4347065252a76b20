#!/bin/bash
# bench.py at several work-item sizes (RT_AMD_CHUNK samples per item); prints kernel ms
OUT=gpurun_out/${1:-chunks}; mkdir -p $OUT
for c in ${CHUNKS:-0 8 17 34 50 100 200}; do
  if [ "$c" = 0 ]; then unset RT_AMD_CHUNK; else export RT_AMD_CHUNK=$c; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 $BARGS > $OUT/c$c.json 2>>$OUT/err.log || { echo "chunk $c failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c$c.json'));print('chunk $c', d['roofline']['kernel_ms'], d['value'])"
done
