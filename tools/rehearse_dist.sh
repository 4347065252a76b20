#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: N ranks on device 0, gloo gathers through host
# memory (RCCL refuses two ranks on one GPU).  Checks the assembled frame against N=1.
OUT=gpurun_out/${1:-rehearse}; mkdir -p $OUT
N=${N:-2}
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --check > $OUT/n1.json 2> $OUT/n1.err || { echo "n1 failed"; tail -5 $OUT/n1.err; exit 1; }
RT_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus $N --steps 3 --warmup 1 --check --dist-backend gloo \
  > $OUT/n$N.json 2> $OUT/n$N.err || { echo "n$N failed"; tail -20 $OUT/n$N.err; exit 1; }
python3 - "$OUT" "$N" <<'PY'
import json, sys
out, n = sys.argv[1], sys.argv[2]
a = json.loads(open(f"{out}/n1.json").read().strip().splitlines()[-1])
b = json.loads(open(f"{out}/n{n}.json").read().strip().splitlines()[-1])
print("n1", a["value"], a["check"]); print(f"n{n}", b["value"], b["n_gpus"], b["check"], b["config"]["parallelism"])
assert b["n_gpus"] == int(n) and b["check"]["finite"] and b["check"]["mean_rgb"] == a["check"]["mean_rgb"], "mismatch"
print("rehearsal ok")
PY
