#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box through the driver's own entry point
# (`python bench.py --gpus N`, which starts the N ranks itself): RT_BENCH_ONE_DEVICE=1 maps every
# rank to device 0 and the gather goes through gloo (RCCL refuses two ranks on one GPU).  The
# assembled frame must be bit-identical (sha16 of its bytes) to the N=1 frame.
# usage: bash tools/rehearse_dist.sh <tag> [config]     env: NS="2 3"
OUT=gpurun_out/${1:-rehearse}; mkdir -p $OUT
CFG=${2:-cornell}
export TMPDIR=/tmp
ARGS="--config $CFG --steps 3 --warmup 1 --warmup-s 0.2 --no-cpu-baseline --no-f32"
timeout -k 10 300 python bench.py $ARGS > $OUT/n1.json 2> $OUT/n1.err || { echo "n1 failed"; tail -5 $OUT/n1.err; exit 1; }
for N in ${NS:-2 3}; do
  RT_BENCH_ONE_DEVICE=1 timeout -k 10 300 python bench.py --gpus $N $ARGS > $OUT/n$N.json 2> $OUT/n$N.err || { echo "n$N failed"; tail -20 $OUT/n$N.err; exit 1; }
done
python3 - "$OUT" ${NS:-2 3} <<'PY'
import json, sys
out, ns = sys.argv[1], sys.argv[2:]
a = json.loads(open(f"{out}/n1.json").read().strip().splitlines()[-1])
print("n1", a["value"], a["check"])
for n in ns:
    b = json.loads(open(f"{out}/n{n}.json").read().strip().splitlines()[-1])
    ab = b.get("abi_device_list") or {}
    print(f"n{n}", b["value"], b["n_gpus"], b["check"], b["config"]["parallelism"])
    print(f"  abi_device_list {ab.get('devices')} {ab.get('ms_per_frame')} ms/frame, sha16 {ab.get('sha16')}, "
          f"allocs {ab.get('device_allocs_timed')}")
    assert b["n_gpus"] == int(n) and b["check"]["finite"] and b["check"]["sha16"] == a["check"]["sha16"], "mismatch"
    assert ab.get("sha16") == a["check"]["sha16"] and ab.get("device_allocs_timed") == 0, "abi device list"
print("rehearsal ok: frames bit-identical to N=1")
PY
