#!/bin/bash
# One rank's share of an N-GPU frame (bench.py --sim-shards N, one process, binary64) for N = 1, 2,
# 4, 8 on Cornell, bunny-Cornell and pawn+fog: bash tools/shard_share_sweep.sh <tag>
# The expected N-GPU speed-up of a config is t(1) / t(N) of these kernel times before the
# gather and launch costs.  env: CFGS="cornell:20 bunny_cornell:5 pawn_fog:3" (config:steps)
O=gpurun_out/${1:-shards}; mkdir -p $O
for cs in ${CFGS:-cornell:20 bunny_cornell:5 pawn_fog:3}; do
  c=${cs%%:*}; st=${cs#*:}
  for s in 1 2 4 8; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-f32 --steps $st --sim-shards $s \
      > $O/${c}_sim_shards_$s.json 2>>$O/err.log || exit 1
  done
done
python3 - $O <<'PY'
import glob, json, os, sys
rows = {}
for f in sorted(glob.glob(sys.argv[1] + "/*_sim_shards_*.json")):
    c, n = os.path.basename(f)[:-5].rsplit("_sim_shards_", 1)
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault(c, {})[int(n)] = d["roofline"]["kernel_ms"]
for c, t in rows.items():
    print(c, " ".join(f"N={n}: {t[n]:.3f} ms (x{t[1] / t[n]:.2f})" for n in sorted(t)))
PY
