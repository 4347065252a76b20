"""Two-level instancing on the GPU: kernel time of bunny_instances (n x n placements of one bunny
object) traced as rt_instances against the same scene with the transforms baked into world
triangles (instance_min=0), both precisions, full 400 x 400 x 64 spp; prints one JSON line per
case."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import raytrace_amd as R  # noqa: E402
from raytrace_amd import scene as S  # noqa: E402
from raytrace_amd import scenes  # noqa: E402

if __name__ == "__main__":
    ns = [int(x) for x in (sys.argv[1:] or ["3", "8"])]
    for n in ns:
        cs, world, seed = scenes.bunny_instances(n=n)
        flats = {"instanced": S.flatten(world), "baked": S.flatten(world, instance_min=0)}
        for prec in ("f64", "f32"):
            imgs = {}
            for kind, flat in flats.items():
                best = None
                for _ in range(3):
                    st = {}
                    t0 = time.time()
                    imgs[kind] = R.raytrace(cs, flat, seed, stats=st, precision=prec)
                    wall = time.time() - t0
                    best = st["kernel_ms"] if best is None else min(best, st["kernel_ms"])
                print(json.dumps({"n": n, "placements": n * n, "kind": kind, "precision": prec,
                                  "prims": len(flat.prims), "instances": len(flat.instances),
                                  "kernel_ms": round(best, 3), "wall_s": round(wall, 3),
                                  "mean": imgs[kind].reshape(-1, 3).mean(0).tolist()}), flush=True)
            a, b = imgs["instanced"].astype(np.float64), imgs["baked"].astype(np.float64)
            rel = (np.abs(a - b) / np.maximum(np.abs(b), 1e-3)).max(-1)
            print(json.dumps({"n": n, "precision": prec, "instanced_vs_baked_frac_le_1e-9": float((rel <= 1e-9).mean()),
                              "frac_le_1e-3": float((rel <= 1e-3).mean())}), flush=True)
