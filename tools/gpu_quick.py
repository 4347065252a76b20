"""Quick GPU sanity check: render small versions of each config on the GPU and compare them
per pixel with the FP64 oracle's Philox mode (same random numbers)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
import raytrace_amd as R  # noqa: E402
from raytrace_amd import scenes  # noqa: E402


def compare(name, cs, world, seed):
    o = oracle.render(cs, world, seed, mode=oracle.RNG_PHILOX)
    out = {}
    for prec in ("f64", "f32"):
        t0 = time.time()
        st = {}
        g = R.raytrace(cs, world, seed, stats=st, precision=prec)
        t1 = time.time()
        d = np.abs(g.astype(np.float64) - o)
        if prec == "f64":
            rel = (d / np.maximum(np.abs(o), 1e-3)).max(-1)
            close = float((rel <= 1e-9).mean())
            tag = "<=1e-9 rel"
        else:
            rel = (d / np.maximum(1.0, np.abs(o))).max(-1)
            close = float((rel < 1e-3).mean())
            tag = "<1e-3"
        print(f"{name} {prec}: {g.shape} gpu {t1 - t0:.2f}s (kernel {st['kernel_ms']:.2f} ms) close({tag})={close:.5f} "
              f"max={rel.max():.3g} mean gpu={g.reshape(-1, 3).mean(0)} oracle={o.reshape(-1, 3).mean(0)}", flush=True)
        out[prec] = close
    return out


if __name__ == "__main__":
    res = {}
    res["cornell"] = compare("cornell", *scenes.cornell_box(spp=16, width=96))
    res["readme"] = compare("readme", *scenes.readme_scene(spp=16, width=120))
    res["demo1"] = compare("demo1", *scenes.demo1(width=120, spp=8))
    res["bunny"] = compare("bunny", *scenes.bunny_cornell(width=64, spp=8))
    res["pawn_fog"] = compare("pawn_fog", *scenes.pawn_fog(width=64, spp=8))
    cs, world, seed = scenes.cornell_box(spp=4, width=50)
    a = R.raytrace(cs, world, seed)
    for devs in ([0, 0], [0, 0, 0]):
        b = R.raytrace(cs, world, seed, devices=devs, row_block=1)
        print(f"device list {devs}: bit-identical={np.array_equal(a, b)}", flush=True)
