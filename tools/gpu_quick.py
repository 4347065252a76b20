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
    t0 = time.time()
    st = {}
    g = R.raytrace(cs, world, seed, stats=st)
    t1 = time.time()
    o = oracle.render(cs, world, seed, mode=oracle.RNG_PHILOX)
    t2 = time.time()
    d = np.abs(g.astype(np.float64) - o)
    rel = d / np.maximum(1.0, np.abs(o))
    close = (rel.max(-1) < 1e-3).mean()
    print(f"{name}: {g.shape} gpu {t1 - t0:.2f}s (kernel {st['kernel_ms']:.2f} ms) oracle {t2 - t1:.2f}s "
          f"close(1e-3)={close:.4f} max={rel.max():.3g} mean gpu={g.reshape(-1, 3).mean(0)} "
          f"oracle={o.reshape(-1, 3).mean(0)}", flush=True)
    return close


if __name__ == "__main__":
    res = {}
    res["cornell"] = compare("cornell", *scenes.cornell_box(spp=16, width=96))
    res["readme"] = compare("readme", *scenes.readme_scene(spp=16, width=120))
    res["demo1"] = compare("demo1", *scenes.demo1(width=120, spp=8))
    res["bunny"] = compare("bunny", *scenes.bunny_cornell(width=64, spp=8))
    res["pawn_fog"] = compare("pawn_fog", *scenes.pawn_fog(width=64, spp=8))
    # full-size Cornell timing
    cs, world, seed = scenes.cornell_box()
    st = {}
    for _ in range(2):
        img = R.raytrace(cs, world, seed, stats=st)
    ms = st["kernel_ms"]
    print(f"cornell 600x600x200: kernel {ms:.2f} ms -> {600 * 600 * 200 / ms / 1e3:.1f} Msamples/s, "
          f"mean {img.reshape(-1, 3).mean(0)}", flush=True)
    print("RESULT", res)
