"""Perlin tables of Graphics.Ray.Noise (Noise.hs:21-92) for the device's noise / marble textures.

* The three fixed permutations permX / permY / permZ are data (`data/perlin_perm.json`,
  extracted from Noise.hs:60-92 by tools/extract_perlin_perm.py).
* The 256 gradients are `evalState (replicateM 256 randomUnitVector) (mkStdGen 666)`
  (Noise.hs:94-98): rejection-sampled unit vectors (Core.hs:54-60) from the splitmix StdGen
  restated in core.py.  Bitwise agreement with the reference's stream is unpinned offline (the
  splitmix restatement is pinned statistically only); tests check it against the
  oracle's independent C restatement.
"""
from __future__ import annotations

import functools
import json
import math
import os

import numpy as np

from .core import mkStdGen

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "perlin_perm.json")


@functools.lru_cache(maxsize=1)
def permutations() -> np.ndarray:
    with open(_DATA) as f:
        d = json.load(f)
    return np.array([d["permX"], d["permY"], d["permZ"]], dtype=np.int32)


def random_unit_vector(gen):
    """randomUnitVector (Core.hs:54-60): V3 ~ randomR (-1, 1) until 1e-8 <= |v|^2 <= 1."""
    while True:
        x, gen = gen.randomR(-1.0, 1.0)
        y, gen = gen.randomR(-1.0, 1.0)
        z, gen = gen.randomR(-1.0, 1.0)
        q = x * x + y * y + z * z
        if 1e-8 <= q <= 1:
            s = math.sqrt(q)
            return (x / s, y / s, z / s), gen


@functools.lru_cache(maxsize=1)
def gradients() -> np.ndarray:
    gen = mkStdGen(666)
    out = np.zeros((256, 3), np.float64)
    for k in range(256):
        out[k], gen = random_unit_vector(gen)
    return out


# include/rt.h rt_perlin
PERLIN_DTYPE = np.dtype([("perm", "<i4", (3, 256)), ("grad", "<f8", (256, 3))], align=True)


def perlin_record() -> np.ndarray:
    rec = np.zeros(1, PERLIN_DTYPE)
    rec[0]["perm"] = permutations()
    rec[0]["grad"] = gradients()
    return rec
