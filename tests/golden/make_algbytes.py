"""Freezes SURVEY.md §8(d)'s algorithmic bytes per sample for every config into
tests/golden/algbytes.json (bench.py reads it for `roofline.achieved`).

  B = sum over segments of [ 32 * BVH nodes visited + 16 * spheres tested + 64 * plane shapes tested
                             + 48 * transform entries + 16 * medium entries + 64 * redirect pdf evals
                             + 32 * material/texture records (hits) ] + 12 / spp (framebuffer)

The counts are the REFERENCE's traversal structure (group folds without culling, median-split
bvhTree, transform / medium boundary entries as in Geometry.hs:298-391), measured by the FP64
oracle in splitmix mode at the config's seed.  Full images for configs 1-2; a fixed random
subset of pixels (all samples each) for the larger configs — the figure is a per-sample mean.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from raytrace_amd import scenes  # noqa: E402
from raytrace_amd.camera import image_height  # noqa: E402

WEIGHTS = {"bvh_nodes": 32, "spheres": 16, "planes": 64, "transforms": 48, "media": 16, "redirect_evals": 64,
           "material_hits": 32}


def bytes_per_sample(cnt, spp):
    s = cnt["samples"]
    return sum(WEIGHTS[k] * cnt[k] for k in WEIGHTS) / s + 12.0 / spp


def main():
    out = {"formula": "B = sum_segments[32 nodes + 16 spheres + 64 planes + 48 transforms + 16 media + "
                      "64 redirect evals + 32 material hits] / samples + 12 / spp",
           "source": "oracle/rt_oracle.c splitmix mode (reference traversal structure)", "configs": {}}
    plan = [("readme", scenes.readme_scene, None), ("cornell", scenes.cornell_box, None),
            ("demo1", scenes.demo1, 4000), ("bunny_cornell", scenes.bunny_cornell, 1500),
            ("pawn_fog", scenes.pawn_fog, 800)]
    for name, fn, npix in plan:
        cs, world, seed = fn()
        h = image_height(cs)
        w = cs.cs_imageWidth
        pix = None
        if npix is not None:
            pix = np.sort(np.random.default_rng(7).choice(w * h, npix, replace=False)).astype(np.int32)
        _, cnt = oracle.render(cs, world, seed, mode=oracle.RNG_SPLITMIX, pixels=pix, nthreads=8, counters=True)
        b = bytes_per_sample(cnt, cs.cs_samplesPerPixel)
        out["configs"][name] = {"bytes_per_sample": b, "segments_per_sample": cnt["segments"] / cnt["samples"],
                                "counts": cnt, "pixels": "all" if pix is None else int(npix),
                                "width": w, "height": h, "spp": cs.cs_samplesPerPixel}
        print(name, round(b, 1), cnt, flush=True)
    with open(os.path.join(HERE, "algbytes.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
