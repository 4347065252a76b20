"""Generates tests/golden/* from the reference's committed renders (run in the build
container only; /root/reference does not exist on the GPU box).

Fixtures written (all data, no reference source):
  png_stats.json          per-image linear means, encoding, quantisation model
  <name>_block8.npy       8x8-block means of the decoded linear image (float32)
  noise_floor.json        seed-to-seed 8x8-block RMSE of the FP64 oracle at the reference spp
                          (oracle splitmix mode, seeds 234/235 and 100/101)
  demo1_worlds.json       (--demo1) the spread of demo1's published-image mean over WORLD seeds:
                          the reference built demo1's world from newStdGen (test/Main.hs:184-185),
                          so only statistics that do not depend on the world's draw can be pinned;
                          the FP64 oracle (splitmix) renders worlds 1..8 at 320x180, 64 spp, each
                          quantised as writeImageSqrt stores it
  demo2_worlds.json       (--demo2) the same for demo2 (test/Main.hs:259-321): its world IS seeded
                          (mkStdGen 1234) but the published demo2.png's random ground boxes and
                          ball cluster are not the ones the restated generator draws (an earlier
                          revision of the code, like the other PNGs), so its mean is
                          pinned against the spread over world seeds 1..8 (oracle, splitmix,
                          160x160, 64 spp, depth 50)

Decoding model (measured on pawn_demo.png's background, whose linear value is analytic):
the 8-bit code v of a value x in [0,1] is min(255, floor(256 x)) after the transfer
function (sRGB for `writeImage`, sqrt for `writeImageSqrt`, Ray.hs:248-260), so the
decoder maps v to the bin centre (v + 0.5) / 256 before inverting the transfer function.
"""
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))

IMAGES = {
    # name: (file, encoding, producing code)
    "example_image": ("example_image.png", "srgb", "README.md:33-61 (seed 100, 600x338, 50 spp, depth 10)"),
    "cornell_box_redirect": ("cornell_box_redirect.png", "sqrt", "test/Main.hs:188-218 cornellBox 200 50 (seed 234)"),
    "cornell_box_noisy": ("cornell_box_noisy.png", "sqrt", "same with cs_redirectTargets = [] (README.md:71)"),
    "demo1": ("demo1.png", "sqrt", "test/Main.hs:136-186 (world from newStdGen: not reproducible)"),
    "pawn_demo": ("pawn_demo.png", "srgb", "test/Main.hs:323-344 (seed 55, 500x500, 400 spp, depth 20)"),
    "demo2": ("demo2.png", "sqrt", "test/Main.hs:259-321 demo2 (world from mkStdGen 1234; 800x800, spp and depth "
                                   "not stated)"),
}


def decode(codes, encoding):
    x = (codes.astype(np.float64) + 0.5) / 256.0
    if encoding == "sqrt":
        return x * x
    return np.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055) ** 2.4)


def block8(a, b=8):
    h, w, _ = a.shape
    return a[: h // b * b, : w // b * b].reshape(h // b, b, w // b, b, 3).mean((1, 3))


def main():
    stats = {"quantisation": "code = min(255, floor(256 * transfer(clamp01(x))))", "images": {}}
    for name, (fn, enc, src) in IMAGES.items():
        codes = np.asarray(Image.open(os.path.join(REF, fn)).convert("RGB"))
        lin = decode(codes, enc)
        stats["images"][name] = {
            "file": fn, "encoding": enc, "source": src, "height": int(codes.shape[0]), "width": int(codes.shape[1]),
            "linear_mean": lin.reshape(-1, 3).mean(0).tolist(),
            "saturated_fraction": float((codes.max(-1) == 255).mean()),
        }
        np.save(os.path.join(HERE, f"{name}_block8.npy"), block8(lin).astype(np.float32))
    with open(os.path.join(HERE, "png_stats.json"), "w") as f:
        json.dump(stats, f, indent=1)
    if "--noise" in sys.argv:
        import oracle
        from raytrace_amd import scenes
        from raytrace_amd.core import mkStdGen
        floors = {}
        for name, fn_scene, enc, seeds in [("cornell_box_redirect", scenes.cornell_box, "sqrt", (234, 235)),
                                           ("example_image", scenes.readme_scene, "srgb", (100, 101))]:
            cs, world, _ = fn_scene()
            imgs = []
            for s in seeds:
                out = oracle.render(cs, world, mkStdGen(s), mode=oracle.RNG_SPLITMIX, nthreads=8)
                x = np.clip(out, 0, 1)
                t = np.sqrt(x) if enc == "sqrt" else np.where(x <= 0.0031308, 12.92 * x, 1.055 * x ** (1 / 2.4) - 0.055)
                imgs.append(decode(np.minimum(np.floor(t * 256), 255), enc))
            d = block8(imgs[0]) - block8(imgs[1])
            floors[name] = {"block8_rmse": np.sqrt((d ** 2).reshape(-1, 3).mean(0)).tolist(), "seeds": list(seeds),
                            "oracle_mode": "splitmix"}
        with open(os.path.join(HERE, "noise_floor.json"), "w") as f:
            json.dump(floors, f, indent=1)
    if "--demo1" in sys.argv:
        import oracle
        from raytrace_amd import scenes
        from raytrace_amd.core import mkStdGen
        means = []
        for w in range(1, 9):
            cs, world, seed = scenes.demo1(width=320, spp=64, seed=w)
            out = oracle.render(cs, world, seed, mode=oracle.RNG_SPLITMIX, nthreads=os.cpu_count())
            t = np.sqrt(np.clip(out, 0, 1))
            lin = decode(np.minimum(np.floor(t * 256), 255), "sqrt")
            means.append(lin.reshape(-1, 3).mean(0).tolist())
            print("world", w, means[-1], flush=True)
        m = np.array(means)
        with open(os.path.join(HERE, "demo1_worlds.json"), "w") as f:
            json.dump({"world_seeds": list(range(1, 9)), "width": 320, "height": 180, "spp": 64, "depth": 50,
                       "oracle_mode": "splitmix", "quantised_linear_mean": means,
                       "mean_over_worlds": m.mean(0).tolist(), "std_over_worlds": m.std(0, ddof=1).tolist()}, f,
                      indent=1)
    if "--demo2" in sys.argv:
        import oracle
        from raytrace_amd import scenes
        from raytrace_amd.core import mkStdGen
        means = []
        earth = scenes.earthmap()
        for w in range(1, 9):
            world, gen2 = scenes.demo2_world(mkStdGen(w), earth)
            cs, _, _ = scenes.demo2(width=160, spp=64, depth=50)
            out = oracle.render(cs, world, gen2, mode=oracle.RNG_SPLITMIX, nthreads=os.cpu_count())
            t = np.sqrt(np.clip(out, 0, 1))
            lin = decode(np.minimum(np.floor(t * 256), 255), "sqrt")
            means.append(lin.reshape(-1, 3).mean(0).tolist())
            print("world", w, means[-1], flush=True)
        m = np.array(means)
        with open(os.path.join(HERE, "demo2_worlds.json"), "w") as f:
            json.dump({"world_seeds": list(range(1, 9)), "width": 160, "height": 160, "spp": 64, "depth": 50,
                       "oracle_mode": "splitmix", "quantised_linear_mean": means,
                       "mean_over_worlds": m.mean(0).tolist(), "std_over_worlds": m.std(0, ddof=1).tolist()}, f,
                      indent=1)
    print("ok")


if __name__ == "__main__":
    main()
