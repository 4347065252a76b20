"""Which depth and spp match the reference's published demo2.png (test/Main.hs:259-321 states only
800 x 800 for it)?  GPU renders of scenes.demo2 at 800 x 800 against tests/golden/demo2_block8.npy
and png_stats.json (the 8-bit sqrt-encoded PNG, decoded), binary64 kernel:

  depth sweep: the quantised image's linear mean and 8x8-block RMSE vs the PNG at a high spp;
  spp estimate: per-pixel RMSE (sqrt-code space) between the PNG and a converged render, against the
  RMSE between two renders of known spp s and different seeds: sigma ~ 1/sqrt(spp), so the PNG's
  spp ~ s (rmse_pair / sqrt(2) / rmse_pub)^2 (the converged render's own noise subtracted).

usage: python tools/demo2_fit.py OUT.jsonl"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import raytrace_amd as R  # noqa: E402
from conftest import as_published, block8  # noqa: E402
from raytrace_amd import scenes  # noqa: E402
from raytrace_amd.core import mkStdGen  # noqa: E402
from raytrace_amd.ray import encode8  # noqa: E402


def main():
    out = open(sys.argv[1], "a")
    gold = np.load(os.path.join(ROOT, "tests", "golden", "demo2_block8.npy")).astype(np.float64)
    with open(os.path.join(ROOT, "tests", "golden", "png_stats.json")) as f:
        pub_mean = np.array(json.load(f)["images"]["demo2"]["linear_mean"])

    def emit(**kw):
        print(json.dumps(kw), flush=True)
        out.write(json.dumps(kw) + "\n")
        out.flush()

    hi_spp = int(os.environ.get("DEMO2_HI_SPP", "2000"))
    for depth in (3, 4, 5, 6, 8, 10, 50):
        cs, world, seed = scenes.demo2(spp=hi_spp, depth=depth)
        t = time.time()
        img = R.raytrace(cs, world, seed)
        dt = time.time() - t
        lin = as_published(img, "sqrt")
        rmse = np.sqrt(((block8(lin) - gold) ** 2).reshape(-1, 3).mean(0))
        emit(kind="depth", depth=depth, spp=hi_spp, seconds=round(dt, 2), mean=lin.reshape(-1, 3).mean(0).tolist(),
             pub_mean=pub_mean.tolist(), block8_rmse=rmse.tolist(), finite=bool(np.isfinite(img).all()))
    # renders for the spp estimate (analysed against demo2.png in the build container, which has
    # the reference: tools/demo2_fit.py --analyse DIR): a converged one and seed pairs of known spp
    d = os.path.join(os.path.dirname(os.path.abspath(sys.argv[1])), "demo2_codes")
    os.makedirs(d, exist_ok=True)
    for depth in [int(x) for x in os.environ.get("DEMO2_DEPTHS", "4,50").split(",")]:
        cs, world, seed = scenes.demo2(spp=hi_spp, depth=depth)
        np.save(os.path.join(d, f"d{depth}_hi.npy"), encode8(R.raytrace(cs, world, seed), "sqrt"))
        for s in (50, 250, 1000):
            for k in (11, 12):
                img = R.raytrace(cs.replace(cs_samplesPerPixel=s), world, mkStdGen(k))
                np.save(os.path.join(d, f"d{depth}_s{s}_k{k}.npy"), encode8(img, "sqrt"))
        emit(kind="saved", depth=depth, dir=d)


def analyse(d):
    """sigma of the PNG against the converged render, vs seed pairs of known spp."""
    from PIL import Image
    pub = np.asarray(Image.open("/root/reference/demo2.png").convert("RGB")).astype(np.float64)
    for depth in (4, 50):
        hi_path = os.path.join(d, f"d{depth}_hi.npy")
        if not os.path.exists(hi_path):
            continue
        hi = np.load(hi_path).astype(np.float64)
        res = {"depth": depth, "rmse_pub_vs_hi": float(np.sqrt(((pub - hi) ** 2).mean()))}
        for s in (50, 250, 1000):
            a = np.load(os.path.join(d, f"d{depth}_s{s}_k11.npy")).astype(np.float64)
            b = np.load(os.path.join(d, f"d{depth}_s{s}_k12.npy")).astype(np.float64)
            res[f"pair_{s}"] = float(np.sqrt(((a - b) ** 2).mean()) / np.sqrt(2))
            res[f"a_vs_hi_{s}"] = float(np.sqrt(((a - hi) ** 2).mean()))
        # the top band (rows 0-199: light, back wall through the fog, the moving sphere) holds no
        # random geometry: there the PNG differs from the converged render by its own noise only
        top = slice(0, 200)
        hi_sig = None
        a = np.load(os.path.join(d, f"d{depth}_s1000_k11.npy")).astype(np.float64)
        b = np.load(os.path.join(d, f"d{depth}_s1000_k12.npy")).astype(np.float64)
        sig1000 = float(np.sqrt(((a[top] - b[top]) ** 2).mean() / 2))
        hi_sig = sig1000 * np.sqrt(1000 / float(os.environ.get("DEMO2_HI_SPP", "2000")))
        pub_hi = float(np.sqrt(((pub[top] - hi[top]) ** 2).mean()))
        sig_pub = float(np.sqrt(max(pub_hi ** 2 - hi_sig ** 2, 1e-9)))
        res.update(top_rmse_pub_vs_hi=pub_hi, top_sigma_1000=sig1000, top_sigma_pub=sig_pub,
                   spp_estimate=round(1000 * (sig1000 / sig_pub) ** 2),
                   top_mean_codes_pub=pub[top].mean((0, 1)).tolist(), top_mean_codes_hi=hi[top].mean((0, 1)).tolist())
        print(json.dumps(res))

if __name__ == "__main__":
    if sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        main()
