"""Bit-identity of two kernel builds: render configs with the in-tree library and with an
experiment library (RT_AMD_LIB), each in its own child process, and compare the images.

usage (GPU box): python tools/image_ab.py raytrace_amd/_lib/exp/librt_amd_X.so [out.json]
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (scene, kwargs): full resolution, reduced samples per pixel
# (the 128-spp cases split each pixel into 32+ items: the kernels' commit aggregation is active)
CASES = [("cornell_box", {"spp": 8}), ("bunny_cornell", {"spp": 4}), ("demo1", {"spp": 4}),
         ("pawn_fog", {"spp": 2}), ("bunny_instances", {}), ("box_gallery", {}),
         ("cornell_box", {"spp": 128}), ("bunny_cornell", {"spp": 128}), ("pawn_fog", {"spp": 128})]


def _tag(name, kw):
    return name + "".join(f"_{k}{v}" for k, v in sorted(kw.items()))


def child(out_dir):
    sys.path.insert(0, ROOT)
    import raytrace_amd as R
    from raytrace_amd import scenes
    for name, kw in CASES:
        cs, world, seed = getattr(scenes, name)(**kw)
        for prec in ("f64", "f32"):
            np.save(os.path.join(out_dir, f"{_tag(name, kw)}_{prec}.npy"),
                    R.raytrace(cs, world, seed, device=0, precision=prec))


def main():
    exp_lib, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/image_ab.json")
    dirs = {}
    for tag, lib in (("base", None), ("exp", exp_lib)):
        d = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"image_ab_{tag}")  # images stay off gpurun_out/
        os.makedirs(d, exist_ok=True)
        env = dict(os.environ, RT_AMD_EXPERIMENTS="1")
        env.pop("RT_AMD_LIB", None)
        if lib:
            env["RT_AMD_LIB"] = os.path.abspath(lib)
        subprocess.run([sys.executable, __file__, "--child", d], check=True, env=env, timeout=600)
        dirs[tag] = d
    res = {}
    for name, kw in CASES:
        name = _tag(name, kw)
        for prec in ("f64", "f32"):
            a = np.load(os.path.join(dirs["base"], f"{name}_{prec}.npy"))
            b = np.load(os.path.join(dirs["exp"], f"{name}_{prec}.npy"))
            same = np.array_equal(a, b, equal_nan=True)
            diff = np.abs(a - b).max(-1)
            res[f"{name}_{prec}"] = {"bit_identical": bool(same), "pixels_differing": int((diff != 0).sum()),
                                     "pixels": int(diff.size), "max_abs_diff": float(np.nanmax(diff))}
            print(name, prec, res[f"{name}_{prec}"], flush=True)
    with open(out, "w") as f:
        json.dump({"exp_lib": exp_lib, "cases": res}, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
