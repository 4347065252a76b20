"""Determinism check of one library build on the GPU box: installs the given librt_amd.so over the
in-tree one (the box's copy is scratch), renders bunny_instances (FP32, 4 spp, 8 x 8 placements)
three times and prints the frames' max difference (0 for a deterministic build) and mean.
usage (on the GPU box): python tools/determinism_check.py <lib.so>"""
import ctypes, os, sys, shutil, numpy as np
sys.path.insert(0, os.getcwd())
lib = sys.argv[1]
shutil.copy(lib, "raytrace_amd/_lib/librt_amd.so")
import raytrace_amd as R
from raytrace_amd import scenes
cs, w, s = scenes.bunny_instances(spp=4, n=8)
imgs = [R.raytrace(cs, w, s, precision="f32") for _ in range(3)]
d01 = float(np.abs(imgs[0] - imgs[1]).max()); d02 = float(np.abs(imgs[0] - imgs[2]).max())
np.save("gpurun_out/dbg_" + os.path.basename(lib) + ".npy", imgs[0])
print(os.path.basename(lib), "self-diff", d01, d02, "mean", imgs[0].mean(), "nan", int(np.isnan(imgs[0]).sum()))
