"""Determinism check of one library build on the GPU box: renders bunny_instances (FP32, 4 spp,
8 x 8 placements: the instanced kernel class that rendered nondeterministically in a round-5
experiment build) three times with the given library (RT_AMD_LIB, the in-tree one untouched) and
prints the frames' max difference (0 for a deterministic build), the mean and the NaN count.
usage (on the GPU box): python tools/determinism_check.py <lib.so> [precision]"""
import os
import sys

import numpy as np

lib = os.path.abspath(sys.argv[1])
prec = sys.argv[2] if len(sys.argv) > 2 else "f32"
os.environ["RT_AMD_EXPERIMENTS"] = "1"
os.environ["RT_AMD_LIB"] = lib
sys.path.insert(0, os.getcwd())
import ctypes  # noqa: E402

from raytrace_amd import _lib  # noqa: E402

_lib.ABI_VERSION = ctypes.CDLL(lib).rt_abi_version()  # (older builds: rt_render and rt_stats are unchanged since v5)
import raytrace_amd as R  # noqa: E402
from raytrace_amd import scenes  # noqa: E402

cs, w, s = scenes.bunny_instances(spp=4, n=8)
imgs = [R.raytrace(cs, w, s, precision=prec) for _ in range(3)]
d01 = float(np.abs(imgs[0] - imgs[1]).max())
d02 = float(np.abs(imgs[0] - imgs[2]).max())
ndiff = int((np.abs(imgs[0] - imgs[1]).max(-1) > 0).sum())
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/det_" + os.path.basename(lib) + ".npy", imgs[0])
print(os.path.basename(lib), prec, "self-diff", d01, d02, "pixels differing", ndiff, "of", imgs[0].shape[0] * imgs[0].shape[1],
      "mean", float(imgs[0].mean()), "nan", int(np.isnan(imgs[0]).sum()), flush=True)
