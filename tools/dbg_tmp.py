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
