"""Nondeterminism probe (diagnostic, GPU box): renders bunny_instances (FP32, 4 spp, n=8) three times
with the library given as argv[1] under each RT_AMD_* knob set in argv[2:] ("base" = none), and
prints per setting the max frame-to-frame difference and the count of differing pixels.
Each setting runs in a child process (the library reads its knobs at scene creation)."""
import json
import os
import subprocess
import sys

CHILD = r'''
import os, sys, shutil, numpy as np
sys.path.insert(0, os.getcwd())
shutil.copy(sys.argv[1], "raytrace_amd/_lib/librt_amd.so")
import raytrace_amd as R
from raytrace_amd import scenes
cs, w, s = scenes.bunny_instances(spp=4, n=8)
imgs = [R.raytrace(cs, w, s, precision="f32") for _ in range(3)]
d = np.abs(imgs[0] - imgs[1]).max(axis=2)
print(float(d.max()), int((d > 0).sum()), float(np.abs(imgs[0] - imgs[2]).max()))
'''

if __name__ == "__main__":
    lib, sets = sys.argv[1], sys.argv[2:] or ["base"]
    for st in sets:
        env = dict(os.environ, RT_AMD_EXPERIMENTS="1")
        if st != "base":
            for kv in st.split(","):
                k, v = kv.split("=")
                env[k] = v
        r = subprocess.run([sys.executable, "-c", CHILD, lib], env=env, capture_output=True, text=True, timeout=200)
        print(json.dumps({"lib": os.path.basename(lib), "set": st, "out": r.stdout.strip(), "rc": r.returncode,
                          "err": r.stderr.strip()[-300:] if r.returncode else ""}), flush=True)
