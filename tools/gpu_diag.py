import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import raytrace_amd as R
from raytrace_amd import scenes
for name, f in [("demo1_120", lambda: scenes.demo1(width=120, spp=8)), ("demo1_160", lambda: scenes.demo1(width=160, spp=8)),
                ("bunny", lambda: scenes.bunny_cornell(width=80, spp=8)), ("pawn_fog", lambda: scenes.pawn_fog(width=80, spp=8))]:
    cs, w, s = f()
    st = {}
    img = R.raytrace(cs, w, s, stats=st)
    print(name, img.shape, np.isfinite(img).all(), img.reshape(-1, 3).mean(0), st, flush=True)
    time.sleep(1)
    print("after sleep", flush=True)
