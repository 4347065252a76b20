"""TEST TOOLING, run by tests/test_sanitizers.py in a subprocess with a sanitizer runtime
preloaded: renders every scene class through the sanitizer builds of the host scene builder +
kernel logic (tests/kernel_emu) and of the FP64 oracle, plus malformed scenes the builder must
reject with an error code.  Exits non-zero (or the sanitizer aborts) on any finding."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(HERE, "kernel_emu")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import emu  # noqa: E402
import oracle  # noqa: E402
import raytrace_amd as R  # noqa: E402
from raytrace_amd import _lib, scenes  # noqa: E402
from raytrace_amd.scene import flatten  # noqa: E402

emu.build = lambda: None      # the sanitizer .so is prebuilt (make sanitize)
oracle.build = lambda force=False: oracle.LIB_PATH
threads = int(os.environ.get("RT_SAN_THREADS", "4"))

cases = [
    scenes.cornell_box(spp=2, width=24), scenes.readme_scene(spp=2, width=24), scenes.demo1(width=32, spp=1),
    scenes.bunny_cornell(width=16, spp=1), scenes.pawn_fog(width=16, spp=1), scenes.noise_test(width=24, spp=1),
    scenes.box_gallery(width=24, spp=2),
]
tex = R.imageTexture(np.random.default_rng(0).random((8, 16, 3)).astype(np.float32))
cases.append((R.defaultCameraSettings(cs_imageWidth=16, cs_samplesPerPixel=2, cs_background=R.sky),
              R.group([R.lambertian(tex) << R.sphere((0, 0, -2), 0.6),
                       R.metal(0.2, tex) << R.moving((0, 0, 0), (0.3, 0, 0), R.sphere((1, 0, -2), 0.4)),
                       R.dielectric(1.5) << R.transform(R.rotateY(R.degrees(30)),
                                                        R.cuboid(R.fromCorners((-1, -1, -3), (0, 0, -2))))]),
              R.mkStdGen(3)))
for cs, world, seed in cases:
    for prec in ("f64", "f32"):
        img = emu.render(cs, world, seed, nthreads=threads, precision=prec)
        assert np.isfinite(img).all()
    ref = oracle.render(cs, world, seed, mode=oracle.RNG_PHILOX, nthreads=threads)
    assert np.isfinite(ref).all()
    oracle.render(cs, world, seed, mode=oracle.RNG_SPLITMIX, nthreads=threads, pixels=np.arange(0, 64, 3))

# malformed scenes: the builder must answer with an error code, never read out of bounds
cs, world, seed = scenes.cornell_box(spp=1, width=8)
flat = flatten(world)
L = emu.lib()
c = _lib.camera_struct(cs)
out = np.zeros((8, 8, 3))
bad = []
p = flat.prims.copy(); p[0]["material"] = 99; bad.append(p)
p = flat.prims.copy(); p[1]["set"] = 5; bad.append(p)
p = flat.prims.copy(); p[2]["kind"] = 7; bad.append(p)
p = flat.prims.copy(); p[3]["motion"] = 3; bad.append(p)
p = flat.prims.copy(); p[4]["p"][0] = np.nan; bad.append(p)
for p in bad:
    flat.prims = p
    sc = _lib.scene_struct(flat)
    ex = _lib.exec_struct()
    rc = L.rt_emu_render(ctypes.byref(c), ctypes.byref(sc), ctypes.c_uint64(1), ctypes.byref(ex),
                         out.ctypes.data_as(ctypes.c_void_p), 2, 0, None, 1)
    assert rc < 0, rc
print("sanitize ok", len(cases), "scenes")
