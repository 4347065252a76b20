"""ctypes front-end of the FP64 oracle (oracle/rt_oracle.c).  TEST INFRASTRUCTURE ONLY:
imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_ORACLE_LIB") or os.path.join(HERE, "_build", "librt_oracle.so")  # env: sanitizer builds (tests/test_sanitizers.py)

RNG_SPLITMIX = 0
RNG_PHILOX = 1

COUNTER_NAMES = ["segments", "bvh_nodes", "spheres", "planes", "transforms", "media", "redirect_evals",
                 "material_hits", "samples"]

_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (idempotent; make decides)."""
    cmd = ["make", "-C", HERE, "-s"]
    if force:
        cmd.append("-B")
    subprocess.run(cmd, check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, P, P, P, P, P, P, P, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, P, ctypes.c_int, ctypes.c_int,
                                    P, P, P, P, P]
        L.oracle_philox.argtypes = [P, P, P]
        L.oracle_perlin_gradients.argtypes = [P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def camera_arrays(cs):
    """CameraSettings -> (cam_d[19], cam_i[5], targets[n,10])."""
    from raytrace_amd.camera import background_of
    bg = background_of(cs)
    cam_d = np.zeros(19, np.float64)
    cam_d[0:3] = cs.cs_center
    cam_d[3:6] = cs.cs_lookAt
    cam_d[6:9] = cs.cs_up
    cam_d[9] = cs.cs_vfov
    cam_d[10] = cs.cs_aspectRatio
    cam_d[11] = cs.cs_defocusAngle
    cam_d[12] = cs.cs_focusDist
    cam_d[13:16] = bg.c0
    cam_d[16:19] = bg.c1
    nt = len(cs.cs_redirectTargets)
    cam_i = np.array([cs.cs_imageWidth, cs.cs_samplesPerPixel, cs.cs_maxRecursionDepth, bg.kind, nt], np.int32)
    tg = np.zeros((max(nt, 1), 10), np.float64)
    for k, (p, q, u, v) in enumerate(cs.cs_redirectTargets):
        tg[k] = [p, *q, *u, *v]
    return cam_d, cam_i, tg


def render(cs, world, seed, mode=RNG_PHILOX, pixels=None, nthreads=None, variant=0, counters=False):
    """Render `pixels` (linear row-major indices; default all) with the oracle.

    seed: a raytrace_amd.core.StdGen.  Philox mode keys the stream with seed.key(), exactly
    as the device path does.  Returns float64 (n, 3) — or (h, w, 3) when pixels is None.
    """
    from raytrace_amd.camera import image_height
    from raytrace_amd.scene import serialize_tree
    t = serialize_tree(world)
    cam_d, cam_i, tg = camera_arrays(cs)
    w = int(cs.cs_imageWidth)
    h = image_height(cs)
    full = pixels is None
    if full:
        pixels = np.arange(w * h, dtype=np.int32)
    pixels = np.ascontiguousarray(pixels, dtype=np.int32)
    out = np.zeros((len(pixels), 3), np.float64)
    cnt = np.zeros(16, np.float64)
    mat_i = np.zeros((max(len(t.materials), 1), 4), np.int32)
    mat_d = np.zeros((max(len(t.materials), 1), 2), np.float64)
    for k, m in enumerate(t.materials):
        mat_i[k, 0] = m["kind"]
        mat_i[k, 1] = m["texture"]
        mat_d[k, 0] = m["param"]
    tex_i = np.zeros((max(len(t.textures), 1), 4), np.int32)
    tex_d = np.zeros((max(len(t.textures), 1), 14), np.float64)
    for k, x in enumerate(t.textures):
        tex_i[k] = [x["kind"], x["nu"], x["nv"], x["image"]]
        tex_d[k, 0:3] = x["c0"]
        tex_d[k, 3:6] = x["c1"]
        tex_d[k, 6:14] = x["params"]
    texels = np.ascontiguousarray(t.texels, dtype=np.float32).reshape(-1, 3)
    if len(texels) == 0:
        texels = np.zeros((1, 3), np.float32)
    if t.perlin is not None:
        perm = np.ascontiguousarray(t.perlin[0]["perm"], dtype=np.int32)
        grad = np.ascontiguousarray(t.perlin[0]["grad"], dtype=np.float64)
    else:
        perm = np.zeros((3, 256), np.int32)
        grad = np.zeros((256, 3), np.float64)
    if mode == RNG_SPLITMIX:
        sa, sb = seed.seed, seed.gamma
    else:
        sa, sb = seed.key(), 0
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    ni = np.ascontiguousarray(t.node_i)
    nd = np.ascontiguousarray(t.node_d)
    rc = lib().oracle_render(_ptr(ni), _ptr(nd), len(ni), t.root, _ptr(t.children), _ptr(mat_i), _ptr(mat_d),
                             _ptr(tex_i), _ptr(tex_d), _ptr(cam_d), _ptr(cam_i), _ptr(tg), mode, variant, sa, sb,
                             _ptr(pixels), len(pixels), nthreads, _ptr(out), _ptr(cnt), _ptr(texels), _ptr(perm),
                             _ptr(grad))
    if rc < 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    res = out.reshape(h, w, 3) if full else out
    if counters:
        return res, dict(zip(COUNTER_NAMES, cnt[: len(COUNTER_NAMES)].tolist()))
    return res


def philox(ctr, key):
    c = np.array(ctr, np.uint32)
    k = np.array(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().oracle_philox(_ptr(c), _ptr(k), _ptr(o))
    return o


if __name__ == "__main__":
    build(force="-B" in sys.argv)
    print(LIB_PATH)


def perlin_gradients():
    """The oracle's restatement of Noise.hs:94-98 (256 x 3)."""
    out = np.zeros((256, 3), np.float64)
    lib().oracle_perlin_gradients(_ptr(out))
    return out
