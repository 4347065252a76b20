"""ctypes front-end of the host emulator of the kernel logic (TEST TOOLING)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("RT_EMU_LIB") or os.path.join(HERE, "_build", "librt_emu.so")  # env: sanitizer builds (tests/test_sanitizers.py)
_lib = None


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.rt_emu_last_error.restype = ctypes.c_char_p
    return _lib


def render(settings, world, seed, n_shards=1, shard=0, row_block=4, nthreads=None, chunk=0, counters=False,
           precision="f64"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from raytrace_amd import _lib as R
    from raytrace_amd.camera import image_height
    from raytrace_amd.ray import _seed64, shard_rows
    from raytrace_amd.scene import FlatScene, flatten
    flat = world if isinstance(world, FlatScene) else flatten(world)
    cs = R.camera_struct(settings)
    sc = R.scene_struct(flat)
    ex = R.exec_struct(0, n_shards, shard, row_block)
    h = image_height(settings)
    rows = shard_rows(h, n_shards, row_block)
    out = np.zeros((rows, int(settings.cs_imageWidth), 3), np.float64 if precision == "f64" else np.float32)
    L = lib()
    cnt = np.zeros(4, np.int64)
    rc = L.rt_emu_render(ctypes.byref(cs), ctypes.byref(sc), ctypes.c_uint64(_seed64(seed)), ctypes.byref(ex),
                         out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(nthreads or min(16, os.cpu_count() or 1)),
                         ctypes.c_int(chunk), cnt.ctypes.data_as(ctypes.c_void_p),
                         ctypes.c_int(1 if precision == "f64" else 0))
    if rc != 0:
        raise RuntimeError(f"rt_emu_render failed {rc}: {L.rt_emu_last_error().decode()}")
    if counters:
        return out, dict(zip(["bvh_nodes", "prims_tested", "segments", "samples"], cnt.tolist()))
    return out


def scene_info(world):
    """n_nodes, surface_nodes, max_depth, n_prims, flat, box groups, surface-prefix primitives and
    the one-class leaf kind (1 static triangles, 2 static spheres, 0 mixed) of the host build of
    `world`."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from raytrace_amd import _lib as R
    from raytrace_amd.scene import FlatScene, flatten
    flat = world if isinstance(world, FlatScene) else flatten(world)
    sc = R.scene_struct(flat)
    info = np.zeros(8, np.int32)
    rc = lib().rt_emu_scene_info(ctypes.byref(sc), info.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise RuntimeError(f"rt_emu_scene_info failed {rc}: {lib().rt_emu_last_error().decode()}")
    return dict(zip(["n_nodes", "surface_nodes", "max_depth", "n_prims", "flat", "boxes", "prefix", "leaf_kind"], info.tolist()))
