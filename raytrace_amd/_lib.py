"""ctypes binding of librt_amd.so (include/rt.h).  The product path has NO CPU fallback: if
the HIP library is missing or fails to load, every render raises RtDeviceError."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .errors import RtDeviceError, RtError, RtInvalid, RtUnsupported

HERE = os.path.dirname(os.path.abspath(__file__))
# RT_AMD_LIB (an experiment build of the library) is honoured only with RT_AMD_EXPERIMENTS set, like
# the library's own RT_AMD_* knobs (rt_internal.h rt_knob)
_EXPERIMENTS = os.environ.get("RT_AMD_EXPERIMENTS", "0") not in ("", "0")
LIB_PATH = (_EXPERIMENTS and os.environ.get("RT_AMD_LIB")) or os.path.join(HERE, "_lib", "librt_amd.so")

RT_OK, RT_E_GENERIC, RT_E_INVALID, RT_E_UNSUPPORTED, RT_E_HIP, RT_E_STACK = 0, -1, -2, -3, -4, -5

EXPORTED = ["rt_abi_version", "rt_last_error", "rt_device_count", "rt_image_height", "rt_shard_rows", "rt_shard_row", "rt_render",
            "rt_scene_create", "rt_scene_destroy", "rt_scene_stats", "rt_render_async", "rt_encode8_async",
            "rt_multi_scene_create", "rt_multi_scene_destroy", "rt_multi_render"]


class RtRedirectTarget(ctypes.Structure):
    _fields_ = [("prob", ctypes.c_double), ("q", ctypes.c_double * 3), ("u", ctypes.c_double * 3),
                ("v", ctypes.c_double * 3)]


class RtCameraSettings(ctypes.Structure):
    _fields_ = [
        ("center", ctypes.c_double * 3), ("look_at", ctypes.c_double * 3), ("up", ctypes.c_double * 3),
        ("vfov", ctypes.c_double), ("aspect_ratio", ctypes.c_double),
        ("image_width", ctypes.c_int32), ("samples_per_pixel", ctypes.c_int32),
        ("max_recursion_depth", ctypes.c_int32), ("background_kind", ctypes.c_int32),
        ("background_c0", ctypes.c_double * 3), ("background_c1", ctypes.c_double * 3),
        ("defocus_angle", ctypes.c_double), ("focus_dist", ctypes.c_double),
        ("n_redirect_targets", ctypes.c_int32), ("pad", ctypes.c_int32),
        ("redirect_targets", ctypes.POINTER(RtRedirectTarget)),
    ]


class RtScene(ctypes.Structure):
    _fields_ = [
        ("n_prims", ctypes.c_int32), ("prims", ctypes.c_void_p),
        ("n_media", ctypes.c_int32), ("media", ctypes.c_void_p),
        ("n_materials", ctypes.c_int32), ("materials", ctypes.c_void_p),
        ("n_textures", ctypes.c_int32), ("textures", ctypes.c_void_p),
        ("n_motions", ctypes.c_int32), ("motions", ctypes.c_void_p),
        ("n_uvframes", ctypes.c_int32), ("uvframes", ctypes.c_void_p),
        ("n_texels", ctypes.c_int32), ("texels", ctypes.c_void_p),
        ("perlin", ctypes.c_void_p),
        ("n_instances", ctypes.c_int32), ("instances", ctypes.c_void_p),
    ]


RT_EXEC_F32 = 1  # rt_exec.flags: FP32 kernel, float output (default: binary64, double output)
RT_EXEC_ENCODE8_SRGB = 2  # rt_render output: uint8 codes of writeImage (sRGB)
RT_EXEC_ENCODE8_SQRT = 4  # rt_render output: uint8 codes of writeImageSqrt
RT_EXEC_SOLO = 8  # rt_render_async: the render runs alone (planned for a short end, as rt_render's)
ENCODINGS = {None: 0, "srgb": RT_EXEC_ENCODE8_SRGB, "sqrt": RT_EXEC_ENCODE8_SQRT}
ABI_VERSION = 6
PRECISIONS = {"f64": np.float64, "f32": np.float32}


class RtExec(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("n_shards", ctypes.c_int32), ("shard", ctypes.c_int32),
                ("row_block", ctypes.c_int32), ("flags", ctypes.c_int32), ("n_devices", ctypes.c_int32),
                ("devices", ctypes.POINTER(ctypes.c_int32))]


class RtStats(ctypes.Structure):
    _fields_ = [("upload_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("samples", ctypes.c_int64), ("bvh_nodes", ctypes.c_int32), ("max_stack", ctypes.c_int32),
                ("device_allocs", ctypes.c_int32), ("kernel_block", ctypes.c_int32)]


_lib = None


def load():
    """Load librt_amd.so; raise RtDeviceError (never fall back) if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RtDeviceError(f"HIP library {LIB_PATH} is not built (run __graft_entry__.build() or "
                            f"make -C raytrace_amd/csrc)")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise RtDeviceError(f"cannot load {LIB_PATH}: {e}") from None
    P = ctypes.c_void_p
    L.rt_abi_version.restype = ctypes.c_int
    L.rt_last_error.restype = ctypes.c_char_p
    L.rt_image_height.argtypes = [ctypes.POINTER(RtCameraSettings)]
    L.rt_shard_rows.argtypes = [ctypes.c_int32, ctypes.POINTER(RtExec)]
    L.rt_shard_row.argtypes = [ctypes.c_int32, ctypes.POINTER(RtExec)]
    L.rt_render.argtypes = [ctypes.POINTER(RtCameraSettings), ctypes.POINTER(RtScene), ctypes.c_uint64,
                            ctypes.POINTER(RtExec), P, ctypes.POINTER(RtStats)]
    L.rt_scene_create.argtypes = [ctypes.POINTER(RtScene), ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]
    L.rt_scene_destroy.argtypes = [P]
    L.rt_scene_stats.argtypes = [P, ctypes.POINTER(RtStats)]
    L.rt_render_async.argtypes = [P, ctypes.POINTER(RtCameraSettings), ctypes.c_uint64, ctypes.POINTER(RtExec), P, P]
    L.rt_encode8_async.argtypes = [P, ctypes.c_int32, P, ctypes.c_int64, ctypes.c_int32, P]
    L.rt_multi_scene_create.argtypes = [ctypes.POINTER(RtScene), ctypes.POINTER(ctypes.c_int32), ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_void_p)]
    L.rt_multi_scene_destroy.argtypes = [P]
    L.rt_multi_render.argtypes = [P, ctypes.POINTER(RtCameraSettings), ctypes.c_uint64, ctypes.POINTER(RtExec), P,
                                  ctypes.POINTER(RtStats)]
    for name in EXPORTED:
        getattr(L, name)
    if L.rt_abi_version() != ABI_VERSION:
        raise RtDeviceError("librt_amd.so ABI version mismatch")
    _lib = L
    return L


def check(rc: int):
    if rc >= 0:
        return rc
    msg = load().rt_last_error().decode(errors="replace")
    cls = {RT_E_INVALID: RtInvalid, RT_E_UNSUPPORTED: RtUnsupported, RT_E_HIP: RtDeviceError}.get(rc, RtError)
    raise cls(f"[{rc}] {msg}")


def camera_struct(cs):
    """CameraSettings -> rt_camera_settings (keeps the target array alive on the struct)."""
    from .camera import background_of
    bg = background_of(cs)
    c = RtCameraSettings()
    c.center[:] = list(map(float, cs.cs_center))
    c.look_at[:] = list(map(float, cs.cs_lookAt))
    c.up[:] = list(map(float, cs.cs_up))
    c.vfov = float(cs.cs_vfov)
    c.aspect_ratio = float(cs.cs_aspectRatio)
    c.image_width = int(cs.cs_imageWidth)
    c.samples_per_pixel = int(cs.cs_samplesPerPixel)
    c.max_recursion_depth = int(cs.cs_maxRecursionDepth)
    c.background_kind = bg.kind
    c.background_c0[:] = list(bg.c0)
    c.background_c1[:] = list(bg.c1)
    c.defocus_angle = float(cs.cs_defocusAngle)
    c.focus_dist = float(cs.cs_focusDist)
    nt = len(cs.cs_redirectTargets)
    arr = (RtRedirectTarget * max(nt, 1))()
    for k, (p, q, u, v) in enumerate(cs.cs_redirectTargets):
        arr[k].prob = float(p)
        arr[k].q[:] = list(map(float, q))
        arr[k].u[:] = list(map(float, u))
        arr[k].v[:] = list(map(float, v))
    c.n_redirect_targets = nt
    c.redirect_targets = ctypes.cast(arr, ctypes.POINTER(RtRedirectTarget))
    c._keep = arr
    return c


def scene_struct(flat):
    """FlatScene (numpy record arrays in rt.h layout) -> rt_scene."""
    s = RtScene()
    keep = []

    def ptr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return a.ctypes.data if len(a) else None

    s.n_prims, s.prims = len(flat.prims), ptr(flat.prims)
    s.n_media, s.media = len(flat.media), ptr(flat.media)
    s.n_materials, s.materials = len(flat.materials), ptr(flat.materials)
    s.n_textures, s.textures = len(flat.textures), ptr(flat.textures)
    s.n_motions, s.motions = len(flat.motions), ptr(flat.motions)
    s.n_uvframes, s.uvframes = len(flat.uvframes), ptr(flat.uvframes)
    texels = np.ascontiguousarray(flat.texels, dtype=np.float32).reshape(-1, 3)
    s.n_texels, s.texels = len(texels), ptr(texels)
    s.perlin = ptr(flat.perlin) if flat.perlin is not None else None
    inst = getattr(flat, "instances", None)
    s.n_instances, s.instances = (len(inst), ptr(inst)) if inst is not None and len(inst) else (0, None)
    s._keep = keep
    return s


def dtype_of(precision: str):
    """Output dtype of a precision ("f64": the reference's binary64, the default; "f32")."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, not {precision!r}")
    return PRECISIONS[precision]


def exec_struct(device=0, n_shards=1, shard=0, row_block=4, precision="f64", devices=None, encode=None,
                solo=False):
    """rt_exec: the row shard, the precision, (rt_render only) a device list and an 8-bit output
    encoding (None: linear RGB; "srgb": writeImage's codes; "sqrt": writeImageSqrt's); `solo`
    (rt_render_async): the render does not overlap another on its device (RT_EXEC_SOLO)."""
    dtype_of(precision)
    if encode not in ENCODINGS:
        raise ValueError(f"encode must be one of {sorted(k for k in ENCODINGS if k)} or None, not {encode!r}")
    e = RtExec()
    e.device, e.n_shards, e.shard, e.row_block = device, n_shards, shard, row_block
    e.flags = (RT_EXEC_F32 if precision == "f32" else 0) | ENCODINGS[encode] | (RT_EXEC_SOLO if solo else 0)
    if devices:
        arr = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
        e.n_devices, e.devices = len(devices), ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32))
        e._keep = arr
    return e
