"""Graphics.Ray's `raytrace` (src/Graphics/Ray.hs:121-238) on the MI355X, plus image IO.

`raytrace(settings, world, seed)` has the reference's argument order and meaning and returns
the h x w x 3 linear-RGB image (row 0 = top, Ray.hs:238 `ix@(j :. i)`), each pixel the mean of
`cs_samplesPerPixel` samples.  It flattens the descriptor tree, calls the C-ABI (`rt_render`)
and raises instead of silently computing anything on the CPU.

`DeviceScene` is the device-resident form (scene uploaded once, renders enqueued on a HIP
stream into caller-owned device memory) used by bench.py and the multi-GPU driver.
"""
from __future__ import annotations

import ctypes
import struct
import zlib

import numpy as np

from . import _lib
from .camera import CameraSettings, image_height
from .core import StdGen, mkStdGen
from .scene import FlatScene, flatten


def _seed64(seed) -> int:
    if isinstance(seed, StdGen):
        return seed.key()
    if isinstance(seed, int):
        return mkStdGen(seed).key()
    raise TypeError("seed must be a StdGen (mkStdGen n) or an int")


def raytrace(settings: CameraSettings, world, seed, device: int = 0, stats: dict | None = None,
             precision: str = "f64", devices=None, row_block: int = 4, encode: str | None = None,
             out: np.ndarray | None = None) -> np.ndarray:
    """Render on the GPU.  Returns (height, width, 3) linear RGB: float64 computed in binary64 as the
    reference does (default), or float32 from the FP32 kernel (precision="f32").  `devices`: a list
    of HIP devices that render the image together from this process (rt_exec device list; rows
    dealt round-robin in blocks of `row_block`); the image is identical to the one-device render.
    `encode` = "srgb" / "sqrt": uint8 codes as writeImage / writeImageSqrt store them, encoded on
    the device after the gather (Ray.hs:248-260; equal to encode8 of the linear render).  `out`: a
    caller-held output array to render into (shape and dtype as returned)."""
    L = _lib.load()
    flat = world if isinstance(world, FlatScene) else flatten(world)
    cs = _lib.camera_struct(settings)
    sc = _lib.scene_struct(flat)
    ex = _lib.exec_struct(device=device, precision=precision, devices=devices,
                          row_block=row_block if devices else 4, encode=encode)
    h = image_height(settings)
    w = int(settings.cs_imageWidth)
    if h <= 0 or w <= 0:
        from .errors import RtInvalid
        raise RtInvalid(f"image size {w}x{h} must be positive")
    rows = _lib.check(L.rt_shard_rows(h, ctypes.byref(ex)))
    if rows != h:
        raise RuntimeError(f"librt_amd.so reports {rows} rows for a {h}-row image")
    out = _out_buffer(out, (h, w, 3), np.uint8 if encode else _lib.dtype_of(precision))
    st = _lib.RtStats()
    _lib.check(L.rt_render(ctypes.byref(cs), ctypes.byref(sc), _seed64(seed), ctypes.byref(ex),
                           out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st)))
    if stats is not None:
        stats.update(upload_ms=st.upload_ms, kernel_ms=st.kernel_ms, total_ms=st.total_ms, samples=st.samples,
                     bvh_nodes=st.bvh_nodes, max_stack=st.max_stack, device_allocs=st.device_allocs,
                     kernel_block=st.kernel_block)
    return out


def render_shard(settings: CameraSettings, world, seed, n_shards: int, shard: int, row_block: int = 4,
                 device: int = 0, precision: str = "f64") -> np.ndarray:
    """Render only the rows of one shard (rt_exec row interleave); returns (rows, width, 3)."""
    L = _lib.load()
    flat = world if isinstance(world, FlatScene) else flatten(world)
    cs = _lib.camera_struct(settings)
    sc = _lib.scene_struct(flat)
    ex = _lib.exec_struct(device=device, n_shards=n_shards, shard=shard, row_block=row_block, precision=precision)
    rows = _lib.check(L.rt_shard_rows(image_height(settings), ctypes.byref(ex)))
    out = np.zeros((rows, int(settings.cs_imageWidth), 3), _lib.dtype_of(precision))
    st = _lib.RtStats()
    _lib.check(L.rt_render(ctypes.byref(cs), ctypes.byref(sc), _seed64(seed), ctypes.byref(ex),
                           out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st)))
    return out


def shard_rows(height: int, n_shards: int, row_block: int) -> int:
    """Padded rows per shard (pure arithmetic, mirrors rt_shard_rows); a single shard is the image."""
    if n_shards == 1:
        return height
    blocks = (height + row_block - 1) // row_block
    return ((blocks + n_shards - 1) // n_shards) * row_block


def shard_row_index(height: int, n_shards: int, shard: int, row_block: int) -> np.ndarray:
    """Global row of every shard-local row (>= height for padding rows); mirrors rt_shard_row."""
    t = np.arange(shard_rows(height, n_shards, row_block))
    return ((t // row_block) * n_shards + shard) * row_block + (t % row_block)


def assemble_shards(tiles, height: int, row_block: int) -> np.ndarray:
    """Un-permute gathered shard tiles [n_shards, rows, width, 3] into the (height, width, 3) image."""
    tiles = np.asarray(tiles)
    n = tiles.shape[0]
    img = np.zeros((height,) + tiles.shape[2:], tiles.dtype)
    for r in range(n):
        rows = shard_row_index(height, n, r, row_block)
        keep = rows < height
        img[rows[keep]] = tiles[r][keep]
    return img


def _out_buffer(out, shape, dtype) -> np.ndarray:
    """The output array: a new one, or the caller's after checking that the library may write the
    whole frame into it (shape, dtype, C-contiguous, writeable)."""
    if out is None:
        return np.zeros(shape, dtype)
    if not isinstance(out, np.ndarray) or out.shape != tuple(shape) or out.dtype != np.dtype(dtype) \
            or not out.flags.c_contiguous or not out.flags.writeable:
        from .errors import RtInvalid
        raise RtInvalid(f"out must be a writeable C-contiguous {np.dtype(dtype)} array of shape {tuple(shape)}")
    return out


class DeviceScene:
    """A scene resident in HBM (rt_scene_create).  Renders are enqueued asynchronously."""

    def __init__(self, world, device: int = 0):
        self._lib = _lib.load()
        self.flat = world if isinstance(world, FlatScene) else flatten(world)
        sc = _lib.scene_struct(self.flat)
        h = ctypes.c_void_p()
        _lib.check(self._lib.rt_scene_create(ctypes.byref(sc), device, ctypes.byref(h)))
        self.handle = h
        self.device = device

    def stats(self) -> dict:
        st = _lib.RtStats()
        _lib.check(self._lib.rt_scene_stats(self.handle, ctypes.byref(st)))
        return dict(upload_ms=st.upload_ms, bvh_nodes=st.bvh_nodes, max_stack=st.max_stack)

    def render_async(self, settings: CameraSettings, seed, out_ptr: int, stream_ptr: int = 0, n_shards: int = 1,
                     shard: int = 0, row_block: int = 4, precision: str = "f64", solo: bool = False):
        """Enqueue a render into the device buffer at out_ptr (rows x width x 3 float64, or float32
        with precision="f32").  Renders are planned for frames that overlap on two or more streams;
        `solo`: this one runs alone on its device (RT_EXEC_SOLO, the synchronous call's plan)."""
        cs = _lib.camera_struct(settings)
        ex = _lib.exec_struct(device=self.device, n_shards=n_shards, shard=shard, row_block=row_block,
                              precision=precision, solo=solo)
        _lib.check(self._lib.rt_render_async(self.handle, ctypes.byref(cs), _seed64(seed), ctypes.byref(ex),
                                             ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream_ptr or None)))

    def close(self):
        if self.handle:
            self._lib.rt_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiDeviceScene:
    """A scene resident on a list of GPUs of this process (rt_multi_scene_create: one host build,
    concurrent uploads).  `render` returns the whole image like `raytrace(..., devices=...)`,
    without rebuilding or re-uploading the scene; shard k renders on devices[k]."""

    def __init__(self, world, devices):
        self._lib = _lib.load()
        self.flat = world if isinstance(world, FlatScene) else flatten(world)
        self.devices = [int(d) for d in devices]
        sc = _lib.scene_struct(self.flat)
        arr = (ctypes.c_int32 * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _lib.check(self._lib.rt_multi_scene_create(ctypes.byref(sc), arr, len(self.devices), ctypes.byref(h)))
        self.handle = h

    def render(self, settings: CameraSettings, seed, precision: str = "f64", row_block: int = 4,
               encode: str | None = None, stats: dict | None = None, out: np.ndarray | None = None) -> np.ndarray:
        """`out`: a caller-held (h, w, 3) C-contiguous buffer of the output dtype, reused across
        renders (a fresh array costs its page faults in the device-to-host copy on every call)."""
        cs = _lib.camera_struct(settings)
        ex = _lib.exec_struct(device=self.devices[0], precision=precision, row_block=row_block, encode=encode)
        h, w = image_height(settings), int(settings.cs_imageWidth)
        out = _out_buffer(out, (h, w, 3), np.uint8 if encode else _lib.dtype_of(precision))
        st = _lib.RtStats()
        _lib.check(self._lib.rt_multi_render(self.handle, ctypes.byref(cs), _seed64(seed), ctypes.byref(ex),
                                             out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st)))
        if stats is not None:
            stats.update(upload_ms=st.upload_ms, kernel_ms=st.kernel_ms, total_ms=st.total_ms, samples=st.samples,
                         device_allocs=st.device_allocs)
        return out

    def close(self):
        if self.handle:
            self._lib.rt_multi_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ image IO (Ray.hs:240-260)

_ENC8 = None


def encode8_thresholds(encoding: str = "srgb") -> np.ndarray:
    """Per 8-bit code k, the smallest binary64 x whose code is >= k under the EXACTLY evaluated
    transfer (raytrace_amd/data/encode8_thresholds.json, tools/gen_encode8_table.py); the device
    epilogue reads the same table (rt_encode8_table.h)."""
    global _ENC8
    if _ENC8 is None:
        import json
        import os
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "encode8_thresholds.json")) as f:
            d = json.load(f)
        _ENC8 = {k: np.array([float.fromhex(x) for x in d[k]]) for k in ("srgb", "sqrt")}
    return _ENC8["sqrt" if encoding == "sqrt" else "srgb"]


def encode8(rgb: np.ndarray, encoding: str = "srgb") -> np.ndarray:
    """8-bit codes as the reference's writers store them: min(255, floor(256 * transfer(clamp01 x)))
    with transfer = sRGB (writeImage) or sqrt (writeImageSqrt), the transfer evaluated exactly (the
    number of code thresholds <= x); NaN -> 0.  Host twin of rt_encode8_async (bit-exact with it)."""
    x = np.asarray(rgb, np.float64)
    thr = encode8_thresholds(encoding)
    codes = np.searchsorted(thr[1:], np.where(np.isnan(x), -1.0, x), side="right")
    return codes.astype(np.uint8)


def _write_png(path: str, codes: np.ndarray):
    h, w, _ = codes.shape
    raw = b"".join(b"\x00" + codes[j].tobytes() for j in range(h))

    def chunk(tag, data):
        c = struct.pack(">I", len(data)) + tag + data
        return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


def writeImage(path: str, image: np.ndarray):
    """Ray.hs:248-252: linear RGB written as sRGB 8-bit PNG."""
    _write_png(path, encode8(image, "srgb"))


def writeImageSqrt(path: str, image: np.ndarray):
    """Ray.hs:256-260: sqrt as the transfer curve (`slightly incorrect`, kept for parity)."""
    _write_png(path, encode8(image, "sqrt"))


def readImage(path: str) -> np.ndarray:
    """Ray.hs:241-245: decode to linear RGB (needs Pillow)."""
    from PIL import Image
    codes = np.asarray(Image.open(path).convert("RGB")).astype(np.float64)
    x = codes / 255.0
    return np.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055) ** 2.4)
