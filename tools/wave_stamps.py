"""Ramp and tail of ONE render launch, wave by wave (diagnostic build: tools/build_variant.sh stamps
-DRT_WAVE_STAMPS): every wave of the persistent grid stamps the wall clock (100 MHz) at its start,
when its grab first finds every queue spent, and at its end.  Per frame (one stream, synchronised,
the stamps read after each launch):
  span      first wave start -> last wave end (the kernel's own duration, launch overhead excluded)
  ramp      wave starts after the first one (p50 / p99 / max)
  drain     the first wave that found the queue spent (every item claimed), from the first start
  tail      drain -> last wave end: the launch's last items, on a machine that empties
  busy      sum over waves of (end - start) / (waves x span): the mean fraction of the grid alive
  alive     waves alive in each tenth of the span (fraction of the grid)
The span split as ramp + work + tail says where the one-stream launch loses against frames
overlapped on two streams (bench.py), which hide both ends.
usage: RT_AMD_EXPERIMENTS=1 RT_AMD_LIB=raytrace_amd/_lib/diag/librt_amd_stamps.so \
       python tools/wave_stamps.py [config] [f64|f32] [frames]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from raytrace_amd import _lib, scenes  # noqa: E402
from raytrace_amd.camera import image_height  # noqa: E402
from raytrace_amd.ray import DeviceScene  # noqa: E402

MAX_WAVES = 16384
TICK_MS = 1e-5  # s_memrealtime: 100 MHz


def frame_stats(raw: np.ndarray) -> dict:
    st = raw.reshape(-1, 4)
    st = st[st[:, 0] != 0]
    t0, td, t1 = st[:, 0].astype(np.int64), st[:, 1].astype(np.int64), st[:, 2].astype(np.int64)
    base = int(t0.min())
    span = int(t1.max()) - base
    start = t0 - base
    drained = td[td != 0]
    first_drain = int(drained.min()) - base if drained.size else span
    end = t1 - base
    bins = 10
    edges = np.linspace(0, span, bins + 1)
    alive = [float(np.mean((start < edges[i + 1]) & (end > edges[i]))) for i in range(bins)]
    xcc = st[:, 3] & 0xF  # HW_REG 20 (XCC_ID) in the low word; the high word is HW_ID
    return {
        "waves": int(st.shape[0]),
        "span_ms": round(span * TICK_MS, 4),
        "ramp_ms": {"p50": round(float(np.percentile(start, 50)) * TICK_MS, 4),
                    "p99": round(float(np.percentile(start, 99)) * TICK_MS, 4),
                    "max": round(int(start.max()) * TICK_MS, 4)},
        "drain_ms": round(first_drain * TICK_MS, 4),
        "tail_ms": round((span - first_drain) * TICK_MS, 4),
        "end_ms": {q: round(float(np.percentile(end, q)) * TICK_MS, 4) for q in (1, 10, 50, 90, 99)},
        "busy": round(float((end - start).sum()) / (st.shape[0] * span), 4),
        "alive_by_tenth": [round(a, 3) for a in alive],
        "waves_per_xcc": np.bincount(xcc.astype(np.int64), minlength=8).tolist(),
    }


if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cornell"
    prec = sys.argv[2] if len(sys.argv) > 2 else "f64"
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    L = _lib.load()
    if not hasattr(L, "rt_stamps_read"):
        sys.exit("the loaded library is not a -DRT_WAVE_STAMPS build")
    cs, world, seed = scenes.CONFIGS[cfg]()
    sc = DeviceScene(world)
    h, w = image_height(cs), int(cs.cs_imageWidth)
    out = torch.empty((h, w, 3), dtype=torch.float64 if prec == "f64" else torch.float32, device="cuda")
    buf = (ctypes.c_ulonglong * (4 * MAX_WAVES))()
    f64 = 1 if prec == "f64" else 0
    for _ in range(30):  # warm-up: clocks settle after a few hundred ms of rendering
        sc.render_async(cs, seed, out.data_ptr(), precision=prec, row_block=1)
    torch.cuda.synchronize()
    L.rt_stamps_read(f64, buf, MAX_WAVES)
    rows = []
    for _ in range(frames):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        sc.render_async(cs, seed, out.data_ptr(), precision=prec, row_block=1)
        ev1.record()
        torch.cuda.synchronize()
        n = L.rt_stamps_read(f64, buf, MAX_WAVES)
        r = frame_stats(np.ctypeslib.as_array(buf)[: 4 * n].copy())
        r["event_ms"] = round(ev0.elapsed_time(ev1), 4)
        rows.append(r)
    keys = ("span_ms", "drain_ms", "tail_ms", "busy", "event_ms")
    summary = {k: round(float(np.median([r[k] for r in rows])), 4) for k in keys}
    print(json.dumps({"config": cfg, "precision": prec, "frames": frames, "median": summary, "per_frame": rows}), flush=True)
