"""The binary64 kernels' FP32 BVH node test (rt_trace.h prep_axis / node_slabs_f32) is
conservative: it enters every box that the exact slab test (rational arithmetic on the same
float box and binary64 ray) enters, so the leaves it tests are a superset of the exact test's and
the closest hit, keyed by (t, order), cannot change.  It must also stay tight: boxes the ray
clearly misses are rejected.  Runs on the host emulator (tests/kernel_emu), no GPU."""
import ctypes
from fractions import Fraction

import numpy as np
import pytest


def exact_accept(o, d, box, tmin, tmax):
    near, far = Fraction(tmin), Fraction(tmax) if np.isfinite(tmax) else None
    for k in range(3):
        b0, b1 = Fraction(float(box[2 * k])), Fraction(float(box[2 * k + 1]))
        ok, dk = Fraction(float(o[k])), Fraction(float(d[k]))
        t0, t1 = (b0 - ok) / dk, (b1 - ok) / dk
        lo, hi = min(t0, t1), max(t0, t1)
        near = max(near, lo)
        far = hi if far is None else min(far, hi)
    return near <= far, near, far


def make_cases(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-300.0, 600.0, (n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d *= rng.uniform(0.05, 20.0, (n, 1))
    small = rng.random((n, 3)) < 0.05  # near-axis-parallel rays
    d[small] = np.sign(d[small]) * 10.0 ** rng.uniform(-12, -3, small.sum())
    tstar = 10.0 ** rng.uniform(-2, 3.3, n)
    p = o + tstar[:, None] * d
    ext = 10.0 ** rng.uniform(-4, 2, (n, 3))
    # boxes around the ray's point at t*: grazing (a face through p, shifted by a few float ulps
    # either way), hit, or missed by a small relative gap
    box = np.empty((n, 6), np.float32)
    mode = rng.integers(0, 3, n)
    for k in range(3):
        pk = p[:, k].astype(np.float32)
        shift = rng.integers(-3, 4, n).astype(np.float32) * np.spacing(np.abs(pk))
        face = pk + shift
        lo_side = rng.random(n) < 0.5
        w = ext[:, k].astype(np.float32)
        gap = np.where(mode == 2, w * np.float32(1e-3), 0).astype(np.float32)
        mn = np.where(lo_side, face + gap, face - w)
        mx = np.where(lo_side, face + w, face - gap)
        mid = mode == 1
        mn = np.where(mid, pk - w, mn)
        mx = np.where(mid, pk + w, mx)
        box[:, 2 * k] = np.minimum(mn, mx)
        box[:, 2 * k + 1] = np.maximum(mn, mx)
    tr = np.stack([np.full(n, 1e-3), np.where(rng.random(n) < 0.3, np.inf,
                                              tstar * rng.uniform(0.5, 2.0, n))], 1)
    return o, d, box, tr


@pytest.mark.parametrize("rcp_ulps", [-1, 0, 1])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fp32_node_test_is_conservative(emu_mod, seed, rcp_ulps):
    """rcp_ulps: the direction reciprocal rounded as IEEE (0) or 1 ulp either way (+-1) — the
    device's v_rcp_f32 is within 1 ulp, so both of its possible results are covered."""
    L = emu_mod.lib()
    f = L.rt_emu_node_test_f64
    f.restype = None
    n = 6000
    o, d, box, tr = make_cases(n, seed)
    acc = np.zeros(n, np.int32)
    dp = ctypes.POINTER(ctypes.c_double)
    L.rt_emu_set_rcp_ulps(rcp_ulps)
    try:
        f(n, o.ctypes.data_as(dp), d.ctypes.data_as(dp), box.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
          tr.ctypes.data_as(dp), acc.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    finally:
        L.rt_emu_set_rcp_ulps(0)
    assert np.all((acc == 0) | (acc == 3)), "the two children (the same box) must agree"
    n_exact = n_clear_miss = n_clear_rejected = 0
    for i in range(n):
        ok, near, far = exact_accept(o[i], d[i], box[i], tr[i, 0], tr[i, 1])
        if ok:
            n_exact += 1
            assert acc[i] == 3, f"case {i}: the exact slab test enters the box, the FP32 test does not"
        elif (near - far) > Fraction(1, 10 ** 5) * (abs(near) + Fraction(float(np.max(np.abs(o[i] / d[i]))))):
            # missed by more than ~30x the pad (5 eps |o / d|, prep_axis) plus the relative margin
            n_clear_miss += 1
            n_clear_rejected += acc[i] == 0
    assert n_exact > n // 5 and n_clear_miss > n // 20, (n_exact, n_clear_miss)
    # tightness: the pad only widens boxes by a few float ulps of |o / d| and t
    assert n_clear_rejected == n_clear_miss, (n_clear_rejected, n_clear_miss)
