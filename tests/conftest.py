import json
import os
import sys

import numpy as np
import pytest

# The tests run the library as callers get it: stray RT_AMD_* variables of the environment (an A/B
# session's knobs, RT_AMD_LIB, the experiments switch) are dropped at session start.  The tests that
# compare code paths set knobs through the `knobs` fixture, which turns the switch on for that test
# only (rt_internal.h rt_knob; test_host_mirror checks the knobs are ignored without it).
for _k in [k for k in os.environ if k.startswith("RT_AMD_")]:
    del os.environ[_k]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "kernel_emu")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture
def knobs(monkeypatch):
    """The library's RT_AMD_* experiment knobs honoured for this test (set them with monkeypatch)."""
    monkeypatch.setenv("RT_AMD_EXPERIMENTS", "1")
    return monkeypatch


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def emu_mod():
    import emu
    emu.build()
    return emu


@pytest.fixture(scope="session")
def golden_stats():
    with open(os.path.join(GOLDEN, "png_stats.json")) as f:
        stats = json.load(f)
    with open(os.path.join(GOLDEN, "noise_floor.json")) as f:
        floors = json.load(f)
    return stats, floors


def decode_codes(codes, encoding):
    """Inverse of the reference writers' 8-bit encoding (bin centre, tests/golden/make_golden.py)."""
    x = (codes.astype(np.float64) + 0.5) / 256.0
    if encoding == "sqrt":
        return x * x
    return np.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055) ** 2.4)


def as_published(img, encoding):
    """Quantise a linear render exactly as writeImage / writeImageSqrt store it, then decode."""
    from raytrace_amd.ray import encode8
    return decode_codes(encode8(img, encoding), encoding)


def block8(a, b=8):
    h, w, _ = a.shape
    return a[: h // b * b, : w // b * b].reshape(h // b, b, w // b, b, 3).mean((1, 3))


def pixel_agreement(img, ref, tol=1e-3):
    """Fraction of pixels whose every channel is within tol (relative above 1) of the oracle."""
    rel = np.abs(img.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))
    return float((rel.max(-1) < tol).mean())


def record_measure(name, rec):
    """Append a GPU test's measured figures to gpurun_out/<name>.jsonl (copied to profiles/ by the
    session): the bars in the tests are derived from these."""
    d = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    except OSError:
        pass
