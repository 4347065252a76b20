"""Sanitizer runs on the host code: the scene builder (rt_build.cpp / rt_bvh.cpp,
which parse caller-supplied scenes) with the kernel logic (tests/kernel_emu), and the FP64
oracle, under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer (the
threaded render loops).  Each run is a subprocess with the sanitizer runtime preloaded into
Python; tests/sanitize_scenes.py renders every scene class and feeds malformed scenes."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _runtime(name):
    out = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True, check=True).stdout.strip()
    if not os.path.isabs(out) or not os.path.exists(out):
        pytest.skip(f"{name} is not available")
    return out


def _build():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "sanitize"], check=True)
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "kernel_emu"), "-s", "sanitize"], check=True)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_under_sanitizers(kind):
    _build()
    env = dict(os.environ)
    env["RT_ORACLE_LIB"] = os.path.join(ROOT, "oracle", "_build", f"librt_oracle_{kind}.so")
    env["RT_EMU_LIB"] = os.path.join(ROOT, "tests", "kernel_emu", "_build", f"librt_emu_{kind}.so")
    if kind == "asan":
        env["LD_PRELOAD"] = _runtime("libasan.so")
        env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1:halt_on_error=1"
        env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    else:
        env["LD_PRELOAD"] = _runtime("libtsan.so")
        env["TSAN_OPTIONS"] = "halt_on_error=1:report_signal_unsafe=0"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sanitize_scenes.py")], env=env,
                       capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0 and "sanitize ok" in r.stdout, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
    assert "WARNING: ThreadSanitizer" not in r.stderr, tail
