"""bench.py's multi-GPU entry (CPU): `--gpus N` without a launcher starts N ranks itself and
refuses, rather than silently measuring fewer GPUs, when it cannot honour N."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


def test_more_gpus_than_visible_is_refused():
    r = _run(["--gpus", "2", "--steps", "1"], {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0
    assert "not measuring" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_launcher_world_size_mismatch_is_refused():
    r = _run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_wait_exited_sees_exits_and_zombies():
    """bench.py times the C-ABI device list only once the other ranks have exited: wait_exited
    returns when the processes are gone or zombies (exited, GPU contexts released, not yet reaped)."""
    import time
    sys.path.insert(0, ROOT)
    import bench
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(0.3)"])
    t0 = time.perf_counter()
    waited = bench.wait_exited([p.pid], timeout_s=20.0)
    assert 0.1 < waited < 10.0 and time.perf_counter() - t0 < 10.0
    # not reaped yet: a zombie counts as exited
    assert bench.wait_exited([p.pid], timeout_s=5.0) < 1.0
    p.wait()
    assert bench.wait_exited([p.pid, 2 ** 22 + 12345], timeout_s=5.0) < 1.0  # gone / never existed
    q = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        assert bench.wait_exited([q.pid], timeout_s=0.5) >= 0.5  # gives up at the timeout
    finally:
        q.kill()
        q.wait()
