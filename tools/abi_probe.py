"""The C-ABI device list timed in a process of its own (no torch.distributed ranks on the card):
bench.py's abi_device_list record for the lists [0], [0, 0], [0, 0, 0] on one GPU, plus the
per-call host wall time split (rt_stats.total_ms vs kernel_ms).  Diagnoses whether the one-GPU
rehearsal's [0] x N time comes from the device list itself or from the rehearsal's other ranks.
usage: python tools/abi_probe.py [config] [frames]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from raytrace_amd import scenes  # noqa: E402
from raytrace_amd.ray import MultiDeviceScene  # noqa: E402

if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cornell"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cs, world, seed = scenes.CONFIGS[cfg]()
    for devs in ([0], [0, 0], [0, 0, 0], [0]):
        rec = bench.abi_device_list(world, cs, seed, devs, "f64", frames)
        # per-call split: host wall vs the library's own total and the slowest shard's kernel
        m = MultiDeviceScene(world, devs)
        try:
            for _ in range(3):
                m.render(cs, seed, precision="f64", row_block=1)
            rows = []
            for _ in range(5):
                st = {}
                t0 = time.perf_counter()
                m.render(cs, seed, precision="f64", row_block=1, stats=st)
                rows.append({"wall_ms": round((time.perf_counter() - t0) * 1e3, 3),
                             "total_ms": round(st["total_ms"], 3), "kernel_ms": round(st["kernel_ms"], 3)})
        finally:
            m.close()
        rec["calls"] = rows
        print(json.dumps({"config": cfg, **rec}), flush=True)
