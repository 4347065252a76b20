"""Device-to-host copy of one binary64 Cornell frame (600 x 600 x 3 doubles, 8.64 MB) into pageable
and into pinned host memory: the part of a synchronous rt_render call after its kernel.
usage (GPU box): python tools/d2h_probe.py"""
import json
import time

import torch

n = 600 * 600 * 3
d = torch.rand(n, dtype=torch.float64, device="cuda")
pageable = torch.empty(n, dtype=torch.float64)
pinned = torch.empty(n, dtype=torch.float64).pin_memory()
out = {}
for name, dst in (("pageable", pageable), ("pinned", pinned)):
    for _ in range(5):
        dst.copy_(d)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        dst.copy_(d)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    out[name + "_ms_median"] = round(ts[len(ts) // 2], 4)
    out[name + "_GBps"] = round(n * 8 / ts[len(ts) // 2] / 1e6, 1)
print(json.dumps({"bytes": n * 8, **out}))
