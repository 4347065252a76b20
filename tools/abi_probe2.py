"""Why the C-ABI device list is slower inside bench.py's N>1 rehearsal than alone (tools/abi_probe.py):
the list [0, 0] timed after each of the things bench.py's rank 0 has done by then.
usage: python tools/abi_probe2.py <mode>   mode: plain | torch | torch_tensors | dist | streams
(one mode per process; tools/gpu_round.sh step `abiprobe2` runs them all)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
    t0 = time.perf_counter()
    if mode != "plain":
        import torch
        torch.cuda.set_device(0)
        if mode == "streams":  # bench.py's rank 0 has created streams of its own by then
            ss = [torch.cuda.Stream() for _ in range(3)]
            for st in ss:
                with torch.cuda.stream(st):
                    torch.ones(16, device="cuda:0").sum()
            torch.cuda.synchronize()
        if mode in ("torch_tensors", "dist"):
            x = [torch.empty((600, 600, 3), dtype=torch.float64, device="cuda:0") for _ in range(4)]
            torch.cuda.synchronize()
            del x
        if mode == "dist":
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("gloo", rank=0, world_size=1)
            dist.barrier()
            dist.destroy_process_group()
    import bench
    from raytrace_amd import scenes
    cs, world, seed = scenes.CONFIGS["cornell"]()
    for devs in ([0], [0, 0]):
        rec = bench.abi_device_list(world, cs, seed, devs, "f64", 10)
        print(json.dumps({"mode": mode, "devices": devs, "ms_per_frame": rec["ms_per_frame"],
                          "kernel_ms_max_device": rec["kernel_ms_max_device"],
                          "affinity": len(os.sched_getaffinity(0)),
                          "threads_env": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "HIP_VISIBLE_DEVICES")}}),
              flush=True)
