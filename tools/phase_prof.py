"""Phase profile of the decoupled BVH kernel (diagnostic build: tools/build_variant.sh prof
-DRT_PHASE_PROF): per-wave shader clocks in the front end (items / camera / segment start), the
traversal rounds and shading, and the lane occupancy of each, for one config and precision.
usage: RT_AMD_EXPERIMENTS=1 RT_AMD_LIB=raytrace_amd/_lib/diag/librt_amd_prof.so python tools/phase_prof.py CONFIG [f32|f64] [frames]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from raytrace_amd import _lib, scenes  # noqa: E402
from raytrace_amd.camera import image_height  # noqa: E402
from raytrace_amd.ray import DeviceScene  # noqa: E402

NAMES = ["front_clk", "trav_clk", "shade_clk", "iters", "rounds", "tracing_lanes", "live_lanes", "shading_lanes",
         "front_lanes", "node_steps", "node_lanes", "leaf_steps", "leaf_lanes", "node_clk", "leaf_clk", "cam_clk",
         "cam_lanes"]

if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "bunny_cornell"
    prec = sys.argv[2] if len(sys.argv) > 2 else "f32"
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    L = _lib.load()
    cs, world, seed = scenes.CONFIGS[cfg]()
    sc = DeviceScene(world)
    h, w = image_height(cs), int(cs.cs_imageWidth)
    out = torch.empty((h, w, 3), dtype=torch.float64 if prec == "f64" else torch.float32, device="cuda")
    buf = (ctypes.c_ulonglong * 32)()
    sc.render_async(cs, seed, out.data_ptr(), precision=prec)  # warm-up
    torch.cuda.synchronize()
    L.rt_prof_read(1 if prec == "f64" else 0, buf, 32)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(frames):
        sc.render_async(cs, seed, out.data_ptr(), precision=prec)
    ev1.record()
    torch.cuda.synchronize()
    n = L.rt_prof_read(1 if prec == "f64" else 0, buf, 32)
    d = dict(zip(NAMES, [buf[i] / frames for i in range(n)]))
    # flat kernel (lane_loop_lockstep): front = commit / grab / item, cam = camera ray, trav = the
    # closest-hit tests of the segment, shade = material, scatter and the sample's sums
    clk = d["front_clk"] + d["trav_clk"] + d["shade_clk"] + d.get("cam_clk", 0)
    r = {"config": cfg, "precision": prec, "ms_per_frame": ev0.elapsed_time(ev1) / frames,
         "share": {k: round(d.get(k, 0) / clk, 4) for k in ("front_clk", "cam_clk", "trav_clk", "shade_clk")},
         "cam_lanes_per_iter": round(d.get("cam_lanes", 0) / max(1, d["iters"]), 2),
         "lanes_tracing_per_round": round(d["tracing_lanes"] / max(1, d["rounds"]), 2),
         "lanes_live_per_round": round(d["live_lanes"] / max(1, d["rounds"]), 2),
         "rounds_per_iter": round(d["rounds"] / max(1, d["iters"]), 3),
         "shading_lanes_per_iter": round(d["shading_lanes"] / max(1, d["iters"]), 2),
         "front_lanes_per_iter": round(d["front_lanes"] / max(1, d["iters"]), 2),
         "clk_per_round": round(d["trav_clk"] / max(1, d["rounds"]), 1),
         "clk_per_iter_front": round(d["front_clk"] / max(1, d["iters"]), 1),
         "clk_per_iter_shade": round(d["shade_clk"] / max(1, d["iters"]), 1),
         "node_steps_per_round": round(d["node_steps"] / max(1, d["rounds"]), 2),
         "lanes_per_node_step": round(d["node_lanes"] / max(1, d["node_steps"]), 2),
         "leaf_steps_per_round": round(d["leaf_steps"] / max(1, d["rounds"]), 2),
         "lanes_per_leaf_step": round(d["leaf_lanes"] / max(1, d["leaf_steps"]), 2),
         "node_clk_share_of_trav": round(d["node_clk"] / max(1, d["trav_clk"]), 3),
         "leaf_clk_share_of_trav": round(d["leaf_clk"] / max(1, d["trav_clk"]), 3),
         "raw": d}
    print(json.dumps(r), flush=True)
