"""Benchmark of the MI355X path-tracing kernel on BASELINE.json's headline config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cornell]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full frame of the config (Cornell box 600x600, 200 spp, depth 50, redirect
target, seed 234 — test/Main.hs:188-218) with the scene already resident in HBM.  With N
ranks (one process per GPU) the frame's rows are dealt to ranks round-robin (--row-block 1)
(rt_exec row interleave) and the framebuffer tiles are gathered to rank 0 over RCCL (one gather
into rank 0's frame) inside the timed region — asynchronously, so frame i+1 renders
while frame i's gather is in flight (two frame buffers); the clock stops after every frame is
rendered AND gathered.
`value` = pixels x spp of all ranks / max-over-ranks time.
The W warm-up frames are followed by more untimed frames until the warm-up has rendered for
--warmup-s seconds (2 by default: the per-frame time only settles after a few hundred ms of
continuous rendering, and a GPU-activity sampler polling about once a second sees the card busy
even when the timed region itself is a fraction of a second); `warmup_frames` / `warmup_s` in the
line say how many ran.

Frames of flat scenes (the Cornell box) alternate between two HIP streams (--streams 2, the
default for them): a frame's last long paths occupy few CUs, and the next frame's persistent
workgroups fill the rest instead of waiting (Cornell +4 % at 1 GPU, +26 % on one rank's share of
an 8-GPU frame).

Precision: the line is measured with the binary64 kernel (`dtype` "f64"), the reference's
arithmetic (`V3 Double`, Core.hs:29-31); the FP32 fast path is measured right after it on the
same frames and reported beside it as `f32_fast_path` (a labelled second record, not `value`).

Extra fields: `roofline` — the physical ceiling of the render kernel: VALU instruction issue
(the kernel's PMC-counted VALU wave-instructions per launch, profiles/pmc_valu.json, scaled to the
samples this launch renders, / its device time per frame from HIP events over the timed region —
`kernel_ms`, the span of the timed frames / frames; `launch_ms` is the average single-launch
duration, longer when two launches overlap — against 256 CUs x 4 SIMDs x one wave64 VALU
instruction per 2 cycles at 2.4 GHz; frac <= 1 by construction; `mix_frac` = the time the VALUs
need for the launch's measured instruction mix at the per-class throughput a full chip sustains
(tools/microbench/valu_rates.hip, profiles/r2/valu_rates.json) / the kernel time), with `traffic` = the PMC-measured
HBM bytes per launch and `hbm_gbs` = traffic / kernel time beside it, and the SURVEY.md §8(d)
algorithmic bytes (the REFERENCE's traversal: every Cornell quad tested every segment) kept as a
labelled `reference_traversal_bytes` figure — it exceeds HBM peak because the kernel reads its
1.4 KB scene from the scalar cache, so it is never `frac`; `cpu_baseline` — the FP64 oracle, the
CPU restatement of the reference's algorithm, on a bounded row sample, rank 0 at N=1 only, on
every core this process may use (os.sched_getaffinity), with a 1-core figure beside it;
`abi_device_list` — the drop-in's own multi-GPU path (what the Haskell binding calls): after the
ranks' measurement rank 0 alone renders the frame through the C ABI's device list over GPUs
0..N-1 (rt_multi_render, host-buffer output) once the other ranks have exited, ms per frame and
the frame digest, which must equal the line's `check.sha16`.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
PUBLISHED_MSAMPLES = {"cornell": 1.2}  # Cornell 600x600x200 with redirect ~1:00 (author's laptop)
METRIC = "Msamples/s (pixels×spp/s) + achieved HBM GB/s, Cornell-box 600×600"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu_info():
    """CPU model, the machine's CPUs, the CPUs this process may run on and the cgroup CPU quota."""
    info = {"host_cpus": os.cpu_count()}
    try:
        info["usable_cpus"] = len(os.sched_getaffinity(0))
    except Exception:
        info["usable_cpus"] = os.cpu_count()
    try:
        with open("/proc/cpuinfo") as f:
            info["cpu_model"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        pass
    return info


def cpu_baseline(config, world_fn, row_stride=6):
    """Time the oracle (binary64 restatement, splitmix draw order) on every `row_stride`-th row, on
    every CPU this process may run on (the reference's `-threaded -N`: one capability per core)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    from raytrace_amd.camera import image_height
    cs, world, seed = world_fn()
    h, w = image_height(cs), cs.cs_imageWidth
    rows = np.arange(0, h, row_stride)
    pix = (rows[:, None] * w + np.arange(w)[None, :]).reshape(-1).astype(np.int32)
    hw = host_cpu_info()
    threads = max(1, hw["usable_cpus"] or 1)
    if hw.get("cgroup_cpu_quota"):  # more threads than the CPU quota only time-share it
        threads = max(1, min(threads, int(round(hw["cgroup_cpu_quota"]))))
    oracle.render(cs, world, seed, mode=oracle.RNG_SPLITMIX, pixels=pix[:64], nthreads=threads)  # warm
    t0 = time.perf_counter()
    oracle.render(cs, world, seed, mode=oracle.RNG_SPLITMIX, pixels=pix, nthreads=threads)
    dt = time.perf_counter() - t0
    samples = len(pix) * cs.cs_samplesPerPixel
    # single-core figure on a tenth of that sample (BASELINE.md §3 asks for both)
    pix1 = pix.reshape(len(rows), w)[::10].reshape(-1)
    t0 = time.perf_counter()
    oracle.render(cs, world, seed, mode=oracle.RNG_SPLITMIX, pixels=pix1, nthreads=1)
    dt1 = time.perf_counter() - t0
    samples1 = len(pix1) * cs.cs_samplesPerPixel
    return {"value": round(samples / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "value_1core": round(samples1 / dt1 / 1e6, 4), **hw,
            "sample": f"{config}: every {row_stride}th row ({len(rows)} rows x {w} px x {cs.cs_samplesPerPixel} spp"
                      f" = {samples / 1e6:.1f} M samples) in {dt:.2f} s, oracle/rt_oracle.c splitmix mode, "
                      f"{threads} threads; 1-core: every {10 * row_stride}th row ({samples1 / 1e6:.2f} M samples)"
                      f" in {dt1:.2f} s"}


# VALU issue ceiling: 256 CUs x 4 SIMD-32 x one wave64 VALU instruction per 2 cycles at the
# 2.4 GHz peak engine clock (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles")
VALU_PEAK_GINST = 256 * 4 * 0.5 * 2.4


def pmc_record(config, precision):
    """The committed PMC summary of the render kernel for (config, precision) (profiles/pmc_valu.json)."""
    path = os.path.join(ROOT, "profiles", "pmc_valu.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None
    return d.get(f"{config}/{precision}")


# instruction class (PMC SQ_INSTS_VALU_<class>) -> the microbenchmark's throughput key
MIX_RATE_KEYS = {"fma_f64": "fma_f64", "mul_f64": "mul_f64", "add_f64": "add_f64", "trans_f64": "rcp_f64",
                 "trans_f32": "sin_f32", "int64": "mad_u64_u32_plus"}


def mix_time_s(mix, total):
    """Seconds the chip's VALUs need for `total` wave-instructions of class mix `mix` at the
    measured per-class throughput (profiles/r2/valu_rates.json); classes not listed (f32 / int32
    arithmetic, moves, selects, compares) at the v_fma_f32 rate."""
    try:
        with open(os.path.join(ROOT, "profiles", "r2", "valu_rates.json")) as f:
            rates = json.load(f)
    except Exception:
        return None
    if not mix:
        return None
    t, used = 0.0, 0.0
    for cls, key in MIX_RATE_KEYS.items():
        n = mix.get(cls, 0.0)
        t += n / (rates[key] * 1e9)
        used += n
    return t + max(0.0, total - used) / (rates["fma_f32"] * 1e9)


def roofline_of(config, precision, kernel_ms, launch_ms, share, samples_per_launch, concurrent):
    """The physical roofline of the render kernel: VALU issue from the committed PMC counts (full
    frame, scaled by `share` = the fraction of the frame's samples this launch renders), measured
    HBM traffic beside it, and the reference-traversal bytes as a labelled figure."""
    with open(os.path.join(ROOT, "tests", "golden", "algbytes.json")) as f:
        alg = json.load(f)["configs"]
    b_sample = (alg.get(config) or alg[config.split("_")[0]])["bytes_per_sample"]  # demo1_1200x800: demo1's
    ref_bytes = b_sample * samples_per_launch
    r = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_GINST, "unit": "G VALU wave-instr/s", "frac": None,
         "traffic": None, "kernel": "rt_render_kernel", "precision": precision, "kernel_ms": round(kernel_ms, 4),
         "launch_ms": round(launch_ms, 4), "concurrent_launches": concurrent,
         "samples_per_launch": samples_per_launch,
         "reference_traversal_bytes": {"bytes_per_sample": round(b_sample, 1), "per_launch": round(ref_bytes),
                                       "gbs_if_read_from_hbm": round(ref_bytes / (kernel_ms * 1e-3) / 1e9, 1),
                                       "note": "SURVEY §8(d) bytes of the reference's traversal; the kernel reads "
                                               "its scene from caches, so this is not HBM traffic"}}
    d = pmc_record(config, precision)
    if d is None:
        return r
    valu = d["valu_insts_per_launch"] * share
    ach = valu / (kernel_ms * 1e-3) / 1e9
    r.update(achieved=round(ach, 1), frac=round(ach / VALU_PEAK_GINST, 4),
             valu_insts_per_launch=round(valu), lane_utilisation=round(d["lane_utilisation"], 4),
             pmc_round=d.get("round"), pmc_share_scale=round(share, 6))
    mt = mix_time_s(d.get("valu_mix_per_launch"), d["valu_insts_per_launch"])
    if mt is not None:
        # the time the VALU needs for this launch's instruction mix at the measured per-class
        # throughput of a full chip (tools/microbench/valu_rates.hip), over the measured time
        r["mix_frac"] = round(mt * share / (kernel_ms * 1e-3), 4)
    if d.get("hbm_bytes_per_launch") is not None:
        traffic = d["hbm_bytes_per_launch"] * share
        r.update(traffic=round(traffic), hbm_gbs=round(traffic / (kernel_ms * 1e-3) / 1e9, 1),
                 hbm_frac=round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    return r


def abi_device_list(world, cs, seed, devices, precision, frames, warmup=2, warmup_s=0.5):
    """The drop-in's own multi-GPU path: ONE process rendering the whole frame through the C ABI's
    device list (rt_multi_scene_create / rt_multi_render: shard k on devices[k], peer-copy gather
    into devices[0], one device-to-host copy), as the Haskell binding calls it (Device.hs passes
    every visible device; the reference's `-threaded -N` analogue, Ray.hs:238).  Host-buffer
    output, so the time includes the device-to-host copy of the frame."""
    import hashlib
    import numpy as np
    from raytrace_amd.ray import MultiDeviceScene
    m = MultiDeviceScene(world, devices)
    try:
        tw, k = time.perf_counter(), 0
        # uploads, occupancy queries, the resident buffers; then at least warmup_s of frames
        # one host buffer for every frame, as a caller rendering repeatedly holds it (a fresh
        # array per call pays its page faults inside the device-to-host copy)
        img = None
        while k < warmup or time.perf_counter() - tw < warmup_s:
            img = m.render(cs, seed, precision=precision, row_block=1, out=img)
            k += 1
        kms, tms, allocs = [], [], 0
        t0 = time.perf_counter()
        for _ in range(frames):
            st = {}
            img = m.render(cs, seed, precision=precision, row_block=1, stats=st, out=img)
            kms.append(st["kernel_ms"])
            tms.append(st["total_ms"])
            allocs += st["device_allocs"]
        dt = time.perf_counter() - t0
    finally:
        m.close()
    samples = img.shape[0] * img.shape[1] * cs.cs_samplesPerPixel
    return {"devices": list(devices), "dtype": precision, "frames": frames,
            "ms_per_frame": round(dt / frames * 1e3, 4), "value": round(samples * frames / dt / 1e6, 2),
            "unit": "Msamples/s", "kernel_ms_max_device": round(sum(kms) / len(kms), 4),
            "library_ms_per_call": round(sum(tms) / len(tms), 4),  # rt_stats.total_ms: inside the C ABI
            "device_allocs_timed": allocs,
            "sha16": hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()[:16],
            "note": "one process, rt_multi_render over the device list (C-ABI drop-in path), host-buffer output "
                    "(one caller-held buffer reused across frames)"}


def abi_helper(args):
    """--abi-helper: build the scene on the CPU, wait for 'go <d0,d1,...>' on stdin (rank 0 sends it
    once the other ranks have exited), time the C-ABI device list over those devices in THIS process
    and print its record as one JSON line.  Never touches a GPU before the go."""
    from raytrace_amd import scenes
    cs, world, seed = scenes.CONFIGS[args.config]()
    cmd = sys.stdin.readline().split()
    if len(cmd) != 2 or cmd[0] != "go":
        return 0  # rank 0 ended without a measurement
    devs = [int(x) for x in cmd[1].split(",")]
    print(json.dumps(abi_device_list(world, cs, seed, devs, args.precision, frames=args.steps)), flush=True)
    return 0


def wait_exited(pids, timeout_s=120.0):
    """Wait until the processes `pids` have exited (gone, or zombies whose GPU contexts are already
    released); returns the seconds waited.  Gives up after timeout_s (the record then carries it)."""
    t0 = time.perf_counter()

    def alive(pid):
        try:
            with open(f"/proc/{pid}/stat") as f:
                return f.read().rsplit(")", 1)[1].split()[0] != "Z"
        except OSError:
            return False

    while any(alive(p) for p in pids) and time.perf_counter() - t0 < timeout_s:
        time.sleep(0.05)
    return time.perf_counter() - t0


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: run this same command as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) and return its exit code.
    Called before this process touches a GPU (counting devices does not initialise one), and the
    ranks are CHILD processes: nothing is exec'd over a process that has initialised the GPU.
    Refuses (non-zero exit, no measurement) when fewer than N GPUs are visible, unless
    RT_BENCH_ONE_DEVICE=1 maps every rank to device 0 (the one-GPU rehearsal)."""
    import socket
    import subprocess
    import torch
    have = torch.cuda.device_count()
    if have < n and os.environ.get("RT_BENCH_ONE_DEVICE") != "1":
        log(f"bench.py: --gpus {n} but only {have} GPU(s) visible; not measuring")
        return 2
    with socket.socket() as s:  # a free rendezvous port
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"bench.py: launching {n} ranks: {' '.join(cmd)}")
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30,
                    help="timed frames (default 30: the Cornell frame is ~5 ms, so the barrier and "
                         "synchronise around the timed region weigh < 0.5 %)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cornell", choices=["cornell", "readme", "demo1", "demo1_1200x800", "bunny_cornell", "pawn_fog"])
    ap.add_argument("--row-block", type=int, default=1,
                    help="rows are dealt to ranks in blocks of this many (1: 600 rows split exactly 8 ways)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"],
                    help="the kernel precision of the line's value (f64: the reference's binary64)")
    ap.add_argument("--no-f32", action="store_true", help="skip the FP32 fast-path record after an f64 line")
    ap.add_argument("--plan", default="auto", choices=["auto", "overlapped", "solo"],
                    help="work plan of each render (rt_exec RT_EXEC_SOLO): auto = solo with one stream, "
                         "overlapped otherwise; tools/pmc_run.sh counts one-stream launches of the "
                         "overlapped plan, the bench line's")
    ap.add_argument("--streams", type=int, default=0, choices=[0, 1, 2, 3, 4],
                    help="frames alternate between this many HIP streams (2: frame i+1 fills the CUs that "
                         "frame i's last long paths leave idle); 0 = auto: 2")
    ap.add_argument("--warmup-s", type=float, default=2.0,
                    help="after the W warm-up frames, keep warming up until the warm-up has rendered this "
                         "many seconds (the per-frame time settles after a few hundred ms); 0: exactly W")
    ap.add_argument("--sim-shards", type=int, default=1,
                    help="diagnostic, one process: render only shard 0 of N (one rank's share of an N-GPU frame)")
    ap.add_argument("--no-abi-devices", action="store_true",
                    help="skip the abi_device_list record (rank 0, after the ranks' measurement)")
    ap.add_argument("--abi-helper", action="store_true",
                    help="internal: the process that times the C-ABI device list for rank 0 (started "
                         "before rank 0 touches a GPU; waits for 'go <devices>' on stdin)")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="nccl (= RCCL, the real path); gloo gathers through host memory (N>1 rehearsal on one "
                         "GPU, with RT_BENCH_ONE_DEVICE=1 mapping every rank to device 0); auto: gloo with "
                         "RT_BENCH_ONE_DEVICE=1, else nccl")
    args = ap.parse_args()
    if args.abi_helper:
        return abi_helper(args)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: start one rank per GPU ourselves (before anything touches a GPU)
        raise SystemExit(spawn_ranks(args.gpus))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_size} ranks; "
                         f"refusing to report a different GPU count than requested")
    one_device = os.environ.get("RT_BENCH_ONE_DEVICE") == "1"
    if args.dist_backend == "auto":
        # RCCL refuses two ranks on one GPU: the one-device rehearsal gathers through gloo
        args.dist_backend = "gloo" if one_device else "nccl"

    # N > 1: rank 0 starts the device-list process now, before this process touches a GPU (it is
    # forked from a process without GPU state), and hands it the devices once the other ranks have
    # exited: the drop-in's caller is a plain process of its own (no torch, no process group)
    helper = None
    if world_size > 1 and int(os.environ.get("RANK", "0")) == 0 and not args.no_abi_devices and args.sim_shards == 1:
        import subprocess
        henv = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        helper = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--abi-helper", "--config", args.config,
                                   "--precision", args.precision, "--steps", str(max(args.steps, 5))],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=henv)

    import torch
    import torch.distributed as dist

    from raytrace_amd import scenes
    from raytrace_amd.camera import image_height
    from raytrace_amd.ray import DeviceScene, assemble_shards, shard_row_index, shard_rows

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n = world_size
    n_sh, sh = (args.sim_shards, 0) if world_size == 1 and args.sim_shards > 1 else (n, rank)
    if one_device:
        local_rank = 0
    elif torch.cuda.device_count() <= local_rank:
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local_rank} but {torch.cuda.device_count()} are visible")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if n > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    fn = scenes.CONFIGS[args.config]
    cs, world, seed = fn()
    h, w, spp = image_height(cs), cs.cs_imageWidth, cs.cs_samplesPerPixel
    scene = DeviceScene(world, device=local_rank)
    rows = shard_rows(h, n_sh, args.row_block)
    if args.streams == 0:
        # two streams for every scene since round 6: with the tail stealing and 1024-lane BVH
        # workgroups, two overlapped BVH launches no longer interfere (bunny's 8-GPU share 18.84 ->
        # 18.00 ms, demo1's 7.90 -> 7.53, pawn+fog's 52.39 -> 51.83; profiles/r6/sweeps/streams)
        args.streams = 2

    def measure(precision):
        """Warm up, then time exactly args.steps frames in `precision`; returns the rank's timings."""
        dtype = torch.float64 if precision == "f64" else torch.float32
        # frame buffers: frame i+1 renders while the RCCL gather of frame i is in flight on the
        # collective's own stream (the compute stream waits for the gather that last read a tile
        # before reusing it).  Two streams at N > 1 take three buffers: gather i starts only after
        # frame i's resolve, which queues behind frame i+1's persistent grid, so with two
        # buffers frame i+2 would wait for that gather and leave frame i+1's tail alone on the CUs
        nbuf = args.streams + (1 if n > 1 and args.streams > 1 else 0) + (1 if n > 1 and args.streams == 1 else 0)
        tiles = [torch.empty((rows, w, 3), dtype=dtype, device=dev) for _ in range(nbuf)]
        # the frame buffers the tiles are gathered into: rank 0 only (the gather's destination)
        gathered = ([torch.empty((n * rows, w, 3), dtype=dtype, device=dev) for _ in range(nbuf)]
                    if n > 1 and rank == 0 else None)
        works = [None] * nbuf
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(args.streams - 1)]
        ev = []
        # N > 1 over RCCL: per timed frame, the gather's completion seen from a probe stream that only
        # waits for it (the compute streams never wait on the probe): render end -> gather done
        probe = torch.cuda.Stream(dev) if n > 1 and args.dist_backend == "nccl" else None
        gev = []
        frame = [0]

        def step(timed):
            b = frame[0] % nbuf
            stream = streams[frame[0] % len(streams)]
            frame[0] += 1
            with torch.cuda.stream(stream):
                frame_step(b, stream, timed)

        def frame_step(b, stream, timed):
            tile = tiles[b]
            if works[b] is not None:
                works[b].wait()  # stream-ordered: the gather that read this tile has completed
                works[b] = None
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            # one stream: frames do not overlap, so each is planned as a lone render (RT_EXEC_SOLO)
            solo = args.plan == "solo" or (args.plan == "auto" and len(streams) == 1)
            scene.render_async(cs, seed, tile.data_ptr(), stream.cuda_stream, n_shards=n_sh, shard=sh,
                               row_block=args.row_block, precision=precision, solo=solo)
            if timed:
                e1.record(stream)
                ev.append((e0, e1))
            if n > 1:
                if args.dist_backend == "nccl":
                    # every rank's tile into rank 0's frame (a gather, not an all-gather;
                    # RCCL point-to-point over each rank's xGMI link to GPU 0)
                    parts = list(gathered[b].chunk(n)) if rank == 0 else None
                    works[b] = dist.gather(tile, gather_list=parts, dst=0, async_op=True)
                    if timed:
                        with torch.cuda.stream(probe):
                            works[b].wait()
                            g = torch.cuda.Event(enable_timing=True)
                            g.record(probe)
                        gev.append((e1, g))
                else:  # rehearsal path: through host memory
                    parts = [torch.empty((rows, w, 3), dtype=dtype) for _ in range(n)] if rank == 0 else None
                    dist.gather(tile.cpu(), gather_list=parts, dst=0)
                    if rank == 0:
                        gathered[b].copy_(torch.cat(parts).to(dev))

        def drain():
            for k in range(nbuf):
                if works[k] is not None:
                    works[k].wait()
                    works[k] = None
            torch.cuda.synchronize(dev)

        # untimed warm-up: W frames, and at least one per stream (a stream's first frame pays for its
        # stream-ordered allocation pool); then, in rounds of doubling length, until the warm-up has
        # kept the GPU busy for --warmup-s seconds: the per-frame time settles only after a few
        # hundred ms of continuous rendering (Cornell 3.56 ms per frame after 2 warm-up frames, 3.47
        # after 100; one rank's share of 8: 0.577 / 0.530 ms).  Ranks agree on every round (the
        # gathers inside the frames must match), so they all run the same number of frames.
        k, warm_frames, warm_s = max(args.warmup, len(streams)), 0, 0.0
        while True:
            tw = time.perf_counter()
            for _ in range(k):
                step(False)
            drain()
            warm_s += time.perf_counter() - tw
            warm_frames += k
            more = warm_s < args.warmup_s and warm_frames < 100000
            if n > 1:
                flag = torch.tensor([int(more)], dtype=torch.int32, device=dev if args.dist_backend == "nccl" else "cpu")
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                more = bool(flag.item())
            if not more:
                break
            k = min(2 * k, 4096)
        if n > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(True)
        drain()  # every frame rendered AND gathered
        if n > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = elapsed_local = time.perf_counter() - t0
        if n > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        # per-launch HIP-event duration, and the device time per frame: the HIP-event span of the
        # timed frames / frames (with --streams 2 consecutive launches overlap, so a launch lasts
        # longer than the device time it costs per frame)
        launch_ms = sum(a.elapsed_time(b) for a, b in ev) / max(1, len(ev))
        kernel_ms = launch_ms
        if ev:
            span = max(ev[0][0].elapsed_time(b) for _, b in ev[-len(streams):])
            kernel_ms = span / len(ev)
        check = None
        if rank == 0:  # (the frame exists on rank 0 only)
            import numpy as np
            last = (frame[0] - 1) % nbuf
            if n > 1:
                parts = gathered[last].view(n, rows, w, 3).cpu().numpy()
                img = assemble_shards(parts, h, args.row_block)
            else:
                img = tiles[last][:h].cpu().numpy() if n_sh == 1 else tiles[last].cpu().numpy()
            import hashlib
            check = {"finite": bool(np.isfinite(img).all()),
                     "mean_rgb": [round(float(x), 5) for x in img.reshape(-1, 3).mean(0)],
                     # digest of the assembled frame's bytes: equal across GPU counts (bit-identical)
                     "sha16": hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()[:16]}
        # per rank (N > 1): which rank and which phase set the max-over-ranks time — its render
        # kernel time per frame, the gathers' completion after its renders, its own wall time
        ranks = None
        if n > 1:
            mine = {"rank": rank, "kernel_ms": round(kernel_ms, 4), "launch_ms": round(launch_ms, 4),
                    "gather_after_render_ms": round(sum(a.elapsed_time(b) for a, b in gev) / len(gev), 4) if gev else None,
                    "ms_per_step_local": round(elapsed_local / args.steps * 1e3, 4)}
            allr = [None] * n
            dist.all_gather_object(allr, mine)
            km = [r["kernel_ms"] for r in allr]
            ranks = {"per_rank": allr, "kernel_ms_min": min(km), "kernel_ms_max": max(km),
                     # the rank whose wall time sets the line's max-over-ranks time, and the one whose
                     # kernels took longest (they differ when the exchange, not the render, is slow)
                     "slowest_rank_wall": max(allr, key=lambda r: r["ms_per_step_local"])["rank"],
                     "slowest_rank_kernel": max(allr, key=lambda r: r["kernel_ms"])["rank"],
                     "note": "kernel_ms: the rank's render device time per frame (HIP events); gather_after_render_ms: "
                             "a frame's render end -> its RCCL gather to rank 0 done on this rank (probe stream, RCCL only); "
                             "ms_per_step_local: the rank's own timed region / frames before the max over ranks"}
        return dict(elapsed=elapsed, launch_ms=launch_ms, kernel_ms=kernel_ms, warm_frames=warm_frames,
                    warm_s=warm_s, check=check, streams=len(streams), ranks=ranks)

    precisions = [args.precision] + (["f32"] if args.precision == "f64" and not args.no_f32 else [])
    res = {p: measure(p) for p in precisions}

    total_samples = h * w * spp
    real_rows = int((shard_row_index(h, n_sh, sh, args.row_block) < h).sum())
    if n_sh != n:  # --sim-shards: the samples of the one shard rendered
        total_samples = real_rows * w * spp
    samples_per_launch = real_rows * w * spp
    share = samples_per_launch / (h * w * spp)  # of the full frame the PMC counts describe
    if rank == 0:
        def record(p):
            r = res[p]
            value = total_samples * args.steps / r["elapsed"] / 1e6
            return value, {"value": round(value, 2), "unit": "Msamples/s", "dtype": p,
                           "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 4),
                           "warmup_frames": r["warm_frames"], "warmup_s": round(r["warm_s"], 3),
                           "roofline": roofline_of(args.config, p, r["kernel_ms"], r["launch_ms"], share,
                                                   samples_per_launch, r["streams"]),
                           "check": r["check"], "ranks": r["ranks"]}
        value, main_rec = record(precisions[0])
        cpu = None
        if n == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(args.config, fn)
            except Exception as e:  # the baseline must never break the bench line
                cpu = {"error": repr(e)}
        pub = PUBLISHED_MSAMPLES.get(args.config)
        line = {
            "metric": METRIC if args.config == "cornell" else f"Msamples/s, {args.config}",
            "value": main_rec["value"], "unit": "Msamples/s", "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "warmup_frames": main_rec["warmup_frames"], "warmup_s": main_rec["warmup_s"],
            "ms_per_step": main_rec["ms_per_step"], "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(value / pub, 1) if pub else None, "dtype": precisions[0],
            "data": "synthetic (reference scene built in-process, no external data)",
            "config": {"workload": f"{args.config} {w}x{h} {spp}spp depth {cs.cs_maxRecursionDepth}",
                       "width": w, "height": h, "spp": spp, "max_depth": cs.cs_maxRecursionDepth,
                       "parallelism": f"rows interleaved over {n} GPU(s), row_block {args.row_block}"
                                      + ((", RCCL gather of the framebuffer to rank 0" if args.dist_backend == "nccl"
                                          else ", gloo gather through host memory (rehearsal)") if n > 1 else "")
                                      + (f" (diagnostic: shard 0 of {n_sh} only)" if n_sh != n else "")},
            "roofline": main_rec["roofline"], "cpu_baseline": cpu, "check": main_rec["check"],
        }
        if main_rec["ranks"] is not None:
            line["ranks"] = main_rec["ranks"]
        if len(precisions) > 1:
            _, f32 = record("f32")
            f32["note"] = "FP32 fast path (rt_exec.flags RT_EXEC_F32), same frames, measured after the f64 line"
            line["f32_fast_path"] = f32
    others = []
    if n > 1:
        pids = [None] * n
        dist.all_gather_object(pids, os.getpid())
        others = [p for r, p in enumerate(pids) if r != rank]
        dist.barrier()
        dist.destroy_process_group()
    scene.close()
    if rank == 0:
        # the drop-in's own multi-GPU path over the same N GPUs, after the ranks' measurement: rank 0
        # alone drives every device through the C-ABI device list once the other ranks have EXITED —
        # a second process holding a context on a GPU (even an idle one) slows the kernels there
        # (one-GPU rehearsal: [0, 0] 13.9 ms per frame beside the idle ranks, 7.05 alone)
        if not args.no_abi_devices and n_sh == n:
            devs = [0] * n if one_device else list(range(n))
            if os.environ.get("RT_BENCH_ABI_DEVICES"):  # diagnostic: another device list (e.g. "0,0")
                devs = [int(x) for x in os.environ["RT_BENCH_ABI_DEVICES"].split(",")]
            try:
                waited = wait_exited(others, timeout_s=120.0)
                if helper is not None:
                    out, _ = helper.communicate("go " + ",".join(map(str, devs)) + "\n", timeout=900)
                    helper = None
                    line["abi_device_list"] = json.loads(out.strip().splitlines()[-1])
                    line["abi_device_list"]["process"] = "its own (started by rank 0 before any GPU call)"
                else:
                    line["abi_device_list"] = abi_device_list(world, cs, seed, devs, precisions[0],
                                                              frames=max(args.steps, 5))
                line["abi_device_list"]["waited_for_ranks_s"] = round(waited, 2)
                line["abi_device_list"]["sha16_equals_line"] = (
                    main_rec["check"] is not None and line["abi_device_list"]["sha16"] == main_rec["check"]["sha16"])
            except Exception as e:  # never break the bench line
                line["abi_device_list"] = {"error": repr(e)}
        print(json.dumps(line), flush=True)
    if helper is not None:  # not used (an error above): let it go
        helper.kill()
        helper.wait()


if __name__ == "__main__":
    main()
