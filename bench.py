#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X ray march on a BASELINE.json config (default
C2, the headline: 256^3 synthetic grid, VCS + original, 1920x1080), plus the
roofline of the dominant kernel and the CPU oracle baseline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5]
                  [--tiling auto|weak|fixed]

A step = one full frame.  With N > 1 ranks the frame is dealt over the ranks --
fixed tiling: learned strips (round 6: rank r renders one contiguous strip of rows, the
strips re-cut from the ranks' measured frame times before timing until their costs are
equal -- compact like a band, balanced like the deal; --layout tiles: the 2-D tile deal,
every 16-row band cut into 16-column blocks, block j of band b -> rank (j + 3b) % N;
--layout bands: whole 16-row bands, band b -> rank b % N); weak tiling: 16-row bands --
each rank renders its share and every frame is gathered to rank 0 over RCCL as RGB8 (3 B
per pixel) and assembled there.  Tiling:
  fixed -- the config's own frame whatever N is (strong scaling; BASELINE C5 is
           defined this way: one 3840x2160 frame tiled over 8 GPUs);
  weak  -- the same view at about N x the pixels (each side x sqrt(N));
  auto  -- fixed for C5, weak for the others (default).
Two frames are in flight (tiles.BandGather: two band buffers, each with its own
stream): the long waves that end frame k overlap the start of frame k+1, and frame
k's gather runs beside frame k+1's render.  Every frame is still rendered in full.
Inputs (scene, camera) are resident in HBM before timing starts; the timed region
ends after the last frame's gather and assembly.  Rank 0 prints ONE JSON line.

`value`/`ms_per_step` are the pipelined throughput; `kernel_ms_first_render` (nothing
learned: grid order, 8x8 tiles), `kernel_ms_grid_order` (grid order, the lane order learned
from earlier launches of the view) and `kernel_ms` (both learned orders) are one launch
timed alone: one pair of HIP events around 200 isolated launches on the launch stream.

roofline: `achieved`/`frac` are the north star's figure for ONE launch as a first render
-- the algorithmic bytes the launch issues (the words the reference walk
reads, counted by the instrumented kernel, minus the existence reads of the crawl
iterations the crawl pass fast-forwards in closed form and never loads:
`algorithmic_bytes_issued_per_launch`, `crawl_iterations_fast_forwarded`) /
`kernel_ms_first_render` / 8 TB/s.  `frac_grid_order` uses `kernel_ms_grid_order`,
`frac_learned_order` `kernel_ms`,
`frac_pipelined` `ms_per_step` (C2 reaches ~1.0 there: its counted 4-B words are
answered by 8-B mask-record loads that mostly hit the vector L1 -- DESIGN.md 6),
`frac_section8d` the unreduced 8(d) bytes.  `dispatch_phases` lists the run's
launch phases in order, so that profiles/roofline_phases.py can recompute every
fraction from a rocprofv3 kernel trace of the same command.
`bound` is the MEASURED limiter, from the round's PMC profile
(profiles/traffic.json, keyed by config, written by profiles/collect_traffic.py):
"valu" when the walk's VALU issue is closer to its roof than the measured HBM
traffic is to the HBM roof (every VCS config: the scene is L2/MALL-resident),
else "hbm".  The line carries both fractions: `hbm_measured_frac` (PMC DRAM
bytes) and `valu_issue_frac` (VALU issue cycles / the chip's SIMD cycles).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
CONFIG_NAMES = ["C1", "C2", "C3", "C4", "C5"]     # voxelraymarcher_amd.CONFIGS (BASELINE.json configs)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="C2", choices=CONFIG_NAMES)
    p.add_argument("--tiling", default="auto", choices=["auto", "weak", "fixed"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--frames-in-flight", type=int, default=0,
                   help="band buffers/streams of the frame pipeline (1 = one frame at a time, for PMC passes; "
                        "default: tiles.pipeline_depth -- 8 for C5, whose frames end in a latency-bound crawl "
                        "pass, else 2; profiles/r03/queues/)")
    p.add_argument("--hw-queues", type=int, default=0,
                   help="hardware queues of this process (GPU_MAX_HW_QUEUES, set before the HIP runtime starts; "
                        "at most 16).  Default: tiles.pipeline_hw_queues -- 16 when the pipeline's streams "
                        "outnumber the runtime's 4 queues -- and an exported GPU_MAX_HW_QUEUES is raised to "
                        "that, never lowered; an explicit --hw-queues sets it as given (clamped to 16, the "
                        "line records requested and effective counts)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="oracle threads (default: the CPUs this process may run on, at most OMP_NUM_THREADS)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes and VALU issue per launch, keyed by config "
                        "(written by profiles/collect_traffic.py)")
    p.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                   help="N > 1 process group: auto/nccl = RCCL over xGMI (one GPU per rank); gloo = the same "
                        "pipeline with the gather staged through host memory (tiles.init_frame_group)")
    p.add_argument("--same-device", action="store_true",
                   help="every rank on cuda:0 (rehearse N ranks on a one-GPU box; needs --backend gloo)")
    p.add_argument("--resolution", default="",
                   help="WxH instead of the config's frame (tests; the same view and scene)")
    p.add_argument("--layout", default="auto", choices=["auto", "bands", "tiles", "strips"],
                   help="how the frame is dealt over N > 1 ranks: 16-row bands, the 2-D tile deal (16-row bands "
                        "cut into --tile-cols column blocks), or learned strips (round 6: one contiguous strip "
                        "of rows per rank, re-cut from the ranks' measured frame times before timing so that "
                        "their costs are equal); auto = strips for fixed tiling, bands for weak")
    p.add_argument("--tile-cols", type=int, default=16, help="column block of the 2-D tile deal (one workgroup)")
    p.add_argument("--exchange", action="store_true",
                   help="run the N > 1 frame exchange (process group, RGB8 pack, gather, rank-0 assembly) even "
                        "with one rank: exercises the RCCL calls on a one-GPU box")
    p.add_argument("--dump-frame", default="",
                   help="rank 0 saves the last frame of the timed loop (.npy): RGB8 [H, W, 3] with N > 1 ranks, "
                        "packed 0x00RRGGBB words [H, W] with one")
    return p.parse_args()


ARGS = parse() if __name__ == "__main__" else None
HW_QUEUES_REQUESTED = None
if ARGS is not None:
    # The frame pipeline's streams must each get a hardware queue of their own, or two
    # frames in flight serialise (profiles/r03/queues/): the queue count is read when the
    # HIP runtime starts, so it is set here, before torch or libvr touch the GPU.
    from voxelraymarcher_amd.tiles import pipeline_depth, pipeline_hw_queues   # (no GPU, no torch.cuda)
    # (the GPU box exports GPU_MAX_HW_QUEUES=4, HIP's default: raised when the pipeline needs more;
    # ranks sharing one GPU (--same-device) keep the default: their queues add up on one device)
    _q = ARGS.hw_queues or (0 if ARGS.same_device else
                            pipeline_hw_queues(ARGS.frames_in_flight or pipeline_depth(ARGS.config),
                                               max(int(os.environ.get("WORLD_SIZE", "1")),
                                                   2 if ARGS.exchange else 1)))
    _have = os.environ.get("GPU_MAX_HW_QUEUES", "")
    if _q and (ARGS.hw_queues or not _have.isdigit() or int(_have) < _q):
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(int(_q), 16))
        if ARGS.hw_queues and ARGS.hw_queues > 16:
            HW_QUEUES_REQUESTED = ARGS.hw_queues

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import (BandGather, frame_resolution, init_frame_group, pipeline_depth,  # noqa: E402
                                       strip_bounds)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
N_SIMD = 1024              # 256 CUs x 4 SIMDs; a wave64 VALU instruction issues over 2 cycles (SIMD-32)
BAND_ROWS = 16             # row bands and the 2-D tile deal's bands: one 16x16 lane-order block high
                           # (8-row bands put two frame strips in one block: C5 rank of 8 0.099 vs
                           # 0.089 ms, C2 weak rank of 8 0.0883 vs 0.0841)
HEADLINE = "Mrays/sec at 1920x1080, 256^3 grid (VCS+original); achieved HBM GB/s"   # BASELINE.json metric
# the learned strip deal (--layout strips): rebalancing rounds, frames timed per round (after
# STRIP_WARM untimed ones: the learned orders of the new strip), strip boundaries on 4-row steps
# (C5 8-rank projection 6.48x with 12 rounds on 4-row steps, 6.40x with 8 on 8-row steps;
# profiles/r06/strips/)
STRIP_ITERS, STRIP_WARM, STRIP_STEPS, STRIP_ALIGN = 12, 16, 80, 4
# the latency cut's lone frames per rank and round (after LAT_WARM untimed ones)
LAT_WARM, LAT_REPS = 4, 7


def learn_strips(pipe, render_rows, W, H, world, rank, dev, stage_host, grouped) -> list:
    """Re-cut pipe's strips from the ranks' frame times (tiles.rebalance_strips): each rank
    times STRIP_STEPS frames of its own strip with pipe.depth frames in flight on pipe's own
    streams (no exchange: a gather would make every rank wait for the slowest), the times
    are all-reduced into one vector, and every rank re-cuts the same strips from it.  Returns
    the rounds' (strips, times); pipe is left with the measured cut whose slowest rank was fastest."""
    from voxelraymarcher_amd.tiles import rebalance_strips
    bounds, est, hist = list(pipe.S), None, []
    nst = len(pipe.streams)
    scratch = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(nst)]
    cur = torch.cuda.current_stream()
    for _ in range(STRIP_ITERS):
        y0, y1 = bounds[rank], bounds[rank + 1]

        def loop(n):
            for i in range(n):
                with torch.cuda.stream(pipe.streams[i % nst]):
                    render_rows(scratch[i % nst], y0, y1)

        for st in pipe.streams:
            st.wait_stream(cur)
        loop(STRIP_WARM)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop(STRIP_STEPS)
        torch.cuda.synchronize()
        t = torch.zeros(world, dtype=torch.float64, device="cpu" if stage_host else dev)
        t[rank] = (time.perf_counter() - t0) / STRIP_STEPS * 1e3
        if grouped:
            dist.all_reduce(t)
        ts = [float(x) for x in t.cpu().tolist()]
        hist.append({"strips": list(bounds), "ms_per_frame": [round(x, 4) for x in ts]})
        bounds, est = rebalance_strips(bounds, ts, STRIP_ALIGN, prior=est)
    # the measured cut whose slowest rank is fastest (the cost model -- uniform within a strip --
    # is coarse where a few rows cost most, C5's crawl rows: its last re-cut is not always the best)
    best = min(hist, key=lambda h: max(h["ms_per_frame"]))
    pipe.set_strips(best["strips"])
    return hist


def learn_latency_strips(pipe, render_rows, W, H, world, rank, dev, stage_host, grouped) -> list:
    """The latency-balanced cut (profiles/rank_projection.py --latency-cut): as learn_strips, but
    each rank times ONE frame of its strip alone (HIP events around the launch on the current
    stream, median of LAT_REPS after LAT_WARM), so the ranks' single-frame latencies are equal --
    the crawl rows' rank gets a short strip.  Returns the rounds; pipe is left with the best cut."""
    from voxelraymarcher_amd.tiles import rebalance_strips
    bounds, est, hist = list(pipe.S), None, []
    buf = torch.empty(W * H, dtype=torch.int32, device=dev)
    cur = torch.cuda.current_stream()
    for _ in range(STRIP_ITERS):
        y0, y1 = bounds[rank], bounds[rank + 1]
        ts = []
        for k in range(LAT_WARM + LAT_REPS):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            render_rows(buf, y0, y1)
            e1.record(cur)
            torch.cuda.synchronize()
            if k >= LAT_WARM:
                ts.append(e0.elapsed_time(e1))
        t = torch.zeros(world, dtype=torch.float64, device="cpu" if stage_host else dev)
        t[rank] = float(np.median(ts))
        if grouped:
            dist.all_reduce(t)
        tv = [float(x) for x in t.cpu().tolist()]
        hist.append({"strips": list(bounds), "lone_ms": [round(x, 4) for x in tv]})
        bounds, est = rebalance_strips(bounds, tv, STRIP_ALIGN, prior=est)
    best = min(hist, key=lambda h: max(h["lone_ms"]))
    pipe.set_strips(best["strips"])
    return hist


def cpu_info() -> dict:
    """The host CPU as lscpu names it, and how many logical CPUs the machine has."""
    info = {"machine_cpus": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() == "Model name":
                info["model"] = v.strip()
            elif k.strip() == "Socket(s)":
                info["sockets"] = int(v.strip())
            elif k.strip() == "Core(s) per socket":
                info["cores_per_socket"] = int(v.strip())
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    return info


def baseline_threads() -> int:
    """All the CPUs this process may use (its affinity mask), capped by
    OMP_NUM_THREADS when set: on a shared GPU box the affinity mask / OMP limit is
    the box's CPU share (16 per GPU), while os.cpu_count() reports the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def _oracle_rate(scene, cam, lit, cfg, threads: int, cpu_seconds: float):
    """Rays per second of the oracle on a bounded sample of the config's frame: 8-row
    bands in a fixed order whose every prefix is spread over the whole frame (band
    97 k mod n for k = 0, 1, ...: a permutation, 97 being prime to the band counts of
    every config), taken until about `cpu_seconds` of CPU time (threads x wall) has
    been spent (at least one band), after one untimed band.  Per-band cost varies a lot
    (C5's crawl rows), so the sample is sized by time, not by a per-ray estimate."""
    W, H = cfg.width, cfg.height
    bands = list(range(0, H, 8))
    n = len(bands)
    step = 97 if n % 97 else 89
    order = [bands[(k * step) % n] for k in range(n)]

    def band(y):
        scene.render(int(cfg.algorithm), cam, lit, W, H, cfg.scale, row_begin=y, row_end=min(H, y + 8),
                     nthreads=threads)
        return (min(H, y + 8) - y) * W

    band(order[0])                                                      # untimed
    rays, i = 0, 0
    t0 = time.perf_counter()
    while True:
        rays += band(order[i % len(order)])
        i += 1
        dt = time.perf_counter() - t0
        if dt * threads >= cpu_seconds:
            break
    return rays, dt, rays / dt / 1e6, i


def cpu_baseline(cfg, xyz, rgb, threads: int) -> dict:
    """The oracle (clean-room C restatement, -O3, OpenMP dynamic over rows) on the host
    cores over the same workload: on `threads` cores (~20 CPU-s) and on
    one core (~6 s)."""
    import oracle
    scene = oracle.Scene(xyz, rgb, int(cfg.store))
    cam = oracle.reference_camera(cfg.width, cfg.height)
    lit = oracle.lighting()
    rays, dt, rate, nbands = _oracle_rate(scene, cam, lit, cfg, threads, 20.0)
    rays1, dt1, rate1, nbands1 = _oracle_rate(scene, cam, lit, cfg, 1, 6.0)
    ci = cpu_info()

    nb = -(-cfg.height // 8)

    def sample(r, k, t, n):
        part = (f"{k} of its {nb} 8-row bands, spread evenly" if k < nb else
                f"the whole frame x{k / nb:.2f}")
        return (f"{r} primary rays of {cfg.name} {cfg.width}x{cfg.height} ({part}) in {t:.2f} s wall on {n} "
                f"thread(s) ({t * n:.1f} CPU-s), oracle/vr_oracle.c -O3 OpenMP")

    return {"value": round(rate, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": sample(rays, nbands, dt, threads),
            "cpu_model": ci.get("model"), "machine_cpus": ci.get("machine_cpus"),
            "threads_note": "all CPUs of this process's affinity mask, capped by OMP_NUM_THREADS (the GPU "
                            "box's CPU share); machine_cpus is the whole host",
            "single_core": {"value": round(rate1, 3), "unit": "Mrays/s", "cores": 1,
                            "sample": sample(rays1, nbands1, dt1, 1)}}


def load_traffic(path: str, cfg_name: str, world: int) -> dict:
    """The round's PMC profile of this config (profiles/traffic.json): {config: {...}},
    or the round-2 single-config form."""
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return {}
    if "config" in tj:                                   # round-2 form: one config
        tj = {tj["config"]: tj}
    t = tj.get(cfg_name, {})
    return t if t.get("world", 1) == world else {}


def main():
    args = ARGS
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    grouped = world > 1 or args.exchange
    dev, backend, stage_host = init_frame_group(world, local, args.backend, args.same_device, force_group=grouped)

    def allreduce(x: float | int, op=dist.ReduceOp.SUM, dtype=torch.float64):
        """A scalar over the ranks (host tensors for gloo, device tensors for RCCL)."""
        t = torch.tensor([x], dtype=dtype, device="cpu" if stage_host else dev)
        if grouped:
            dist.all_reduce(t, op=op)
        return t.item()

    def barrier():
        if grouped:
            dist.barrier()

    cfg = vr.CONFIGS[args.config]
    tiling = args.tiling if args.tiling != "auto" else ("fixed" if cfg.name == "C5" else "weak")
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store, device=dev.index)
    W0, H0 = (int(v) for v in args.resolution.lower().split("x")) if args.resolution else (cfg.width, cfg.height)
    W, H = frame_resolution(W0, H0, world, tiling)
    cam = vr.Camera.reference(W, H)
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    stream = torch.cuda.current_stream()
    # N > 1: bands travel as the RGB8 framebuffer (writeColorToFramebuffer's format, 3 B per
    # pixel): rank 0 ends each frame with the RGB8 image
    depth = args.frames_in_flight or pipeline_depth(args.config)
    layout = args.layout if args.layout != "auto" else ("strips" if tiling == "fixed" else "bands")
    band_rows = BAND_ROWS
    strips0 = strip_bounds([1.0] * H, world, STRIP_ALIGN) if (layout == "strips" and grouped) else None
    pipe = BandGather(W, H, band_rows, rank, world, dev, depth=depth, rgb8=grouped, stage_host=stage_host,
                      tile_cols=args.tile_cols if layout == "tiles" else 0, exchange=grouped, strips=strips0)
    tcols = pipe.T          # 0: row bands or strips (every N = 1 run without --exchange)
    strip = pipe.S is not None

    def prepare(c):
        """The launch of view `c` with its arguments made once (renderer.PreparedRender: the
        timed loop's host path per frame is one ctypes call on the slot's stream)."""
        if strip:
            y0, y1 = pipe.rows()
            return vr.PreparedRender(scene, cfg.algorithm, c, lit, info, W, H, row_begin=y0, row_end=y1)
        return vr.PreparedRender(scene, cfg.algorithm, c, lit, info, W, H, band_rows=band_rows, rank=rank,
                                 nranks=world, tile_cols=tcols)

    # A moving view: the same camera with its eye moved by 1, 2 and 3 ulps in x,
    # one per frame in turn, so no two consecutive launches -- and no launch slot's successive
    # uses (16 slots, 3 views) -- see the same view: nothing is learned (no work or lane order,
    # no crawl-pass skip), every frame renders as a first render does, as for a moving camera.
    moving = []
    for k in (1, 2, 3):
        c = vr.Camera.reference(W, H)
        bits = np.array([c.raw.origin[0]], dtype=np.float32).view(np.uint32) + np.uint32(k)
        c.raw.origin[0] = float(bits.view(np.float32)[0])
        moving.append(c)
    moving_step = [0]

    # algorithmic bytes of THIS rank's launch (its bands; instrumented kernel,
    # untimed) and of the whole frame (sum over ranks); `stats`: the part of
    # them the crawl pass credits for crawl iterations it fast-forwards in closed form
    # (their existence reads are counted, never issued)
    # Learned strips: re-cut the strips from every rank's measured frame time of its own strip
    # (pipelined, no exchange), STRIP_ITERS times (tiles.rebalance_strips), so that the ranks'
    # costs are equal -- every rank computes the same cut from the same all-reduced times
    strip_hist = []
    if strip:
        strip_hist = learn_strips(pipe, lambda buf, y0, y1: vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H,
                                                                         buf, y0, y1),
                                  W, H, world, rank, dev, stage_host, grouped)
    render = prepare(cam)                       # (after the strips are learned: their rows are final)
    moving_prep = [prepare(c) for c in moving]

    def render_moving(buf, stream=None):
        moving_prep[moving_step[0] % 3](buf, stream)
        moving_step[0] += 1
    render_moving.vr_stream_arg = True

    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    stats = torch.zeros(2, dtype=torch.int64, device=dev)
    if strip:
        vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, pipe.bufs[0], *pipe.rows(), counter=ctr, stats=stats)
    else:
        vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, pipe.bufs[0], band_rows=band_rows, rank=rank,
                     nranks=world, counter=ctr, stats=stats, tile_cols=tcols)
    torch.cuda.synchronize()
    launch_bytes = int(ctr.item())
    ff_iters, ff_bytes = (int(x) for x in stats.cpu().tolist())
    issued_bytes = launch_bytes - ff_bytes
    frame_bytes = int(allreduce(launch_bytes, dtype=torch.int64))
    frame_issued = int(allreduce(issued_bytes, dtype=torch.int64))

    for _ in range(args.warmup):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()

    def iso_phase():
        # kernel-only timing of this rank's launch on the launch stream (HIP events; the
        # events bracket the whole launch: tile pass + crawl pass), at least 200 launches:
        # enough samples for kernel_ms, and the GPU reaches its loaded clock before the
        # timed loop starts (a short --steps run otherwise measures the clock ramp of a
        # GPU that sat idle while the host built the scene)
        # Launches on ONE stream run one after the other, so vr_render's AUTO schedule dispatches
        # their heaviest tile groups first (from costs an earlier launch of the slot recorded:
        # the untimed launches below make them); the pipelined loop's launches overlap on
        # BandGather's streams and run in grid order (include/vr.h vr_schedule).  The same
        # launches in grid order are timed too (kernel_ms_grid_order).
        # One event pair brackets each phase of n_iso launches (an event pair around every
        # launch adds ~10 us of event processing to each, profiles/r04/run1: 160.6 vs 150.8 us):
        # kernel_ms = phase time / n_iso -- each launch's tile and crawl passes plus the
        # dispatch gaps between back-to-back launches on one stream.
        n_iso = max(args.steps, 200)
        # A first render of the view, n_iso times: what the device learned (work and lane orders,
        # include/vr.h vr_forget_orders) is dropped before every launch, so each one renders as
        # the reference's one-frame CLI run does (Main.cu:105-163) -- grid order, 8x8 tiles
        ev_first = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev_first[0].record(stream)
        for _ in range(n_iso):
            vr.forget_orders(dev.index)
            render(pipe.bufs[0])
        ev_first[1].record(stream)
        for _ in range(40):
            render(pipe.bufs[0])

        def render_grid(buf):
            if strip:
                vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, buf, *pipe.rows(), stream=stream,
                             schedule=vr.Schedule.GRID)
                return
            vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, buf, band_rows=band_rows, rank=rank, nranks=world,
                         stream=stream, schedule=vr.Schedule.GRID, tile_cols=tcols)

        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev_grid = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for (a, b), fn in ((ev_grid, render_grid), (ev, render)):
            a.record(stream)
            for _ in range(n_iso):
                fn(pipe.bufs[0])
            b.record(stream)
        torch.cuda.synchronize()
        # (the events are read after the timed loop: reading 200 of them takes ~17 ms,
        # long enough for an idle GPU to drop its clock before the timed loop starts)
        # (the W warmup steps stay BEFORE this phase: moved to just before the timed loop
        # they made a 20-step loop slower, 0.1196-0.1205 -> 0.128 ms per step on one box,
        # profiles/r03/driver_ab/; again in round 6, 0.1035-0.1055 -> 0.1109-0.1116,
        # profiles/r06/driver/late_warmup.txt)
        return ev, ev_grid, ev_first, n_iso

    # (before the timed loop: the learned orders of the device's 16 launch slots are made here --
    # after the timed loop instead, the loop's first frames make them, 0.1019-0.1057 -> 0.160 ms
    # per step at 20 steps, profiles/r06/driver/iso_after.txt)
    ev, ev_grid, ev_first, n_iso = iso_phase()

    # N > 1: latency of ONE frame, first launch -> gathered and assembled on
    # rank 0, without the overlap of the pipelined loop
    frame_latency_ms = None
    if grouped:
        lat = []
        for _ in range(5):
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipe.step(render)
            pipe.drain()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        frame_latency_ms = allreduce(float(np.median(lat)) * 1e3, op=dist.ReduceOp.MAX)

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.step(render)
    t_enq = time.perf_counter() - t0            # host time to enqueue every frame
    pipe.drain()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    dt = allreduce(dt, op=dist.ReduceOp.MAX)
    ms_per_step = dt / args.steps * 1e3
    kern_ms = ev[0].elapsed_time(ev[1]) / n_iso
    kern_grid_ms = ev_grid[0].elapsed_time(ev_grid[1]) / n_iso
    kern_first_ms = ev_first[0].elapsed_time(ev_first[1]) / n_iso
    mrays = W * H / (ms_per_step * 1e-3) / 1e6
    if args.dump_frame and rank == 0:
        np.save(args.dump_frame, pipe.last_frame().cpu().numpy())

    # the same pipelined loop with the moving view (nothing learned; after the timed loop)
    barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        pipe.step(render_moving)
    pipe.drain()
    torch.cuda.synchronize()
    barrier()
    dt_mov = allreduce(time.perf_counter() - t1, op=dist.ReduceOp.MAX)
    ms_moving = dt_mov / args.steps * 1e3

    # N > 1 with learned strips: a second cut, balanced on one frame's latency instead of the
    # pipelined rate, and the latency of one frame on it (after the timed loops: the strips and
    # the learned orders of their views change)
    frame_latency_cut_ms, lat_hist = None, []
    thr_strips = list(pipe.S) if strip else None
    if strip and grouped:
        lat_hist = learn_latency_strips(pipe, lambda buf, y0, y1: vr.render_ex(scene, cfg.algorithm, cam, lit, info,
                                                                               W, H, buf, y0, y1),
                                        W, H, world, rank, dev, stage_host, grouped)
        render_lat = prepare(cam)
        for _ in range(16):                     # the new strip's orders learned
            pipe.step(render_lat)
        pipe.drain()
        lat = []
        for _ in range(5):
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipe.step(render_lat)
            pipe.drain()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        frame_latency_cut_ms = allreduce(float(np.median(lat)) * 1e3, op=dist.ReduceOp.MAX)
        if args.dump_frame and rank == 0:           # (the last frame on the latency cut, for the tests)
            root, ext = os.path.splitext(args.dump_frame)
            np.save(root + ".latency_cut" + (ext or ".npy"), pipe.last_frame().cpu().numpy())

    if rank == 0:
        def gbs(nbytes, ms):
            return nbytes / (ms * 1e-3) / 1e9
        # The roofline's numerator: the bytes this launch's walks stand for minus
        # the existence reads of crawl iterations the crawl pass fast-forwards in closed form
        # (it never issues them).  Its duration: one launch on its own as a first render, as
        # the reference's CLI makes (Main.cu:105-163), with no work or lane order learned from
        # earlier launches of the view.  (With frames in flight a launch's events also span
        # the other frame's work, so no per-launch duration exists there; the pipelined rate
        # is frac_pipelined.)
        achieved = gbs(issued_bytes, kern_first_ms)
        tj = load_traffic(args.traffic_json, cfg.name, world)
        traffic = tj.get("hbm_bytes_per_launch")
        roof = {"bound": None, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "achieved_basis": "algorithmic bytes issued per launch (SURVEY 8(d): the words the reference walk "
                                  "reads, counted by the instrumented kernel, minus the existence reads of crawl "
                                  "iterations fast-forwarded in closed form) / the mean duration of one launch "
                                  "alone as a first render (kernel_ms_first_render: learned orders dropped before "
                                  "every launch; tile pass + crawl pass, one HIP event pair on the launch stream "
                                  "around the phase's back-to-back launches) -- mostly served from L2/MALL, not HBM",
                "algorithmic_bytes_per_launch": launch_bytes,
                "algorithmic_bytes_issued_per_launch": issued_bytes,
                "crawl_iterations_fast_forwarded": ff_iters,
                "algorithmic_bytes_per_frame": frame_bytes, "algorithmic_bytes_issued_per_frame": frame_issued,
                "frac_grid_order": round(gbs(issued_bytes, kern_grid_ms) / HBM_PEAK_GBS, 4),
                "frac_learned_order": round(gbs(issued_bytes, kern_ms) / HBM_PEAK_GBS, 4),
                "frac_pipelined": round(gbs(issued_bytes, ms_per_step) / HBM_PEAK_GBS, 4),
                "frac_pipelined_moving_view": round(gbs(issued_bytes, ms_moving) / HBM_PEAK_GBS, 4),
                "frac_section8d": round(gbs(launch_bytes, kern_first_ms) / HBM_PEAK_GBS, 4),
                "fracs_basis": "the same issued bytes over kernel_ms_grid_order (one launch alone in grid order "
                               "with the lane order learned from earlier launches of the view), kernel_ms (one "
                               "launch alone, heaviest tile groups first as well) and ms_per_step (the pipelined "
                               "frame rate); frac_section8d: the full SURVEY 8(d) count over "
                               "kernel_ms_first_render (crawl iterations credited as if loaded). "
                               "profiles/roofline_phases.py recomputes frac, frac_grid_order and "
                               "frac_learned_order from a rocprofv3 kernel trace of the same run. "
                               "frac_pipelined_moving_view: over ms_per_step_moving_view (nothing learned). "
                               "Every frac here is a REFERENCE-EQUIVALENT WORD RATE, cache-served: the 4-B words "
                               "the reference walk reads, answered by 8-B mask-record loads that mostly hit the "
                               "vector L1 / L2 (the scene is L2/MALL-resident), over the HBM peak as SURVEY 8(d) "
                               "defines the roofline -- not HBM traffic (hbm_measured_frac is); above 1 it is "
                               "cache-served words, and the roof that binds is bound / bound_frac",
                }
        hbm_frac = valu_frac = None
        if traffic:
            # what HBM actually serves (PMC DRAM bytes per launch, profiles/)
            hbm = traffic / (kern_ms * 1e-3) / 1e9
            hbm_frac = hbm / HBM_PEAK_GBS
            roof.update({"hbm_measured_gbs": round(hbm, 1), "hbm_measured_frac": round(hbm_frac, 4),
                         "algorithmic_over_hbm_bytes": round(launch_bytes / traffic, 1),
                         "traffic_kernel": tj.get("kernel"),
                         "traffic_basis": "PMC (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction) of ONE launch alone of "
                                          "the tile-pass kernel named in traffic_kernel (the lone-frame occupancy "
                                          "variant), profiles/traffic.json"})
        if tj.get("valu_insts_per_launch") and tj.get("grbm_gui_active_per_launch") and tj.get("rocprof_avg_ns"):
            # VALU issue of the dependent walk: 2 cycles per wave64 instruction on each of the
            # 1024 SIMD-32s, at the clock the profile measured (GRBM_GUI_ACTIVE sums the 8 XCDs)
            cyc = tj["grbm_gui_active_per_launch"] / 8.0
            ghz = cyc / tj["rocprof_avg_ns"]
            valu_cyc = 2.0 * tj["valu_insts_per_launch"]
            valu_frac = valu_cyc / (N_SIMD * cyc)
            roof["valu_issue_frac"] = round(valu_frac, 4)                       # one launch alone
            roof["valu_issue_frac_pipelined"] = round(valu_cyc / (N_SIMD * ghz * ms_per_step * 1e6), 4)
            roof["valu_insts_per_launch"] = tj["valu_insts_per_launch"]
            roof["profile_clock_ghz"] = round(ghz, 3)
            if tj.get("lane_util") is not None:
                roof["valu_lane_utilisation"] = tj["lane_util"]
                # the share of the chip's VALU lane-slots doing a lane's work: issue x lane utilisation
                roof["valu_useful_frac"] = round(valu_frac * tj["lane_util"], 4)
                roof["valu_useful_frac_pipelined"] = round(roof["valu_issue_frac_pipelined"] * tj["lane_util"], 4)
        if hbm_frac is not None and valu_frac is not None:
            roof["bound"] = "valu" if valu_frac >= hbm_frac else "hbm"
            roof["bound_basis"] = ("the measured limiter: VALU issue fraction vs measured HBM fraction "
                                   f"({valu_frac:.3f} vs {hbm_frac:.3f}, profiles/traffic.json)")
            # how close the kernel is to the roof that binds: for VALU the share of the chip's
            # lane-slots doing a lane's work (issue x lane utilisation) of one launch alone, from
            # the PMC pass of the build traffic_kernel / traffic_build name; for HBM the measured
            # DRAM fraction
            if roof["bound"] == "valu":
                roof["bound_frac"] = roof.get("valu_useful_frac", round(valu_frac, 4))
                roof["bound_frac_basis"] = ("valu_useful_frac: VALU issue fraction x lane utilisation of one "
                                            "launch alone (PMC SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU, "
                                            "GRBM_GUI_ACTIVE; profiles/traffic.json)")
            else:
                roof["bound_frac"] = round(hbm_frac, 4)
                roof["bound_frac_basis"] = "hbm_measured_frac (PMC DRAM bytes per launch)"
            if tj.get("build"):
                roof["traffic_build"] = tj["build"]
                import hashlib
                with open(vr.LIB_PATH, "rb") as f:
                    roof["traffic_build_matches"] = tj["build"].endswith(hashlib.sha256(f.read()).hexdigest()[:16])
        else:
            roof["bound"] = "valu" if cfg.store == vr.StorageType.VOXEL_CLUSTER_STORE else "hbm"
            roof["bound_basis"] = "no PMC profile of this config in profiles/traffic.json: by store"
        metric = HEADLINE if cfg.name == "C2" else \
            (f"Mrays/sec at {cfg.width}x{cfg.height}, {cfg.grid}^3 grid ({cfg.store.name}+{cfg.algorithm.name}); "
             f"achieved HBM GB/s")
        gather = ("RCCL gather" if backend == "nccl" else "gloo gather staged through host memory") + \
            (" (ranks sharing cuda:0)" if args.same_device else "")
        deal = (f"learned strips x{world} (rank r renders rows [b_r, b_r+1), b = {pipe.S}, cut by measured cost)"
                if strip else
                f"2-D tile deal x{world} ({band_rows}x{tcols} blocks, block j of {band_rows}-row band b -> rank (j + "
                f"{pipe.stride}b) % {world})" if tcols else f"row-band tiles x{world}")
        par = deal + (f" + {gather} of the RGB8 tiles to rank 0 (overlapped with the next frame)" if grouped else "")
        line = {
            "metric": metric,
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            # value / ms_per_step render the SAME view every step, so the learned per-view
            # orders (work order, lane order) and the crawl-pass skip apply (include/vr.h
            # vr_forget_orders); the moving view renders every frame from scratch
            "view": "repeated identical view (learned per-view work/lane orders and crawl skip apply)",
            "value_moving_view": round(W * H / (ms_moving * 1e-3) / 1e6, 2),
            "ms_per_step_moving_view": round(ms_moving, 4),
            "moving_view_basis": "the same pipelined loop, steps frames, the camera eye moved by 1, 2, 3 ulps in "
                                 "x in turn: no launch sees the view its predecessor or its slot's previous launch "
                                 "saw, so nothing is learned (every frame a first render, as for a moving camera)",
            "higher_is_better": True,
            "scaling": "strong" if tiling == "fixed" else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-hash voxel grid, SURVEY.md 8(d))",
            "config": {"workload": f"{cfg.name}: {cfg.notes}, {W}x{H}" + (
                           "" if world == 1 or tiling == "fixed" else f" (the same view at x{world} pixels, weak "
                                                                       f"scaling)"),
                       "grid": cfg.grid, "width": W, "height": H, "tiling": tiling,
                       "store": cfg.store.name, "algorithm": cfg.algorithm.name, "scale": cfg.scale,
                       "voxels": int(len(rgb)), "parallelism": par, "layout": "strips" if strip else ("tiles" if tcols else "bands"),
                       "frames_in_flight": pipe.depth,
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "runtime default")},
            "kernel_ms": round(kern_ms, 4),
            "kernel_ms_grid_order": round(kern_grid_ms, 4),
            "kernel_ms_first_render": round(kern_first_ms, 4),
            "kernel_ms_basis": f"{n_iso} launches one after the other on one stream, one HIP event pair around them "
                               "(each: tile pass + crawl pass): kernel_ms with the AUTO schedule (heaviest tile "
                               "groups first and the lane order, both learned from earlier launches of the same "
                               "view), kernel_ms_grid_order in grid order with the learned lane order, "
                               "kernel_ms_first_render with what the device learned dropped before every launch "
                               "(vr_forget_orders: grid order, 8x8 tiles -- a first render)",
            "kernel_mrays_per_s": round(W * H / world / (kern_first_ms * 1e-3) / 1e6, 2),
            "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
            "roofline": roof,
            # the non-instrumented launches of this run in order, per phase (a rocprofv3 kernel
            # trace of the same command splits into them: profiles/roofline_phases.py)
            "dispatch_phases": {"strip_calibration": STRIP_ITERS * (STRIP_WARM + STRIP_STEPS) if strip else 0,
                                "warmup": args.warmup, "iso_first": n_iso, "untimed": 40, "iso_grid": n_iso,
                                "iso_learned": n_iso,
                                "latency": 5 if grouped else 0, "timed": args.steps, "moving": args.steps,
                                "latency_cut": (STRIP_ITERS * (LAT_WARM + LAT_REPS) + 16 + 5) if lat_hist else 0},
        }
        if strip:
            line["config"]["strip_bounds"] = thr_strips
            line["config"]["strip_calibration"] = strip_hist
            if lat_hist:
                line["config"]["latency_strip_bounds"] = pipe.S
                line["config"]["latency_calibration"] = lat_hist
        if HW_QUEUES_REQUESTED is not None:
            line["config"]["hw_queues_requested"] = HW_QUEUES_REQUESTED
        if frame_latency_ms is not None:
            line["frame_latency_ms"] = round(frame_latency_ms, 4)
        if frame_latency_cut_ms is not None:
            line["frame_latency_ms_latency_cut"] = round(frame_latency_cut_ms, 4)
            line["frame_latency_basis"] = ("frame_latency_ms: one frame first launch -> gathered on rank 0 on the "
                                           "throughput cut (config.strip_bounds); _latency_cut: the same on strips "
                                           "re-cut from the ranks' lone-frame times (config.latency_strip_bounds)")
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, xyz, rgb, args.cpu_threads or baseline_threads())
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
