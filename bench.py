#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X ray march on BASELINE.json's headline
config (C2: 256^3 synthetic grid, VCS + original, 1920x1080), plus the
roofline of the dominant kernel and the CPU oracle baseline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]

A step = one full frame.  N = 1: the C2 frame exactly.  N > 1 (one rank per
GPU, torch.distributed.run, RCCL): weak scaling over image tiles -- the same
view at N x the pixels (each side x sqrt(N), ~1920x1080 per GPU), rows split
into interleaved 8-row bands (band b -> rank b % N), and every frame gathered
to rank 0 over RCCL as RGB8 (3 B per pixel) and assembled there.  Two frames are in flight
(tiles.BandGather: two band buffers, each with its own stream): the long waves
that end frame k overlap the start of frame k+1, and frame k's gather runs beside
frame k+1's render.  Every frame is still rendered in full.  Inputs (scene,
camera) are resident in HBM before timing starts; the timed region ends after
the last frame's gather and assembly.  Rank 0 prints ONE JSON line.

`value`/`ms_per_step` are the pipelined throughput; `kernel_ms` is one launch
timed alone (HIP events on the launch stream, nothing overlapping).
roofline.achieved = the algorithmic bytes of one launch / that
launch's average duration `kernel_ms` (the figure rocprofv3's per-dispatch
duration reproduces); `achieved_pipelined` = the same bytes x launches per second
in the timed loop (two launches overlap there).  The scene is
L2/MALL-resident, so those bytes are mostly served on-die: the roofline also
carries the PMC-measured HBM bytes (traffic, hbm_measured_*) and the VALU-issue
fraction that actually bounds the walk (valu_issue_frac), both from the
round's profile (profiles/traffic.json, written by profiles/collect_traffic.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather, weak_scaled_resolution  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
BAND_ROWS = 8              # one wave tile high


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="C2", choices=sorted(vr.CONFIGS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--frames-in-flight", type=int, default=2,
                   help="band buffers/streams of the frame pipeline (1 = one frame at a time, for PMC passes)")
    p.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (default min(16, cpus))")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch (written by profiles/collect_traffic.py)")
    return p.parse_args()


def _oracle_rate(scene, cam, lit, cfg, threads: int, cpu_seconds: float):
    """Whole frames of the config, repeated until about `cpu_seconds` of CPU
    time (threads x wall) has been spent, after one untimed frame."""
    t0 = time.perf_counter()
    scene.render(int(cfg.algorithm), cam, lit, cfg.width, cfg.height, cfg.scale, nthreads=threads)
    first = time.perf_counter() - t0
    reps = int(min(60, max(1, np.ceil(cpu_seconds / max(first * threads, 1e-3)))))
    t0 = time.perf_counter()
    for _ in range(reps):
        scene.render(int(cfg.algorithm), cam, lit, cfg.width, cfg.height, cfg.scale, nthreads=threads)
    dt = time.perf_counter() - t0
    return reps, dt, cfg.width * cfg.height * reps / dt / 1e6


def cpu_baseline(cfg, xyz, rgb, threads: int) -> dict:
    """Oracle (clean-room C restatement, OpenMP dynamic over 8x8 tiles) on the
    host cores over the same workload: on `threads` cores (~16
    CPU-s) and on one core (~4 s)."""
    import oracle
    scene = oracle.Scene(xyz, rgb, int(cfg.store))
    cam = oracle.reference_camera(cfg.width, cfg.height)
    lit = oracle.lighting()
    reps, dt, rate = _oracle_rate(scene, cam, lit, cfg, threads, 16.0)
    reps1, dt1, rate1 = _oracle_rate(scene, cam, lit, cfg, 1, 4.0)
    rays = cfg.width * cfg.height * reps
    return {"value": round(rate, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{reps} full {cfg.width}x{cfg.height} frames of {cfg.name} ({rays} primary rays, "
                      f"{dt * threads:.1f} CPU-s), oracle/vr_oracle.c -O2 OpenMP {threads} threads, {dt:.2f} s wall",
            "single_core": {"value": round(rate1, 3), "unit": "Mrays/s", "cores": 1,
                            "sample": f"{reps1} full frames, {dt1:.2f} s"}}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = vr.CONFIGS[args.config]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store, device=local)
    W, H = weak_scaled_resolution(cfg.width, cfg.height, world)
    cam = vr.Camera.reference(W, H)
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    stream = torch.cuda.current_stream()
    # N > 1: bands travel as the RGB8 framebuffer (writeColorToFramebuffer's format, 3 B per
    # pixel): rank 0 ends each frame with the RGB8 image
    pipe = BandGather(W, H, BAND_ROWS, rank, world, dev, depth=args.frames_in_flight, rgb8=world > 1)

    def render(buf):   # on the current stream (BandGather's slot stream in the loops)
        vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, BAND_ROWS, rank, world, buf)

    # algorithmic bytes of THIS rank's launch (its bands; instrumented kernel,
    # untimed) and of the whole frame (sum over ranks)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, pipe.bufs[0], band_rows=BAND_ROWS, rank=rank,
                 nranks=world, counter=ctr)
    torch.cuda.synchronize()
    launch_bytes = int(ctr.item())
    if world > 1:
        dist.all_reduce(ctr)
    frame_bytes = int(ctr.item())

    for _ in range(args.warmup):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()

    # kernel-only timing of this rank's launch on the launch stream (HIP events),
    # at least 200 launches (~35 ms of C2 work): enough samples for kernel_ms, and
    # the GPU reaches its loaded clock before the timed loop starts (a short
    # --steps run otherwise measures the clock ramp of a GPU that sat idle while
    # the host built the scene)
    n_iso = max(args.steps, 200)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_iso)]
    for a, b in ev:
        a.record(stream)
        render(pipe.bufs[0])
        b.record(stream)
    torch.cuda.synchronize()
    # (the events are read after the timed loop: reading 200 of them takes ~17 ms,
    # long enough for an idle GPU to drop its clock before the timed loop starts)

    # N > 1: latency of ONE frame, first launch -> gathered and assembled on
    # rank 0, without the overlap of the pipelined loop
    frame_latency_ms = None
    if world > 1:
        lat = []
        for _ in range(5):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipe.step(render)
            pipe.drain()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        frame_latency_ms = float(np.median(lat)) * 1e3

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    kern_all = [a.elapsed_time(b) for a, b in ev]
    kern_ms = float(np.mean(kern_all))
    kern_median = float(np.median(kern_all))
    mrays = W * H / (ms_per_step * 1e-3) / 1e6

    if rank == 0:
        achieved = launch_bytes / (ms_per_step * 1e-3) / 1e9          # launches overlap: pipelined rate
        achieved_isolated = launch_bytes / (kern_ms * 1e-3) / 1e9
        traffic, tj = None, {}
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("config") == cfg.name and tj.get("world") == world:
                traffic = tj.get("hbm_bytes_per_launch")
            else:
                tj = {}
        except (OSError, ValueError):
            pass
        roof = {"bound": "hbm", "achieved": round(achieved_isolated, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved_isolated / HBM_PEAK_GBS, 4), "traffic": traffic,
                "achieved_basis": "algorithmic bytes per launch (SURVEY 8(d): the words the reference walk reads, "
                                  "counted by the instrumented kernel) / the launch's average duration (kernel_ms, "
                                  "HIP events on the launch stream)",
                "achieved_pipelined": round(achieved, 1),
                "frac_pipelined": round(achieved / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": launch_bytes, "algorithmic_bytes_per_frame": frame_bytes}
        if traffic:
            # what HBM actually serves: the scene is L2/MALL-resident, so the measured
            # DRAM bytes (PMC, profiles/) are a small fraction of the algorithmic ones
            hbm = traffic / (kern_ms * 1e-3) / 1e9                      # per launch, as achieved
            roof.update({"hbm_measured_gbs": round(hbm, 1), "hbm_measured_frac": round(hbm / HBM_PEAK_GBS, 4),
                         "algorithmic_over_hbm_bytes": round(launch_bytes / traffic, 1)})
        if tj.get("valu_insts_per_launch") and tj.get("grbm_gui_active_per_launch") and tj.get("rocprof_avg_ns"):
            # the limiter: VALU issue of the dependent walk (2 cycles per wave64
            # instruction on each of the 1024 SIMD-32s) at the clock the profile measured
            cyc = tj["grbm_gui_active_per_launch"] / 8.0                 # GRBM sums the 8 XCDs
            ghz = cyc / tj["rocprof_avg_ns"]
            valu_cyc = 2.0 * tj["valu_insts_per_launch"]
            roof["limiter"] = "VALU issue and memory latency of the per-pixel walk (not HBM bandwidth)"
            roof["valu_issue_frac"] = round(valu_cyc / (1024 * ghz * ms_per_step * 1e6), 4)
            roof["valu_issue_frac_isolated"] = round(valu_cyc / (1024 * cyc), 4)
            roof["profile_clock_ghz"] = round(ghz, 3)
        line = {
            "metric": "Mrays/sec at 1920x1080, 256^3 grid (VCS+original); achieved HBM GB/s",
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-hash voxel grid, SURVEY.md 8(d))",
            "config": {"workload": f"{cfg.name}: {cfg.notes}" + (
                           "" if world == 1 else f"; the same view at {W}x{H} (x{world} pixels, weak scaling)"),
                       "grid": cfg.grid, "width": W, "height": H,
                       "store": cfg.store.name, "algorithm": cfg.algorithm.name, "scale": cfg.scale,
                       "voxels": int(len(rgb)), "parallelism": f"row-band tiles x{world}" +
                       (" + RCCL gather of the RGB8 bands to rank 0 (overlapped with the next frame)"
                        if world > 1 else ""),
                       "frames_in_flight": pipe.depth},
            "kernel_ms": round(kern_ms, 4),
            "kernel_ms_median": round(kern_median, 4),
            "kernel_mrays_per_s": round(W * H / world / (kern_ms * 1e-3) / 1e6, 2),
            "roofline": roof,
        }
        if frame_latency_ms is not None:
            line["frame_latency_ms"] = round(frame_latency_ms, 4)
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(cfg, xyz, rgb, threads)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
