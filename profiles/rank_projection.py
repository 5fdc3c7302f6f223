#!/usr/bin/env python3
"""Projected N-GPU frame time of a fixed-tiling config from ONE GPU: each rank r of N
renders only its own 8-row bands (vr_render_bands(r, N), band b -> rank b % N, plus
the RGB8 pack it sends), pipelined exactly as bench.py runs it (tiles.BandGather's
frames in flight), timed alone on the box's one MI355X.  The N-GPU frame rate is set
by the slowest rank (its gather to rank 0 runs beside the next frame),
so max over ranks of the per-rank frame time is the projection -- without the RCCL
gather, which no one-GPU box can run (profiles/r03/rccl/).

The single-frame latency projection (round 4): each rank's ONE frame alone on the GPU
(render of its bands + RGB8 pack, then synchronise), median over --latency-reps launches in
grid order (a first render) and with the learned heaviest-first order; the N-GPU latency is
the slowest rank's (the gather to rank 0 adds its own ~27 us per rank over xGMI).

  python profiles/rank_projection.py [--config C5] [--world 8] [--steps 100]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

p = argparse.ArgumentParser()
p.add_argument("--config", default="C5")
p.add_argument("--world", type=int, default=8)
p.add_argument("--steps", type=int, default=100)
p.add_argument("--warmup", type=int, default=20)
p.add_argument("--frames-in-flight", type=int, default=0, help="default: tiles.pipeline_depth (bench.py's)")
p.add_argument("--ranks", default="", help="comma-separated subset of ranks (default: all)")
p.add_argument("--band-rows", type=int, default=16, help="bench.py's BAND_ROWS")
p.add_argument("--layout", default="tiles", choices=["tiles", "bands", "strips"],
               help="tiles: the 2-D deal (round 5); bands: row bands; strips: the learned cost-balanced "
                    "contiguous strips (round 6: rank r renders rows [b_r, b_r+1), the cuts re-made from the "
                    "ranks' measured frame times --strip-iters times, tiles.rebalance_strips)")
p.add_argument("--strip-iters", type=int, default=12, help="strips: rebalancing rounds")
p.add_argument("--strip-steps", type=int, default=80, help="strips: pipelined frames timed per rank per round")
p.add_argument("--strip-align", type=int, default=4)
p.add_argument("--latency-cut", action="store_true",
               help="strips: also learn a second cut from the ranks' LONE-frame times (grid order, a first "
                    "render: the single frame of the reference's CLI) and project one frame's latency with it")
p.add_argument("--tile-cols", type=int, default=16)
p.add_argument("--latency-reps", type=int, default=30)
p.add_argument("--tiling", default="fixed", choices=["fixed", "weak"],
               help="weak: the frame bench.py --tiling weak renders at --world ranks (each side x sqrt(N))")
a = p.parse_args()

from voxelraymarcher_amd.tiles import pipeline_depth, pipeline_hw_queues  # noqa: E402  (no GPU yet)
depth = a.frames_in_flight or pipeline_depth(a.config)
_q = pipeline_hw_queues(depth)
if _q and not (os.environ.get("GPU_MAX_HW_QUEUES", "").isdigit() and int(os.environ["GPU_MAX_HW_QUEUES"]) >= _q):
    os.environ["GPU_MAX_HW_QUEUES"] = str(_q)      # as bench.py: before the HIP runtime starts

import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402

cfg = vr.CONFIGS[a.config]
dev = torch.device("cuda", 0)
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
if a.tiling == "weak":
    from voxelraymarcher_amd.tiles import frame_resolution
    W, H = frame_resolution(W, H, a.world, "weak")
cam = vr.Camera.reference(W, H)
lit = vr.setup_constant_values()
info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
B = a.band_rows
T = a.tile_cols if a.layout == "tiles" else 0
STRIPS = a.layout == "strips"
bounds = None
if STRIPS:
    from voxelraymarcher_amd.tiles import rebalance_strips, strip_bounds  # noqa: E402
    bounds = strip_bounds([1.0] * H, a.world, a.strip_align)     # equal heights to start
words = (W * H if STRIPS else
         vr.tile_buffer_words(W, H, B, T, a.world) if T else vr.band_buffer_words(W, H, B, a.world))


# ONE pipeline (its streams) for every run: a second BandGather's new streams may share a
# hardware queue (4 per process on the box) and serialise its frames (seen: the second
# pipeline of a process ran C2's rank at 2x the time of every later one)
pipe = BandGather(W, H, B, 0, 1, dev, depth=depth)
pipe.bufs = [torch.empty(max(words, vr.band_buffer_words(W, H, B, 1)), dtype=torch.int32, device=dev)
             for _ in range(depth)]
packed = [torch.empty(words * 3, dtype=torch.uint8, device=dev) for _ in range(depth)]


def send_words():
    """Words each rank sends (equal on every rank: one gather); strips pad to the tallest."""
    if STRIPS:
        return W * max(bounds[r + 1] - bounds[r] for r in range(a.world))
    return words


def run(rank, nranks, steps):
    k = [0]

    def render(buf):
        if STRIPS and nranks > 1:
            vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, buf, bounds[rank], bounds[rank + 1])
        elif T and nranks > 1:
            vr.render_tiles(scene, cfg.algorithm, cam, lit, info, W, H, B, T, rank, nranks, buf)
        else:
            vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, B, rank, nranks, buf)
        if nranks > 1:                                  # the send side of bench.py's N > 1 step
            vr.pack_rgb8(buf[:send_words()], out=packed[k[0] % depth][:3 * send_words()])
        k[0] += 1

    for _ in range(a.warmup):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def lone(rank, nranks, schedule):
    """One frame alone: render + pack on one stream, HIP events around it, median."""
    st = torch.cuda.current_stream()
    buf = pipe.bufs[0]

    def once():
        if STRIPS and nranks > 1:
            vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, buf, bounds[rank], bounds[rank + 1],
                         stream=st, schedule=schedule)
        else:
            vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, buf, band_rows=B, rank=rank, nranks=nranks,
                         stream=st, schedule=schedule, tile_cols=T if nranks > 1 else 0)
        if nranks > 1:
            vr.pack_rgb8(buf[:send_words()], out=packed[0][:3 * send_words()])

    for _ in range(20):
        once()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.latency_reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        once()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


single = run(0, 1, a.steps)
single_lone = {k: lone(0, 1, s) for k, s in (("grid", vr.Schedule.GRID), ("learned", vr.Schedule.HEAVIEST_FIRST))}
calibration = []
if STRIPS:
    # the learned strip deal: each round times every rank's strip pipelined and re-cuts
    est = None
    for it in range(a.strip_iters):
        ts = [run(r, a.world, a.strip_steps) for r in range(a.world)]
        calibration.append({"bounds": list(bounds), "ms_per_frame": [round(t, 4) for t in ts]})
        print(json.dumps({"strip_round": it, **calibration[-1]}), flush=True)
        bounds, est = rebalance_strips(bounds, ts, a.strip_align, prior=est)
    # as bench.py: the measured cut whose slowest rank was fastest
    bounds = min(calibration, key=lambda c: max(c["ms_per_frame"]))["bounds"]
ranks = []
for r in ([int(x) for x in a.ranks.split(",")] if a.ranks else range(a.world)):
    ms = run(r, a.world, a.steps)
    lg = lone(r, a.world, vr.Schedule.GRID)
    ll = lone(r, a.world, vr.Schedule.HEAVIEST_FIRST)
    ranks.append({"rank": r, "ms_per_frame": round(ms, 4),
                  "lone_frame_ms_grid": round(lg, 4), "lone_frame_ms_learned": round(ll, 4)})
    print(json.dumps(ranks[-1]), flush=True)
latency_cut = None
if STRIPS and a.latency_cut:
    # the latency-balanced strips: the same rebalancing, from each rank's lone frame time
    thr_bounds, cal_l, est = bounds, [], None
    bounds = strip_bounds([1.0] * H, a.world, a.strip_align)
    for it in range(a.strip_iters):
        ts = [lone(r, a.world, vr.Schedule.GRID) for r in range(a.world)]
        cal_l.append({"bounds": list(bounds), "lone_ms_grid": [round(t, 4) for t in ts]})
        print(json.dumps({"latency_round": it, **cal_l[-1]}), flush=True)
        bounds, est = rebalance_strips(bounds, ts, a.strip_align, prior=est)
    bounds = min(cal_l, key=lambda c: max(c["lone_ms_grid"]))["bounds"]
    lg = [lone(r, a.world, vr.Schedule.GRID) for r in range(a.world)]
    ll = [lone(r, a.world, vr.Schedule.HEAVIEST_FIRST) for r in range(a.world)]
    latency_cut = {"bounds": bounds, "calibration": cal_l,
                   "lone_frame_ms_grid": [round(x, 4) for x in lg], "lone_frame_ms_learned": [round(x, 4) for x in ll],
                   "projected_lone_frame_ms": {"grid": round(max(lg), 4), "learned": round(max(ll), 4)},
                   "projected_latency_speedup": {"grid": round(single_lone["grid"] / max(lg), 2),
                                                 "learned": round(single_lone["learned"] / max(ll), 2)}}
    print(json.dumps({"latency_cut": latency_cut}), flush=True)
    bounds = thr_bounds
slow = max(x["ms_per_frame"] for x in ranks)
slow_lg = max(x["lone_frame_ms_grid"] for x in ranks)
slow_ll = max(x["lone_frame_ms_learned"] for x in ranks)
mean = sum(x["ms_per_frame"] for x in ranks) / len(ranks)
mean_lg = sum(x["lone_frame_ms_grid"] for x in ranks) / len(ranks)
print(json.dumps({"config": a.config, "width": W, "height": H, "world": a.world, "band_rows": B,
                  "layout": a.layout, "tile_cols": T, "strip_bounds": bounds, "strip_calibration": calibration,
                  "slowest_over_mean": round(slow / mean, 3), "slowest_over_mean_lone_grid": round(slow_lg / mean_lg, 3),
                  "frames_in_flight": depth,
                  "steps": a.steps, "one_gpu_ms_per_frame": round(single, 4),
                  "projected_ms_per_frame": slow, "projected_speedup": round(single / slow, 2),
                  "projected_mrays_per_s": round(W * H / (slow * 1e-3) / 1e6, 1),
                  "one_gpu_lone_frame_ms": {k: round(v, 4) for k, v in single_lone.items()},
                  "projected_lone_frame_ms": {"grid": slow_lg, "learned": slow_ll},
                  "projected_latency_speedup": {"grid": round(single_lone["grid"] / slow_lg, 2),
                                                "learned": round(single_lone["learned"] / slow_ll, 2)},
                  "latency_cut": latency_cut,
                  "note": "max over ranks of each rank's own pipelined frame time on one GPU; RCCL gather not "
                          "included (overlapped with the next frame in bench.py)"}), flush=True)
