#!/usr/bin/env python3
"""Where the driver's short (20-step) bench line loses time against the 200-step rate:
the same C2 timed loop as bench.py (two frames in flight, BandGather), repeated, with
  A  bench.py as it is: drain() joins both frame streams into the current stream, then
     torch.cuda.synchronize();
  B  no join: the device-wide synchronize alone ends the timed region (it waits for every
     stream; the join only orders later work on the current stream);
  C  B, and the first two frames' streams do not wait for the current stream (it was just
     synchronized: there is nothing to wait for).
Variants interleaved, `reps` timed loops each; prints medians (ms per step).
  python profiles/r06/driver_overhead.py [--steps 20] [--reps 15]"""
from __future__ import annotations

import argparse
import statistics
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--config", default="C2")
    a = ap.parse_args()
    cfg = vr.CONFIGS[a.config]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store)
    W, H = cfg.width, cfg.height
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    dev = torch.device("cuda", 0)
    pipe = BandGather(W, H, 16, 0, 1, dev, depth=2)

    def render(buf):
        vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, 16, 0, 1, buf)

    for _ in range(300):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()

    def run(v):
        torch.cuda.synchronize()
        if v == "C":
            pipe.k = pipe.depth           # (slot 0 first; no join of the idle current stream)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            pipe.step(render)
        if v == "A":
            pipe.drain()
        else:
            pipe.pending.clear()
            pipe.k = 0
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    res = {v: [] for v in "ABC"}
    for _ in range(a.reps):
        for v in "ABC":
            res[v].append(run(v))
    for v, xs in res.items():
        print(f"{v}: median {statistics.median(xs):.4f} ms/step  min {min(xs):.4f}  ({a.steps} steps, {a.reps} reps)")


if __name__ == "__main__":
    main()
