#!/usr/bin/env python3
"""bench.py's phase sequence for N = 1 (warmup steps, isolated launches with
HIP events, timed pipelined loop), with one phase changed at a time, to find
what a short timed loop (the driver's --steps 20 --warmup 5) pays for.
  python profiles/bench_phase_probe.py [C2]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
cfg = vr.CONFIGS[name]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
cam = vr.Camera.reference(W, H)
lit = vr.setup_constant_values()
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
dev = torch.device("cuda", 0)


def run(variant, K=20, Wm=5):
    pipe = BandGather(W, H, 8, 0, 1, dev, depth=2)
    stream = torch.cuda.current_stream()

    def render(buf):
        vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, 8, 0, 1, buf)

    if variant == "isolated_first":
        for _ in range(K):
            render(pipe.bufs[0])
        torch.cuda.synchronize()
    for _ in range(Wm):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    if variant in ("bench", "side_stream_isolated"):
        s = stream if variant == "bench" else pipe.streams[0]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        with torch.cuda.stream(s):
            for a, b in ev:
                a.record(s)
                render(pipe.bufs[0])
                b.record(s)
        torch.cuda.synchronize()
        _ = [a.elapsed_time(b) for a, b in ev]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


for rnd in range(3):
    for variant in ("bench", "isolated_first", "side_stream_isolated", "no_isolated"):
        print(f"[{rnd}] {variant:22s} K=20: {run(variant):.4f} ms/step", flush=True)
