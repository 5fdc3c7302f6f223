#!/usr/bin/env python3
"""The 20-step C2 timed loop of bench.py right after its isolated phases (640 back-to-back
launches on one stream), with an idle gap of G ms between them, interleaved over G; and after
a short pipelined run instead (no isolated phases).  Prints the median ms per step per gap."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import torch  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402

cfg = vr.CONFIGS["C2"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
pipe = BandGather(W, H, 16, 0, 1, torch.device("cuda", 0), depth=2)
render = vr.PreparedRender(scene, cfg.algorithm, cam, lit, info, W, H, band_rows=16)
for _ in range(5):
    pipe.step(render)
pipe.drain()
torch.cuda.synchronize()


def iso():
    for _ in range(200):
        vr.forget_orders(0)
        render(pipe.bufs[0])
    for _ in range(40):
        render(pipe.bufs[0])
    for _ in range(200):
        vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, pipe.bufs[0], band_rows=16, schedule=vr.Schedule.GRID)
    for _ in range(200):
        render(pipe.bufs[0])
    torch.cuda.synchronize()


def timed(steps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


gaps = [0, 2, 10, 50, 200]
res = {g: [] for g in gaps}
res["no_iso"] = []
for rep in range(6):
    for g in gaps:
        iso()
        if g:
            time.sleep(g / 1e3)
        res[g].append(timed())
    time.sleep(0.2)
    for _ in range(3):
        timed(20)
    res["no_iso"].append(timed())
for k, v in res.items():
    print(f"gap {k} ms: median {statistics.median(v):.4f} ms/step  ({' '.join(f'{x:.4f}' for x in v)})", flush=True)
