#!/usr/bin/env python3
"""How the bench's per-frame time depends on the step count (the fixed cost of
starting from and draining to an idle GPU): bench.py's timed loop, repeated for
several step counts, plus the host time spent enqueuing one step.
  python profiles/steps_probe.py [C2] [depth]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = vr.CONFIGS[name]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
cam = vr.Camera.reference(W, H)
lit = vr.setup_constant_values()
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
dev = torch.device("cuda", 0)
pipe = BandGather(W, H, 8, 0, 1, dev, depth=depth)


def render(buf):
    vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, 8, 0, 1, buf)


for _ in range(10):
    pipe.step(render)
pipe.drain()
torch.cuda.synchronize()
for K in (5, 20, 50, 200, 20):
    res = []
    host = []
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            pipe.step(render)
        th = time.perf_counter()
        pipe.drain()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res.append((t1 - t0) / K * 1e3)
        host.append((th - t0) / K * 1e3)
    print(f"{name} depth={depth} K={K}: ms/step " + " ".join(f"{r:.4f}" for r in res) +
          f" | host enqueue ms/step {min(host):.4f}", flush=True)
