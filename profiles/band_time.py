#!/usr/bin/env python3
"""Event-timed renders of chosen 8-row bands of a config (tuning probe).
  python profiles/band_time.py C5 704 0 1000"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

cfg = vr.CONFIGS[sys.argv[1]]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
lit = vr.setup_constant_values()
W, H = cfg.width, cfg.height
cam = vr.Camera.reference(W, H)
out = torch.empty(8 * W, dtype=torch.int32, device="cuda")
for r0 in [int(a) for a in sys.argv[2:]]:
    vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, r0, r0 + 8, kernel=vr.Kernel.TILE)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in ev:
        a.record()
        vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, r0, r0 + 8, kernel=vr.Kernel.TILE)
        b.record()
    torch.cuda.synchronize()
    print(f"{cfg.name} rows [{r0},{r0 + 8}): {np.median([a.elapsed_time(b) for a, b in ev]):.3f} ms", flush=True)
