#!/usr/bin/env python3
"""Event-timed tiny launches: is there a fixed per-launch cost?"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr
cfg = vr.CONFIGS["C2"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
lit = vr.setup_constant_values()
for (W, H, r0, r1) in [(8, 8, 0, 8), (1920, 1080, 0, 1), (1920, 1080, 0, 8), (1920, 1080, 540, 548), (1920, 1080, 0, 1080)]:
    cam = vr.Camera.reference(W, H)
    out = torch.empty((r1 - r0) * W, dtype=torch.int32, device="cuda")
    for k in (vr.Kernel.TILE, vr.Kernel.PERSISTENT):
        vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, r0, r1, kernel=k)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(); vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, r0, r1, kernel=k); b.record()
        torch.cuda.synchronize()
        print(f"{W}x{H} rows[{r0},{r1}) {k.name:10s} median {np.median([a.elapsed_time(b) for a, b in ev]):.4f} ms", flush=True)
