#!/usr/bin/env python3
"""Kernel time vs image size for one scene/view (tail-effect probe)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr
cfg = vr.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
lit = vr.setup_constant_values()
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
for W, H in [(960, 540), (1920, 1080), (3840, 2160), (7680, 4320)]:
    cam = vr.Camera.reference(W, H)
    out = torch.empty(W * H, dtype=torch.int32, device="cuda")
    for k in (vr.Kernel.TILE, vr.Kernel.PERSISTENT):
        vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, kernel=k)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(); vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, kernel=k); b.record()
        torch.cuda.synchronize()
        ms = np.mean([a.elapsed_time(b) for a, b in ev])
        print(f"{cfg.name} {W}x{H} {k.name:10s} {ms:8.3f} ms  {W*H/ms/1e3:8.1f} Mrays/s", flush=True)
