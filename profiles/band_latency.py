#!/usr/bin/env python3
"""Single-wave critical path: render one 8-row band of the C2 1080p frame
(240 waves spread over 60 CUs, no contention) -- its kernel time is the
slowest wave's walk alone.  Run under rocprofv3 --kernel-trace for durations.
  python profiles/band_latency.py 352 592 96 1000"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

cfg = vr.CONFIGS["C2"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
lit = vr.setup_constant_values()
W, H = cfg.width, cfg.height
cam = vr.Camera.reference(W, H)
for r0 in [int(a) for a in sys.argv[1:]]:
    out = torch.empty(8 * W, dtype=torch.int32, device="cuda")
    for _ in range(12):
        vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, r0, r0 + 8, kernel=vr.Kernel.TILE)
    torch.cuda.synchronize()
    print("band", r0, "done", flush=True)
