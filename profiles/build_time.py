#!/usr/bin/env python3
"""Scene build wall time, host vs device builder, per config."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

torch.cuda.init()
for name in sys.argv[1:] or ["C2", "C4", "C5"]:
    cfg = vr.CONFIGS[name]
    xyz, rgb = cfg.voxels()
    for build in (vr.Build.DEVICE, vr.Build.HOST, vr.Build.DEVICE):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s = vr.create_scene(xyz, rgb, cfg.store, build=build)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"{name} {cfg.store.name:20s} {len(rgb):9d} voxels  {build.name:6s} build {dt * 1e3:9.1f} ms", flush=True)
        s.close()
