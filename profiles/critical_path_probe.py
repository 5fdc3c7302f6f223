#!/usr/bin/env python3
"""Kernel time of a single 8-row band (one wave per tile, no contention) vs the
full frame: isolates the critical path of the slowest waves."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr
cfg = vr.CONFIGS["C2"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)


def t(W, H, r0, r1, shadows=True, reps=10):
    cam = vr.Camera.reference(W, H)
    lit = vr.setup_constant_values(use_shadows=shadows)
    out = torch.empty((r1 - r0) * W, dtype=torch.int32, device="cuda")
    vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, r0, r1)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(); vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, r0, r1); b.record()
    torch.cuda.synchronize()
    return np.median([a.elapsed_time(b) for a, b in ev])


for (W, H, r) in [(960, 540, 208), (1920, 1080, 48)]:
    for sh in (True, False):
        print(f"{W}x{H} shadows={sh}: full {t(W, H, 0, H, sh):.3f} ms   band[{r},{r+8}) {t(W, H, r, r + 8, sh):.3f} ms"
              f"   one tile-row of 8 px at x-range full", flush=True)
print(f"empty band (rows 0-8, sky): {t(1920, 1080, 0, 8):.3f} ms")
