#!/usr/bin/env python3
"""Does any second kernel after the render cost a fixed ~tens of us?  Times
render alone vs render + a 1-element vr_pack_rgb8 on the same stream."""
import os
import sys

import numpy as np
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
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
one = out[:1]


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return np.mean([a.elapsed_time(b) for a, b in ev])


r = lambda: vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, kernel=vr.Kernel.TILE)
print("render alone      %.4f ms" % t(r))
print("render + pack(1)  %.4f ms" % t(lambda: (r(), vr.pack_rgb8(one))))
print("pack(1) alone     %.4f ms" % t(lambda: vr.pack_rgb8(one)))
