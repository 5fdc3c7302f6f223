#!/usr/bin/env python3
"""Wave-level execution counts of one frame from a VR_DIAG build
(profiles/build_variant.sh diag -- -DVR_DIAG): how many times a wave ran each
loop body and each per-walk / per-ray block.  Multiplied by the blocks' static
VALU counts (profiles/loop_isa.py) this splits the kernel's SQ_INSTS_VALU into
loop and non-loop work.
  VR_LIBRARY=voxelraymarcher_amd/ab/libvr_diag.so python profiles/wave_counts.py [C2]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd import _capi  # noqa: E402

NAMES = {0: "primary VCS walks (sign-specialised)", 1: "primary VCS walks (generic)",
         2: "primary loop iterations (sign-specialised)", 3: "primary loop iterations (generic)",
         4: "shadow VCS walks (specialised)", 5: "shadow VCS walks (generic)",
         6: "shadow loop iterations (specialised)", 7: "shadow loop iterations (generic)",
         8: "grid_original calls (primary)", 9: "grid_original calls (shadow)",
         10: "primary region rounds", 11: "primary null-region skips", 12: "shadow region rounds",
         13: "shadow null-region skips", 14: "primary() calls", 15: "entry-clip iterations",
         16: "shadow walks started", 17: "primary longest-axis walks", 18: "primary longest-axis iterations",
         19: "shadow longest-axis walks", 20: "shadow longest-axis iterations",
         21: "longest-axis iterations with a jumping lane",
         22: "primary iterations, no lane skipping", 23: "primary iterations, every lane skipping",
         24: "shadow iterations, no lane skipping", 25: "shadow iterations, every lane skipping"}

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
cfg = vr.CONFIGS[name]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
cam = vr.Camera.reference(W, H)
lit = vr.setup_constant_values()
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
lib = _capi.lib()
buf = (ctypes.c_ulonglong * 32)()
vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, kernel=vr.Kernel.TILE)
assert lib.vr_diag_fetch(buf, 1) == 0
vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out, kernel=vr.Kernel.TILE)
assert lib.vr_diag_fetch(buf, 1) == 0
waves = ((W + 7) // 8) * ((H + 7) // 8)
print(f"{name} {W}x{H}: {waves} waves")
for k in range(32):
    if buf[k]:
        print(f"  [{k:2d}] {NAMES.get(k, '?'):45s} {buf[k]:12d}  ({buf[k] / waves:8.2f} per wave)")
