#!/usr/bin/env python3
"""Frames/s of render -> PNG at C2 1920x1080:
  render only | render + FrameWriter (pipelined) | render + the reference's
  sequence (pack, blocking D2H into pageable memory, encode, then next frame)."""
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
cfg = vr.CONFIGS["C2"]
W, H = cfg.width, cfg.height
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
words = torch.empty(W * H, dtype=torch.int32, device="cuda")
tmp = tempfile.mkdtemp()


def render():
    vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, out=words)


for _ in range(5):
    render()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(K):
    render()
torch.cuda.synchronize()
r_only = (time.perf_counter() - t) / K

with vr.FrameWriter(W, H, depth=3) as fw:          # warm the encoder threads and pinned buffers
    render(); fw.submit(words, os.path.join(tmp, "w.png"))
torch.cuda.synchronize()
t = time.perf_counter()
with vr.FrameWriter(W, H, depth=3) as fw:
    for k in range(K):
        render()
        fw.submit(words, os.path.join(tmp, f"p{k % 4}.png"))
pipe = (time.perf_counter() - t) / K

t = time.perf_counter()
for k in range(K):
    render()
    host = vr.pack_rgb8(words).cpu().numpy()          # blocking copy into pageable memory
    vr.write_png(os.path.join(tmp, f"s{k % 4}.png"), host.reshape(H, W, 3))
seq = (time.perf_counter() - t) / K
size = os.path.getsize(os.path.join(tmp, "p0.png"))
print(f"C2 {W}x{H}: render only {r_only * 1e3:.3f} ms/frame; render+FrameWriter {pipe * 1e3:.2f} ms/frame "
      f"({1 / pipe:.0f} frames/s); render+blocking output {seq * 1e3:.2f} ms/frame ({1 / seq:.0f} frames/s); "
      f"png {size} B", flush=True)
