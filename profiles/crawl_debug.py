#!/usr/bin/env python3
"""Crawl-pass diagnostics for a debug libvr build (VR_LIBRARY; the crawl pass
writes (plain iterations | fast-forward count << 20) instead of colours):
distribution over the deferred pixels of C5."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

cfg = vr.CONFIGS["C5"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
vr.run_raymarching_kernel(scene, cfg.algorithm, vr.Camera.reference(W, H), vr.setup_constant_values(),
                          vr.VoxelSceneInfo((0, 0, 0), cfg.scale), W, H, out)
torch.cuda.synchronize()
img = out.cpu().numpy().view(np.uint32).reshape(H, W)
band = img[680:720]
plain = band & 0xFFFFF
ffn = (band >> 20) & 0x7FF
sel = (band >> 31) == 1
print("crawl-pass pixels:", int(sel.sum()), " with no fast-forward:", int((sel & (ffn == 0)).sum()))
for name, a in (("plain iterations", plain[sel]), ("fast-forwards", ffn[sel])):
    print(f"{name}: min {a.min()} median {np.median(a):.0f} p90 {np.percentile(a, 90):.0f} max {a.max()} mean {a.mean():.1f}")
