#!/usr/bin/env python3
"""Wave-divergence study on the CPU oracle's per-pixel work counters: a wave
(8x8 pixel tile) runs its primary walk until its longest lane finishes, then
its shadow walk likewise, so its cost ~ max over lanes.  Prints lane
efficiency = sum(lane iterations) / (64 * sum(per-wave max iterations)).
  python profiles/divergence.py [C2] [tile_w tile_h]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import voxelraymarcher_amd as vr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
cfg = vr.CONFIGS[name]
xyz, rgb = cfg.voxels()
sc = oracle.Scene(xyz, rgb, int(cfg.store))
W, H = cfg.width, cfg.height
st = sc.pixel_stats(int(cfg.algorithm), oracle.reference_camera(W, H), oracle.lighting(), W, H, cfg.scale)
it = st[..., 6].astype(np.float64)          # iterations: [H, W, 2]
print(f"{name} {W}x{H}: mean iterations primary {it[..., 0].mean():.2f} shadow {it[..., 1].mean():.2f}; "
      f"max primary {it[..., 0].max():.0f} shadow {it[..., 1].max():.0f}")
shapes = [(8, 8), (16, 4), (4, 16), (32, 2), (64, 1)]
if len(sys.argv) > 3:
    shapes = [(int(sys.argv[2]), int(sys.argv[3]))]
for tw, th in shapes:
    Hc, Wc = H - H % th, W - W % tw
    t = it[:Hc, :Wc].reshape(Hc // th, th, Wc // tw, tw, 2).transpose(0, 2, 1, 3, 4).reshape(-1, th * tw, 2)
    mx = t.max(axis=1)                      # [waves, 2]
    eff = t.sum(axis=(1, 2)).sum() / (th * tw * mx.sum())
    eff_p = t[..., 0].sum() / (th * tw * mx[:, 0].sum())
    eff_s = t[..., 1].sum() / (th * tw * mx[:, 1].sum())
    joint = t.sum(axis=2).max(axis=1)       # if primary+shadow were one fused loop per lane
    eff_j = t.sum() / (th * tw * joint.sum())
    print(f"  tile {tw}x{th}: lane efficiency {eff:.3f} (primary {eff_p:.3f}, shadow {eff_s:.3f}); "
          f"fused primary+shadow loop {eff_j:.3f}; wave-iterations/frame {mx.sum():.3e} (fused {joint.sum():.3e})")
