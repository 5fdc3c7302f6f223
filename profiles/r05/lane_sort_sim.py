#!/usr/bin/env python3
"""The learned lane order (vr_march.hip lane_pixel, perm_kernel) on the oracle's per-pixel
work: how many wave-iterations does the tile pass issue when each 16x16 pixel block's 256
pixels are dealt to its four waves heaviest first, instead of one 8x8 tile per wave?

  cost of a wave = max over its lanes of primary iterations + max of shadow iterations
  (the primary and shadow walks are separate loops: a wave runs each until its slowest lane
  ends); lanes are sorted by their pixel's total iterations p + s, and by the weight
  perm_kernel uses, max(p, s) + (p + s) / 8.

  python profiles/r05/lane_sort_sim.py [C2 C3 C4 ...]   (CPU: the oracle's per-pixel statistics)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import voxelraymarcher_amd as vr  # noqa: E402


def wave_iterations(it, sort, weight=lambda p, s: p + s):
    H, W = it.shape[:2]
    Hc, Wc = -(-H // 16) * 16, -(-W // 16) * 16
    pad = np.zeros((Hc, Wc, 2))
    pad[:H, :W] = it
    blk = pad.reshape(Hc // 16, 16, Wc // 16, 16, 2).transpose(0, 2, 1, 3, 4).reshape(-1, 256, 2)
    if sort:
        order = np.argsort(-weight(blk[..., 0], blk[..., 1]), axis=1, kind="stable")
        waves = np.take_along_axis(blk, order[..., None], axis=1).reshape(-1, 4, 64, 2)
    else:   # four 8x8 tiles: rows 0-7 / 8-15 x columns 0-7 / 8-15
        waves = blk.reshape(-1, 2, 8, 2, 8, 2).transpose(0, 1, 3, 2, 4, 5).reshape(-1, 4, 64, 2)
    return waves.max(axis=2).sum()


for name in sys.argv[1:] or ["C2", "C3", "C4"]:
    cfg = vr.CONFIGS[name]
    xyz, rgb = cfg.voxels()
    sc = oracle.Scene(xyz, rgb, int(cfg.store))
    W, H = cfg.width, cfg.height
    it = sc.pixel_stats(int(cfg.algorithm), oracle.reference_camera(W, H), oracle.lighting(), W, H,
                        cfg.scale)[..., 6].astype(np.float64)
    sc.close()
    tiles, lanes = wave_iterations(it, False), wave_iterations(it, True)
    # the weight perm_kernel uses: max(p, s) + (p + s) / 8 (integer, as the kernel computes it)
    kern = wave_iterations(it, True, lambda p, s: np.maximum(p, s) + np.floor((p + s) / 8))
    print(f"{name} {W}x{H}: 8x8 tiles {tiles:.4g} wave-iterations, 16x16 blocks heaviest first {lanes:.4g} "
          f"(ratio {lanes / tiles:.3f}; weight max(p,s)+(p+s)/8: {kern:.4g}, {kern / tiles:.3f}); lane iterations "
          f"{it.sum():.4g}, utilisation {it.sum() / 64 / tiles:.3f} -> {it.sum() / 64 / lanes:.3f}", flush=True)
