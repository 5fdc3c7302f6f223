#!/usr/bin/env python3
"""Load balance of the fixed-frame C5 tiling (BASELINE configs[4]: one 3840x2160 frame
over N GPUs) from the oracle's per-pixel work (CPU only):
  per rank, for band heights B and the round-robin deal band b -> rank b % N,
  - walk iterations outside crawls (the tile pass's work; a wave costs its slowest lane),
  - crawling pixels (walks past 4096 iterations: the crawl pass's records, whose
    latency chain ends the frame).
  python profiles/band_balance.py [N] [algo]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
import voxelraymarcher_amd as vr  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
algo = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cfg = vr.CONFIGS["C5"]
xyz, rgb = cfg.voxels()
sc = oracle.Scene(xyz, rgb, 0)
W, H = cfg.width, cfg.height
st = sc.pixel_stats(algo, oracle.reference_camera(W, H), oracle.lighting(), W, H, cfg.scale)
it = st[..., 6].sum(-1).astype(np.int64)                 # [H, W] iterations per pixel
crawl = it > 4096
# a wave (8x8 tile) costs its slowest lane: per-tile max of the non-crawl pixels
tile = np.where(crawl, 0, it).reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))   # [H/8, W/8]
print(f"C5 algo {algo}: {int(crawl.sum())} crawling pixels in rows "
      f"{sorted(set((np.nonzero(crawl)[0] // 8 * 8).tolist()))[:20]}...")
for B in (8, 16, 32, 64):
    nb = -(-H // B)
    wave_cost = np.zeros(N)
    crawls = np.zeros(N, np.int64)
    for b in range(nb):
        r = b % N
        rows = slice(b * B, min(H, (b + 1) * B))
        crawls[r] += int(crawl[rows].sum())
        wave_cost[r] += tile[b * B // 8:min(H, (b + 1) * B) // 8].sum()
    print(f"B={B:3d}: tile-pass work max/mean {wave_cost.max() / wave_cost.mean():.3f}; crawl records per rank "
          f"{crawls.tolist()} (max/mean {crawls.max() / max(crawls.mean(), 1e-9):.2f})")
