#!/usr/bin/env python3
"""Can a first render get the learned work order's gain without a prior launch? (VERDICT r4
item 4.)  A list-scheduling model of the tile pass on the oracle's per-pixel work:

  cost of a tile group = max over its two 8x8 waves of (max primary + max shadow iterations)
  (a wave walks its primary rays until its slowest lane ends, then its shadow rays; a
  workgroup's slot is held until its slower wave ends), P = 3584 workgroup slots (256 CUs x
  4 SIMDs x 7 waves / 2 waves per workgroup), duration = 2 us + 0.45 us per iteration
  (~0.45 us per dependent iteration at full load).

It prints the modelled frame time for grid order, the heaviest-first order made from the
true costs (what the learned order approximates), and for orders made from predictors a
first render could compute without walking the frame: a perfect background classifier,
block means of the TRUE costs (an upper bound for any smooth geometric predictor), and the
true cost with Gaussian noise.  On C2 the costs are dominated by per-ray luck (a ray slipping
through gaps between random voxels), so only a per-tile estimate within ~10 iterations
recovers the gain -- and a walk that produces one is itself a ~200-iteration dependent
chain (its longest sampled ray), as long as the frame's own critical path.

  python profiles/r05/first_render_sim.py [C2]     (CPU: the oracle's per-pixel statistics)
"""
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import voxelraymarcher_amd as vr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
cfg = vr.CONFIGS[name]
xyz, rgb = cfg.voxels()
sc = oracle.Scene(xyz, rgb, int(cfg.store))
W, H = cfg.width, cfg.height
it = sc.pixel_stats(int(cfg.algorithm), oracle.reference_camera(W, H), oracle.lighting(), W, H,
                    cfg.scale)[..., 6].astype(np.float64)
Hc, Wc = -(-H // 8) * 8, -(-W // 16) * 16
pad = np.zeros((Hc, Wc, 2))
pad[:H, :W] = it
tiles = pad.reshape(Hc // 8, 8, Wc // 8, 8, 2).transpose(0, 2, 1, 3, 4).reshape(Hc // 8, Wc // 8, 64, 2)
wave = tiles.max(axis=2).sum(-1)
grp = wave.reshape(Hc // 8, Wc // 16, 2).max(-1)
cost = grp.reshape(-1)
n = cost.size
fused = tiles.sum(-1).max(axis=2).reshape(Hc // 8, Wc // 16, 2).max(-1).reshape(-1)


def sim(order, c=cost, P=3584, a=2.0, b=0.45):
    slots = [0.0] * P
    end = 0.0
    for i in order:
        s = heapq.heappop(slots)
        e = s + a + b * c[i]
        end = max(end, e)
        heapq.heappush(slots, e)
    return end


grid = np.arange(n)
print(f"{name} {W}x{H}: {n} tile groups, cost mean {cost.mean():.1f} p50 {np.median(cost):.0f} "
      f"p90 {np.percentile(cost, 90):.0f} max {cost.max():.0f} iterations")
print(f"  grid order                      {sim(grid):7.1f} us")
print(f"  heaviest first (true costs)     {sim(np.argsort(-cost, kind='stable')):7.1f} us")
print(f"  random order                    {sim(np.random.default_rng(0).permutation(n)):7.1f} us")
for T in (3, 20, 40):
    o = np.concatenate([grid[cost > T], grid[cost <= T]])
    print(f"  cost > {T:2d} first (classifier)   {sim(o):7.1f} us")
for k in (2, 4):
    hh, ww = grp.shape[0] // k * k, grp.shape[1] // k * k
    blk = grp[:hh, :ww].reshape(hh // k, k, ww // k, k).mean(axis=(1, 3))
    prox = np.zeros_like(grp)
    prox[:hh, :ww] = np.kron(blk, np.ones((k, k)))
    print(f"  {k}x{k}-group block mean of costs   {sim(np.argsort(-prox.reshape(-1), kind='stable')):7.1f} us")
for sd in (10, 30, 60):
    p = cost + np.random.default_rng(1).normal(0, sd, n)
    print(f"  true cost + N(0, {sd:2d})           {sim(np.argsort(-p, kind='stable')):7.1f} us")
print(f"  per-lane fused primary->shadow: max wave cost {fused.max():.0f} (separate: {cost.max():.0f}); "
      f"heaviest first {sim(np.argsort(-fused, kind='stable'), c=fused):7.1f} us")
