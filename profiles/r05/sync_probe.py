#!/usr/bin/env python3
"""Round trip of one small launch on an idle GPU: synchronize, host clock, launch, synchronize,
host clock -- what a timed region pays at its two ends beyond its kernels (bench.py's 20-step
line: the kernels' span is 97 us per frame, the wall clock 104.5; profiles/r05/misc/driver_trace/).
  python profiles/r05/sync_probe.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import voxelraymarcher_amd as vr  # noqa: E402

x = torch.zeros(1 << 20, device="cuda")
torch.cuda.synchronize()


def rt(fn, n=50, idle_s=0.0):
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        if idle_s:
            time.sleep(idle_s)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return np.median(ts), np.percentile(ts, 90)


print("empty sync            %.1f us (p90 %.1f)" % rt(lambda: None))
print("tiny torch kernel     %.1f us (p90 %.1f)" % rt(lambda: x.add_(1.0)))
print("tiny kernel, 1 ms idle %.1f us (p90 %.1f)" % rt(lambda: x.add_(1.0), idle_s=1e-3))
print("tiny kernel, 10 ms idle %.1f us (p90 %.1f)" % rt(lambda: x.add_(1.0), idle_s=1e-2))
cfg = vr.CONFIGS["C1"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = 64, 64
cam, lit, info = vr.Camera.reference(W, H), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
for _ in range(40):
    vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out)
print("64x64 render (tile + crawl pass) %.1f us (p90 %.1f)" %
      rt(lambda: vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out)))
s = torch.cuda.Stream()
def on_side():
    with torch.cuda.stream(s):
        x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
print("tiny kernel on a side stream + wait_stream %.1f us (p90 %.1f)" % rt(on_side))
scene.close()
