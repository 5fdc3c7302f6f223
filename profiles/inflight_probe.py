#!/usr/bin/env python3
"""Frames in flight: K frames of one config rendered back-to-back on S streams
(frame i on stream i % S, its own output buffer), wall time bracketed by
device synchronisation.  S = 1 is the serial frame loop; S > 1 lets the tail of
frame i (a few long waves) overlap the start of frame i+1.  Prints frames/s,
Mrays/s and whether every frame equals the serial frame.
  python profiles/inflight_probe.py [C2] [K] [tile|rewalk]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
name, _, algo_override = name.partition(":")      # e.g. C5:longestaxis
K = int(sys.argv[2]) if len(sys.argv) > 2 else 60
kern = {"tile": vr.Kernel.TILE, "rewalk": vr.Kernel.TILE_REWALK}[sys.argv[3] if len(sys.argv) > 3 else "tile"]
cfg = vr.CONFIGS[name]
if algo_override:
    import dataclasses
    cfg = dataclasses.replace(cfg, algorithm=vr.parse_algorithm(algo_override))
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
cam = vr.Camera.reference(W, H)
lit = vr.setup_constant_values()
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
ref = torch.empty(W * H, dtype=torch.int32, device="cuda")
vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, ref)
torch.cuda.synchronize()
_w = torch.arange(1, W * H + 1, dtype=torch.int64, device="cuda")
print(f"{name} frame digest {int((ref.to(torch.int64) * _w).sum())} {int(ref.to(torch.int64).sum())}", flush=True)
for S in (1, 2, 3, 4):
    streams = [torch.cuda.Stream() for _ in range(S)]
    outs = [torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in range(S)]
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            vr.run_raymarching_kernel(scene, cfg.algorithm, cam, lit, info, W, H, outs[i % S], stream=streams[i % S],
                                      kernel=kern)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    ok = all(torch.equal(o, ref) for o in outs)
    print(f"{name} {kern.name} streams={S}: {dt / K * 1e3:.4f} ms/frame, {K / dt:.0f} frames/s, "
          f"{W * H * K / dt / 1e6:.0f} Mrays/s, frames equal: {ok}", flush=True)
