#!/usr/bin/env python3
"""Profiling driver: render one BASELINE config `--iters` times (kernel only,
inputs resident), one launch after another on one stream, printing the HIP-event
average per launch.  `--warmup` untimed launches come first: they give every
launch slot its heaviest-first work order (include/vr.h vr_schedule; the AUTO
schedule of serialised launches), so the timed launches run as bench.py's
kernel_ms launches do.  Run under rocprofv3 by profiles/r03/profile_round.sh;
profiles/trace_avg.py averages the timed (last --iters) dispatches of the trace."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="C2")
p.add_argument("--iters", type=int, default=20)
p.add_argument("--warmup", type=int, default=40)
p.add_argument("--no-shadows", action="store_true")
p.add_argument("--algo", choices=["original", "longestaxis"], default=None)
p.add_argument("--store", choices=["vcs", "hashtable"], default=None)
p.add_argument("--kernel", choices=["auto", "tile", "rewalk"], default="auto")
p.add_argument("--world", type=int, default=1, help="> 1: render only --rank's share of the 2-D tile deal")
p.add_argument("--rank", type=int, default=0)
a = p.parse_args()
kern = {"auto": vr.Kernel.AUTO, "tile": vr.Kernel.TILE, "rewalk": vr.Kernel.TILE_REWALK}[a.kernel]
cfg = vr.CONFIGS[a.config]
store = cfg.store if a.store is None else vr.parse_storage(a.store)
algo = cfg.algorithm if a.algo is None else vr.parse_algorithm(a.algo)
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, store)
W, H = cfg.width, cfg.height
cam = vr.Camera.reference(W, H)
lit = vr.setup_constant_values(use_shadows=not a.no_shadows)
info = vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()


def render():
    if a.world > 1:     # one rank's tiles (8-row bands, 16-column blocks), as bench.py's fixed tiling
        vr.render_tiles(scene, algo, cam, lit, info, W, H, 8, 16, a.rank, a.world, out)
    else:
        vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, out, kernel=kern)


for _ in range(1 + a.warmup):
    render()
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
for e0, e1 in ev:
    e0.record(s)
    render()
    e1.record(s)
torch.cuda.synchronize()
ms = [e0.elapsed_time(e1) for e0, e1 in ev]
o64 = out.to(torch.int64)
digest = int(((o64 & 0xFFFFFFFF) * torch.arange(1, W * H + 1, device=out.device, dtype=torch.int64)).sum()) & 0xFFFFFFFFFFFF
print(f"{a.config} {a.kernel} {store.name} {algo.name} shadows={not a.no_shadows}: mean {np.mean(ms):.4f} ms "
      f"median {np.median(ms):.4f} min {np.min(ms):.4f} ms -> {W * H / np.mean(ms) / 1e3:.1f} Mrays/s "
      f"digest {digest:012x}", flush=True)
