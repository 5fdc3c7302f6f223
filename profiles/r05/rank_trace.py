#!/usr/bin/env python3
"""One rank of a fixed-tiling config on one GPU, for a rocprofv3 kernel trace: WARM frames
pipelined, STEPS frames pipelined (tiles.BandGather, bench.py's depth), then LONE frames one
at a time (render + RGB8 pack, synchronised).  profiles/r05/rank_trace_split.py splits the
trace by these counts: GPU busy fraction and per-kernel time of the pipelined phase, and the
tile-pass / crawl-pass / pack timeline of each lone frame.
  rocprofv3 --kernel-trace -d <dir> -o run -- python3 profiles/r05/rank_trace.py --rank 1"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
p = argparse.ArgumentParser()
p.add_argument("--config", default="C5")
p.add_argument("--world", type=int, default=8)
p.add_argument("--rank", type=int, default=1)
p.add_argument("--layout", default="tiles", choices=["tiles", "bands"])
p.add_argument("--steps", type=int, default=100)
p.add_argument("--warm", type=int, default=20)
p.add_argument("--lone", type=int, default=30)
p.add_argument("--frames-in-flight", type=int, default=0)
a = p.parse_args()
from voxelraymarcher_amd.tiles import pipeline_depth, pipeline_hw_queues  # noqa: E402
depth = a.frames_in_flight or pipeline_depth(a.config)
q = pipeline_hw_queues(depth, a.world)
if q:
    os.environ["GPU_MAX_HW_QUEUES"] = str(q)
import torch  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402

cfg = vr.CONFIGS[a.config]
dev = torch.device("cuda", 0)
scene = vr.create_scene(*cfg.voxels(), cfg.store)
W, H, B, T = cfg.width, cfg.height, 8, (16 if a.layout == "tiles" else 0)
cam, lit, info = vr.Camera.reference(W, H), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
words = vr.tile_buffer_words(W, H, B, T, a.world) if T else vr.band_buffer_words(W, H, B, a.world)
pipe = BandGather(W, H, B, 0, 1, dev, depth=depth)
pipe.bufs = [torch.empty(words, dtype=torch.int32, device=dev) for _ in range(depth)]
packed = [torch.empty(words * 3, dtype=torch.uint8, device=dev) for _ in range(depth)]
k = [0]


def render(buf):
    if T:
        vr.render_tiles(scene, cfg.algorithm, cam, lit, info, W, H, B, T, a.rank, a.world, buf)
    else:
        vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, B, a.rank, a.world, buf)
    vr.pack_rgb8(buf, out=packed[k[0] % depth])
    k[0] += 1


for n in (a.warm, a.steps):
    for _ in range(n):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
st = torch.cuda.current_stream()
for _ in range(a.lone):
    vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, pipe.bufs[0], band_rows=B, rank=a.rank, nranks=a.world,
                 stream=st, schedule=vr.Schedule.GRID, tile_cols=T)
    vr.pack_rgb8(pipe.bufs[0], out=packed[0])
    torch.cuda.synchronize()
print(f"done {a.config} rank {a.rank}/{a.world} {a.layout} depth {depth}", flush=True)
