#!/usr/bin/env python3
"""RCCL probe on a ONE-GPU box: bench.py's N > 1 frame path (tiles.BandGather with
RGB8 bands, dist.gather over the "nccl" backend = RCCL) run by `world` ranks that
all share cuda:0, compared byte for byte with the single-rank frame.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 profiles/rccl_probe.py [--config C2] [--frames 6]

RCCL may refuse two ranks on one device (the "duplicate GPU" check it shares with
NCCL); the probe then prints that error as its result line and exits 3, so the call
tells which case it was.  Not a test (tests/ run one process per GPU box)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C2")
    p.add_argument("--frames", type=int, default=6)
    a = p.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", device_id=dev)
        dist.barrier()
    except Exception as e:            # RCCL's answer to two ranks on one device
        if rank == 0:
            print(json.dumps({"rccl_two_ranks_one_gpu": "refused", "error": str(e)[:400]}), flush=True)
        sys.exit(3)
    cfg = vr.CONFIGS[a.config]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store, device=0)
    W, H = cfg.width, cfg.height
    cam = vr.Camera.reference(W, H)
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    got = []
    pipe = BandGather(W, H, 8, rank, world, dev, depth=2, rgb8=True,
                      on_frame=(lambda f: got.append(f.clone())) if rank == 0 else None)

    def render(buf):
        vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, 8, rank, world, buf)

    for _ in range(a.frames):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    ok = None
    if rank == 0:
        whole = torch.empty(W * H, dtype=torch.int32, device=dev)
        vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, 8, 0, 1, whole)
        want = vr.pack_rgb8(whole).view(H, W, 3)
        torch.cuda.synchronize()
        ok = [bool(torch.equal(g, want)) for g in got]
    dist.barrier()
    if rank == 0:
        print(json.dumps({"rccl_two_ranks_one_gpu": "ran", "world": world, "config": a.config,
                          "frames": len(got), "frames_equal_single_rank": ok,
                          "rccl_version": ".".join(map(str, torch.cuda.nccl.version()))}), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if rank != 0 or (ok and all(ok)) else 1)


if __name__ == "__main__":
    main()
