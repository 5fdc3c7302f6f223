#!/usr/bin/env python3
"""Localise parity-fuzz mismatches (tests/fuzz_cases.py): for each seed x store x
algorithm, the GPU frame's pixels and algorithmic bytes against the oracle's; on a
byte mismatch, the rows whose byte counts differ (one counted GPU launch per row)
with the oracle's per-pixel bytes of those rows.
  python profiles/fuzz_bytes_probe.py [first_seed] [n_seeds]     (seeds >= 5000: make_wide_case)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import voxelraymarcher_amd as vr  # noqa: E402
from tests.fuzz_cases import make_case, make_wide_case  # noqa: E402
from tests.helpers import gpu_render, oracle_camera_from, oracle_lighting_from  # noqa: E402

first = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 48
for seed in range(first, first + n):
    c = make_wide_case(seed) if seed >= 5000 else make_case(seed)
    cam = vr.Camera(c.eye, c.look_at, c.up, c.fov, c.aspect)
    lit = vr.setup_constant_values(use_shadows=c.shadows, use_point_light=c.point, light_position=c.light_pos,
                                   light_direction=c.light_dir, light_color=c.light_color)
    info = vr.VoxelSceneInfo(c.translation, c.scale)
    ocam, olit = oracle_camera_from(cam), oracle_lighting_from(lit)
    for store in (vr.StorageType.VOXEL_CLUSTER_STORE, vr.StorageType.HASH_TABLE):
        ref = oracle.Scene(c.xyz, c.rgb, int(store))
        gpu = vr.create_scene(c.xyz, c.rgb, store)
        for algo in (vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS):
            want, ob = ref.render(int(algo), ocam, olit, c.W, c.H, c.scale, c.translation)
            got, gb = gpu_render(gpu, algo, cam, lit, info, c.W, c.H, count=True)
            rec = {"seed": seed, "store": store.name, "algo": algo.name, "pixels_equal": bool(np.array_equal(got, want)),
                   "gpu_bytes": gb, "oracle_bytes": ob}
            if gb != ob:
                rows = []
                for y in range(c.H):
                    w1, b1 = ref.render(int(algo), ocam, olit, c.W, c.H, c.scale, c.translation, y, y + 1)
                    g1, gb1 = gpu_render(gpu, algo, cam, lit, info, c.W, c.H, y, y + 1, count=True)
                    if gb1 != b1:
                        px = np.arange(c.W, dtype=np.uint32)
                        _, pb = ref.render_pixels(int(algo), ocam, olit, c.W, c.H, c.scale, px,
                                                  np.full(c.W, y, np.uint32), c.translation)
                        rows.append({"y": y, "gpu": gb1, "oracle": b1, "pixel_bytes": [int(v) for v in pb]})
                rec["rows"] = rows
            print(json.dumps(rec), flush=True)
        gpu.close()
torch.cuda.synchronize()
