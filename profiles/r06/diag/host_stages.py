#!/usr/bin/env python3
"""Host stage times of each launch in bench.py's timed loop (a VR_HOST_PROF build, e.g.
VR_LIBRARY=voxelraymarcher_amd/ab/libvr_hostprof.so): the C2 sequence of bench.py -- W
pipelined warmup steps, the isolated phases on the current stream, then the timed 20-step
loop (prepared launches on the pipeline's slot streams) -- and per timed launch the stamps
vr_host.cpp launch() takes: entry, slot leased, `alone` queried, view key, orders, crawl
key, kernel launch begin / end (us from the loop's first launch entry)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import torch  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402

cfg = vr.CONFIGS["C2"]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
pipe = BandGather(W, H, 16, 0, 1, torch.device("cuda", 0), depth=2)
render = vr.PreparedRender(scene, cfg.algorithm, cam, lit, info, W, H, band_rows=16)
fetch = vr.lib().vr_host_prof_fetch
fetch.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
for _ in range(5):
    pipe.step(render)
pipe.drain()
torch.cuda.synchronize()


def iso(n_first=200):
    for _ in range(n_first):
        vr.forget_orders(0)
        render(pipe.bufs[0])
    for _ in range(40):
        render(pipe.bufs[0])
    for _ in range(200):
        vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, pipe.bufs[0], band_rows=16, schedule=vr.Schedule.GRID)
    for _ in range(200):
        render(pipe.bufs[0])
    torch.cuda.synchronize()


for rep in range(4):
    if rep < 2:
        iso()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = []
    for _ in range(20):
        a = time.perf_counter()
        pipe.step(render)
        steps.append((time.perf_counter() - a) * 1e6)
    pipe.drain()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20 * 1e3
    buf = (ctypes.c_uint64 * (8 * 20))()
    n = fetch(buf, 20)
    rows = [list(buf[8 * i:8 * i + 8]) for i in range(n)]
    base = rows[0][0]
    print(f"rep {rep} ({'after the isolated phases' if rep < 2 else 'after a timed loop'}): {dt:.4f} ms/step; "
          f"python step us: {' '.join(f'{x:.0f}' for x in steps[:6])} ...", flush=True)
    for i, r in enumerate(rows[:6]):
        d = [(r[j] - r[j - 1]) / 1e3 if r[j] and r[j - 1] else -1 for j in range(1, 8)]
        print(f"  launch {i}: entry +{(r[0] - base) / 1e3:8.1f} us; stages " + " ".join(f"{x:7.1f}" for x in d),
              flush=True)
