#!/usr/bin/env python3
"""Per-record cost of the crawl pass (C5) from a VR_CRAWL_PROF build (clock reads around
each record only -- no per-iteration counters, so the timing is the product's):
  bash profiles/build_variant.sh cprof -- -DVR_CRAWL_PROF
  VR_LIBRARY=voxelraymarcher_amd/ab/libvr_cprof.so python profiles/crawl_prof.py [C5] [algo]
For every record of the last crawl pass: shader cycles spent on it (clock64 around the
record), its plain loop iterations in the crawl pass (those not fast-forwarded), the
crawl_run calls that applied steps and their loop trips.  Prints distributions and the
records on the critical path (the slowest ones)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voxelraymarcher_amd as vr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C5"
cfg = vr.CONFIGS[name]
algo = cfg.algorithm if len(sys.argv) <= 2 else vr.RayMarchAlgorithm[sys.argv[2]]
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
cam, lit, info = vr.Camera.reference(W, H), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
out = torch.empty(W * H, dtype=torch.int32, device="cuda")
lib = vr.lib()
fn = lib.vr_crawl_prof_fetch
fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
fn.restype = ctypes.c_int
buf = np.zeros(16384 * 8, dtype=np.uint32)
for _ in range(3):
    vr.render_ex(scene, algo, cam, lit, info, W, H, out, schedule=vr.Schedule.GRID)
torch.cuda.synchronize()
ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
ev[0].record()
vr.render_ex(scene, algo, cam, lit, info, W, H, out, schedule=vr.Schedule.GRID)
ev[1].record()
torch.cuda.synchronize()
print(f"{name} {algo.name}: one launch {ev[0].elapsed_time(ev[1]):.3f} ms")
assert fn(buf.ctypes.data, 16384) == 0
p = buf.reshape(-1, 8)
p = p[p[:, 0] > 0]
t0 = p[:, 4].astype(np.int64)
t1 = p[:, 5].astype(np.int64)
base = t0.min()
start_us, dur_us, end_us = (t0 - base) / 100.0, (t1 - t0) / 100.0, (t1 - base) / 100.0
cyc = p[:, 0].astype(np.float64)
plain = (p[:, 1] & 0x7FFFFFFF).astype(np.float64)
rew = (p[:, 1] >> 31).astype(bool)
runs, trips = p[:, 2].astype(np.float64), p[:, 3].astype(np.float64)
print(f"records {len(p)} (walked from the start: {int(rew.sum())})")
print(f"  last record ends {end_us.max():.1f} us after the first starts; starts spread over {start_us.max():.1f} us")
for nm, a in (("start us", start_us), ("dur us", dur_us), ("kcycles", cyc / 1e3), ("plain iters", plain),
              ("crawl runs", runs), ("run trips", trips)):
    print(f"  {nm:12s} min {a.min():9.1f} p50 {np.median(a):9.1f} p90 {np.percentile(a, 90):9.1f} "
          f"p99 {np.percentile(a, 99):9.1f} max {a.max():9.1f} mean {a.mean():9.1f}")
A = np.stack([plain, runs, trips, np.ones_like(plain)], axis=1)
coef, *_ = np.linalg.lstsq(A, cyc, rcond=None)
print(f"  cycles ~ {coef[0]:.0f}/plain iter + {coef[1]:.0f}/run + {coef[2]:.0f}/trip + {coef[3]:.0f}")
top = np.argsort(-cyc)[:12]
A = np.stack([plain, runs, trips, np.ones_like(plain)], axis=1)
coef, *_ = np.linalg.lstsq(A, dur_us, rcond=None)
print(f"  dur_us ~ {coef[0]:.3f}/plain iter + {coef[1]:.3f}/run + {coef[2]:.3f}/trip + {coef[3]:.2f}")
top = np.argsort(-end_us)[:12]
print("  last to end: start_us dur_us kcycles plain runs trips")
for i in top:
    print(f"    {start_us[i]:8.1f} {dur_us[i]:8.1f} {cyc[i] / 1e3:9.1f} {plain[i]:7.0f} {runs[i]:6.0f} {trips[i]:6.0f}"
          f"{'  (rewalk)' if rew[i] else ''}")
