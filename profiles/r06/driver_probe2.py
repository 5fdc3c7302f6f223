#!/usr/bin/env python3
"""Where the driver's 20-step C2 line (bench.py --steps 20 --warmup 5) loses time against the
pipelined rate, split on ONE clock pair: host perf_counter around the timed loop as bench.py
takes it, plus HIP events recorded on the current stream at t0 (a marker the idle GPU runs as
soon as it sees it) and after drain().  Per rep:
  host_ms      t0 -> synchronize() returned (bench.py's dt)
  gpu_ms       marker at t0 -> marker after the last frame (GPU clock)
  first_enq_us host time of the first pipe.step (Python + launch)
  enq_us       host time to enqueue all steps
The difference host - gpu is the start-up latency of the first submission plus the wake-up of
the final synchronize; gpu - steps x steady is the pipeline's fill and drain.
  --spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before torch starts (the host thread spins on
          completion instead of sleeping on an interrupt)
  python profiles/r06/driver_probe2.py [--steps 20] [--reps 30] [--spin]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--config", default="C2")
ap.add_argument("--spin", action="store_true")
ap.add_argument("--prelude", action="store_true", help="also time runs that follow bench.py's isolated phase "
                "(n launches one after the other on the current stream), interleaved with plain runs")
ap.add_argument("--lean", action="store_true", help="also time a lean step: pre-built ctypes arguments, raw stream "
                "handles, pre-made join events (no torch stream context, no per-step Event)")
a = ap.parse_args()
if a.spin:
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))      # hipDeviceScheduleSpin
    print(json.dumps({"hipSetDeviceFlags_spin_rc": rc}), flush=True)

import torch  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402
from voxelraymarcher_amd.tiles import BandGather  # noqa: E402


def main():
    cfg = vr.CONFIGS[a.config]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store)
    W, H = cfg.width, cfg.height
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    dev = torch.device("cuda", 0)
    pipe = BandGather(W, H, 16, 0, 1, dev, depth=2)

    def render(buf):
        vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, 16, 0, 1, buf)

    for _ in range(300):
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()

    def run(steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(cur)
        pipe.step(render)
        t1 = time.perf_counter()
        for _ in range(steps - 1):
            pipe.step(render)
        t2 = time.perf_counter()
        pipe.drain()
        e1.record(cur)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        return {"host_ms": (t3 - t0) * 1e3, "gpu_ms": e0.elapsed_time(e1), "first_enq_us": (t1 - t0) * 1e6,
                "enq_us": (t2 - t0) * 1e6}

    if a.lean:
        import ctypes as C
        from voxelraymarcher_amd._capi import lib, f3
        fn = lib().vr_render_bands
        pre = (scene.handle, int(cfg.algorithm), C.byref(cam.raw), C.byref(lit), f3(info.translation),
               int(info.scale), W, H, 16, 0, 1)
        sp = [C.c_void_p(st.cuda_stream) for st in pipe.streams]
        bp = [C.c_void_p(b.data_ptr()) for b in pipe.bufs]
        joins = [torch.cuda.Event() for _ in pipe.streams]

        def lean_step(k):
            slot = k % 2
            if k < 2:
                joins[slot].record(cur)
                pipe.streams[slot].wait_event(joins[slot])
            if fn(*pre, bp[slot], sp[slot]):
                raise RuntimeError("vr_render_bands")

        def run_lean(steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(cur)
            lean_step(0)
            t1 = time.perf_counter()
            for k in range(1, steps):
                lean_step(k)
            t2 = time.perf_counter()
            for st in pipe.streams:
                cur.wait_stream(st)
            e1.record(cur)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            return {"host_ms": (t3 - t0) * 1e3, "gpu_ms": e0.elapsed_time(e1), "first_enq_us": (t1 - t0) * 1e6,
                    "enq_us": (t2 - t0) * 1e6}

        for _ in range(50):
            run_lean(2)
        rl, rb = [], []
        for _ in range(a.reps):
            rb.append(run(a.steps))
            rl.append(run_lean(a.steps))
        for name, rs in (("bench_step", rb), ("lean_step", rl)):
            med = {k: round(statistics.median(r[k] for r in rs), 4) for k in rs[0]}
            print(json.dumps({"variant": name, "median": med, "host_ms_per_step": round(med["host_ms"] / a.steps, 5),
                              "host_minus_gpu_us": round((med["host_ms"] - med["gpu_ms"]) * 1e3, 1)}), flush=True)
    if a.prelude:
        def iso(n, schedule):
            for _ in range(n):
                vr.render_ex(scene, cfg.algorithm, cam, lit, info, W, H, pipe.bufs[0], band_rows=16, schedule=schedule)
        variants = {"plain": lambda: None,
                    "after_200_learned": lambda: iso(200, vr.Schedule.AUTO),
                    "after_200_grid": lambda: iso(200, vr.Schedule.GRID),
                    "after_200_first": lambda: [(vr.forget_orders(0), iso(1, vr.Schedule.AUTO)) for _ in range(200)]}
        res = {k: [] for k in variants}
        for _ in range(a.reps):
            for k, f in variants.items():
                f()
                res[k].append(run(a.steps))
        for k, rs in res.items():
            med = {q: round(statistics.median(r[q] for r in rs), 4) for q in rs[0]}
            print(json.dumps({"variant": k, "median": med, "host_ms_per_step": round(med["host_ms"] / a.steps, 5),
                              "max_host_ms_per_step": round(max(r["host_ms"] for r in rs) / a.steps, 5)}), flush=True)
    steady = statistics.median(run(200)["gpu_ms"] / 200 for _ in range(5))
    rs = [run(a.steps) for _ in range(a.reps)]
    med = {k: round(statistics.median(r[k] for r in rs), 4) for k in rs[0]}
    out = {"steps": a.steps, "reps": a.reps, "spin": a.spin, "steady_ms_per_frame_200": round(steady, 5),
           "median": med, "host_ms_per_step": round(med["host_ms"] / a.steps, 5),
           "host_minus_gpu_us": round((med["host_ms"] - med["gpu_ms"]) * 1e3, 1),
           "fill_drain_us": round((med["gpu_ms"] - a.steps * steady) * 1e3, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
