"""Shared helpers: render one configuration through the HIP path (C ABI) and
through the CPU oracle with identical inputs."""
from __future__ import annotations

import os

import numpy as np

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def oracle_camera_from(cam) -> "oracle.OrCamera":
    """Copy a vr.Camera's fields into the oracle struct (same host math, checked separately)."""
    c = oracle.OrCamera()
    for f in ("origin", "lower_left", "horizontal", "vertical", "forward"):
        for i in range(3):
            getattr(c, f)[i] = getattr(cam.raw, f)[i]
    return c


def oracle_lighting_from(lit) -> "oracle.OrLighting":
    o = oracle.OrLighting()
    for f in ("light_dir", "light_color", "light_pos"):
        for i in range(3):
            getattr(o, f)[i] = getattr(lit, f)[i]
    o.use_point_light = lit.use_point_light
    o.use_shadows = lit.use_shadows
    return o


def gpu_render(scene, algo, cam, lit, info, W, H, row_begin=0, row_end=None, count=False, kernel=None, defer_cap=0):
    import torch

    import voxelraymarcher_amd as vr
    row_end = H if row_end is None else row_end
    kernel = vr.Kernel.AUTO if kernel is None else kernel
    out = torch.full(((row_end - row_begin) * W,), -1, dtype=torch.int32, device="cuda")
    nbytes = None
    if count or defer_cap:
        ctr = torch.zeros(1, dtype=torch.int64, device="cuda") if count else None
        vr.render_ex(scene, algo, cam, lit, info, W, H, out, row_begin, row_end, counter=ctr, kernel=kernel,
                     defer_cap=defer_cap)
        torch.cuda.synchronize()
        nbytes = int(ctr.item()) if count else None
    else:
        vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, out, row_begin, row_end, kernel=kernel)
        torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), nbytes


def diff_report(got: np.ndarray, want: np.ndarray, W: int, row_begin: int = 0) -> str:
    bad = np.flatnonzero(got != want)
    if bad.size == 0:
        return "identical"
    lines = [f"{bad.size} of {got.size} pixels differ"]
    for i in bad[:8]:
        lines.append(f"  (x={i % W}, y={row_begin + i // W}): gpu=0x{int(got[i]):08x} oracle=0x{int(want[i]):08x}")
    return "\n".join(lines)
