"""The tile pass's occupancy variants, forced (vr_render_opts.occupancy, include/vr.h).

With frames in flight the AUTO schedule renders with the in-flight occupancy variant of a walk
where a build has one (vr_march.hip TileWaves, march_kernel<..., true>: rounds 4-5 ran the
cuckoo `original` walk at 8 waves per SIMD and the VCS `longestaxis` walk at 7; since round 6
every walk is fastest in flight with its lone kernel, so the default build launches that), but
AUTO picks it only when another stream's launch is still running, which a test cannot arrange
deterministically.  VR_OCCUPANCY_IN_FLIGHT forces it: every frame here is rendered through the
in-flight path and must equal the committed oracle digest (tests/golden/frames.json) and the
lone variant's frame, pixel for pixel.
  C4: CuckooHashTable::lookupVoxel (CuckooHashTable.cuh:59-76) in rayMarchVoxelGrid
      (Renderer.cuh:260-336), the whole 1920x1080 frame over the 20 M-voxel store;
  C3: rayMarchVoxelGridLongestAxis / performVoxelSpaceJump (Renderer.cuh:696-915), the
      whole 1920x1080 frame;
  C5 longest axis: the whole 3840x2160 frame (its crawl rows walk up to 1.4 million
      iterations, deferred to the crawl pass) and the committed longest walks
      (tests/golden/c5_crawl_pixels.json).
The VCS `original` walk never had an in-flight variant (8 waves measured slower); forcing it
renders with the lone kernel, which is checked too."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

from tests.helpers import GOLDEN, diff_report

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")
FRAMES = {f["name"]: f for f in json.load(open(os.path.join(GOLDEN, "frames.json")))["frames"]}


def render(scene, cfg, algo, occupancy, row_begin=0, row_end=None, schedule=None):
    import torch
    W, H = cfg.width, cfg.height
    row_end = H if row_end is None else row_end
    out = torch.full(((row_end - row_begin) * W,), -1, dtype=torch.int32, device="cuda")
    vr.render_ex(scene, algo, vr.Camera.reference(W, H), vr.setup_constant_values(),
                 vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale), W, H, out, row_begin, row_end,
                 occupancy=occupancy, schedule=schedule if schedule is not None else vr.Schedule.AUTO)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def digest(img):
    return hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()


@pytest.mark.parametrize("name,cfg_name,algo", [("C4", "C4", vr.RayMarchAlgorithm.ORIGINAL),
                                                ("C3", "C2", vr.RayMarchAlgorithm.LONGEST_AXIS),
                                                ("C2", "C2", vr.RayMarchAlgorithm.ORIGINAL)])
def test_in_flight_variant_full_frame(name, cfg_name, algo):
    cfg = vr.CONFIGS[cfg_name]
    scene = vr.create_scene(*cfg.voxels(), cfg.store)
    lone = render(scene, cfg, algo, vr.Occupancy.LONE)
    assert digest(lone) == FRAMES[name]["sha256"], name
    for schedule in (vr.Schedule.GRID, vr.Schedule.HEAVIEST_FIRST):
        hi = render(scene, cfg, algo, vr.Occupancy.IN_FLIGHT, schedule=schedule)
        assert np.array_equal(hi, lone), f"{name} in-flight variant: " + diff_report(hi, lone, cfg.width)
        assert digest(hi) == FRAMES[name]["sha256"], name
    scene.close()


def test_in_flight_variant_c5_longest_axis():
    """C5, longest axis, forced in-flight variant (the lone kernel unless a build makes one): the whole 4K frame
    against the committed digest, and the committed longest walks (rows 696-711)."""
    cfg = vr.CONFIGS["C5"]
    scene = vr.create_scene(*cfg.voxels(), vr.StorageType.VOXEL_CLUSTER_STORE)
    algo = vr.RayMarchAlgorithm.LONGEST_AXIS
    full = render(scene, cfg, algo, vr.Occupancy.IN_FLIGHT)
    assert digest(full) == FRAMES["C5-longestaxis"]["sha256"]
    rows = render(scene, cfg, algo, vr.Occupancy.IN_FLIGHT, 696, 712)
    assert np.array_equal(rows, full[696 * cfg.width:712 * cfg.width])
    fx = json.load(open(os.path.join(GOLDEN, "c5_crawl_pixels.json")))["pixels"]
    n = 0
    for p in fx:
        if p["algo"] == int(algo):
            assert int(rows[(p["y"] - 696) * cfg.width + p["x"]]) == p["colour"], p
            n += 1
    assert n > 0
    scene.close()


def test_occupancy_rejects_unknown_value():
    import torch
    cfg = vr.CONFIGS["C1"]
    scene = vr.create_scene(*cfg.voxels(), cfg.store)
    out = torch.empty(64 * 64, dtype=torch.int32, device="cuda")
    with pytest.raises(vr.VrError):
        vr.render_ex(scene, cfg.algorithm, vr.Camera.reference(64, 64), vr.setup_constant_values(),
                     vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale), 64, 64, out, occupancy=3)
    scene.close()
