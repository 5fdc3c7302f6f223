"""GPU test of the tile pass's heaviest-first work order (vr_host.cpp, KView::order):
each launch slot keeps an order of the tile groups made from the costs an earlier
launch of that slot recorded, and the tile pass renders tile group order[i] in
workgroup i.  Any permutation must render the same pixels, including an order made
for a different view of the same grid size and orders remade while other launches
are in flight.  Every frame below must equal the serial render and, for the
reference view, the committed oracle digest."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FRAMES = {f["name"]: f for f in json.load(open(os.path.join(GOLDEN, "frames.json")))["frames"]}


@pytest.mark.parametrize("algo", [vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS],
                         ids=lambda a: a.name)
def test_ordered_launches_two_views_in_flight(algo):
    cfg = vr.CONFIGS["C2"]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store)
    W, H = cfg.width, cfg.height
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    # the reference view and a second view of the same size (its heavy tiles elsewhere)
    cams = [vr.Camera.reference(W, H),
            vr.Camera((-3.0, 5.0, 8.0), (1.0, -1.0, -2.0), (0.0, 1.0, 0.0), 50.0, W / H)]
    refs = []
    for cam in cams:
        out = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
        vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, out)
        torch.cuda.synchronize()
        refs.append(out.clone())
    name = "C2" if algo == vr.RayMarchAlgorithm.ORIGINAL else "C3"
    img = refs[0].cpu().numpy().view(np.uint32)
    assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == FRAMES[name]["sha256"]
    # 48 launches (three uses of each of the ring's 16 slots) on two streams, the two views
    # alternating in runs of three: each view's orders are learned within its runs (a launch
    # whose previous launch rendered the same view) and used only for that view
    streams = [torch.cuda.Stream() for _ in range(2)]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    n = 48
    outs = [torch.full((W * H,), -1, dtype=torch.int32, device="cuda") for _ in range(n)]
    which = [(i // 3) % 2 for i in range(n)]
    for i in range(n):
        # (launches overlapping on two streams: AUTO would pick grid order; force the order)
        vr.render_ex(scene, algo, cams[which[i]], lit, info, W, H, outs[i], stream=streams[i % 2],
                     schedule=vr.Schedule.HEAVIEST_FIRST)
    torch.cuda.synchronize()
    bad = [i for i in range(n) if not torch.equal(outs[i], refs[which[i]])]
    assert not bad, f"{len(bad)} of {n} ordered launches differ from the serial render (first: {bad[:5]})"
    scene.close()


def test_ordered_launches_grid_change():
    # orders are per view: frame sizes alternating in runs of two (each view's orders made on
    # its repeats) never use an order of another size
    cfg = vr.CONFIGS["C1"]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store)
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    sizes = [(320, 240), (336, 200), (64, 8)]
    refs = {}
    for W, H in sizes:
        out = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
        vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, vr.Camera.reference(W, H), lit, info, W, H,
                                  out)
        torch.cuda.synchronize()
        refs[(W, H)] = out.clone()
    for i in range(96):
        W, H = sizes[(i // 2) % 3]
        out = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
        vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, vr.Camera.reference(W, H), lit, info, W, H,
                                  out)
        torch.cuda.synchronize()
        assert torch.equal(out, refs[(W, H)]), f"launch {i} ({W}x{H})"
    scene.close()


def test_schedules_render_identical_pixels():
    # AUTO on one stream (heaviest first), explicit grid order and explicit heaviest first,
    # each repeated past the ring's 16 slots, against the committed oracle digest
    cfg = vr.CONFIGS["C2"]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store)
    W, H = cfg.width, cfg.height
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    out = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
    for sched in (vr.Schedule.AUTO, vr.Schedule.GRID, vr.Schedule.HEAVIEST_FIRST):
        for i in range(20):
            out.fill_(-1)
            vr.render_ex(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out, schedule=sched)
            torch.cuda.synchronize()
            img = out.cpu().numpy().view(np.uint32)
            assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == FRAMES["C2"]["sha256"], \
                (sched.name, i)
    with pytest.raises(vr.VrError):
        vr.render_ex(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out, schedule=7)
    scene.close()


@pytest.mark.parametrize("store", ["vcs", "hashtable"])
def test_lane_order_ragged_frames(store):
    # the lane order (vr_march.hip lane_pixel) deals each 16x16 block's pixels to its four
    # waves heaviest first once a slot has recorded the grid's per-pixel walk lengths: ragged
    # frames (partial blocks at the right edge, an odd number of tile-group rows whose last
    # block row keeps the identity order) must render the same pixels with it as without
    cfg = vr.CONFIGS["C1"]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, vr.parse_storage(store))
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    for W, H in [(200, 37), (17, 250), (333, 41)]:
        cam = vr.Camera.reference(W, H)
        for algo in (vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS):
            ref = None
            for i in range(40):       # past two uses of each of the ring's 16 slots
                out = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
                vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, out)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                assert torch.equal(out, ref), (store, W, H, algo.name, i)
    scene.close()


def test_forget_orders_first_render_and_view_keys():
    # vr_forget_orders drops what the device learned: the next launch is a first render; the
    # orders come back after repeated launches of the view and are never used for another view
    # of the same grid size -- every frame stays the oracle's
    cfg = vr.CONFIGS["C2"]
    xyz, rgb = cfg.voxels()
    scene = vr.create_scene(xyz, rgb, cfg.store)
    W, H = cfg.width, cfg.height
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    cams = [vr.Camera.reference(W, H),
            vr.Camera((-3.0, 5.0, 8.0), (1.0, -1.0, -2.0), (0.0, 1.0, 0.0), 50.0, W / H)]
    out = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
    refs = []
    for cam in cams:
        vr.forget_orders(0)
        out.fill_(-1)
        vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out)
        torch.cuda.synchronize()
        refs.append(out.clone())
    img = refs[0].cpu().numpy().view(np.uint32)
    assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == FRAMES["C2"]["sha256"]
    seq = [0] * 40 + [1] * 3 + [0] * 20 + ["forget", 0, 0] + [1, 0] * 10
    for i, k in enumerate(seq):
        if k == "forget":
            vr.forget_orders(0)
            continue
        out.fill_(-1)
        vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, cams[k], lit, info, W, H, out)
        torch.cuda.synchronize()
        assert torch.equal(out, refs[k]), (i, k)
    scene.close()
