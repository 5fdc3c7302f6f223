"""GPU test of the per-launch scratch slots (vr_host.cpp SlotRing): each slot's
crawl-pass deferral list and its work-order buffers, fenced by per-slot events;
both passes of a launch run on the launch's own stream (with launches in flight
the crawl pass takes 8 records per wave).  Many launches in flight on several
streams at once, far more of them than the ring has slots, must each render
exactly the frame one serial launch renders: a slot shared by two launches in
flight would mix their deferred records (wrong or zero pixels), and a missing
fence would let a frame be read before its crawl pass wrote it."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")


@pytest.fixture(scope="module")
def c5_scene():
    cfg = vr.CONFIGS["C5"]
    xyz, rgb = cfg.voxels()
    return cfg, vr.create_scene(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE)


@pytest.mark.parametrize("kernel", [vr.Kernel.TILE, vr.Kernel.TILE_REWALK], ids=lambda k: k.name)
@pytest.mark.parametrize("algo", [vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS],
                         ids=lambda a: a.name)
def test_launches_in_flight_on_three_streams(c5_scene, kernel, algo):
    # C5 rows 696-712 defer thousands of crawling rays per launch (test_gpu_parity.test_c5_crawl_rows)
    cfg, scene = c5_scene
    W, H, r0, r1 = cfg.width, cfg.height, 696, 712
    cam = vr.Camera.reference(W, H)
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    words = (r1 - r0) * W
    ref = torch.full((words,), -1, dtype=torch.int32, device="cuda")
    vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, ref, r0, r1, kernel=kernel)
    torch.cuda.synchronize()
    ref_np = ref.cpu().numpy()
    assert np.count_nonzero(ref_np) > 0
    depth, frames = 3, 70                       # 70 launches > the ring's 16 slots; 16 % 3 != 0
    streams = [torch.cuda.Stream() for _ in range(depth)]
    outs = [torch.full((words,), -1, dtype=torch.int32, device="cuda") for _ in range(frames)]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    for i in range(frames):
        vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, outs[i], r0, r1, stream=streams[i % depth],
                                  kernel=kernel)
    torch.cuda.synchronize()
    bad = [i for i in range(frames) if not torch.equal(outs[i], ref)]
    assert not bad, f"{len(bad)} of {frames} launches differ from the serial render (first: {bad[:5]})"
    # the slots are clean afterwards: one more serial launch still matches
    last = torch.full((words,), -1, dtype=torch.int32, device="cuda")
    vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, last, r0, r1, kernel=kernel)
    torch.cuda.synchronize()
    assert torch.equal(last, ref)


def test_crawl_skip_safety_net(c5_scene):
    """The crawl-pass skip's safety net (vr_host.cpp launch, vr_march.hip deferral_report).
    Every slot first learns a view that defers nothing (C5's top rows: each slot's last crawl
    pass reports 0).  Then the next launch is forced to skip its crawl pass on C5's crawl rows,
    as a wrong skip would: its deferred pixels stay 0 (the frame differs).  Its tile pass
    reports the deferral, so that slot stops skipping: every later launch of the view -- 40,
    so each of the 16 slots comes round at least twice -- equals the serial frame, and the
    records the skipped launch left never reach a frame (they carry its launch id).  Without
    the report the forced slot would skip the crawl pass of this view every 16th launch."""
    cfg, scene = c5_scene
    W, H = cfg.width, cfg.height
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    algo = vr.RayMarchAlgorithm.ORIGINAL
    dev = torch.cuda.current_device()

    def frame(r0, r1):
        out = torch.full(((r1 - r0) * W,), -1, dtype=torch.int32, device="cuda")
        vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, out, r0, r1)
        torch.cuda.synchronize()
        return out

    vr.forget_orders(dev)
    quiet = frame(0, 16)
    for _ in range(40):                          # every slot's crawl pass reports 0 deferrals
        assert torch.equal(frame(0, 16), quiet)
    ref = frame(696, 712)
    assert int((ref == 0).sum()) < ref.numel()
    vr.debug_skip_next_crawl(dev)
    skipped = frame(696, 712)
    assert not torch.equal(skipped, ref), "the forced skip left every deferred pixel shaded"
    bad = [i for i in range(40) if not torch.equal(frame(696, 712), ref)]
    assert not bad, f"launches after the forced skip differ from the serial frame: {bad}"
    assert torch.equal(frame(0, 16), quiet)


def test_crawl_skip_key_inputs(c5_scene):
    """The crawl-pass skip is keyed by everything that decides deferral (vr_host.cpp view_key,
    crawl_key): one camera and row range, rendered 40 times with TILE and TILE_REWALK
    alternating on a scene where it defers nothing (the C2 grid: every slot learns to skip),
    then 40 times on C5's scene, where the same view defers thousands of crawling rays, then
    on the first scene again.  Every frame equals that scene's serial first render (which
    test_gpu_parity pins to the oracle): a key without the scene would skip C5's crawl pass."""
    cfg, c5 = c5_scene
    c2 = vr.create_scene(*vr.CONFIGS["C2"].voxels(), vr.StorageType.VOXEL_CLUSTER_STORE)
    W, H, r0, r1 = cfg.width, cfg.height, 696, 712
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    algo = vr.RayMarchAlgorithm.ORIGINAL
    kernels = [vr.Kernel.TILE, vr.Kernel.TILE_REWALK]

    def frame(scene, kernel):
        out = torch.full(((r1 - r0) * W,), -1, dtype=torch.int32, device="cuda")
        vr.run_raymarching_kernel(scene, algo, cam, lit, info, W, H, out, r0, r1, kernel=kernel)
        torch.cuda.synchronize()
        return out

    vr.forget_orders(torch.cuda.current_device())
    refs = {id(s): frame(s, vr.Kernel.TILE) for s in (c2, c5)}
    assert not torch.equal(refs[id(c2)], refs[id(c5)])
    for scene in (c2, c5, c2):
        bad = [i for i in range(40) if not torch.equal(frame(scene, kernels[i % 2]), refs[id(scene)])]
        assert not bad, f"scene {'C5' if scene is c5 else 'C2'}: launches {bad} differ"


def test_render_refuses_graph_capture(c5_scene):
    """vr_render* on a stream that is capturing a graph returns VR_E_INVALID before enqueuing
    anything (include/vr.h): the slot ring's event wait/record and the work order's host-side
    bookkeeping would be baked into the graph and not replay.  The capture itself stays
    usable: it ends cleanly, and a render after it is exact."""
    cfg, scene = c5_scene
    W, H = 64, 48
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    ref = vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H).clone()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    err = None
    with torch.cuda.graph(g, stream=s):
        try:
            vr.render_ex(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out, stream=s)
        except vr.VrError as e:
            err = e
    assert err is not None and err.code == -1 and "captur" in str(err)
    torch.cuda.synchronize()
    vr.render_ex(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_crawl_stats_credit_unloaded_reads(c5_scene):
    """vr_render_opts.stats_dev: [0] crawl iterations fast-forwarded in closed form, [1] the
    existence-read bytes credited without a load -- 4 per fast-forwarded iteration plus 4 per
    crawl-pass skip step answered from the LDS cluster bits (round 5) -- a part of the
    counted bytes.  C5's crawl rows have both; a frame that defers nothing has neither."""
    cfg, scene = c5_scene
    W, H = cfg.width, cfg.height
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    out = torch.empty(16 * W, dtype=torch.int32, device="cuda")
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.zeros(2, dtype=torch.int64, device="cuda")
    vr.render_ex(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out, 696, 712, counter=ctr, stats=st)
    torch.cuda.synchronize()
    n, b, total = int(st[0]), int(st[1]), int(ctr.item())
    assert n > 1_000_000 and b > 4 * n and b < total, (n, b, total)
    ctr.zero_()
    st.zero_()
    vr.render_ex(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out, 0, 16, counter=ctr, stats=st)
    torch.cuda.synchronize()
    assert int(st[0]) == 0 and int(st[1]) == 0 and int(ctr.item()) > 0


@pytest.mark.parametrize("algo", [vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS],
                         ids=lambda a: a.name)
def test_prepared_render_in_the_frame_pipeline(c5_scene, algo):
    """renderer.PreparedRender (the bench's per-frame host path): arguments made once, the
    launch enqueued on the BandGather slot stream it is handed (no torch stream context).
    Every frame of a pipelined run -- the crawl rows, with the moving-view rotation of three
    prepared views -- equals render_ex's frame of the same view, and a camera changed in place
    re-aims the next call."""
    from voxelraymarcher_amd.tiles import BandGather
    cfg, scene = c5_scene
    W, H, r0, r1 = cfg.width, cfg.height, 688, 720
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    cams = []
    for k in (0, 1, 2):
        c = vr.Camera.reference(W, H)
        bits = np.array([c.raw.origin[0]], dtype=np.float32).view(np.uint32) + np.uint32(k)
        c.raw.origin[0] = float(bits.view(np.float32)[0])
        cams.append(c)
    words = (r1 - r0) * W
    refs = []
    for c in cams:
        ref = torch.full((words,), -1, dtype=torch.int32, device="cuda")
        vr.render_ex(scene, algo, c, lit, info, W, H, ref, r0, r1)
        refs.append(ref)
    torch.cuda.synchronize()
    preps = [vr.PreparedRender(scene, algo, c, lit, info, W, H, row_begin=r0, row_end=r1) for c in cams]
    assert preps[0].vr_stream_arg
    pipe = BandGather(W, r1 - r0, 16, 0, 1, torch.device("cuda", 0), depth=3)
    pipe.bufs = [torch.full((words,), -1, dtype=torch.int32, device="cuda") for _ in range(3)]
    got, k_box = [], [0]

    def render(buf, stream=None):
        preps[k_box[0] % 3](buf, stream)
    render.vr_stream_arg = True
    for k in range(24):
        k_box[0] = k
        pipe.step(render)
        if len(pipe.pending) == pipe.depth:    # the oldest frame in flight: step k - 2's
            slot = pipe.pending[0]
            pipe.streams[slot].synchronize()
            got.append((k - pipe.depth + 1, pipe.bufs[slot].clone()))
            torch.cuda.current_stream().synchronize()   # (the copy is done before the slot renders again)
    pipe.drain()
    torch.cuda.synchronize()
    bad = [k for k, f in got if not torch.equal(f, refs[k % 3])]
    assert len(got) >= 20 and not bad, f"frames {bad[:5]} differ from render_ex's"
    # the struct is passed by reference: moving camera 0 onto camera 1's eye gives camera 1's frame
    cams[0].raw.origin[0] = cams[1].raw.origin[0]
    out = torch.full((words,), -1, dtype=torch.int32, device="cuda")
    preps[0](out)
    torch.cuda.synchronize()
    assert torch.equal(out, refs[1])
    with pytest.raises(ValueError):
        preps[0](torch.empty(words - 1, dtype=torch.int32, device="cuda"))
