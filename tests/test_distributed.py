"""Multi-rank path on CPU (gloo, world_size 2 and 3): every rank produces its
interleaved row bands of a known frame, rank 0 gathers and reassembles, and
the result equals the frame.  Mirrors bench.py's N > 1 step (render_bands ->
gather -> assemble_bands) without a GPU."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import voxelraymarcher_amd as vr
from voxelraymarcher_amd.tiles import assemble_bands, assemble_tiles, owned_rows, tile_rank_buffer


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frame = (torch.arange(W * H, dtype=torch.int64) * 2654435761 % (1 << 24)).to(torch.int32).reshape(H, W)
    words = vr.band_buffer_words(W, H, B, world)
    buf = torch.zeros(words, dtype=torch.int32)
    view = buf.view(-1, W)
    for i, y in enumerate(owned_rows(H, B, rank, world)):
        view[i] = frame[y]
    gathered = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        img = assemble_bands(torch.stack(gathered), W, H, B)
        q.put((bool(torch.equal(img, frame)), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_band_gather_reassembles(world):
    W, H, B = 64, 45, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok
    assert tmax == world - 1


def _pipeline_worker(rank, world, port, W, H, B, frames, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from voxelraymarcher_amd.tiles import BandGather

    def expected(k):
        return ((torch.arange(W * H, dtype=torch.int64) * 2654435761 + 977 * k) % (1 << 24)).to(torch.int32).reshape(H, W)

    got = []
    pipe = BandGather(W, H, B, rank, world, "cpu", depth=2, on_frame=lambda f: got.append(f.clone()))
    k_box = [0]

    def render(buf):
        view = buf.view(-1, W)
        img = expected(k_box[0])
        for i, y in enumerate(owned_rows(H, B, rank, world)):
            view[i] = img[y]

    for k in range(frames):
        k_box[0] = k
        pipe.step(render)
    pipe.drain()
    if rank == 0:
        q.put([bool(torch.equal(g, expected(k))) for k, g in enumerate(got)])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_band_gather_pipeline_overlapped(world):
    """BandGather (bench.py's N > 1 step): frames stay intact and in order with
    two band buffers in flight."""
    W, H, B, frames = 48, 61, 8, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, W, H, B, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [True] * frames


def test_weak_scaled_resolution():
    from voxelraymarcher_amd.tiles import weak_scaled_resolution
    assert weak_scaled_resolution(1920, 1080, 1) == (1920, 1080)
    assert weak_scaled_resolution(1920, 1080, 4) == (3840, 2160)
    for n in (2, 8):
        w, h = weak_scaled_resolution(1920, 1080, n)
        assert abs(w * h / (1920 * 1080) - n) < 0.01 * n
        assert abs(w / h - 16 / 9) < 1e-3


def test_band_gather_single_rank_is_the_frame():
    from voxelraymarcher_amd.tiles import BandGather
    W, H, B = 40, 21, 8
    got = []
    pipe = BandGather(W, H, B, 0, 1, "cpu", on_frame=lambda f: got.append(f.clone()))
    ref = torch.arange(W * H, dtype=torch.int32).reshape(H, W)

    def render(buf):
        buf.view(-1, W)[:H] = ref

    pipe.step(render)
    pipe.step(render)
    pipe.drain()
    assert len(got) == 2 and all(torch.equal(g, ref) for g in got)


def test_fixed_tiling_eight_ranks_4k():
    """BASELINE C5 as defined: ONE 3840x2160 frame over 8 ranks (bench.py --tiling fixed,
    the default for C5): 8-row bands dealt round-robin, gathered over gloo to rank 0 and
    assembled -- the frame comes back whole."""
    from voxelraymarcher_amd.tiles import frame_resolution
    world = 8
    W, H = frame_resolution(3840, 2160, world, "fixed")
    assert (W, H) == (3840, 2160)
    assert frame_resolution(3840, 2160, world, "weak") != (3840, 2160)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, 8, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, tmax = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok and tmax == world - 1


def test_pipeline_policy():
    """Frames in flight per config and the hardware queues they need (bench.py sets
    GPU_MAX_HW_QUEUES from these before the HIP runtime starts)."""
    from voxelraymarcher_amd.tiles import pipeline_depth, pipeline_hw_queues
    assert pipeline_depth("C2") == 2 and pipeline_depth("C5") == 8
    assert pipeline_hw_queues(2) == 0 and pipeline_hw_queues(3) == 0
    assert pipeline_hw_queues(pipeline_depth("C5")) >= pipeline_depth("C5") + 2
    # N > 1: rank 0's assembly stream and the RCCL stream join the two frame streams
    assert pipeline_hw_queues(2, 8) >= 2 + 3


def _tile_worker(rank, world, port, W, H, B, T, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frame = (torch.arange(W * H, dtype=torch.int64) * 2654435761 % (1 << 24)).to(torch.int32).reshape(H, W)
    buf = tile_rank_buffer(frame, rank, world, B, T)
    assert buf.numel() == vr.tile_buffer_words(W, H, B, T, world)
    gathered = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    if rank == 0:
        img = assemble_tiles(torch.stack(gathered), W, H, B, T)
        q.put(bool(torch.equal(img, frame)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,T", [(2, 64, 45, 16), (3, 100, 37, 8), (8, 3840, 2160, 16)])
def test_tile_gather_reassembles(world, W, H, T):
    """The 2-D tile deal (bench.py's N > 1 layout for fixed tiling; the 8-rank case is C5's
    3840x2160 frame): each rank's tile buffer, gathered over gloo and assembled on rank 0,
    gives the frame back."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tile_worker, args=(r, world, port, W, H, 8, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok


def _tile_pipeline_worker(rank, world, port, W, H, B, T, frames, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from voxelraymarcher_amd.tiles import BandGather

    def expected(k):
        return ((torch.arange(W * H, dtype=torch.int64) * 2654435761 + 977 * k) % (1 << 24)).to(torch.int32).reshape(H, W)

    got = []
    pipe = BandGather(W, H, B, rank, world, "cpu", depth=2, on_frame=lambda f: got.append(f.clone()), tile_cols=T)
    assert pipe.T == T
    k_box = [0]

    def render(buf):
        buf.copy_(tile_rank_buffer(expected(k_box[0]), rank, world, B, T))

    for k in range(frames):
        k_box[0] = k
        pipe.step(render)
    pipe.drain()
    if rank == 0:
        q.put([bool(torch.equal(g, expected(k))) for k, g in enumerate(got)])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_gather_pipeline_overlapped(world):
    """BandGather with the 2-D tile deal: frames intact and in order, two in flight."""
    W, H, B, T, frames = 72, 61, 8, 16, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tile_pipeline_worker, args=(r, world, port, W, H, B, T, frames, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [True] * frames


def _exchange_worker(rank, world, port, q):
    """One rank with the exchange forced (bench.py --exchange): the gather/assembly path runs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from voxelraymarcher_amd.tiles import BandGather
    W, H, B = 40, 21, 8
    ref = torch.arange(W * H, dtype=torch.int32).reshape(H, W)
    got = []
    for T in (0, 16):
        pipe = BandGather(W, H, B, 0, 1, "cpu", on_frame=lambda f: got.append(f.clone()), tile_cols=T,
                          exchange=True)
        assert pipe.x and pipe.T == T

        def render(buf, T=T):
            if T:
                buf.copy_(tile_rank_buffer(ref, 0, 1, B, T))
            else:
                buf.view(-1, W)[:H] = ref
        pipe.step(render)
        pipe.drain()
    q.put(len(got) == 2 and all(torch.equal(g, ref) for g in got))
    dist.destroy_process_group()


def test_forced_exchange_single_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_exchange_worker, args=(0, 1, _free_port(), q))
    p.start()
    ok = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0 and ok


def _strip_pipeline_worker(rank, world, port, W, H, frames, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from voxelraymarcher_amd.tiles import BandGather, rebalance_strips, strip_bounds

    def expected(k):
        return ((torch.arange(W * H, dtype=torch.int64) * 2654435761 + 977 * k) % (1 << 24)).to(torch.int32).reshape(H, W)

    # the learned strip deal as bench.py makes it: equal strips, then re-cut from every rank's
    # (here: made-up, rank-dependent) frame times, the same on every rank (all_reduce of the vector)
    bounds = strip_bounds([1.0] * H, world, 8)
    got = []
    pipe = BandGather(W, H, 8, rank, world, "cpu", depth=2, on_frame=lambda f: got.append(f.clone()), strips=bounds)
    k_box = [0]

    def render(buf):
        y0, y1 = pipe.rows()
        buf[:(y1 - y0) * W].copy_(expected(k_box[0])[y0:y1].reshape(-1))

    for k in range(frames):                      # frames on the equal strips
        k_box[0] = k
        pipe.step(render)
    pipe.drain()
    t = torch.zeros(world, dtype=torch.float64)
    t[rank] = (bounds[rank + 1] - bounds[rank]) * (1.0 + rank)
    dist.all_reduce(t)
    new, _ = rebalance_strips(bounds, t.tolist(), 8)
    pipe.set_strips(new)
    for k in range(frames, 2 * frames):          # frames on the re-cut strips
        k_box[0] = k
        pipe.step(render)
    pipe.drain()
    if rank == 0:
        q.put(([bool(torch.equal(g, expected(k))) for k, g in enumerate(got)], bounds, new))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_strip_gather_pipeline_overlapped(world):
    """BandGather with the learned strip deal (round 6): frames intact and in order, two in
    flight, before and after the strips are re-cut from the ranks' times (set_strips); the
    re-cut gives the slower (higher-rank) strips fewer rows."""
    W, H, frames = 40, 77, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strip_pipeline_worker, args=(r, world, port, W, H, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, b0, b1 = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [True] * (2 * frames)
    assert b1 != b0 and (b1[world] - b1[world - 1]) < (b0[world] - b0[world - 1])
