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
from voxelraymarcher_amd.tiles import assemble_bands, owned_rows


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
