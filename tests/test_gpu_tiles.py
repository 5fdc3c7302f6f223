"""GPU test of BandGather's rank-0 stream logic (bench.py's N > 1 step): the
gather is emulated by an asynchronous copy on its own stream (one GPU cannot
host two RCCL ranks), delayed with a spin so that any missing stream wait --
band buffer re-rendered before its gather finished, receive buffer gathered
into before its un-interleaving copy finished, frame read before the side
stream finished -- shows up as a wrong or out-of-order frame."""
from __future__ import annotations

import pytest
import torch

import voxelraymarcher_amd as vr
from voxelraymarcher_amd import tiles
from voxelraymarcher_amd.tiles import BandGather, owned_rows

pytestmark = pytest.mark.gpu


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


@pytest.mark.parametrize("rgb8", [False, True], ids=["words", "rgb8"])
def test_band_gather_rank0_side_stream(monkeypatch, rgb8):
    W, H, B, R, frames = 64, 77, 8, 3, 9
    dev = torch.device("cuda", 0)

    def expected(k):
        return ((torch.arange(W * H, dtype=torch.int64, device=dev) * 2654435761 + 977 * k) % (1 << 24)) \
            .to(torch.int32).reshape(H, W)

    def rank_buffer(k, r, n):
        words = n // 3 if rgb8 else n
        buf = torch.zeros(words, dtype=torch.int32, device=dev)
        rows = owned_rows(H, B, r, R)
        buf.view(-1, W)[:len(rows)] = expected(k)[torch.tensor(rows, device=dev)]
        return vr.pack_rgb8(buf) if rgb8 else buf

    gstream = torch.cuda.Stream(dev)
    kbox = [0]
    sent, keep = [], []

    def fake_gather(tensor, gather_list, dst=0, async_op=True):
        k = kbox[0]
        others = [rank_buffer(k, r, tensor.numel()) for r in range(1, R)]
        gstream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(gstream):
            torch.cuda._sleep(2_000_000)          # a slow link
            gather_list[0].copy_(tensor)
            for r in range(1, R):
                gather_list[r].copy_(others[r - 1])
            ev = torch.cuda.Event()
            ev.record(gstream)
        sent.append(k)
        keep.append(others)                      # used on gstream: keep them out of the allocator
        return _Work(ev)

    import torch.distributed as dist
    monkeypatch.setattr(dist, "gather", fake_gather)
    got = []
    pipe = BandGather(W, H, B, 0, R, dev, depth=2, on_frame=lambda f: got.append(f.clone()), rgb8=rgb8)
    assert pipe.side is not None

    def render(buf):
        torch.cuda._sleep(200_000)
        view = buf.view(-1, W)
        rows = owned_rows(H, B, 0, R)
        view[:len(rows)] = expected(kbox[0])[torch.tensor(rows, device=dev)]

    for k in range(frames):
        kbox[0] = k
        pipe.step(render)
    pipe.drain()
    torch.cuda.synchronize()
    assert sent == list(range(frames))
    assert len(got) == frames
    for k, g in enumerate(got):
        want = vr.pack_rgb8(expected(k).reshape(-1)).view(H, W, 3) if rgb8 else expected(k)
        assert torch.equal(g, want), f"frame {k} differs"
    assert tiles is not None
