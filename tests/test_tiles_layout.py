"""CPU tests of the 2-D tile deal (include/vr.h vr_render_tiles / vr_assemble_tiles,
voxelraymarcher_amd/tiles.py): the library's buffer sizes and default stride equal the
Python mirror's, the deal is a bijection between frame pixels and the ranks' buffer slots,
every rank gets a share of every band, and a frame dealt out and assembled comes back
whole.  No GPU: the device assembly kernel is compared with this in tests/test_gpu_tiles_deal.py."""
from __future__ import annotations

import ctypes

import pytest
import torch

import voxelraymarcher_amd as vr
from voxelraymarcher_amd.tiles import (assemble_tiles, deal_stride, tile_local_width, tile_rank_buffer,
                                       tile_source_index, tile_words)

CASES = [(64, 45, 8, 16, 2), (64, 45, 8, 16, 3), (200, 150, 8, 8, 5), (97, 41, 4, 24, 8), (3840, 2160, 8, 16, 8),
         (1920, 1080, 8, 16, 4), (33, 7, 3, 5, 6), (16, 8, 8, 16, 1), (3840, 2160, 16, 16, 8)]


@pytest.mark.parametrize("W,H,B,T,R", CASES)
def test_library_sizes_match_python(W, H, B, T, R):
    assert vr.tile_buffer_words(W, H, B, T, R) == tile_words(W, H, B, T, R)
    assert vr.deal_stride_default(R) % R == deal_stride(R)
    assert tile_words(W, H, B, T, R) == -(-H // B) * B * tile_local_width(W, T, R)


@pytest.mark.parametrize("W,H,B,T,R", CASES[:7])
def test_deal_is_a_bijection_and_spreads_every_band(W, H, B, T, R):
    words = tile_words(W, H, B, T, R)
    idx = tile_source_index(W, H, B, T, R)
    assert idx.numel() == W * H and idx.unique().numel() == W * H
    assert int(idx.min()) >= 0 and int(idx.max()) < R * words
    ranks = (idx // words).reshape(H, W)
    nblk = -(-W // T)
    for b in range(-(-H // B)):
        owners = set(ranks[b * B].tolist())
        assert len(owners) == min(R, nblk)            # every band is spread over the ranks
    # balance: per rank, pixels within one column block per band of the mean
    counts = torch.bincount(ranks.reshape(-1), minlength=R)
    assert int(counts.max() - counts.min()) <= T * B * -(-H // B)


@pytest.mark.parametrize("W,H,B,T,R", CASES[:7])
def test_dealt_frame_reassembles(W, H, B, T, R):
    frame = (torch.arange(W * H, dtype=torch.int64) * 2654435761 % (1 << 24)).to(torch.int32).reshape(H, W)
    parts = torch.stack([tile_rank_buffer(frame, r, R, B, T) for r in range(R)])
    assert torch.equal(assemble_tiles(parts, W, H, B, T), frame)
    # as RGB8 (3 elements per pixel), the exchanged form
    rgb = torch.stack([(frame >> 16) & 255, (frame >> 8) & 255, frame & 255], -1).to(torch.uint8)
    prgb = torch.stack([torch.stack([(p >> 16) & 255, (p >> 8) & 255, p & 255], -1).to(torch.uint8).reshape(-1)
                        for p in parts])
    assert torch.equal(assemble_tiles(prgb, W, H, B, T).reshape(H, W, 3), rgb)


def test_explicit_stride():
    W, H, B, T, R = 96, 40, 8, 8, 4
    frame = torch.arange(W * H, dtype=torch.int32).reshape(H, W)
    for s in (1, 2, 3, 5):
        parts = torch.stack([tile_rank_buffer(frame, r, R, B, T, stride=s) for r in range(R)])
        assert torch.equal(assemble_tiles(parts, W, H, B, T, stride=s), frame)


def test_tile_entry_points_validate_arguments():
    """No GPU needed: argument errors are reported before any device work."""
    lib = vr.lib()
    cam = vr.Camera.reference(64, 64)
    lit = vr.setup_constant_values()
    tr = (ctypes.c_float * 3)(0, 0, 0)
    assert lib.vr_render_tiles(None, 1, ctypes.byref(cam.raw), ctypes.byref(lit), tr, 1, 64, 64, 8, 0, 0, 2,
                               None, None) == -1
    assert lib.vr_assemble_tiles(None, None, 4, 64, 64, 8, 16, 2, 0, None) == -1
    buf = ctypes.create_string_buffer(16)
    assert lib.vr_assemble_tiles(buf, buf, 5, 64, 64, 8, 16, 2, 0, None) == -1
    assert b"elem_bytes" in lib.vr_last_error()
    assert lib.vr_assemble_tiles(buf, buf, 4, 64, 64, 8, 128, 2, 0, None) == -1
    assert lib.vr_tile_buffer_words(64, 64, 8, 0, 2) == 0


def test_strip_bounds_balance_and_alignment():
    """The cost-balanced contiguous deal (tiles.strip_bounds): strips are contiguous, cover
    every row once, start on aligned rows, and their costs are as equal as the alignment
    allows -- an expensive band of rows (C5's crawl rows) gets a short strip."""
    from voxelraymarcher_amd.tiles import strip_bounds
    H = 2160
    cost = [1.0] * H
    for y in range(680, 720):
        cost[y] = 10.0
    b = strip_bounds(cost, 8, 8)
    assert b[0] == 0 and b[-1] == H and all(b[i] < b[i + 1] for i in range(8))
    assert all(x % 8 == 0 for x in b[:-1])
    per = [sum(cost[b[r]:b[r + 1]]) for r in range(8)]
    assert max(per) / (sum(per) / 8) < 1.05, per
    assert min(b[r + 1] - b[r] for r in range(8)) < 200 < max(b[r + 1] - b[r] for r in range(8))
    # uniform costs: equal heights (to the alignment)
    u = strip_bounds([1.0] * 1080, 4, 8)
    assert [u[r + 1] - u[r] for r in range(4)] == [272, 264, 272, 272] or max(
        u[r + 1] - u[r] for r in range(4)) - min(u[r + 1] - u[r] for r in range(4)) <= 8


def test_rebalance_strips_converges():
    """tiles.rebalance_strips: timing each strip and re-cutting moves rows from the slow ranks to
    the fast ones; on a fixed hidden cost it reaches max/mean < 1.05 in a few rounds."""
    from voxelraymarcher_amd.tiles import rebalance_strips, strip_bounds
    H, N = 2160, 8
    true = [0.2 + (3.0 if 600 <= y < 760 else 0.0) + (0.0 if y > 1700 else 1.0) for y in range(H)]
    b = strip_bounds([1.0] * H, N, 8)
    est = None
    for _ in range(6):
        t = [sum(true[b[r]:b[r + 1]]) for r in range(N)]
        b, est = rebalance_strips(b, t, 8, prior=est)
    t = [sum(true[b[r]:b[r + 1]]) for r in range(N)]
    assert max(t) / (sum(t) / N) < 1.05, t


def test_assemble_strips_roundtrip():
    import torch

    from voxelraymarcher_amd.tiles import assemble_strips
    W, H = 37, 53
    frame = torch.arange(W * H * 3, dtype=torch.int64).reshape(H, W * 3)
    b = [0, 8, 24, 53]
    mh = max(b[i + 1] - b[i] for i in range(3))
    parts = torch.full((3, mh * W * 3), -1, dtype=torch.int64)
    for r in range(3):
        h = b[r + 1] - b[r]
        parts[r, :h * W * 3] = frame[b[r]:b[r + 1]].reshape(-1)
    assert torch.equal(assemble_strips(parts, b, W, 3), frame)
