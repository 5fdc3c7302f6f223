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
