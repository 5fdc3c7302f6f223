"""Multi-GPU image tiling: interleaved row bands (band b -> rank b % R) and
their reassembly after the gather.  SURVEY.md 8(e): pixels are independent,
the voxel store is replicated per GPU, and the only exchange is the final
gather of the framebuffer to rank 0.
"""
from __future__ import annotations

import torch

from .renderer import band_buffer_words


def bands_per_rank(height: int, band_rows: int, nranks: int) -> int:
    nb = -(-height // band_rows)
    return -(-nb // nranks)


def assemble_bands(parts: torch.Tensor, width: int, height: int, band_rows: int) -> torch.Tensor:
    """parts: [R, words] per-rank band buffers (vr_render_bands layout) -> [height, width] frame."""
    R = parts.shape[0]
    per = bands_per_rank(height, band_rows, R)
    expect = band_buffer_words(width, height, band_rows, R)
    if parts.shape[1] != expect or per * band_rows * width != expect:
        raise ValueError(f"band buffers have {parts.shape[1]} words, expected {expect}")
    img = parts.reshape(R, per, band_rows, width).permute(1, 0, 2, 3).reshape(per * R * band_rows, width)
    return img[:height]


def owned_rows(height: int, band_rows: int, rank: int, nranks: int) -> list[int]:
    """Frame rows rendered by `rank` (for tests and accounting)."""
    rows = []
    nb = -(-height // band_rows)
    for b in range(rank, nb, nranks):
        rows.extend(range(b * band_rows, min(height, (b + 1) * band_rows)))
    return rows
