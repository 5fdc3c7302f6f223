"""The 2-D tile deal on the GPU (include/vr.h vr_render_tiles, vr_assemble_tiles): every
rank's tile buffer rendered through the C ABI, assembled by the device kernel (packed words
and RGB8) and by the host-side mirror (tiles.assemble_tiles), equals the single full
render -- odd frame sizes, several rank counts, block widths and strides, both stores and
algorithms.  (C5's 4K frame over 8 ranks: tests/test_gpu_parity.py.)"""
from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import diff_report, gpu_render

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def c1():
    return vr.CONFIGS["C1"].voxels()


@pytest.mark.parametrize("R,B,T,stride", [(1, 8, 16, 0), (2, 8, 16, 0), (3, 8, 8, 0), (5, 8, 24, 0), (8, 8, 16, 0),
                                          (4, 4, 8, 3), (8, 8, 8, 5), (6, 16, 16, 0), (8, 16, 16, 0)])
@pytest.mark.parametrize("store", [vr.StorageType.VOXEL_CLUSTER_STORE, vr.StorageType.HASH_TABLE],
                         ids=lambda s: s.name)
def test_tiles_reassemble(c1, R, B, T, stride, store):
    from voxelraymarcher_amd.tiles import assemble_tiles
    cfg = vr.CONFIGS["C1"]
    W, H = 203, 150       # neither a multiple of the block nor of the band
    scene = vr.create_scene(*c1, store)
    cam, lit, info = vr.Camera.reference(W, H), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
    for algo in (vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS):
        full, _ = gpu_render(scene, algo, cam, lit, info, W, H)
        words = vr.tile_buffer_words(W, H, B, T, R)
        parts = torch.full((R, words), -7, dtype=torch.int32, device="cuda")
        for r in range(R):
            if stride == 0 and B == 8:
                vr.render_tiles(scene, algo, cam, lit, info, W, H, B, T, r, R, parts[r])
            else:
                vr.render_ex(scene, algo, cam, lit, info, W, H, parts[r], band_rows=B, rank=r, nranks=R,
                             tile_cols=T, deal_stride=stride)
        frame = torch.full((H, W), -9, dtype=torch.int32, device="cuda")
        vr.assemble_tiles_device(parts, frame, 4, W, H, B, T, R, stride)
        torch.cuda.synchronize()
        img = frame.cpu().numpy().view(np.uint32).reshape(-1)
        assert np.array_equal(img, full), f"{algo.name} R={R}: " + diff_report(img, full, W)
        host = assemble_tiles(parts.cpu(), W, H, B, T, stride).numpy().view(np.uint32).reshape(-1)
        assert np.array_equal(host, full)
        # slots past the frame are written as 0 (no -7 left anywhere)
        assert int((parts == -7).sum()) == 0
        # RGB8: the form the ranks exchange
        rgb_parts = torch.stack([vr.pack_rgb8(parts[r]) for r in range(R)])
        rgb = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
        vr.assemble_tiles_device(rgb_parts, rgb, 3, W, H, B, T, R, stride)
        torch.cuda.synchronize()
        f = full.reshape(H, W)
        want = np.stack([(f >> 16) & 0xFF, (f >> 8) & 0xFF, f & 0xFF], -1).astype(np.uint8)
        assert np.array_equal(rgb.cpu().numpy(), want)
    scene.close()


def test_tiles_counted_bytes_sum_to_the_frame(c1):
    """The algorithmic bytes of the ranks' tile launches add up to the full frame's."""
    cfg = vr.CONFIGS["C1"]
    W, H, B, T, R = 160, 120, 8, 16, 3
    scene = vr.create_scene(*c1, vr.StorageType.VOXEL_CLUSTER_STORE)
    cam, lit, info = vr.Camera.reference(W, H), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
    _, full = gpu_render(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, count=True)
    total = 0
    for r in range(R):
        buf = torch.empty(vr.tile_buffer_words(W, H, B, T, R), dtype=torch.int32, device="cuda")
        ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
        vr.render_ex(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, buf, band_rows=B, rank=r,
                     nranks=R, tile_cols=T, counter=ctr)
        torch.cuda.synchronize()
        total += int(ctr.item())
    # every pixel of the buffers past the frame counts nothing; every frame pixel once
    assert total == full
    scene.close()


@pytest.mark.parametrize("R", [3, 8])
def test_tiles_with_learned_orders(c1, R):
    """Each rank's tile buffer rendered 40 times in a row (so the slots learn its work and lane
    orders, include/vr.h vr_forget_orders) equals its first render, for the 16x16 deal bench.py
    uses and both algorithms; the assembled frame of the last renders equals the full render."""
    cfg = vr.CONFIGS["C1"]
    W, H, B, T = 203, 150, 16, 16
    scene = vr.create_scene(*c1, vr.StorageType.VOXEL_CLUSTER_STORE)
    cam, lit, info = vr.Camera.reference(W, H), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
    for algo in (vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS):
        full, _ = gpu_render(scene, algo, cam, lit, info, W, H)
        words = vr.tile_buffer_words(W, H, B, T, R)
        parts = torch.full((R, words), -7, dtype=torch.int32, device="cuda")
        for r in range(R):
            first = None
            for i in range(40):
                buf = torch.full((words,), -7, dtype=torch.int32, device="cuda")
                vr.render_tiles(scene, algo, cam, lit, info, W, H, B, T, r, R, buf)
                torch.cuda.synchronize()
                if first is None:
                    first = buf.clone()
                assert torch.equal(buf, first), (algo.name, R, r, i)
            parts[r] = first
        frame = torch.full((H, W), -9, dtype=torch.int32, device="cuda")
        vr.assemble_tiles_device(parts, frame, 4, W, H, B, T, R)
        torch.cuda.synchronize()
        img = frame.cpu().numpy().view(np.uint32).reshape(-1)
        assert np.array_equal(img, full), f"{algo.name} R={R}: " + diff_report(img, full, W)
    scene.close()
