"""GPU scene build: the device builder (vr_build.hip) must
produce byte-identical scene images to the host builder for both stores --
including the cuckoo placement, which the algorithmic byte count depends on --
and report the same input errors."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")
torch = pytest.importorskip("torch")

STORES = [vr.StorageType.VOXEL_CLUSTER_STORE, vr.StorageType.HASH_TABLE]


def both(xyz, rgb, store):
    d = vr.create_scene(xyz, rgb, store, build=vr.Build.DEVICE)
    h = vr.create_scene(xyz, rgb, store, build=vr.Build.HOST)
    return d, h


@pytest.mark.parametrize("store", STORES, ids=lambda s: s.name)
@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_device_build_matches_host(cfg, store):
    xyz, rgb = vr.CONFIGS[cfg].voxels()
    d, h = both(xyz, rgb, store)
    assert d.info() == h.info()
    assert d.digest() == h.digest()


def test_device_build_matches_host_c4_hashtable():
    xyz, rgb = vr.CONFIGS["C4"].voxels()
    d, h = both(xyz, rgb, vr.StorageType.HASH_TABLE)
    assert d.info() == h.info() and d.digest() == h.digest()


def test_device_build_matches_host_c5_vcs():
    xyz, rgb = vr.CONFIGS["C5"].voxels()
    d, h = both(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE)
    assert d.info() == h.info() and d.digest() == h.digest()


@pytest.mark.parametrize("store", STORES, ids=lambda s: s.name)
def test_device_build_negative_coords_and_duplicates(store):
    rng = np.random.default_rng(5)
    xyz = rng.integers(-700, 300, size=(200_000, 3)).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=200_000).astype(np.uint32)
    xyz[100_000:120_000] = xyz[:20_000]          # later duplicates must win
    d, h = both(xyz, rgb, store)
    assert d.info() == h.info() and d.digest() == h.digest()


@pytest.mark.parametrize("store", STORES, ids=lambda s: s.name)
def test_device_build_empty_and_device_inputs(store):
    e = vr.create_scene(np.zeros((0, 3), np.int32), np.zeros(0, np.uint32), store, build=vr.Build.DEVICE)
    assert e.info()["voxel_count"] == 0 and e.info()["region_count"] == 0
    xyz, rgb = vr.CONFIGS["C1"].voxels()
    g = vr.create_scene(torch.from_numpy(xyz).cuda(), torch.from_numpy(rgb.astype(np.int32)).cuda(), store)
    h = vr.create_scene(xyz, rgb, store, build=vr.Build.HOST)
    assert g.digest() == h.digest()


def test_device_build_errors():
    xyz = np.array([[0, 0, 0], [1, 1, 1]], np.int32)
    with pytest.raises(vr.VrError) as e:
        vr.create_scene(xyz, np.array([5, 1 << 24], np.uint32), vr.StorageType.VOXEL_CLUSTER_STORE, build=vr.Build.DEVICE)
    assert e.value.code == -1 and "index 1" in str(e.value)
    far = np.array([[0, 0, 0], [64 * 1100, 0, 0]], np.int32)
    with pytest.raises(vr.VrError) as e:
        vr.create_scene(far, np.array([1, 2], np.uint32), vr.StorageType.HASH_TABLE, build=vr.Build.DEVICE)
    assert e.value.code == -1


@pytest.mark.parametrize("build", [vr.Build.DEVICE, vr.Build.HOST], ids=["device", "host"])
def test_vcs_region_limit(build):
    """VCS walks address cluster masks by a 32-bit byte offset (64 KB per occupied
    region): a VCS scene may hold at most 65 536 occupied regions; more is an error.
    (The hash store has no bound -- test_hash_scene_past_the_vcs_bound.)"""
    g = np.arange(41, dtype=np.int32) * 64
    xyz = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)   # 68 921 regions
    rgb = np.full(len(xyz), 7, np.uint32)
    with pytest.raises(vr.VrError) as e:
        vr.create_scene(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE, build=build)
    assert e.value.code == -1 and "65536" in str(e.value)
    if build != vr.Build.DEVICE:
        return
    # the largest allowed scene (4 GB of masks) builds -- when the device has room for it
    import torch
    free, _ = torch.cuda.mem_get_info()
    if free < 12 * (1 << 30):
        pytest.skip(f"{free >> 30} GiB free: the 65 536-region scene needs ~5 GiB with its build buffers")
    ok = vr.create_scene(xyz[:65536], rgb[:65536], vr.StorageType.VOXEL_CLUSTER_STORE, build=build)
    assert ok.info()["region_count"] == 65536
    # ... and renders: a camera inside the region of largest id (stored last: region index
    # 65535, whose masks start at byte offset 65535 << 16, the edge of the 32-bit offset)
    # looks at its one voxel, at the region's corner
    import oracle
    from tests.helpers import gpu_render, oracle_camera_from, oracle_lighting_from
    D = 41
    rid = (xyz[:65536, 0] // 64) + (xyz[:65536, 1] // 64) * D + (xyz[:65536, 2] // 64) * D * D
    corner = xyz[:65536][int(np.argmax(rid))].astype(float)
    cam = vr.Camera(tuple(corner + 20.0), tuple(corner), (0.0, 1.0, 0.0), 20.0, 1.0)
    lit = vr.setup_constant_values()
    ref = oracle.Scene(xyz[:65536], rgb[:65536], 0)
    for algo in (vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS):
        want, wb = ref.render(int(algo), oracle_camera_from(cam), oracle_lighting_from(lit), 16, 16, 1)
        got, gb = gpu_render(ok, algo, cam, lit, vr.VoxelSceneInfo((0.0, 0.0, 0.0), 1), 16, 16, count=True)
        assert np.array_equal(got, want) and gb == wb
        assert np.count_nonzero(want) > 0          # the last region's voxel is hit
    ok.close()
    # the hash store at the bound: its last region's filter at byte offset 65535 << 15
    okh = vr.create_scene(xyz[:65536], rgb[:65536], vr.StorageType.HASH_TABLE, build=build)
    assert okh.info()["region_count"] == 65536
    refh = oracle.Scene(xyz[:65536], rgb[:65536], 1)
    for algo in (vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS):
        want, wb = refh.render(int(algo), oracle_camera_from(cam), oracle_lighting_from(lit), 16, 16, 1)
        got, gb = gpu_render(okh, algo, cam, lit, vr.VoxelSceneInfo((0.0, 0.0, 0.0), 1), 16, 16, count=True)
        assert np.array_equal(got, want) and gb == wb
        assert np.count_nonzero(want) > 0
    okh.close()


@pytest.mark.parametrize("build", [vr.Build.DEVICE, vr.Build.HOST], ids=["device", "host"])
def test_hash_scene_past_the_vcs_bound(build):
    """The cuckoo store has no region bound (as the reference's CuckooHashTable per region):
    52^3 = 140 608 occupied regions, one voxel each, so the key-presence filter (32 KB per
    region) runs past 4 GB and the last regions' filter words lie beyond any 32-bit offset.
    A camera in the region of largest id sees its voxel exactly as the oracle does (pixels
    and algorithmic bytes), both algorithms, both builders."""
    import torch

    import oracle
    from tests.helpers import gpu_render, oracle_camera_from, oracle_lighting_from
    free, _ = torch.cuda.mem_get_info()
    if free < 16 * (1 << 30):
        pytest.skip(f"{free >> 30} GiB free: the 140 608-region hash scene needs ~6 GiB")
    D = 52
    g = np.arange(D, dtype=np.int32) * 64
    xyz = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3) + 5
    rgb = (np.arange(len(xyz), dtype=np.uint32) * 2654435761 & 0xFFFFFF).astype(np.uint32)
    scene = vr.create_scene(xyz, rgb, vr.StorageType.HASH_TABLE, build=build)
    assert scene.info()["region_count"] == D ** 3 > 131072
    rid = (xyz[:, 0] // 64) + (xyz[:, 1] // 64) * D + (xyz[:, 2] // 64) * D * D
    corner = xyz[int(np.argmax(rid))].astype(float)
    cam = vr.Camera(tuple(corner + 20.0), tuple(corner), (0.0, 1.0, 0.0), 20.0, 1.0)
    lit = vr.setup_constant_values()
    ref = oracle.Scene(xyz, rgb, 1)
    for algo in (vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS):
        want, wb = ref.render(int(algo), oracle_camera_from(cam), oracle_lighting_from(lit), 16, 16, 1)
        got, gb = gpu_render(scene, algo, cam, lit, vr.VoxelSceneInfo((0.0, 0.0, 0.0), 1), 16, 16, count=True)
        assert np.array_equal(got, want) and gb == wb
        assert np.count_nonzero(want) > 0          # the last region's voxel is hit
        got2, _ = gpu_render(scene, algo, cam, lit, vr.VoxelSceneInfo((0.0, 0.0, 0.0), 1), 16, 16)
        assert np.array_equal(got2, want)
    scene.close()


def test_device_built_scene_renders_like_oracle():
    """End to end: a scene built on the GPU renders bit-exactly (C1 frame, both stores)."""
    import oracle
    from tests.helpers import gpu_render, oracle_camera_from, oracle_lighting_from
    cfg = vr.CONFIGS["C1"]
    xyz, rgb = cfg.voxels()
    cam, lit = vr.Camera.reference(cfg.width, cfg.height), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    for store in STORES:
        g = vr.create_scene(xyz, rgb, store, build=vr.Build.DEVICE)
        want, wb = oracle.Scene(xyz, rgb, int(store)).render(int(vr.RayMarchAlgorithm.ORIGINAL), oracle_camera_from(cam),
                                                            oracle_lighting_from(lit), cfg.width, cfg.height, cfg.scale)
        got, gb = gpu_render(g, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, cfg.width, cfg.height, 0, cfg.height,
                             count=True)
        assert np.array_equal(got, want) and gb == wb
