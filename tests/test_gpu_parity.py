"""GPU parity: the HIP ray march (through the C ABI) against the CPU oracle,
bit-exact on the packed 0x00RRGGBB words, plus the algorithmic byte count of
the instrumented kernel against the oracle's count."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from tests.helpers import diff_report, gpu_render, oracle_camera_from, oracle_lighting_from

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")

STORES = [vr.StorageType.VOXEL_CLUSTER_STORE, vr.StorageType.HASH_TABLE]
ALGOS = [vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS]
KERNELS = [vr.Kernel.PERSISTENT, vr.Kernel.TILE]


def check_frame(xyz, rgb, store, algo, W, H, scale, cam=None, lit=None, translation=(0.0, 0.0, 0.0),
                row_begin=0, row_end=None, count=True, oracle_scene=None, gpu_scene=None, kernels=KERNELS):
    row_end = H if row_end is None else row_end
    cam = cam or vr.Camera.reference(W, H)
    lit = lit or vr.setup_constant_values()
    info = vr.VoxelSceneInfo(translation, scale)
    scene = gpu_scene or vr.create_scene(xyz, rgb, store)
    ref = oracle_scene or oracle.Scene(xyz, rgb, int(store))
    want, obytes = ref.render(int(algo), oracle_camera_from(cam), oracle_lighting_from(lit), W, H, scale,
                              translation, row_begin, row_end)
    for kernel in kernels:
        got, gbytes = gpu_render(scene, algo, cam, lit, info, W, H, row_begin, row_end, count=count, kernel=kernel)
        assert np.array_equal(got, want), f"{kernel.name}: " + diff_report(got, want, W, row_begin)
        if count:
            assert gbytes == obytes, f"{kernel.name}: algorithmic bytes: gpu {gbytes} != oracle {obytes}"
        got2, _ = gpu_render(scene, algo, cam, lit, info, W, H, row_begin, row_end, count=False, kernel=kernel)
        assert np.array_equal(got2, want), f"{kernel.name} (uncounted): " + diff_report(got2, want, W, row_begin)
    return want


@pytest.fixture(scope="module")
def c1():
    return vr.CONFIGS["C1"].voxels()


@pytest.fixture(scope="module")
def c2():
    return vr.CONFIGS["C2"].voxels()


@pytest.mark.parametrize("store", STORES, ids=lambda s: s.name)
@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_c1_full_frame(c1, store, algo):
    cfg = vr.CONFIGS["C1"]
    img = check_frame(*c1, store, algo, cfg.width, cfg.height, cfg.scale)
    assert 0.2 < np.mean(img != 0) < 0.9


@pytest.mark.parametrize("store", STORES, ids=lambda s: s.name)
@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_c2_quarter_res(c2, store, algo):
    cfg = vr.CONFIGS["C2"]
    check_frame(*c2, store, algo, 480, 270, cfg.scale)


@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_c2_full_res_vcs(c2, algo):
    """BASELINE configs C2 (original) and C3 (longest axis) at 1920x1080, whole frame."""
    cfg = vr.CONFIGS["C2"]
    check_frame(*c2, vr.StorageType.VOXEL_CLUSTER_STORE, algo, cfg.width, cfg.height, cfg.scale)


def test_c4_dense_hashtable_rows():
    """C4 (512^3 dense, every region/cluster populated): a band of rows at full width."""
    cfg = vr.CONFIGS["C4"]
    xyz, rgb = cfg.voxels()
    assert len(rgb) > 15_000_000
    check_frame(xyz, rgb, vr.StorageType.HASH_TABLE, vr.RayMarchAlgorithm.ORIGINAL, cfg.width, cfg.height,
                cfg.scale, row_begin=500, row_end=532)


def test_c5_sparse_rows():
    """C5 (1024^3 sparse, D = 16): rows of the 4K frame, both algorithms."""
    cfg = vr.CONFIGS["C5"]
    xyz, rgb = cfg.voxels()
    g = vr.create_scene(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE)
    o = oracle.Scene(xyz, rgb, 0)
    assert g.info()["diameter"] == 16
    for algo in ALGOS:
        check_frame(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE, algo, cfg.width, cfg.height, cfg.scale,
                    row_begin=1000, row_end=1016, oracle_scene=o, gpu_scene=g)


def test_c5_crawl_rows():
    """C5 rows 696-712: thousands of rays that creep through empty clusters by
    RN(EPSILON * d) per iteration (o pinned on a cluster plane), most of
    them until the 65 536-iteration budget -- including a ties-to-even crawl at
    (792, 709).  The tile pass defers them (with the walk's state at the crawl) and
    the crawl pass resumes and fast-forwards them;
    pixels and algorithmic bytes must still equal the oracle's plain walk."""
    cfg = vr.CONFIGS["C5"]
    xyz, rgb = cfg.voxels()
    g = vr.create_scene(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE)
    o = oracle.Scene(xyz, rgb, 0)
    for algo in ALGOS:
        # TILE resumes each deferred crawl from its record; TILE_REWALK walks the pixel
        # from its start (the fallback for crawls whose voxel the record cannot pin)
        check_frame(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE, algo, cfg.width, cfg.height, cfg.scale,
                    row_begin=696, row_end=712, oracle_scene=o, gpu_scene=g,
                    kernels=KERNELS + [vr.Kernel.TILE_REWALK])


def test_count_variant_pixels_identical(c2):
    cfg = vr.CONFIGS["C2"]
    scene = vr.create_scene(*c2, vr.StorageType.VOXEL_CLUSTER_STORE)
    cam, lit, info = vr.Camera.reference(480, 270), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
    a, _ = gpu_render(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, 480, 270, count=False)
    b, n = gpu_render(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, 480, 270, count=True)
    assert np.array_equal(a, b) and n > 0


@pytest.mark.parametrize("nranks,band", [(1, 8), (2, 8), (3, 8), (4, 16), (8, 8)])
def test_band_partition_reassembles(c1, nranks, band):
    """vr_render_bands on every rank, interleaved back, equals the single full render."""
    import torch
    cfg = vr.CONFIGS["C1"]
    W, H = 200, 150   # H not a multiple of the band
    scene = vr.create_scene(*c1, vr.StorageType.VOXEL_CLUSTER_STORE)
    cam, lit, info = vr.Camera.reference(W, H), vr.setup_constant_values(), vr.VoxelSceneInfo((0, 0, 0), cfg.scale)
    full, _ = gpu_render(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H)
    words = vr.band_buffer_words(W, H, band, nranks)
    parts = []
    for r in range(nranks):
        buf = torch.full((words,), -7, dtype=torch.int32, device="cuda")
        vr.render_bands(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, band, r, nranks, buf)
        parts.append(buf)
    torch.cuda.synchronize()
    from voxelraymarcher_amd.tiles import assemble_bands
    img = assemble_bands(torch.stack(parts), W, H, band).cpu().numpy().view(np.uint32).reshape(-1)
    assert np.array_equal(img, full)


# ------------------------------------------------------------------ edge cases

def test_empty_scene():
    xyz = np.zeros((0, 3), np.int32)
    rgb = np.zeros(0, np.uint32)
    for store in STORES:
        for algo in ALGOS:
            img = check_frame(xyz, rgb, store, algo, 64, 48, 4)
            assert not img.any()


def test_single_voxel_and_negative_coords():
    rng = np.random.default_rng(7)
    xyz = np.concatenate([rng.integers(-70, 60, size=(3000, 3)), np.array([[0, 0, 0], [-1, -1, -1], [63, 64, 65]])])
    rgb = rng.integers(0, 1 << 24, size=len(xyz), dtype=np.uint32)
    cam = vr.Camera((90.0, 40.0, 100.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 70.0, 4.0 / 3.0)
    for store in STORES:
        for algo in ALGOS:
            check_frame(xyz, rgb, store, algo, 160, 120, 1, cam=cam)


def test_duplicates_last_wins():
    xyz = np.array([[5, 5, 5], [5, 5, 5], [6, 5, 5]], np.int32)
    rgb = np.array([0xFF0000, 0x00FF00, 0x0000FF], np.uint32)
    cam = vr.Camera((20.0, 12.0, 22.0), (5.0, 5.0, 5.0), (0.0, 1.0, 0.0), 30.0, 1.0)
    for store in STORES:
        img = check_frame(xyz, rgb, store, vr.RayMarchAlgorithm.ORIGINAL, 64, 64, 1, cam=cam)
        assert img.any()


@pytest.mark.parametrize("store", STORES, ids=lambda s: s.name)
@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_lighting_variants(c1, store, algo):
    cfg = vr.CONFIGS["C1"]
    for shadows, point in ((False, False), (True, True), (False, True)):
        lit = vr.setup_constant_values(use_shadows=shadows, use_point_light=point, light_position=(40.0, 90.0, 30.0))
        check_frame(*c1, store, algo, 96, 96, cfg.scale, lit=lit)


LIGHTS = [((-1.0, -1.0, -1.0), (1.0, 1.0, 1.0)),     # equal negative components: one-division shadow walk, d < 0
          ((0.0, 1.0, 0.0), (1.0, 1.0, 1.0)),        # two zero components: guarded shadow divisions
          ((1.0, 1.0, 0.0), (0.5, 1.0, 0.25)),       # long-axis tie x = y (strict '>' picks y)
          ((-1.0, 2.0, -0.5), (1.0, 0.75, 2.0)),     # negative steps, channel overflow clamps by truncation
          ((0.0, -1.0, 1.0), (1.0, 1.0, 1.0))]


@pytest.mark.parametrize("store", STORES, ids=lambda s: s.name)
@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_light_direction_and_color(c1, c2, store, algo):
    """the setupConstantValues block as parameters -- light
    direction (through makeUnitVector) and colour change shading and the shadow walk."""
    for i, (d, col) in enumerate(LIGHTS):
        lit = vr.setup_constant_values(light_direction=d, light_color=col)
        check_frame(*c1, store, algo, 96, 96, vr.CONFIGS["C1"].scale, lit=lit)
        if i < 3:
            check_frame(*c2, store, algo, 240, 136, vr.CONFIGS["C2"].scale, lit=lit, kernels=[vr.Kernel.TILE])


@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_camera_inside_grid_and_translation(c1, algo):
    cam = vr.Camera((2.0, 2.5, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 90.0, 1.5)
    for store in STORES:
        check_frame(*c1, store, algo, 120, 80, 9, cam=cam, translation=(-1.0, -0.5, 0.25))


@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_axis_aligned_views(c1, algo):
    """Rays (nearly) parallel to grid planes: zero / tiny direction components."""
    views = [((32.0, 32.0, 200.0), (32.0, 32.0, 0.0), (0.0, 1.0, 0.0)),
             ((32.0, 300.0, 32.0), (32.0, 0.0, 32.0), (0.0, 0.0, 1.0)),
             ((-150.0, 31.5, 31.5), (10.0, 31.5, 31.5), (0.0, 1.0, 0.0))]
    for eye, at, up in views:
        cam = vr.Camera(eye, at, up, 20.0, 1.0)
        for store in STORES:
            check_frame(*c1, store, algo, 65, 65, 1, cam=cam)
