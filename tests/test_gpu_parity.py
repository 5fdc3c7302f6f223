"""GPU parity: the HIP ray march (through the C ABI) against the CPU oracle,
bit-exact on the packed 0x00RRGGBB words, plus the algorithmic byte count of
the instrumented kernel against the oracle's count."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from tests.helpers import GOLDEN, diff_report, gpu_render, oracle_camera_from, oracle_lighting_from

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")

STORES = [vr.StorageType.VOXEL_CLUSTER_STORE, vr.StorageType.HASH_TABLE]
ALGOS = [vr.RayMarchAlgorithm.ORIGINAL, vr.RayMarchAlgorithm.LONGEST_AXIS]
KERNELS = [vr.Kernel.TILE]
FRAMES = {f["name"]: f for f in json.load(open(os.path.join(GOLDEN, "frames.json")))["frames"]}


def check_frame(xyz, rgb, store, algo, W, H, scale, cam=None, lit=None, translation=(0.0, 0.0, 0.0),
                row_begin=0, row_end=None, count=True, oracle_scene=None, gpu_scene=None, kernels=KERNELS,
                want=None, defer_caps=(0,)):
    """The GPU frame (every kernel; counted and uncounted; every deferral-list capacity)
    equals the oracle's pixels and algorithmic bytes.  want = (pixels, bytes) already
    rendered by the oracle, else rendered here."""
    row_end = H if row_end is None else row_end
    cam = cam or vr.Camera.reference(W, H)
    lit = lit or vr.setup_constant_values()
    info = vr.VoxelSceneInfo(translation, scale)
    scene = gpu_scene or vr.create_scene(xyz, rgb, store)
    if want is None:
        ref = oracle_scene or oracle.Scene(xyz, rgb, int(store))
        want = ref.render(int(algo), oracle_camera_from(cam), oracle_lighting_from(lit), W, H, scale,
                          translation, row_begin, row_end)
    want, obytes = want
    for kernel in kernels:
        for cap in defer_caps:
            tag = f"{kernel.name} defer_cap={cap}"
            got, gbytes = gpu_render(scene, algo, cam, lit, info, W, H, row_begin, row_end, count=count,
                                     kernel=kernel, defer_cap=cap)
            assert np.array_equal(got, want), f"{tag}: " + diff_report(got, want, W, row_begin)
            if count:
                assert gbytes == obytes, f"{tag}: algorithmic bytes: gpu {gbytes} != oracle {obytes}"
            got2, _ = gpu_render(scene, algo, cam, lit, info, W, H, row_begin, row_end, count=False, kernel=kernel,
                                 defer_cap=cap)
            assert np.array_equal(got2, want), f"{tag} (uncounted): " + diff_report(got2, want, W, row_begin)
    return want


def check_golden(name, img, nbytes):
    """The frame equals the committed oracle digest (tests/golden/frames.json)."""
    g = FRAMES[name]
    assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == g["sha256"], name
    assert nbytes == g["algorithmic_bytes"], name


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
    """BASELINE configs C2 (original) and C3 (longest axis) at 1920x1080, whole frame,
    against the live oracle and the committed digest."""
    cfg = vr.CONFIGS["C2"]
    want = check_frame(*c2, vr.StorageType.VOXEL_CLUSTER_STORE, algo, cfg.width, cfg.height, cfg.scale)
    scene = vr.create_scene(*c2, vr.StorageType.VOXEL_CLUSTER_STORE)
    got, n = gpu_render(scene, algo, vr.Camera.reference(cfg.width, cfg.height), vr.setup_constant_values(),
                        vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale), cfg.width, cfg.height, count=True)
    assert np.array_equal(got, want)
    check_golden("C2" if algo == vr.RayMarchAlgorithm.ORIGINAL else "C3", got, n)


def test_c4_dense_hashtable_full_frame():
    """C4 (512^3 dense, every region/cluster populated, ~400 MB cuckoo store): the
    whole 1920x1080 frame, pixels and algorithmic bytes, live oracle and digest."""
    cfg = vr.CONFIGS["C4"]
    xyz, rgb = cfg.voxels()
    assert len(rgb) > 15_000_000
    scene = vr.create_scene(xyz, rgb, vr.StorageType.HASH_TABLE)
    want = check_frame(xyz, rgb, vr.StorageType.HASH_TABLE, vr.RayMarchAlgorithm.ORIGINAL, cfg.width, cfg.height,
                       cfg.scale, gpu_scene=scene)
    check_golden("C4", want, FRAMES["C4"]["algorithmic_bytes"])
    got, n = gpu_render(scene, vr.RayMarchAlgorithm.ORIGINAL, vr.Camera.reference(cfg.width, cfg.height),
                        vr.setup_constant_values(), vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale), cfg.width,
                        cfg.height, count=True)
    check_golden("C4", got, n)


@pytest.fixture(scope="module")
def c5():
    """C5 scene on the GPU and in the oracle, and the oracle's full 4K frames (both
    algorithms; no iteration budget: every cluster-skip crawl runs to its end)."""
    cfg = vr.CONFIGS["C5"]
    xyz, rgb = cfg.voxels()
    g = vr.create_scene(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE)
    o = oracle.Scene(xyz, rgb, 0)
    cam, lit = oracle.reference_camera(cfg.width, cfg.height), oracle.lighting()
    frames = {a: o.render(int(a), cam, lit, cfg.width, cfg.height, cfg.scale) for a in ALGOS}
    return cfg, xyz, rgb, g, o, frames


@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_c5_full_frame(c5, algo):
    """C5 (1024^3 sparse, D = 16) at 3840x2160: every pixel and the algorithmic bytes,
    including ~6 500 (original) / ~4 300 (longest axis) walks of 65 536 to 1.4 million
    iterations -- cluster-skip crawls that the tile pass hands to the crawl pass."""
    cfg, xyz, rgb, g, o, frames = c5
    want = check_frame(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE, algo, cfg.width, cfg.height, cfg.scale,
                       gpu_scene=g, want=frames[algo])
    check_golden("C5" if algo == vr.RayMarchAlgorithm.ORIGINAL else "C5-longestaxis", want, frames[algo][1])


@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_c5_crawl_rows(c5, algo):
    """C5 rows 696-712: thousands of rays that creep through empty clusters by
    RN(EPSILON * d) per iteration (o pinned on a cluster plane) for up to 1.4
    million iterations -- including a ties-to-even crawl at (792, 709).  The tile pass
    defers them (original: with the walk's state at the crawl; longest axis: past the
    tile budget) and the crawl pass fast-forwards them exactly.  TILE_REWALK walks every
    deferred pixel from its start; defer_cap 64 overflows the deferral list, so the
    crawl pass finds most pixels by their marker in the frame."""
    cfg, xyz, rgb, g, o, frames = c5
    W = cfg.width
    want = (frames[algo][0][696 * W:712 * W], None)
    check_frame(xyz, rgb, vr.StorageType.VOXEL_CLUSTER_STORE, algo, cfg.width, cfg.height, cfg.scale,
                row_begin=696, row_end=712, gpu_scene=g, count=False, want=want,
                kernels=[vr.Kernel.TILE, vr.Kernel.TILE_REWALK], defer_caps=(0, 64))


def test_c5_crawl_pixels_fixture(c5):
    """The committed longest C5 walks (tests/golden/c5_crawl_pixels.json: oracle colour
    per pixel, up to 1.4 million iterations) appear in the GPU's 4K frame."""
    cfg, xyz, rgb, g, o, frames = c5
    fx = json.load(open(os.path.join(GOLDEN, "c5_crawl_pixels.json")))["pixels"]
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    cam, lit = vr.Camera.reference(cfg.width, cfg.height), vr.setup_constant_values()
    for algo in ALGOS:
        got, _ = gpu_render(g, algo, cam, lit, info, cfg.width, cfg.height, 696, 712)
        for p in fx:
            if p["algo"] == int(algo):
                assert int(got[(p["y"] - 696) * cfg.width + p["x"]]) == p["colour"], p


@pytest.mark.parametrize("layout", ["tiles", "bands", "strips"])
def test_c5_eight_rank_emulation(c5, layout):
    """C5 as BASELINE defines it -- the fixed 3840x2160 frame over 8 ranks -- emulated on
    one GPU: each rank's buffer, assembled, equals the oracle's frame.  layout "tiles":
    the 2-D deal bench.py uses (16x16 blocks, block j of band b -> rank (j + 3b) % 8;
    vr_render_tiles + the device assembly kernel), both algorithms; "bands": 8-row bands
    dealt round-robin (vr_render_bands); "strips": the learned strip deal (round 6, the fixed
    tiling default) with the cut the calibration made on an MI355X (profiles/r06/strips/): rank
    r renders rows [b_r, b_r+1) (vr_render_ex), both algorithms, assembled by the host copies."""
    import torch

    from voxelraymarcher_amd.tiles import assemble_bands
    cfg, xyz, rgb, g, o, frames = c5
    W, H, R, T = cfg.width, cfg.height, 8, 16
    B = 16 if layout == "tiles" else 8
    cam, lit = vr.Camera.reference(W, H), vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    for algo in (ALGOS if layout != "bands" else [vr.RayMarchAlgorithm.ORIGINAL]):
        if layout == "strips":
            from voxelraymarcher_amd.tiles import assemble_strips
            b = [0, 216, 464, 688, 840, 1056, 1296, 1632, 2160]
            mh = max(b[r + 1] - b[r] for r in range(R))
            parts = torch.full((R, mh * W), -7, dtype=torch.int32, device="cuda")
            for r in range(R):
                vr.render_ex(g, algo, cam, lit, info, W, H, parts[r], b[r], b[r + 1])
            torch.cuda.synchronize()
            img = assemble_strips(parts, b, W).cpu().numpy().view(np.uint32).reshape(-1)
        elif layout == "tiles":
            words = vr.tile_buffer_words(W, H, B, T, R)
            parts = torch.full((R, words), -7, dtype=torch.int32, device="cuda")
            for r in range(R):
                vr.render_tiles(g, algo, cam, lit, info, W, H, B, T, r, R, parts[r])
            frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
            vr.assemble_tiles_device(parts, frame, 4, W, H, B, T, R)
            torch.cuda.synchronize()
            img = frame.cpu().numpy().view(np.uint32).reshape(-1)
        else:
            words = vr.band_buffer_words(W, H, B, R)
            parts = []
            for r in range(R):
                buf = torch.full((words,), -7, dtype=torch.int32, device="cuda")
                vr.render_bands(g, algo, cam, lit, info, W, H, B, r, R, buf)
                parts.append(buf)
            torch.cuda.synchronize()
            img = assemble_bands(torch.stack(parts), W, H, B).cpu().numpy().view(np.uint32).reshape(-1)
        want = frames[algo][0]
        assert np.array_equal(img, want), f"{layout} {algo.name}: " + diff_report(img, want, W)


def test_alias_rays():
    """Longest-axis rays whose first region probe is outside the region with a `short`
    cluster id that aliases into the directory (VoxelClusterStore.cuh:21-24,93-99; the
    kernel's lookup_aliased path): the committed oracle frames (tests/golden/alias_rays.json)."""
    fx = json.load(open(os.path.join(GOLDEN, "alias_rays.json")))
    d = np.load(os.path.join(GOLDEN, fx["scene"]))
    scene = vr.create_scene(d["xyz"], d["rgb"], vr.StorageType.VOXEL_CLUSTER_STORE)
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), fx["scale"])
    W, H = fx["width"], fx["height"]
    for c in fx["cameras"]:
        cam = vr.Camera(c["eye"], c["at"], fx["up"], fx["fov"], fx["aspect"])
        got, n = gpu_render(scene, vr.RayMarchAlgorithm.LONGEST_AXIS, cam, lit, info, W, H, count=True)
        assert got.tolist() == c["pixels"], c
        assert n == c["algorithmic_bytes"], c


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


def test_never_ending_walks():
    """A camera whose rays have NaN directions (plain-data vr_camera: image plane =
    eye): most walks never finish in the reference (the NaN position repeats the
    region loop's, entry clip's or cluster skip's state forever).  The tile pass hands
    them to the crawl pass at its budget; the crawl pass detects the unchanged loop
    state and writes 0 with 4 bytes, as the oracle does; the one config whose walks
    do finish renders as usual."""
    from tests.test_oracle import nan_camera
    xyz, rgb = vr.CONFIGS["C1"].voxels()
    cam = vr.Camera.reference(64, 64)
    for f in ("origin", "lower_left"):
        for i in range(3):
            getattr(cam.raw, f)[i] = 1.0
    for f in ("horizontal", "vertical", "forward"):
        for i in range(3):
            getattr(cam.raw, f)[i] = 0.0
    ocam = nan_camera()
    lit = vr.setup_constant_values()
    for store in STORES:
        ref = oracle.Scene(xyz, rgb, int(store))
        for algo in ALGOS:
            want = ref.render(int(algo), ocam, oracle_lighting_from(lit), 64, 64, 12)
            check_frame(xyz, rgb, store, algo, 64, 64, 12, cam=cam, lit=lit, want=want, defer_caps=(0, 16))


@pytest.mark.parametrize("algo", ALGOS, ids=lambda a: a.name)
def test_degenerate_light_direction(c1, algo):
    """vr_lighting is plain data: a caller may hand a light direction that is not a unit
    vector.  With (1e-6, 1e-6, 1e-6) (and colour 1e6, so that lit pixels are not 0) every
    shadow step's EPSILON * d is ~1e-10: a cluster-skip crawl barely moves, and a crawl
    that moved no coordinate would never finish.  GPU and oracle agree on every pixel and
    byte, and the frame renders in well under the test's bound: no walk loop runs to the
    crawl pass's 2^30-iteration hang guard ("Walks that never finish")."""
    import time
    lit = vr.setup_constant_values()
    for i in range(3):
        lit.light_dir[i] = 1e-6
        lit.light_color[i] = 1e6
    torch = pytest.importorskip("torch")
    t0 = time.perf_counter()
    for store in STORES:
        check_frame(*c1, store, algo, 96, 96, vr.CONFIGS["C1"].scale, lit=lit, defer_caps=(0, 16))
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 60.0
