"""CPU tests of the oracle (oracle/vr_oracle.c): known-answer tests of the
reference's integer functions, storage lookups against a dict, the committed
golden fixtures, and a cross-check against the independent Python
restatement (tests/pyref.py) on sampled rays of every store x algorithm."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from tests import pyref
from tests.helpers import GOLDEN


def py_hash1(key: int, offset: int) -> int:
    """CuckooHashTable.cuh:181-190 evaluated with explicit int32 wrap-around."""
    w = pyref.wrap32
    k = w(key)
    k = w(w(k + 0x7ed55d16) + w(k << 12))
    k = w((k ^ 0xc761c23c) ^ (k >> 19))
    k = w(w(k + 0x165667b1) + w(k << 5))
    k = w(w(k + 0xd3a2646c) ^ w(k << 9))
    k = w(w(k + 0xfd7046c5) + w(k << 3))
    k = w((k ^ 0xb55a4f09) ^ (k >> 16))
    return w(k + offset)


def py_hash2(key: int, prime: int) -> int:
    """CuckooHashTable.cuh:193-202."""
    w = pyref.wrap32
    k = w(key)
    k = w((k ^ 61) ^ (k >> 16))
    k = w(k + w(k << 3))
    k = w(k ^ (k >> 4))
    k = w(k * prime)
    k = w(k ^ (k >> 15))
    return k


def test_hash_functions_match_python_restatement():
    rng = np.random.default_rng(3)
    keys = [0, 1, 61, 0x7FFFFFFF, -1, -2147483648, 1 << 30] + rng.integers(-2**31, 2**31, 300).tolist()
    primes = [668265261, 12289, 50331653]
    for k in keys:
        for off in (0, 7, 24):
            assert oracle.hash1(k, off) == py_hash1(k, off), k
        for p in primes:
            assert oracle.hash2(k, p) == py_hash2(k, p), (k, p)


def test_hash_known_answers():
    """Pinned values (committed fixture) so a change to either restatement is caught."""
    kat = json.load(open(os.path.join(GOLDEN, "hash_kat.json")))
    for row in kat["hash1"]:
        assert oracle.hash1(row["key"], row["offset"]) == row["value"]
    for row in kat["hash2"]:
        assert oracle.hash2(row["key"], row["prime"]) == row["value"]


def test_cluster_id_and_point_packing():
    L = oracle.lib()
    for x, y, z in [(0, 0, 0), (7, 7, 7), (8, 0, 0), (63, 63, 63), (8, 16, 24)]:
        assert L.or_cluster_id(x, y, z) == ((x // 8) << 6) | ((y // 8) << 3) | (z // 8)
        assert L.or_generate_3d_point(x, y, z) == (x << 20) | (y << 10) | z
    assert L.or_cluster_id(63, 63, 63) == 511


@pytest.mark.parametrize("store", [oracle.STORE_VCS, oracle.STORE_HASHTABLE])
def test_storage_lookup_matches_dict(store):
    rng = np.random.default_rng(11)
    xyz = rng.integers(-100, 140, size=(5000, 3)).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=5000).astype(np.uint32)
    truth = {}
    for (x, y, z), c in zip(xyz.tolist(), rgb.tolist()):
        truth[(x, y, z)] = c            # later duplicates win
    sc = oracle.Scene(xyz, rgb, store)
    for (x, y, z), c in list(truth.items())[:1500]:
        r = (int(np.floor(x / 64)), int(np.floor(y / 64)), int(np.floor(z / 64)))
        assert sc.lookup(r, (x % 64, y % 64, z % 64)) == c
    for _ in range(1500):
        x, y, z = rng.integers(-100, 140, size=3).tolist()
        if (x, y, z) in truth:
            continue
        r = (int(np.floor(x / 64)), int(np.floor(y / 64)), int(np.floor(z / 64)))
        assert sc.lookup(r, (x % 64, y % 64, z % 64)) == oracle.EMPTY


def _golden_scene():
    d = np.load(os.path.join(GOLDEN, "c1_scene.npz"))
    return d["xyz"], d["rgb"]


def test_golden_images():
    """The oracle reproduces the committed C1 frames (all 4 store x algorithm)."""
    meta = json.load(open(os.path.join(GOLDEN, "golden.json")))
    xyz, rgb = _golden_scene()
    lit = oracle.lighting()
    for case in meta["frames"]:
        W, H = case["width"], case["height"]
        sc = oracle.Scene(xyz, rgb, case["store"])
        img, nbytes = sc.render(case["algo"], oracle.reference_camera(W, H), lit, W, H, case["scale"])
        assert hashlib.sha256(img.tobytes()).hexdigest() == case["sha256"], case["name"]
        assert nbytes == case["algorithmic_bytes"], case["name"]
        want = np.load(os.path.join(GOLDEN, case["file"]))["pixels"]
        assert np.array_equal(img, want.reshape(-1))


def _pyref_camera(cam):
    return (pyref.V(*cam.origin), pyref.V(*cam.lower_left), pyref.V(*cam.horizontal), pyref.V(*cam.vertical))


@pytest.mark.parametrize("store", [oracle.STORE_VCS, oracle.STORE_HASHTABLE])
@pytest.mark.parametrize("algo", [oracle.ALGO_ORIGINAL, oracle.ALGO_LONGESTAXIS])
def test_oracle_matches_python_restatement(store, algo):
    """Two independent transcriptions of Renderer.cuh agree pixel for pixel, and on each
    ray's algorithmic bytes."""
    xyz, rgb = _golden_scene()
    W, H, scale = 256, 256, 12
    cam = oracle.reference_camera(W, H)
    rng = np.random.default_rng(100 + 2 * store + algo)
    px = rng.integers(0, W, 120)
    py = rng.integers(0, H, 120)
    sc = oracle.Scene(xyz, rgb, store)
    ps = _pyref_scene(sc, xyz, rgb, store)
    for shadows, point in ((True, False), (False, True)):
        lit = oracle.lighting(use_shadows=shadows, use_point_light=point, light_position=(40.0, 90.0, 30.0))
        plit = pyref.Lighting(shadows, point, (40.0, 90.0, 30.0))
        _rays_agree(sc, ps, algo, cam, lit, plit, W, H, scale, px.astype(np.uint32), py.astype(np.uint32),
                    where=(shadows, point))


def test_oracle_matches_python_restatement_negative_and_translated():
    rng = np.random.default_rng(5)
    xyz = rng.integers(-80, 70, size=(2500, 3)).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=2500).astype(np.uint32)
    cam = oracle.camera((90.0, 40.0, 100.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 70.0, 4.0 / 3.0)
    tr = (-1.0, -0.5, 0.25)
    for store in (0, 1):
        sc = oracle.Scene(xyz, rgb, store)
        ps = _pyref_scene(sc, xyz, rgb, store)
        px = rng.integers(0, 160, 60).astype(np.uint32)
        py = rng.integers(0, 120, 60).astype(np.uint32)
        for algo in (0, 1):
            _rays_agree(sc, ps, algo, cam, oracle.lighting(), pyref.Lighting(), 160, 120, 1, px, py, translation=tr,
                        where=store)


def test_scene_geometry_rules():
    """minCoord/maxCoord start at 0 and are scalars over all axes (VoxelSceneCPU.cuh:28-35,129-130)."""
    sc = oracle.Scene(np.array([[200, 5, 5]], np.int32), np.array([1], np.uint32), 0)
    assert (sc.min_coord, sc.diameter) == (0, 4)
    sc = oracle.Scene(np.array([[-1, 5, 5], [5, 300, 5]], np.int32), np.array([1, 2], np.uint32), 0)
    assert (sc.min_coord, sc.diameter) == (-1, 6)
    assert sc.region_count == 2


# ---------------------------------------------------------------- round 3: walks without a budget

def _cfg_scene(name):
    """A config's synthetic scene from libvr's host generator (vr_synth_generate,
    checked against the numpy restatement tests/synth_ref.py in test_capi.py)."""
    import voxelraymarcher_amd.renderer as R
    cfg = R.CONFIGS[name]
    return cfg, cfg.voxels()


def test_crawl_run_matches_plain_steps():
    """pyref.crawl_run (exact rational closed form of a cluster-skip crawl) equals
    stepping p_i <- RN(p_i + RN(EPSILON * d_i)) one iteration at a time, on random
    crawls: pinned axis on its cluster's lower plane, positions in every binade of
    the region, ties-to-even steps included.  (All trials are stepped together.)"""
    rng = np.random.default_rng(42)
    F = np.float32
    P, C, Q, N, LO = [], [], [], [], []
    for trial in range(1500):
        lo = [int(v) for v in rng.integers(0, 8, 3) * 8]
        pin = int(rng.integers(0, 3))
        d = rng.normal(size=3)
        d[pin] = -abs(d[pin]) * (10.0 ** -rng.uniform(1.5, 4))    # small negative: EPSILON * d cannot move it
        d = (d / np.linalg.norm(d)).astype(np.float32)
        if trial % 7 == 0:                                        # c / ulp = k + 1/2 somewhere
            d[(pin + 1) % 3] = F(-(2 ** -18) * 1.5 / 1e-4)
        p = [F(lo[i] + rng.uniform(0, 8) * (rng.uniform() ** 3)) for i in range(3)]
        p[pin] = F(lo[pin])
        c = [F(pyref.EPS * F(d[i])) for i in range(3)]
        if F(p[pin] + c[pin]) != p[pin]:
            continue
        n, q = pyref.crawl_run(pyref.V(*p), pyref.V(*d), lo)
        if not n or n > 20000:            # (the longest batches: test_c5_crawl_pixels_python_restatement)
            continue
        P.append(p); C.append(c); Q.append([q[i] for i in range(3)]); N.append(n); LO.append(lo)
    x, c, n, lo = np.array(P, F), np.array(C, F), np.array(N), np.array(LO, np.float64)
    assert len(n) > 600
    for t in range(int(n.max())):
        act = n > t
        x[act] = (x[act] + c[act]).astype(F)                      # float32 adds, rounded per step
        xa = x[act].astype(np.float64)
        assert ((xa >= lo[act]) & (xa < lo[act] + 8)).all()
    assert np.array_equal(x, np.array(Q, F))


def test_c5_crawl_pixels_python_restatement():
    """The 100 longest C5 walks per algorithm (rows 696-711, up to 1.4 million
    iterations; committed in tests/golden/c5_crawl_pixels.json): the plain C oracle
    (every iteration walked, no budget) and the Python restatement (crawls in exact
    closed form) agree on colour, iteration count and the committed values."""
    cfg, (xyz, rgb) = _cfg_scene("C5")
    fx = json.load(open(os.path.join(GOLDEN, "c5_crawl_pixels.json")))["pixels"]
    sc = oracle.Scene(xyz, rgb, 0)
    ps = pyref.Scene(xyz, rgb, 0)
    W, H = cfg.width, cfg.height
    cam, lit = oracle.reference_camera(W, H), oracle.lighting()
    pc = _pyref_camera(cam)
    for algo in (1, 0):
        rows = [p for p in fx if p["algo"] == algo]
        assert len(rows) == 100 and min(p["iterations"] for p in rows) > 100_000
        px = np.array([p["x"] for p in rows], np.uint32)
        py = np.array([p["y"] for p in rows], np.uint32)
        got, b = sc.render_pixels(algo, cam, lit, W, H, cfg.scale, px, py)
        for i, p in enumerate(rows):
            assert int(got[i]) == p["colour"] and int(b[i]) == p["bytes"], p
            col, its = pyref.render_pixel(ps, pyref.Lighting(), pc, W, H, p["x"], p["y"], cfg.scale, algo == 0,
                                          iters=True)
            assert (col, its) == (p["colour"], p["iterations"]), (p, col, its)
            _, nb = pyref.render_pixel(ps, pyref.Lighting(), pc, W, H, p["x"], p["y"], cfg.scale, algo == 0,
                                       nbytes=True)
            assert nb == p["bytes"], (p, nb)


def _pyref_scene(sc, xyz, rgb, store):
    """The Python restatement of the same voxels; a cuckoo store takes the oracle build's
    placement (which table a key sits in) -- the only input the byte rule needs from a
    builder (CuckooHashTable.cuh:59-76: a key in table 2 costs key1 + key2 + val2)."""
    return pyref.Scene(xyz, rgb, store, placement=(lambda r, k: sc.cuckoo_table(r, k)[0]) if store == 1 else None)


def _rays_agree(sc, ps, algo, cam, lit, plit, W, H, scale, px, py, translation=(0.0, 0.0, 0.0), where=""):
    """Colour AND SURVEY 8(d) bytes of every ray: the C oracle vs the Python restatement."""
    got, b = sc.render_pixels(algo, cam, lit, W, H, scale, px, py, translation=translation)
    pc = _pyref_camera(cam)
    hits = 0
    for i in range(len(px)):
        col, nb = pyref.render_pixel(ps, plit, pc, W, H, int(px[i]), int(py[i]), scale,
                                     algo == oracle.ALGO_LONGESTAXIS, translation=translation, nbytes=True)
        assert (int(got[i]), int(b[i])) == (col, nb), (where, algo, int(px[i]), int(py[i]), hex(int(got[i])), hex(col),
                                                       int(b[i]), nb)
        hits += col != 0
    return hits


@pytest.mark.parametrize("algo", [oracle.ALGO_ORIGINAL, oracle.ALGO_LONGESTAXIS])
def test_c2_c3_rays_python_restatement(algo):
    """120 sampled rays of the C2 (original) / C3 (longest axis) 1920x1080 frame, both stores:
    colours and per-ray algorithmic bytes equal."""
    cfg, (xyz, rgb) = _cfg_scene("C2")
    W, H = cfg.width, cfg.height
    cam, lit = oracle.reference_camera(W, H), oracle.lighting()
    rng = np.random.default_rng(7 + algo)
    px = rng.integers(0, W, 120).astype(np.uint32)
    py = rng.integers(0, H, 120).astype(np.uint32)
    for store in (0, 1):
        sc = oracle.Scene(xyz, rgb, store)
        ps = _pyref_scene(sc, xyz, rgb, store)
        assert _rays_agree(sc, ps, algo, cam, lit, pyref.Lighting(), W, H, cfg.scale, px, py, where=store) > 20


def test_c4_rays_bytes_python_restatement():
    """>= 100 rays of the C4 frame (512^3 dense cuckoo store, 20 M voxels, hashtable +
    original): colours and per-ray bytes, the Python restatement's cuckoo byte rule over
    the oracle build's placement."""
    cfg, (xyz, rgb) = _cfg_scene("C4")
    W, H = cfg.width, cfg.height
    sc = oracle.Scene(xyz, rgb, 1)
    ps = _pyref_scene(sc, xyz, rgb, 1)
    del xyz, rgb
    cam, lit = oracle.reference_camera(W, H), oracle.lighting()
    rng = np.random.default_rng(44)
    px = rng.integers(0, W, 110).astype(np.uint32)
    py = rng.integers(0, H, 110).astype(np.uint32)
    assert _rays_agree(sc, ps, oracle.ALGO_ORIGINAL, cam, lit, pyref.Lighting(), W, H, cfg.scale, px, py) > 40


def test_rehashed_cuckoo_region_bytes_python_restatement():
    """A cuckoo region whose build needs a rehash (8 keys that share both default hash
    slots: the eviction chain passes createCuckooHashTable's limit, CuckooHashTable.cuh:
    112-123, and a new prime/offset is drawn) beside a dense block in the next region:
    every pixel of a 48x40 frame from two views, both algorithms, agrees in colour and
    bytes -- lookups into table 2 cost 4 B more -- and rays do hit the rehashed keys."""
    keys = [(0, 15, 63), (0, 36, 33), (0, 57, 6), (0, 60, 63), (3, 3, 45), (3, 12, 57), (3, 15, 48), (3, 45, 9)]
    g = np.stack(np.meshgrid(np.arange(64, 72), np.arange(0, 20), np.arange(20, 44), indexing="ij"), -1).reshape(-1, 3)
    xyz = np.concatenate([np.array(keys), g]).astype(np.int32)
    rgb = (np.arange(len(xyz), dtype=np.uint32) * 2654435761 % (1 << 24)).astype(np.uint32)
    sc = oracle.Scene(xyz, rgb, 1)
    assert sc.cuckoo_table(0, 0)[1], "region 0 is expected to need a rehash"
    tables = [sc.cuckoo_table(0, (x << 20) | (y << 10) | z)[0] for x, y, z in keys]
    assert set(tables) == {1, 2}
    ps = _pyref_scene(sc, xyz, rgb, 1)
    W, H = 48, 40
    px, py = np.meshgrid(np.arange(W, dtype=np.uint32), np.arange(H, dtype=np.uint32))
    px, py = px.reshape(-1), py.reshape(-1)
    hit_keys = 0
    for eye, at in (((-3.0, 40.0, 30.0), (4.0, 32.0, 30.0)), ((40.0, 70.0, 80.0), (2.0, 30.0, 30.0))):
        cam = oracle.camera(eye, at, (0.0, 1.0, 0.0), 70.0, W / H)
        for algo in (oracle.ALGO_ORIGINAL, oracle.ALGO_LONGESTAXIS):
            _rays_agree(sc, ps, algo, cam, oracle.lighting(use_shadows=False), pyref.Lighting(shadows=False), W, H, 1,
                        px, py, where=eye)
            img, _ = sc.render(algo, cam, oracle.lighting(use_shadows=False), W, H, 1)
            hit_keys += int(np.count_nonzero(img != 0))
    assert hit_keys > 0


def test_alias_rays_python_restatement():
    """Rays that probe outside their region where the `short` cluster id aliases into
    the directory (tests/golden/alias_rays.json): the oracle reproduces the committed
    frames, reports the aliased probes, and the Python restatement agrees on every pixel
    and on each frame's algorithmic bytes."""
    fx = json.load(open(os.path.join(GOLDEN, "alias_rays.json")))
    d = np.load(os.path.join(GOLDEN, fx["scene"]))
    sc = oracle.Scene(d["xyz"], d["rgb"], 0)
    ps = pyref.Scene(d["xyz"], d["rgb"], 0)
    lit = oracle.lighting()
    W, H = fx["width"], fx["height"]
    n_alias = 0
    for c in fx["cameras"]:
        cam = oracle.camera(c["eye"], c["at"], fx["up"], fx["fov"], fx["aspect"])
        img, nbytes = sc.render(0, cam, lit, W, H, 1)
        assert img.tolist() == c["pixels"] and nbytes == c["algorithmic_bytes"]
        st = sc.pixel_stats(0, cam, lit, W, H, 1)
        al = np.flatnonzero(st[..., 8].sum(-1).reshape(-1))
        assert al.tolist() == c["alias_pixels"]
        n_alias += len(al)
        total = 0
        for i in range(W * H):
            want, nb = pyref.render_pixel(ps, pyref.Lighting(), _pyref_camera(cam), W, H, i % W, i // W, 1, True,
                                          nbytes=True)
            assert want == c["pixels"][i], (c["eye"], i)
            total += nb
        assert total == c["algorithmic_bytes"], c["eye"]       # the aliasing slow path's bytes too
    assert n_alias >= 100


@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5", "C5-longestaxis"])
def test_frame_digests(name):
    """The oracle's full frames of the GPU configs reproduce the committed digests
    (tests/golden/frames.json) -- the fixtures the GPU tests check against."""
    g = {f["name"]: f for f in json.load(open(os.path.join(GOLDEN, "frames.json")))["frames"]}[name]
    cfg, (xyz, rgb) = _cfg_scene(g["scene"])
    sc = oracle.Scene(xyz, rgb, g["store"])
    img, nbytes = sc.render(g["algo"], oracle.reference_camera(g["width"], g["height"]), oracle.lighting(),
                            g["width"], g["height"], g["scale"])
    assert hashlib.sha256(img.tobytes()).hexdigest() == g["sha256"]
    assert nbytes == g["algorithmic_bytes"]


def nan_camera():
    """A camera whose every ray has a NaN direction: image plane = eye (ro - eye = 0,
    normalize(0) = 0/0).  vr_camera / or_camera are plain data, so a caller can hand
    the renderer this; the reference's walks then never finish for most scenes: the
    NaN position keeps floorf(NaN / 64) = 0, so the region loop (or the entry clip, or
    performVoxelSpaceJump's cluster skip) repeats its state forever."""
    cam = oracle.OrCamera()
    for i in range(3):
        cam.origin[i] = cam.lower_left[i] = 1.0
        cam.horizontal[i] = cam.vertical[i] = cam.forward[i] = 0.0
    return cam


def test_never_ending_walks():
    """Walks that never finish render 0 with only the pixel write counted (4 B), in
    both restatements; walks of the same camera that do finish (the hashtable's
    longest-axis walk hits a voxel at grid (0,0,1)) are rendered as usual."""
    xyz, rgb = _golden_scene()
    cam = nan_camera()
    pc = (pyref.V(1, 1, 1), pyref.V(1, 1, 1), pyref.V(0, 0, 0), pyref.V(0, 0, 0))
    ended = 0
    for store in (0, 1):
        sc = oracle.Scene(xyz, rgb, store)
        ps = pyref.Scene(xyz, rgb, store)
        for algo in (0, 1):
            img, nbytes = sc.render(algo, cam, oracle.lighting(), 4, 4, 12)
            assert not img.any()
            ended += nbytes > 64
            if not (store == 1 and algo == 0):
                assert nbytes == 16 * 4, (store, algo)
            assert pyref.render_pixel(ps, pyref.Lighting(), pc, 4, 4, 1, 2, 12, algo == 0) == 0
    assert ended == 1
    # no region at (0,0,0): the entry clip's state repeats
    sc = oracle.Scene(np.array([[100, 100, 100]], np.int32), np.array([5], np.uint32), 0)
    img, nbytes = sc.render(1, cam, oracle.lighting(), 4, 4, 1)
    assert not img.any() and nbytes == 64


@pytest.mark.parametrize("seed", list(range(1000, 1012)) + list(range(5000, 5006)))
def test_fuzz_cases_python_restatement(seed):
    """The GPU fuzz cases (tests/fuzz_cases.py: random scenes, cameras, scales,
    translations, light blocks): the oracle and the independent Python restatement
    agree on 24 sampled pixels per store x algorithm."""
    from tests.fuzz_cases import make_case, make_wide_case
    c = make_wide_case(seed) if seed >= 5000 else make_case(seed)
    cam = oracle.camera(c.eye, c.look_at, c.up, c.fov, c.aspect)
    plit = pyref.Lighting(c.shadows, c.point, c.light_pos)
    if c.light_dir is not None:
        plit.L = pyref.V(*c.light_dir).unit()                 # Main.cu:28 makeUnitVector
    plit.LC = pyref.V(*c.light_color)
    lit = oracle.lighting(use_shadows=c.shadows, use_point_light=c.point, light_position=c.light_pos)
    for i in range(3):
        lit.light_dir[i] = float(plit.L.x[i])
        lit.light_color[i] = float(plit.LC.x[i])
    rng = np.random.default_rng(seed)
    px = rng.integers(0, c.W, 24).astype(np.uint32)
    py = rng.integers(0, c.H, 24).astype(np.uint32)
    pc = _pyref_camera(cam)
    for store in (oracle.STORE_VCS, oracle.STORE_HASHTABLE):
        sc = oracle.Scene(c.xyz, c.rgb, store)
        ps = _pyref_scene(sc, c.xyz, c.rgb, store)
        for algo in (oracle.ALGO_ORIGINAL, oracle.ALGO_LONGESTAXIS):
            _rays_agree(sc, ps, algo, cam, lit, plit, c.W, c.H, c.scale, px, py, translation=c.translation,
                        where=(seed, store))


def test_cycle_detection_finds_every_period():
    """The region-level loops' never-finishes test (Brent's cycle detection, oracle
    cycle_step = the kernels' Ctx::cycle_step): a state sequence that
    repeats with any prefix and period is found within about twice (prefix + period)
    rounds -- round 4 compared each round with the one before only (period 1) -- and a
    sequence that never repeats is never reported."""
    L = oracle.lib()
    for prefix in range(0, 40, 3):
        for period in range(1, 40, 2):
            r = L.or_cycle_selftest(prefix, period, 100000)
            assert r > 0, (prefix, period)
            assert r >= max(prefix, 1) + period - 1, (prefix, period, r)   # not before a repeat exists
            assert r <= 2 * (prefix + period) + period + 2, (prefix, period, r)
    assert L.or_cycle_selftest(0, 1, 10) == 1                               # a fixed point: at once
    assert L.or_cycle_selftest(5, 0, 200000) == -1
