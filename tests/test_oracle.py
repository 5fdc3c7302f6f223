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
    """Two independent transcriptions of Renderer.cuh agree pixel for pixel."""
    xyz, rgb = _golden_scene()
    W, H, scale = 256, 256, 12
    cam = oracle.reference_camera(W, H)
    rng = np.random.default_rng(100 + 2 * store + algo)
    px = rng.integers(0, W, 120)
    py = rng.integers(0, H, 120)
    sc = oracle.Scene(xyz, rgb, store)
    ps = pyref.Scene(xyz, rgb, store)
    for shadows, point in ((True, False), (False, True)):
        lit = oracle.lighting(use_shadows=shadows, use_point_light=point, light_position=(40.0, 90.0, 30.0))
        plit = pyref.Lighting(shadows, point, (40.0, 90.0, 30.0))
        got, _ = sc.render_pixels(algo, cam, lit, W, H, scale, px, py)
        for i in range(len(px)):
            want = pyref.render_pixel(ps, plit, _pyref_camera(cam), W, H, int(px[i]), int(py[i]), scale,
                                      algo == oracle.ALGO_LONGESTAXIS)
            assert int(got[i]) == want, (int(px[i]), int(py[i]), hex(int(got[i])), hex(want))


def test_oracle_matches_python_restatement_negative_and_translated():
    rng = np.random.default_rng(5)
    xyz = rng.integers(-80, 70, size=(2500, 3)).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=2500).astype(np.uint32)
    cam = oracle.camera((90.0, 40.0, 100.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 70.0, 4.0 / 3.0)
    tr = (-1.0, -0.5, 0.25)
    for store in (0, 1):
        sc = oracle.Scene(xyz, rgb, store)
        ps = pyref.Scene(xyz, rgb, store)
        px = rng.integers(0, 160, 60)
        py = rng.integers(0, 120, 60)
        for algo in (0, 1):
            got, _ = sc.render_pixels(algo, cam, oracle.lighting(), 160, 120, 1, px, py, translation=tr)
            for i in range(len(px)):
                want = pyref.render_pixel(ps, pyref.Lighting(), _pyref_camera(cam), 160, 120, int(px[i]), int(py[i]),
                                          1, algo == 0, translation=tr)
                assert int(got[i]) == want


def test_scene_geometry_rules():
    """minCoord/maxCoord start at 0 and are scalars over all axes (VoxelSceneCPU.cuh:28-35,129-130)."""
    sc = oracle.Scene(np.array([[200, 5, 5]], np.int32), np.array([1], np.uint32), 0)
    assert (sc.min_coord, sc.diameter) == (0, 4)
    sc = oracle.Scene(np.array([[-1, 5, 5], [5, 300, 5]], np.int32), np.array([1, 2], np.uint32), 0)
    assert (sc.min_coord, sc.diameter) == (-1, 6)
    assert sc.region_count == 2
