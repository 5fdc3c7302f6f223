"""CPU check of the crawl-voxel recovery behind the crawl pass's resume
(vr_march.hip crawl_voxel): a crawl iteration stepped o <- RN(o + c),
c = RN(EPSILON * d); the deferral record keeps only the stepped position, and
the voxel q = trunc(old o) is recovered from it as the truncation shared by
every float within 4 steps of RN(o - c) that steps to o, or declared ambiguous
(the crawl pass then walks the pixel from its start).  The restatement below
follows the device code operation by operation in float32; on random and
adversarial inputs every recovered q must equal the true one."""
from __future__ import annotations

import numpy as np

F = np.float32
EPS = F(0.0001)


def crawl_voxel(on: np.float32, c: np.float32):
    e = F(on - c)
    if F(e + F(2.0 ** -20)) < F(1.0):
        return 0
    found, ok = -1, True
    eb = np.array([e], dtype=np.float32).view(np.uint32)[0]
    for k in range(-4, 5):
        x = np.array([np.uint32(int(eb) + k)], dtype=np.uint32).view(np.float32)[0]
        if not (x >= 0) or F(x + c) != on:
            continue
        t = int(np.trunc(x))
        ok &= found < 0 or t == found
        found = t
    return found if ok and found >= 0 else None


def _check(o_prev: np.ndarray, d: np.ndarray):
    amb = 0
    for op, dd in zip(o_prev, d):
        c = F(EPS * dd)
        on = F(op + c)
        q = crawl_voxel(on, c)
        if q is None:
            amb += 1
            continue
        assert q == int(np.trunc(op)), (float(op), float(dd), q)
    return amb


def test_random_positions_recover_exactly():
    rng = np.random.default_rng(7)
    o_prev = rng.uniform(0.0, 64.0, 200_000).astype(np.float32)
    d = rng.uniform(-1.0, 1.0, 200_000).astype(np.float32)
    amb = _check(o_prev, d)
    assert amb < 50          # ambiguity needs an integer within a few ulps


def test_positions_next_to_integers():
    """The hard cases: old coordinates on, just below and just above integers (the
    pinned plane axis of a crawl sits exactly on a multiple of 8)."""
    rng = np.random.default_rng(11)
    ks = rng.integers(0, 64, 20_000).astype(np.float32)
    steps = rng.integers(-3, 4, 20_000)
    o_prev = (ks.view(np.uint32).astype(np.int64) + steps).clip(0).astype(np.uint32).view(np.float32)
    o_prev = np.where(o_prev < 64.0, o_prev, F(63.5)).astype(np.float32)
    d = rng.choice(np.array([1e-4, 3e-3, 0.01, 0.07, 0.3, 0.577, 0.99], dtype=np.float32), 20_000)
    d = (d * rng.choice(np.array([-1.0, 1.0], dtype=np.float32), 20_000)).astype(np.float32)
    _check(o_prev, d)


def test_pinned_axis_is_exact():
    """An axis EPSILON * d cannot move (the crawl's plane): q is the plane itself."""
    for k in (8.0, 16.0, 24.0, 32.0, 40.0, 48.0, 56.0):
        for dd in (1e-3, -1e-3, 2e-3, -4e-4):
            c = F(EPS * F(dd))
            on = F(F(k) + c)
            assert on == F(k)            # |c| < ulp(k) / 2: the axis is pinned
            assert crawl_voxel(on, c) == int(k)
