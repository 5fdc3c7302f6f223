"""numpy restatement of the synthetic voxel-grid generator,
used to check vr_synth_generate (libvr.so) and to build fixtures without a GPU.

  h(stream, k) = splitmix64((seed << 34) | (stream << 32) | k)
  u = (h >> 40) * 2^-24
  voxel (x,y,z) exists iff u(h(0, region id)) < p_r and u(h(1, cluster id)) < p_c
                           and u(h(2, x<<20|y<<10|z)) < p_v
  colour = h(3, key) & 0xFFFFFF
Ids: region rx + ry*NR + rz*NR^2 (NR = N/64); cluster cx + cy*NC + cz*NC^2 (NC = N/8).
Output order: regions z-y-x major, then clusters z-y-x, then voxels z-y-x.
"""
from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def h(seed: int, stream: int, k: np.ndarray) -> np.ndarray:
    base = np.uint64(((seed << 34) | (stream << 32)) & 0xFFFFFFFFFFFFFFFF)
    return splitmix64(base | np.asarray(k, dtype=np.uint64))


def draw(seed, stream, k, p):
    return (h(seed, stream, k) >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0) < p


def synth(n: int, p_r: float, p_c: float, p_v: float, seed: int):
    NR, NC = n // 64, n // 8
    xs, cs = [], []
    r = np.arange(NR ** 3)
    rx, ry, rz = r % NR, (r // NR) % NR, r // (NR * NR)
    keep = draw(seed, 0, rx + ry * NR + rz * NR * NR, p_r)
    a = np.arange(8)
    for i in np.flatnonzero(keep):
        cz, cy, cx = np.meshgrid(rz[i] * 8 + a, ry[i] * 8 + a, rx[i] * 8 + a, indexing="ij")
        cx, cy, cz = cx.ravel(), cy.ravel(), cz.ravel()
        ck = draw(seed, 1, cx + cy * NC + cz * NC * NC, p_c)
        for j in np.flatnonzero(ck):
            z, y, x = np.meshgrid(cz[j] * 8 + a, cy[j] * 8 + a, cx[j] * 8 + a, indexing="ij")
            x, y, z = x.ravel().astype(np.uint64), y.ravel().astype(np.uint64), z.ravel().astype(np.uint64)
            key = (x << np.uint64(20)) | (y << np.uint64(10)) | z
            vk = draw(seed, 2, key, p_v)
            xs.append(np.stack([x[vk], y[vk], z[vk]], 1).astype(np.int32))
            cs.append((h(seed, 3, key[vk]) & np.uint64(0xFFFFFF)).astype(np.uint32))
    if not xs:
        return np.zeros((0, 3), np.int32), np.zeros(0, np.uint32)
    return np.concatenate(xs), np.concatenate(cs)
