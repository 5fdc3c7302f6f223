"""Seeded random render cases for the parity fuzz tests (tests/test_gpu_fuzz.py on the
GPU, tests/test_oracle.py::test_fuzz_cases_python_restatement on the CPU).

Each case draws what the reference's interface lets a caller vary:
the voxel set (sparse points plus dense blocks, anywhere in a box that may reach
negative coordinates), the camera of Camera::Camera (Camera.cuh:11-23; eye outside or
inside the scene, sometimes on integer / cluster-plane coordinates so that walks start
on grid planes), the image size, VoxelSceneInfo's scale and translation
(VoxelSceneInfo.cuh:5-15), and the setupConstantValues block (Main.cu:26-42: light
direction -- including axis-aligned, equal-component and zero-component ones --,
colour, point light, shadows).  Pure numpy: no GPU, no libvr."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class Case:
    seed: int
    xyz: np.ndarray
    rgb: np.ndarray
    eye: tuple
    look_at: tuple
    up: tuple
    fov: float
    W: int
    H: int
    scale: int
    translation: tuple
    shadows: bool
    point: bool
    light_dir: tuple | None          # None: the reference's normalize(1, 1, 1)
    light_pos: tuple
    light_color: tuple
    notes: list = field(default_factory=list)

    @property
    def aspect(self) -> float:
        return float(np.float32(self.W) / np.float32(self.H))


def _voxels(rng, lo, ext):
    parts, centres = [], []
    n_sparse = int(rng.integers(0, 1500))
    parts.append(rng.integers(0, ext, size=(n_sparse, 3)))
    for _ in range(int(rng.integers(2, 8))):                  # dense blocks
        size = rng.integers(2, max(3, ext // 2), size=3)
        corner = rng.integers(0, np.maximum(ext - size, 1), size=3)
        g = np.stack(np.meshgrid(*[np.arange(s) for s in size], indexing="ij"), -1).reshape(-1, 3)
        keep = rng.random(len(g)) < rng.uniform(0.05, 1.0)
        parts.append(g[keep] + corner)
        centres.append(corner + size / 2.0)
    xyz = (np.concatenate(parts) + lo).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=len(xyz), dtype=np.uint32)
    return xyz, rgb, np.array(centres) + lo


def _light_dir(rng):
    k = int(rng.integers(0, 6))
    if k == 0:
        return None
    if k == 1:                                               # equal magnitudes, random signs
        return tuple(float(s) for s in rng.choice([-1.0, 1.0], size=3))
    if k == 2:                                               # axis-aligned
        d = [0.0, 0.0, 0.0]
        d[int(rng.integers(0, 3))] = float(rng.choice([-1.0, 1.0]))
        return tuple(d)
    if k == 3:                                               # one zero component
        d = rng.normal(size=3)
        d[int(rng.integers(0, 3))] = 0.0
        return tuple(float(v) for v in d)
    return tuple(float(v) for v in rng.normal(size=3))


def make_case(seed: int) -> Case:
    rng = np.random.default_rng(seed)
    ext = int(rng.choice([24, 48, 80, 130]))
    lo = rng.integers(-90, 40, size=3)
    xyz, rgb, blocks = _voxels(rng, lo, ext)
    scale = int(rng.choice([1, 1, 2, 3, 7]))
    notes = []
    # the scene as the march sees it: local = (world - translation) * scale, so place
    # the camera in world units around the voxels' centre / scale
    translation = (0.0, 0.0, 0.0)
    if rng.random() < 0.5:
        translation = tuple(float(v) for v in np.round(rng.uniform(-3, 3, size=3) * 4) / 4)
    centre = (lo + ext / 2.0) / scale + np.array(translation)
    d = rng.normal(size=3)
    d /= np.linalg.norm(d)
    dist = rng.uniform(0.2, 2.5) * ext / scale
    eye = centre + d * dist
    if rng.random() < 0.3:                                   # on grid / cluster planes
        q = float(rng.choice([1.0, 8.0, 0.5]))
        eye = np.round(eye * scale / q) * q / scale
        notes.append(f"eye snapped to {q}")
    look = centre + rng.normal(size=3) * ext / scale * 0.2
    if rng.random() < 0.6:                                   # at one of the dense blocks
        look = blocks[int(rng.integers(0, len(blocks)))] / scale + np.array(translation)
    if rng.random() < 0.2:                                   # look along an axis
        a = int(rng.integers(0, 3))
        look = eye.copy()
        look[a] += float(rng.choice([-1.0, 1.0])) * ext
        notes.append("axis view")
    fwd = look - eye
    up = (0.0, 1.0, 0.0)
    if abs(fwd[1]) > 0.95 * np.linalg.norm(fwd):
        up = (0.0, 0.0, 1.0)
    W, H = int(rng.integers(24, 80)), int(rng.integers(16, 64))
    return Case(seed=seed, xyz=xyz, rgb=rgb, eye=tuple(float(v) for v in eye),
                look_at=tuple(float(v) for v in look), up=up, fov=float(rng.uniform(15.0, 110.0)), W=W, H=H,
                scale=scale, translation=translation, shadows=bool(rng.random() < 0.8),
                point=bool(rng.random() < 0.3), light_dir=_light_dir(rng),
                light_pos=tuple(float(v) for v in centre + rng.normal(size=3) * ext / scale),
                light_color=tuple(float(v) for v in np.round(rng.uniform(0.0, 2.0, size=3) * 8) / 8), notes=notes)


def make_wide_case(seed: int) -> Case:
    """A scene over several 64^3 regions with empty regions between its blocks (the
    null-region skip, region advance and entry clip of rayMarchVoxelScene,
    Renderer.cuh:338-434), seen from up to four scene widths away."""
    rng = np.random.default_rng(seed)
    ext = int(rng.choice([200, 320, 500]))
    lo = rng.integers(-260, 60, size=3)
    parts, centres = [], []
    for _ in range(int(rng.integers(2, 7))):
        size = rng.integers(2, 40, size=3)
        corner = rng.integers(0, ext - size, size=3)
        g = np.stack(np.meshgrid(*[np.arange(s) for s in size], indexing="ij"), -1).reshape(-1, 3)
        keep = rng.random(len(g)) < rng.uniform(0.05, 1.0)
        parts.append(g[keep] + corner)
        centres.append(corner + size / 2.0 + lo)
    parts.append(rng.integers(0, ext, size=(int(rng.integers(0, 3000)), 3)))
    xyz = (np.concatenate(parts) + lo).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=len(xyz), dtype=np.uint32)
    scale = int(rng.choice([1, 1, 2, 4]))
    translation = (0.0, 0.0, 0.0) if rng.random() < 0.5 else \
        tuple(float(v) for v in np.round(rng.uniform(-9, 9, size=3) * 2) / 2)
    tr = np.array(translation)
    centre = (lo + ext / 2.0) / scale + tr
    d = rng.normal(size=3)
    d /= np.linalg.norm(d)
    look = centres[int(rng.integers(0, len(centres)))] / scale + tr
    if rng.random() < 0.5:                                   # from outside the scene
        eye = centre + d * rng.uniform(0.6, 4.0) * ext / scale
    else:                                                    # near a block, across regions
        eye = look + d * rng.uniform(20.0, 150.0) / scale
    fwd = look - eye
    up = (0.0, 0.0, 1.0) if abs(fwd[1]) > 0.95 * np.linalg.norm(fwd) else (0.0, 1.0, 0.0)
    W, H = int(rng.integers(32, 96)), int(rng.integers(24, 72))
    return Case(seed=seed, xyz=xyz, rgb=rgb, eye=tuple(float(v) for v in eye), look_at=tuple(float(v) for v in look),
                up=up, fov=float(rng.uniform(5.0, 70.0)), W=W, H=H, scale=scale, translation=translation,
                shadows=bool(rng.random() < 0.8), point=bool(rng.random() < 0.3), light_dir=_light_dir(rng),
                light_pos=tuple(float(v) for v in centre + rng.normal(size=3) * ext / scale),
                light_color=(1.0, 1.0, 1.0), notes=["wide"])
