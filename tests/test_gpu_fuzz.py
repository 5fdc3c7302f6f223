"""GPU parity fuzz: seeded random scenes, cameras, image sizes, scales, translations
and lighting blocks (tests/fuzz_cases.py), every store x algorithm, the HIP frame
(counted and uncounted, through the C ABI) against the oracle's pixels and
algorithmic bytes -- bit-exact.  Widens the hand-picked cases of test_gpu_parity.py
to views the reference's interface allows but no fixed case covers."""
from __future__ import annotations

import pytest

import oracle
from tests.fuzz_cases import make_case, make_wide_case
from tests.helpers import oracle_camera_from, oracle_lighting_from
from tests.test_gpu_parity import ALGOS, STORES, check_frame

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")

SEEDS = list(range(1000, 1200))
WIDE_SEEDS = list(range(5000, 5100))


@pytest.mark.parametrize("seed", SEEDS + WIDE_SEEDS)
def test_random_views(seed):
    c = make_wide_case(seed) if seed >= 5000 else make_case(seed)
    cam = vr.Camera(c.eye, c.look_at, c.up, c.fov, c.aspect)
    lit = vr.setup_constant_values(use_shadows=c.shadows, use_point_light=c.point, light_position=c.light_pos,
                                   light_direction=c.light_dir, light_color=c.light_color)
    for store in STORES:
        ref = oracle.Scene(c.xyz, c.rgb, int(store))
        gpu = vr.create_scene(c.xyz, c.rgb, store)
        for algo in ALGOS:
            want = ref.render(int(algo), oracle_camera_from(cam), oracle_lighting_from(lit), c.W, c.H, c.scale,
                              c.translation)
            check_frame(c.xyz, c.rgb, store, algo, c.W, c.H, c.scale, cam=cam, lit=lit, translation=c.translation,
                        gpu_scene=gpu, want=want)
        gpu.close()
