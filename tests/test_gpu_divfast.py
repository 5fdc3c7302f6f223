"""The walk loops divide with vr::div_fast (the IEEE division sequence with the
per-direction reciprocal hoisted, vr_device.h).  Check on the device that it is
bit-identical to the correctly rounded `/` for every float numerator of its
domain (2^-90 <= |n| < 2^20, both signs) and 2018 divisors (edge cases + random
ones over [2^-64, 2^20]): ~3.7e12 pairs, exhaustive in n (a few seconds)."""
from __future__ import annotations

import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_div_fast_matches_ieee_division():
    exe = os.path.join(ROOT, "voxelraymarcher_amd", "bin", "div_check")
    assert os.path.exists(exe), "build with make -C voxelraymarcher_amd/csrc"
    r = subprocess.run([exe, "2000"], capture_output=True, text=True, timeout=300)
    assert r.returncode in (0, 1), r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["pairs"] > 3e12
    assert res["mismatches"] == 0, res
