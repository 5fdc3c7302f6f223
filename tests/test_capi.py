"""CPU tests of the product's C ABI (libvr.so) -- no compute calls that need
a GPU: every symbol include/vr.h declares is exported, the host-side camera
equals the oracle's, the synthetic generator equals its numpy restatement,
the .vox reader follows VoxelFile.cuh's parse rules, and device entry points
fail loudly (no CPU fallback) when no GPU is present."""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np
import pytest
import torch

import oracle
import voxelraymarcher_amd as vr
from voxelraymarcher_amd import _capi
from tests.synth_ref import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "vr.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vr_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = vr.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f"{n} declared in vr.h but not exported"
        assert n in _capi.SIGNATURES, f"{n} has no ctypes signature"
    out = os.popen(f"nm -D --defined-only {vr.LIB_PATH}").read()
    exported = set(re.findall(r" T (vr_[a-z0-9_]+)", out))
    assert set(names) <= exported
    assert lib.vr_version().decode().startswith("voxelraymarcher_amd")


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_capi.VrCamera) == 60
    assert ctypes.sizeof(_capi.VrLighting) == 44
    assert ctypes.sizeof(_capi.VrRenderOpts) == 72          # round 5: + occupancy, tile deal
    assert _capi.VrRenderOpts.reserved.offset + 4 == _capi.VR_RENDER_OPTS_MIN_SIZE
    assert _capi.VrRenderOpts.occupancy.offset == 56 and _capi.VrRenderOpts.reserved2.offset == 68
    assert ctypes.sizeof(_capi.VrSynthParams) == 40
    assert f"#define VR_RENDER_OPTS_MIN_SIZE {_capi.VR_RENDER_OPTS_MIN_SIZE}u" in open(
        os.path.join(ROOT, "include", "vr.h")).read()


def test_render_opts_versioning():
    """vr_render_opts carries its size (include/vr.h): vr_render_opts_init fills it, and a
    struct laid out as before the field existed (its first word is `kernel`, 0..3) is
    refused with VR_E_INVALID before any other argument is looked at -- no field is read
    past the caller's struct."""
    o = _capi.VrRenderOpts()
    _capi.check(vr.lib().vr_render_opts_init(ctypes.byref(o)), "init")
    assert o.struct_size == ctypes.sizeof(o) and o.nranks == 1 and o.row_end == 0xFFFFFFFF
    assert (o.kernel, o.schedule, o.defer_cap, o.reserved) == (0, 0, 0, 0) and not o.bytes_dev and not o.stats_dev
    assert (o.occupancy, o.tile_cols, o.deal_stride, o.reserved2) == (0, 0, 0, 0)

    class OldOpts(ctypes.Structure):      # the round-3 layout
        _fields_ = [("kernel", ctypes.c_uint32), ("row_begin", ctypes.c_uint32), ("row_end", ctypes.c_uint32),
                    ("band_rows", ctypes.c_uint32), ("rank", ctypes.c_uint32), ("nranks", ctypes.c_uint32),
                    ("bytes_dev", ctypes.c_void_p), ("defer_cap", ctypes.c_uint32), ("schedule", ctypes.c_uint32)]
    old = OldOpts(3, 0, 16, 8, 0, 1, None, 0, 0)
    lib = vr.lib()
    rc = lib.vr_render_ex(None, 1, None, None, None, 1, 16, 16, ctypes.cast(ctypes.byref(old),
                          ctypes.POINTER(_capi.VrRenderOpts)), None, None)
    assert rc == -1 and b"struct_size" in lib.vr_last_error()
    o.reserved = 1
    assert lib.vr_render_ex(None, 1, None, None, None, 1, 16, 16, ctypes.byref(o), None, None) == -1
    assert b"reserved" in lib.vr_last_error()


@pytest.mark.parametrize("W,H", [(1920, 1080), (256, 256), (3840, 2160), (97, 41)])
def test_camera_matches_oracle_bitwise(W, H):
    a = vr.Camera.reference(W, H).as_floats()
    o = oracle.reference_camera(W, H)
    b = np.array([list(o.origin), list(o.lower_left), list(o.horizontal), list(o.vertical), list(o.forward)],
                 dtype=np.float32)
    assert a.tobytes() == b.tobytes()


def test_lighting_defaults():
    lit = vr.setup_constant_values()
    L = np.float32(1.0) / np.sqrt(np.float32(3.0))
    assert [np.float32(v) for v in lit.light_dir] == [np.float32(1.0) / np.float32(np.sqrt(np.float32(3.0)))] * 3
    assert abs(float(lit.light_dir[0]) - float(L)) < 1e-7
    assert list(lit.light_color) == [1.0, 1.0, 1.0]
    assert list(lit.light_pos) == [10.0, 10.0, -10.0]
    assert (lit.use_point_light, lit.use_shadows) == (0, 1)
    o = oracle.lighting()
    assert bytes(lit) == bytes(o)


@pytest.mark.parametrize("d", [(1.0, 1.0, 1.0), (0.0, 1.0, 0.0), (-1.0, 2.0, -0.5), (3e-20, 1e-20, -2e-20)])
def test_light_direction_is_make_unit_vector(d):
    """Main.cu:28 makeUnitVector = v / sqrtf(x*x+y*y+z*z) in fp32 (Vector3.cuh:79,162-165)."""
    f = np.float32
    x, y, z = (f(c) for c in d)
    ln = np.sqrt(f(f(f(x * x) + f(y * y)) + f(z * z)), dtype=np.float32)
    want = [f(x / ln), f(y / ln), f(z / ln)]
    lit = vr.setup_constant_values(light_direction=d, light_color=(0.5, 1.0, 2.0))
    assert [f(v) for v in lit.light_dir] == want
    assert list(lit.light_color) == [0.5, 1.0, 2.0]
    if d == (1.0, 1.0, 1.0):
        assert list(lit.light_dir) == list(oracle.lighting().light_dir)
    with pytest.raises(vr.VrError):
        vr.setup_constant_values(light_direction=(0.0, 0.0, 0.0))


@pytest.mark.parametrize("name", ["C1", "C2", "C5"])
def test_synth_generator_matches_numpy(name):
    cfg = vr.CONFIGS[name]
    a = cfg.voxels()
    b = synth(cfg.grid, cfg.p_region, cfg.p_cluster, cfg.p_voxel, cfg.seed)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert int(a[1].max()) < (1 << 24)


def test_synth_rejects_bad_grid():
    with pytest.raises(vr.VrError):
        vr.synth_scene(100, 1, 1, 1, 1)


def test_vox_roundtrip_and_parse_rules(tmp_path):
    xyz = np.array([[1, 2, 3], [-4, 5, -6], [70, 0, 130]], np.int32)
    rgb = np.array([0x123456, 0, 0xFFFFFF], np.uint32)
    p = str(tmp_path / "scene.vox")
    vr.write_voxel_file(p, xyz, rgb)
    a, b = vr.read_voxel_file(p)
    assert np.array_equal(a, xyz) and np.array_equal(b, rgb)
    # VoxelFile.cuh:11-35: empty fields skipped, short lines ignored, trailing junk after digits ignored
    q = str(tmp_path / "odd.vox")
    open(q, "w").write("1,2,3,4\r\n,,5,,6,7,8,\n9,9\n\n  10 , 11,12,13xyz\n-1,-2,-3,-4\n")
    a, b = vr.read_voxel_file(q)
    assert a.tolist() == [[1, 2, 3], [5, 6, 7], [10, 11, 12], [-1, -2, -3]]
    assert b.tolist() == [4, 8, 13, 0xFFFFFFFC]
    bad = str(tmp_path / "bad.vox")
    open(bad, "w").write("1,2,3,4\n1,x,3,4\n")
    with pytest.raises(vr.VrError) as e:
        vr.read_voxel_file(bad)
    assert e.value.code == -6
    with pytest.raises(vr.VrError) as e:
        vr.read_voxel_file(str(tmp_path / "missing.vox"))
    assert e.value.code == -4


def test_band_buffer_words():
    assert vr.band_buffer_words(1920, 1080, 8, 1) == 1920 * 1080
    assert vr.band_buffer_words(1920, 1080, 8, 8) == 17 * 8 * 1920     # 135 bands -> 17 per rank
    assert vr.band_buffer_words(10, 10, 8, 3) == 8 * 10
    assert vr.band_buffer_words(10, 10, 0, 3) == 0


def test_forget_orders_checks_device_index():
    # host bookkeeping only (no HIP call): valid indices succeed with or without a GPU
    vr.forget_orders(0)
    vr.forget_orders(63)
    for bad in (-1, 64):
        with pytest.raises(vr.VrError):
            vr.forget_orders(bad)


def test_assemble_bands_cpu():
    from voxelraymarcher_amd.tiles import assemble_bands, owned_rows
    W, H, B = 7, 29, 4
    img = torch.arange(W * H, dtype=torch.int32).reshape(H, W)
    for R in (1, 2, 3, 5, 8):
        words = vr.band_buffer_words(W, H, B, R)
        parts = torch.full((R, words), -1, dtype=torch.int32)
        for r in range(R):
            rows = owned_rows(H, B, r, R)
            buf = parts[r].view(-1, W)
            for i, y in enumerate(rows):
                buf[i] = img[y]
        assert torch.equal(assemble_bands(parts, W, H, B), img)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_device_calls_fail_loudly_without_gpu():
    with pytest.raises(vr.VrError) as e:
        vr.create_scene(np.zeros((1, 3), np.int32), np.zeros(1, np.uint32), vr.StorageType.VOXEL_CLUSTER_STORE)
    assert e.value.code == -2


def test_cli_binary_built():
    exe = os.path.join(ROOT, "voxelraymarcher_amd", "bin", "VoxelRaymarcher")
    assert os.access(exe, os.X_OK)
    out = os.popen(f"{exe} --help").read()
    assert "hashtable|vcs" in out
    for flag in ("--no-shadows", "--point-light", "--light-dir", "--light-color"):
        assert flag in out
    r = os.popen(f"{exe} --light-dir 1,2 2>&1; echo rc=$?").read()
    assert "needs X,Y,Z" in r and "rc=2" in r


def test_cli_converts_scene_to_vxb(tmp_path):
    exe = os.path.join(ROOT, "voxelraymarcher_amd", "bin", "VoxelRaymarcher")
    xyz, rgb = vr.CONFIGS["C1"].voxels()
    src, dst = str(tmp_path / "scene.vox"), str(tmp_path / "scene.vxb")
    vr.write_voxel_file(src, xyz, rgb)
    assert os.system(f"{exe} --scene {src} --write-vxb {dst} > /dev/null") == 0
    a, b = vr.read_voxel_file(dst)
    assert np.array_equal(a, xyz) and np.array_equal(b, rgb)


def test_binary_scene_roundtrip_and_detection(tmp_path):
    """.vxb sidecar: same voxels, same order, auto-detected."""
    rng = np.random.default_rng(7)
    xyz = rng.integers(-300, 300, size=(5000, 3)).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=5000).astype(np.uint32)
    xyz[17] = xyz[3]                        # a duplicate: order must survive
    p = str(tmp_path / "scene.vxb")
    vr.write_binary_scene(p, xyz, rgb)
    a, b = vr.read_voxel_file(p)
    assert np.array_equal(a, xyz) and np.array_equal(b, rgb)
    q = str(tmp_path / "empty.vxb")
    vr.write_binary_scene(q, np.zeros((0, 3), np.int32), np.zeros(0, np.uint32))
    a, b = vr.read_voxel_file(q)
    assert a.shape == (0, 3) and b.shape == (0,)
    bad = str(tmp_path / "trunc.vxb")
    open(bad, "wb").write(open(p, "rb").read()[:1000])
    with pytest.raises(vr.VrError) as e:
        vr.read_voxel_file(bad)
    assert e.value.code == -6


def test_parallel_csv_parse_matches_python(tmp_path):
    """A multi-MB .vox is split across threads: voxels in file order and the
    first error's line number exactly as a sequential reading gives them."""
    rng = np.random.default_rng(11)
    n = 400_000
    xyz = rng.integers(-2000, 2000, size=(n, 3)).astype(np.int32)
    rgb = rng.integers(0, 1 << 24, size=n).astype(np.uint32)
    lines = [f"{x},{y},{z},{c}" for (x, y, z), c in zip(xyz.tolist(), rgb.tolist())]
    # sprinkle ignorable lines and odd-but-valid forms at chunk-boundary-ish places
    for i in (0, 1, n // 7, n // 3, n // 2, n - 1):
        lines.insert(i, "")
    lines.insert(n // 5, "1,2")
    lines.insert(n // 4, ",,9,,8,,7,,6,")
    p = str(tmp_path / "big.vox")
    open(p, "w").write("\n".join(lines) + "\n")
    a, b = vr.read_voxel_file(p)
    want = [[int(t) for t in l.replace(",", " ").split()] for l in lines if len([t for t in l.split(",") if t]) > 3]
    assert a.shape[0] == len(want)
    assert np.array_equal(a, np.array([w[:3] for w in want], np.int32))
    assert np.array_equal(b, np.array([w[3] for w in want], np.uint32))
    bad_at = 300_000
    lines[bad_at] = "1,2,zz,4"
    open(p, "w").write("\n".join(lines) + "\n")
    with pytest.raises(vr.VrError) as e:
        vr.read_voxel_file(p)
    assert e.value.code == -6 and f":{bad_at + 1}:" in str(e.value)
