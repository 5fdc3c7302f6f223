"""Frame output on the GPU: device RGB8 pack, the
pipelined FrameWriter, and the CLI end to end (scene file -> output.png with
the lighting flags), all checked pixel-for-pixel against the oracle."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

import oracle
from tests.helpers import oracle_camera_from, oracle_lighting_from
from tests.test_png import decode_png

pytestmark = pytest.mark.gpu

vr = pytest.importorskip("voxelraymarcher_amd")
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "voxelraymarcher_amd", "bin", "VoxelRaymarcher")


def words_to_rgb(words: np.ndarray, W: int, H: int) -> np.ndarray:
    w = words.astype(np.uint32).reshape(H, W)
    return np.stack([(w >> 16) & 0xFF, (w >> 8) & 0xFF, w & 0xFF], -1).astype(np.uint8)


def test_pack_rgb8_matches_numpy():
    rng = np.random.default_rng(3)
    words = rng.integers(0, 1 << 32, size=1920 * 1080 + 7, dtype=np.uint64).astype(np.uint32)
    got = vr.pack_rgb8(torch.from_numpy(words.view(np.int32)).cuda()).cpu().numpy()
    assert np.array_equal(got.reshape(-1, 3), words_to_rgb(words, words.size, 1).reshape(-1, 3))


def test_frame_writer_pipeline(tmp_path):
    cfg = vr.CONFIGS["C1"]
    xyz, rgb = cfg.voxels()
    W, H = 160, 120
    scene = vr.create_scene(xyz, rgb, vr.StorageType.HASH_TABLE)
    ref = oracle.Scene(xyz, rgb, int(vr.StorageType.HASH_TABLE))
    lit = vr.setup_constant_values()
    info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
    words = torch.empty(W * H, dtype=torch.int32, device="cuda")   # one buffer, reused every frame
    eyes = [(6.0 + 0.5 * k, 2.0 + 0.25 * k, 6.0 - 0.3 * k) for k in range(6)]
    with vr.FrameWriter(W, H, depth=2) as fw:
        for k, eye in enumerate(eyes):
            cam = vr.Camera(eye, (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 60.0, W / H)
            vr.run_raymarching_kernel(scene, vr.RayMarchAlgorithm.ORIGINAL, cam, lit, info, W, H, out=words)
            fw.submit(words, str(tmp_path / f"f{k}.png"))
    assert fw.written == [str(tmp_path / f"f{k}.png") for k in range(len(eyes))]
    for k, eye in enumerate(eyes):
        cam = vr.Camera(eye, (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 60.0, W / H)
        want, _ = ref.render(int(vr.RayMarchAlgorithm.ORIGINAL), oracle_camera_from(cam), oracle_lighting_from(lit),
                             W, H, cfg.scale)
        got = decode_png(open(tmp_path / f"f{k}.png", "rb").read())
        assert np.array_equal(got, words_to_rgb(want, W, H)), f"frame {k}"


@pytest.mark.parametrize("store,algo,flags,lit_kw", [
    ("hashtable", "original", [], {}),
    ("vcs", "longestaxis", [], {}),
    ("vcs", "original", ["--no-shadows", "--point-light", "40,90,30"],
     dict(use_shadows=False, use_point_light=True, light_position=(40.0, 90.0, 30.0))),
    ("hashtable", "longestaxis", ["--light-dir", "1,1,0", "--light-color", "0.5,1,0.25"],
     dict(light_direction=(1.0, 1.0, 0.0), light_color=(0.5, 1.0, 0.25))),
])
def test_cli_end_to_end(tmp_path, store, algo, flags, lit_kw):
    """Main.cu:176-229: scale, storage and algorithm arguments, scene file in,
    output.png out; the PNG's pixels equal the oracle's frame."""
    cfg = vr.CONFIGS["C1"]
    xyz, rgb = cfg.voxels()
    scene_path = str(tmp_path / "scene.vox")
    vr.write_voxel_file(scene_path, xyz, rgb)
    W, H = 200, 150
    out = str(tmp_path / "output.png")
    r = subprocess.run([EXE, str(cfg.scale), store, algo, "--scene", scene_path, "--width", str(W), "--height", str(H),
                        "--out", out] + flags, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Execution Time for Ray Marching Algorithm is" in r.stdout
    lit = vr.setup_constant_values(**lit_kw)
    st = vr.parse_storage(store)
    want, _ = oracle.Scene(xyz, rgb, int(st)).render(int(vr.parse_algorithm(algo)),
                                                    oracle_camera_from(vr.Camera.reference(W, H)),
                                                    oracle_lighting_from(lit), W, H, cfg.scale)
    got = decode_png(open(out, "rb").read())
    assert np.array_equal(got, words_to_rgb(want, W, H))


@pytest.mark.parametrize("store,algo", [("vcs", "original"), ("hashtable", "longestaxis")])
def test_cli_gpus_rccl_path(tmp_path, store, algo):
    """`VoxelRaymarcher ... --gpus 1`: the native multi-GPU host (csrc/cli/multi_gpu.cpp) --
    the 2-D tile deal per device, RGB8 pack, ncclCommInitAll + ncclGather to device 0, the
    assembly kernel -- with one rank on this one-GPU box; the PNG equals the oracle's frame."""
    cfg = vr.CONFIGS["C1"]
    xyz, rgb = cfg.voxels()
    scene_path = str(tmp_path / "scene.vox")
    vr.write_voxel_file(scene_path, xyz, rgb)
    W, H = 232, 150                        # not a multiple of the 16-pixel tiles: edge blocks
    out = str(tmp_path / "output.png")
    r = subprocess.run([EXE, str(cfg.scale), store, algo, "--scene", scene_path, "--width", str(W), "--height", str(H),
                        "--out", out, "--gpus", "1", "--repeat", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "on 1 GPU(s), tiled + RCCL gather" in r.stdout, r.stdout
    lit = vr.setup_constant_values()
    want, _ = oracle.Scene(xyz, rgb, int(vr.parse_storage(store))).render(
        int(vr.parse_algorithm(algo)), oracle_camera_from(vr.Camera.reference(W, H)), oracle_lighting_from(lit), W, H,
        cfg.scale)
    got = decode_png(open(out, "rb").read())
    assert np.array_equal(got, words_to_rgb(want, W, H))


def test_cli_gpus_more_than_visible(tmp_path):
    """--gpus N above the visible device count is refused before any work (exit 2)."""
    n = torch.cuda.device_count()
    r = subprocess.run([EXE, "1", "vcs", "original", "--synth", "64", "--width", "64", "--height", "64",
                        "--out", str(tmp_path / "o.png"), "--gpus", str(n + 1)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert f"--gpus {n + 1}" in r.stderr and "visible" in r.stderr
    assert not os.path.exists(tmp_path / "o.png")
