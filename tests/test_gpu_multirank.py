"""The N > 1 frame path of bench.py, executed with real renders on the one GPU a test box
has.  RCCL refuses two ranks on one device, so 2 and 3 ranks share cuda:0
through a gloo group whose gather is staged through host memory
(tiles.init_frame_group / BandGather(stage_host=True)); everything else is the code path
the driver's multi-GPU run takes: bench.py under torch.distributed.run, vr_render_bands of
each rank's interleaved 8-row bands, the RGB8 pack (writeColorToFramebuffer,
Renderer.cuh:1024-1031), the gather, rank 0's assembly on its side stream, the
single-frame latency loop and the MAX-over-ranks timing.  Rank 0's last assembled RGB8
frame must equal the oracle's frame packed to RGB8, byte for byte."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_rgb8(cfg_name: str, W: int, H: int) -> np.ndarray:
    import oracle
    import voxelraymarcher_amd as vr
    cfg = vr.CONFIGS[cfg_name]
    xyz, rgb = cfg.voxels()
    ref = oracle.Scene(xyz, rgb, int(cfg.store))
    try:
        words, _ = ref.render(int(cfg.algorithm), oracle.reference_camera(W, H), oracle.lighting(), W, H, cfg.scale)
    finally:
        ref.close()
    w = np.asarray(words, dtype=np.uint32).reshape(H, W)
    return np.stack([(w >> 16) & 0xFF, (w >> 8) & 0xFF, w & 0xFF], axis=-1).astype(np.uint8)


def _run_bench(world, extra, tmp_path, W=480, H=270):
    dump = tmp_path / "frame.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "4", "--warmup", "2", "--config", "C2", "--tiling", "fixed",
           "--resolution", f"{W}x{H}", "--no-cpu-baseline", "--dump-frame", str(dump)] + extra
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, f"bench.py over {world} ranks failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), np.load(dump)


@pytest.mark.parametrize("layout", ["tiles", "strips"])
def test_rccl_gather_one_rank(tmp_path, layout):
    """The RCCL branch of the N > 1 path on a one-GPU box (RCCL refuses two ranks on one
    device): bench.py --exchange --backend nccl starts a one-rank nccl process group
    (init_process_group("nccl", device_id=...), tiles.init_frame_group), renders the 2-D tile
    layout (or the learned strips, fixed tiling's default since round 6: calibrated, then one
    strip), packs RGB8, gathers it with dist.gather on the slot stream over RCCL, and rank 0
    assembles it (vr_assemble_tiles / the strip copies) on its side stream; the frame equals
    the oracle's, byte for byte."""
    W, H = 480, 270
    line, got = _run_bench(1, ["--exchange", "--backend", "nccl", "--layout", layout], tmp_path, W, H)
    assert line["n_gpus"] == 1 and "RCCL gather" in line["config"]["parallelism"]
    assert line["config"]["layout"] == layout and line["dispatch_phases"]["latency"] == 5
    want = _oracle_rgb8("C2", W, H)
    assert got.shape == (H, W, 3) and got.dtype == np.uint8
    bad = int(np.count_nonzero(np.any(got != want, axis=-1)))
    assert bad == 0, f"{bad} of {W * H} pixels of the RCCL-gathered RGB8 frame differ from the oracle"


@pytest.mark.parametrize("world,layout", [(2, "tiles"), (3, "tiles"), (2, "bands"), (2, "strips"), (3, "strips")])
def test_bench_frame_path_ranks_share_one_gpu(world, layout, tmp_path):
    W, H = 480, 270
    dump = tmp_path / "frame.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "4", "--warmup", "2", "--config", "C2", "--tiling", "fixed",
           "--resolution", f"{W}x{H}", "--backend", "gloo", "--same-device", "--no-cpu-baseline",
           "--layout", layout, "--dump-frame", str(dump)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, f"bench.py over {world} ranks failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["scaling"] == "strong"
    assert (line["config"]["width"], line["config"]["height"]) == (W, H)
    assert line["frame_latency_ms"] > 0 and line["ms_per_step"] > 0 and line["value"] > 0
    assert "gloo" in line["config"]["parallelism"] and line["config"]["layout"] == layout
    assert line["dispatch_phases"]["latency"] == 5
    if layout == "strips":                   # learned: calibrated, re-cut, every row dealt once
        b = line["config"]["strip_bounds"]
        assert len(b) == world + 1 and b[0] == 0 and b[-1] == H and all(b[i] < b[i + 1] for i in range(world))
        assert len(line["config"]["strip_calibration"]) >= 1
        # the second, latency-balanced cut (round 6): its own strips, its one-frame latency, and
        # its last assembled frame equal to the oracle's too
        lb = line["config"]["latency_strip_bounds"]
        assert len(lb) == world + 1 and lb[0] == 0 and lb[-1] == H and all(lb[i] < lb[i + 1] for i in range(world))
        assert line["frame_latency_ms_latency_cut"] > 0 and len(line["config"]["latency_calibration"]) >= 1
        got_l = np.load(str(dump).replace(".npy", ".latency_cut.npy"))
        assert np.array_equal(got_l, _oracle_rgb8("C2", W, H)), "latency-cut frame differs from the oracle"
    # the frame's algorithmic bytes are the sum over the ranks' bands (all-reduced)
    assert line["roofline"]["algorithmic_bytes_per_frame"] > line["roofline"]["algorithmic_bytes_per_launch"]
    got = np.load(dump)
    want = _oracle_rgb8("C2", W, H)
    assert got.shape == (H, W, 3) and got.dtype == np.uint8
    bad = int(np.count_nonzero(np.any(got != want, axis=-1)))
    assert bad == 0, f"{bad} of {W * H} pixels of the {world}-rank RGB8 frame differ from the oracle"
