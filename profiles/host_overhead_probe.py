import os, sys, time, json
sys.path.insert(0, "/root/repo")
import numpy as np, torch
import voxelraymarcher_amd as vr
from voxelraymarcher_amd.tiles import BandGather
cfg = vr.CONFIGS["C2"]; xyz, rgb = cfg.voxels(); scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = 1920, 1080; cam = vr.Camera.reference(W, H); lit = vr.setup_constant_values(); info = vr.VoxelSceneInfo((0,0,0), cfg.scale)
pipe = BandGather(W, H, 8, 0, 1, torch.device("cuda", 0), depth=2)
def render(buf): vr.render_bands(scene, cfg.algorithm, cam, lit, info, W, H, 8, 0, 1, buf)
for _ in range(50): pipe.step(render)
pipe.drain(); torch.cuda.synchronize()
# host cost of one render_bands call and one pipe.step, GPU kept busy
ts = []
for _ in range(200):
    t = time.perf_counter(); render(pipe.bufs[0]); ts.append(time.perf_counter() - t)
torch.cuda.synchronize()
ts2 = []
for _ in range(200):
    t = time.perf_counter(); pipe.step(render); ts2.append(time.perf_counter() - t)
pipe.drain(); torch.cuda.synchronize()
print(json.dumps({"render_bands_us_median": np.median(ts)*1e6, "pipe_step_us_median": np.median(ts2)*1e6,
                  "render_bands_us_p90": np.percentile(ts, 90)*1e6, "pipe_step_us_p90": np.percentile(ts2, 90)*1e6}))
