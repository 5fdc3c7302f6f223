#!/usr/bin/env python3
"""Diagnostic: frames of C5 crawl rows rendered with 3 views in rotation, on 3 streams in
flight / on one stream, through render_ex / PreparedRender, each checked against a lone
render_ex of its view.  Prints the mismatching frame indices per variant."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import voxelraymarcher_amd as vr  # noqa: E402

cfg = vr.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C5"]
algo = cfg.algorithm
xyz, rgb = cfg.voxels()
scene = vr.create_scene(xyz, rgb, cfg.store)
W, H = cfg.width, cfg.height
r0, r1 = (688, 720) if cfg.name == "C5" else (0, H)
lit = vr.setup_constant_values()
info = vr.VoxelSceneInfo((0.0, 0.0, 0.0), cfg.scale)
cams = []
for k in (0, 1, 2):
    c = vr.Camera.reference(W, H)
    bits = np.array([c.raw.origin[0]], dtype=np.float32).view(np.uint32) + np.uint32(k)
    c.raw.origin[0] = float(bits.view(np.float32)[0])
    cams.append(c)
words = (r1 - r0) * W
refs = []
for c in cams:
    ref = torch.full((words,), -1, dtype=torch.int32, device="cuda")
    vr.render_ex(scene, algo, c, lit, info, W, H, ref, r0, r1)
    torch.cuda.synchronize()
    refs.append(ref)
print("refs differ between views:", [not torch.equal(refs[0], refs[i]) for i in (1, 2)], flush=True)
preps = [vr.PreparedRender(scene, algo, c, lit, info, W, H, row_begin=r0, row_end=r1) for c in cams]


def run(name, nviews, nstreams, use_prep, frames=30):
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    outs = [torch.full((words,), -1, dtype=torch.int32, device="cuda") for _ in range(frames)]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    for i in range(frames):
        v = i % nviews
        st = streams[i % nstreams]
        if use_prep:
            preps[v](outs[i], st)
        else:
            vr.render_ex(scene, algo, cams[v], lit, info, W, H, outs[i], r0, r1, stream=st)
    torch.cuda.synchronize()
    bad = [i for i in range(frames) if not torch.equal(outs[i], refs[i % nviews])]
    nz = [int((outs[i] != refs[i % nviews]).sum()) for i in bad[:4]]
    print(f"{name}: views {nviews} streams {nstreams} prep {use_prep}: bad {bad[:10]} ({len(bad)}) diff px {nz}",
          flush=True)


for nv in (1, 3):
    for ns in (1, 3):
        for up in (False, True):
            run("v", nv, ns, up)
