#!/usr/bin/env python3
"""A/B timing of alternative libvr.so builds (tuning only): each build runs in a
child process (VR_LIBRARY selects the library) on the same config and box.
  python profiles/ab_probe.py C2 voxelraymarcher_amd/libvr.so /tmp/libvr_variant.so"""
import os
import subprocess
import sys

cfg = sys.argv[1]
for lib in sys.argv[2:]:
    env = dict(os.environ, VR_LIBRARY=os.path.abspath(lib))
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "profile_kernel.py"),
                        "--config", cfg, "--iters", "30", "--kernel", "tile"], env=env, capture_output=True, text=True,
                       timeout=300)
    print(f"{lib}: {r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]}", flush=True)
