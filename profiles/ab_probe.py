#!/usr/bin/env python3
"""A/B timing of VR_EXPERIMENT variants (tuning only): each variant runs in a
child process (the env var is read per launch) on the same config.
  python profiles/ab_probe.py C2 0 1 [2 ...]
A variant "lib:<path>" runs that build of libvr.so instead (VR_LIBRARY)."""
import os
import subprocess
import sys

cfg = sys.argv[1]
for e in sys.argv[2:]:
    env = dict(os.environ, VR_LIBRARY=e[4:]) if e.startswith("lib:") else dict(os.environ, VR_EXPERIMENT=e)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "profile_kernel.py"),
                        "--config", cfg, "--iters", "30", "--kernel", "tile"], env=env, capture_output=True, text=True,
                       timeout=300)
    print(f"VR_EXPERIMENT={e}: {r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]}", flush=True)
