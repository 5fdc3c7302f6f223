#!/usr/bin/env python3
"""A/B timing of alternative libvr.so builds (tuning only): each build runs in a
child process (VR_LIBRARY selects the library) on the same config and box.
  python profiles/ab_probe.py C2[,C3,...] voxelraymarcher_amd/libvr.so /tmp/libvr_variant.so [--rounds R]
Rounds interleave the builds (A B A B ...) so clock drift hits every build alike;
the digest is a position-weighted checksum of the frame (equal digests = same pixels)."""
import os
import subprocess
import sys

args = sys.argv[1:]
rounds = 1
if "--rounds" in args:
    i = args.index("--rounds")
    rounds = int(args[i + 1])
    del args[i:i + 2]
cfgs, libs = args[0].split(","), args[1:]
for rnd in range(rounds):
    for cfg in cfgs:
        for lib in libs:
            env = dict(os.environ, VR_LIBRARY=os.path.abspath(lib))
            r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "profile_kernel.py"),
                                "--config", cfg, "--iters", "30", "--kernel", "tile"], env=env, capture_output=True,
                               text=True, timeout=300)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
            print(f"[{rnd}] {os.path.basename(lib)}: {line}", flush=True)
