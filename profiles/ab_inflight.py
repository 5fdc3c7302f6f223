#!/usr/bin/env python3
"""A/B of library builds (VR_LIBRARY) under profiles/inflight_probe.py: every
build in its own child process, rounds interleaved.
  python profiles/ab_inflight.py C2 K lib1.so lib2.so ... [--rounds R]"""
import os
import subprocess
import sys

args = sys.argv[1:]
rounds = 1
if "--rounds" in args:
    i = args.index("--rounds")
    rounds = int(args[i + 1])
    del args[i:i + 2]
cfg, K, libs = args[0], args[1], args[2:]
here = os.path.dirname(os.path.abspath(__file__))
for rnd in range(rounds):
    for lib in libs:
        env = dict(os.environ, VR_LIBRARY=os.path.abspath(lib))
        r = subprocess.run([sys.executable, os.path.join(here, "inflight_probe.py"), cfg, K], env=env,
                           capture_output=True, text=True, timeout=600)
        lines = [l for l in r.stdout.splitlines() if "streams=1" in l or "streams=2" in l or "digest" in l] or [r.stderr[-400:]]
        for l in lines:
            print(f"[{rnd}] {os.path.basename(lib)}: {l}", flush=True)
