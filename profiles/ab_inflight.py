#!/usr/bin/env python3
"""A/B of library builds (VR_LIBRARY) under profiles/inflight_probe.py: every
build in its own child process, rounds interleaved.  A build may carry
environment settings: lib.so:VAR=VAL[,VAR=VAL...] (e.g. libvr.so:VR_CRAWL_STREAM=0).
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
    for spec in libs:
        lib, _, extra = spec.partition(":")
        env = dict(os.environ, VR_LIBRARY=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in extra.split(",") if kv)
        r = subprocess.run([sys.executable, os.path.join(here, "inflight_probe.py"), cfg, K], env=env,
                           capture_output=True, text=True, timeout=600)
        lines = [l for l in r.stdout.splitlines() if "streams=1" in l or "streams=2" in l or "digest" in l] or [r.stderr[-400:]]
        for l in lines:
            print(f"[{rnd}] {os.path.basename(lib)}{':' + extra if extra else ''}: {l}", flush=True)
