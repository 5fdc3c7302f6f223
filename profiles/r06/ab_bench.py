#!/usr/bin/env python3
"""A/B of library builds through bench.py itself: every build in its own child process
(VR_LIBRARY), rounds interleaved (A B A B ...), one summary line per run:
ms_per_step (pipelined), kernel_ms (learned order), kernel_ms_grid_order, frac.
  python profiles/r05/ab_bench.py C4 lib1.so[:VAR=VAL,...] lib2.so ... [--rounds R] [--steps N]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
args = sys.argv[1:]
opts = {"--rounds": "2", "--steps": "200"}
for k in list(opts):
    if k in args:
        i = args.index(k)
        opts[k] = args[i + 1]
        del args[i:i + 2]
cfg, libs = args[0], args[1:]
for rnd in range(int(opts["--rounds"])):
    for spec in libs:
        lib, _, extra = spec.partition(":")
        env = dict(os.environ, VR_LIBRARY=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in extra.split(",") if kv)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--no-cpu-baseline",
                            "--steps", opts["--steps"]], env=env, capture_output=True, text=True, timeout=600)
        js = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if not js:
            print(f"[{rnd}] {os.path.basename(lib)}: FAILED {r.stderr[-400:]}", flush=True)
            continue
        d = json.loads(js[-1])
        ro = d["roofline"]
        print(f"[{rnd}] {os.path.basename(lib)}{':' + extra if extra else ''}: {cfg} ms/step {d['ms_per_step']:.4f} "
              f"kernel_ms {d['kernel_ms']:.4f} grid {d['kernel_ms_grid_order']:.4f} "
              f"first {d.get('kernel_ms_first_render', 0):.4f} frac {ro['frac']:.3f} "
              f"learned {ro['frac_learned_order']:.3f} bytes {ro['algorithmic_bytes_per_launch']}", flush=True)
