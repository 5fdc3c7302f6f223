#!/bin/bash
# Is a rank's loss of efficiency locality?  C5 over 8 ranks: the 2-D tile deal (16x16 blocks)
# vs contiguous strips (270-row bands: rank r renders rows 270r..270r+269, the most compact and
# the least balanced deal).  Efficiency = sum over ranks of their pipelined frame times / the
# one-GPU frame time (1.0 = no loss).
set -u
O=${1:-gpurun_out/r06deal}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u profiles/rank_projection.py --config C5 --world 8 --layout bands --band-rows 270 --latency-reps 5 > $O/strips.jsonl 2> $O/strips.err || { tail -5 $O/strips.err; exit 1; }
timeout -k 10 300 python -u profiles/rank_projection.py --config C5 --world 8 --layout tiles --tile-cols 64 --band-rows 64 --latency-reps 5 > $O/tiles64.jsonl 2> $O/tiles64.err || { tail -5 $O/tiles64.err; exit 1; }
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
for f in ["strips", "tiles64"]:
    rows = [json.loads(l) for l in open(f"{O}/{f}.jsonl")]
    ranks = [r for r in rows if "rank" in r]
    s = rows[-1]
    tot = sum(r["ms_per_frame"] for r in ranks)
    print(f, "per-rank", [r["ms_per_frame"] for r in ranks], "sum", round(tot, 4), "1gpu", s["one_gpu_ms_per_frame"], "eff", round(s["one_gpu_ms_per_frame"] / tot, 3), "speedup", s["projected_speedup"])
PY
