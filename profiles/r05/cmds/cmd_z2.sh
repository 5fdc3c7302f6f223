#!/bin/bash
# C2 weak scaling at 8 ranks (5431x3055-ish frame, row bands), ranks 1 and 2 on one GPU:
# 8- vs 16-row bands (the driver's SCALE run is this configuration).
set -o pipefail
O=${1:-gpurun_out/r05z2}
mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 600 "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; echo "$n: $(head -2 $O/$n.jsonl | tr '\n' ' ')"; tail -1 $O/$n.jsonl | cut -c1-420; }
run weak_b8 python profiles/rank_projection.py --config C2 --world 8 --ranks 1,2 --layout bands --band-rows 8 --tiling weak
run weak_b16 python profiles/rank_projection.py --config C2 --world 8 --ranks 1,2 --layout bands --band-rows 16 --tiling weak
