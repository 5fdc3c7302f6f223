#!/bin/bash
# C5 rank 1,2 of 8 (2-D tile deal): 16-row bands (a 16x16 lane block is one frame block)
# vs 8-row bands.
set -o pipefail
O=${1:-gpurun_out/r05v}
mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 600 "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; echo "$n: $(head -2 $O/$n.jsonl | tr '\n' ' ')"; tail -1 $O/$n.jsonl | cut -c1-330; }
run b16 python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2 --band-rows 16
run b8 python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2
VR_LANE_ORDER=0 run b16_nolane python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2 --band-rows 16
