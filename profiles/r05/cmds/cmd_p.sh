#!/bin/bash
# 8-rank C5 projection (2-D tile deal) with the lane order.
set -o pipefail
O=${1:-gpurun_out/r05p}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python profiles/rank_projection.py --config C5 --world 8 > $O/proj_C5_w8_lane.jsonl 2> $O/proj.err || { tail -20 $O/proj.err; exit 1; }
tail -1 $O/proj_C5_w8_lane.jsonl
