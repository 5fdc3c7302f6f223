#!/bin/bash
# Where does a C5 rank's per-frame time go?  Rank 1 of 8 (pipelined + lone), tile deal vs
# row bands, lane order on/off.
set -o pipefail
O=${1:-gpurun_out/r05s}
mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 600 "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; echo "$n: $(head -1 $O/$n.jsonl)"; tail -1 $O/$n.jsonl | cut -c1-400; }
run tiles python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2
run bands python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2 --layout bands
VR_LANE_ORDER=0 run tiles_nolane python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2
