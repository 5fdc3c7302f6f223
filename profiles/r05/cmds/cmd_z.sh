#!/bin/bash
# C2 over 8 ranks (one GPU, ranks 1 and 2): row bands of 8 vs 16 rows (a 16x16 lane block
# then spans one band), and the 16x16 tile deal.
set -o pipefail
O=${1:-gpurun_out/r05z}
mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 600 "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; echo "$n: $(head -2 $O/$n.jsonl | tr '\n' ' ')"; tail -1 $O/$n.jsonl | cut -c1-300; }
run bands8 python profiles/rank_projection.py --config C2 --world 8 --ranks 1,2 --layout bands --band-rows 8
run bands16 python profiles/rank_projection.py --config C2 --world 8 --ranks 1,2 --layout bands --band-rows 16
run tiles16 python profiles/rank_projection.py --config C2 --world 8 --ranks 1,2 --layout tiles --band-rows 16
