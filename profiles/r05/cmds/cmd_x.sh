#!/bin/bash
# C5 rank 1,2 of 8: deal block shapes around 16x16 (band rows x tile columns).
set -o pipefail
O=${1:-gpurun_out/r05x}
mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 600 "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; echo "$n: $(head -2 $O/$n.jsonl | tr '\n' ' ')"; }
run b32t16 python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2 --band-rows 32
run b16t32 python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2 --band-rows 16 --tile-cols 32
run b16t16 python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2 --band-rows 16
run b32t32 python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2 --band-rows 32 --tile-cols 32
