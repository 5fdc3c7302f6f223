#!/bin/bash
# Round-6 PMC profile of every config's tile pass (profiles/r06/profile_round.sh -> traffic.json,
# with the library build it ran) and the 8-rank C5 projection (profiles/rank_projection.py).
set -u
O=${1:-gpurun_out/r06pmc}
mkdir -p $O
export TMPDIR=/tmp
bash profiles/r06/profile_round.sh $O C2 C3 C4 C5 || exit 1
timeout -k 10 300 python -u profiles/rank_projection.py --config C5 --world 8 > $O/proj_C5_w8.jsonl 2> $O/proj.err || { tail -5 $O/proj.err; exit 1; }
tail -2 $O/proj_C5_w8.jsonl
