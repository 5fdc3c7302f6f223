#!/bin/bash
# A/B of library builds on one box: bench.py per config per library, alternated R rounds.
#   bash profiles/r04/ab_libs.sh <out> <rounds> <configs (comma)> <lib> [lib ...]
set -o pipefail
O=$1; R=$2; CF=$3; shift 3
mkdir -p $O
for r in $(seq 1 $R); do
  for C in ${CF//,/ }; do
    for L in "$@"; do
      n=$(basename $L .so)
      VR_LIBRARY=$L timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > $O/${C}_${n}_$r.json 2> $O/${C}_${n}_$r.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/${C}_${n}_$r.json').read().strip().splitlines()[-1]); print('$C', '$n', 'round $r', 'grid_ms', d['kernel_ms_grid_order'], 'learned_ms', d['kernel_ms'], 'frame_ms', d['ms_per_step'])" | tee -a $O/ab.txt
    done
  done
done
