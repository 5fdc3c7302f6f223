#!/bin/bash
# A/B of the XCD-aware grid order (VR_XCD_CHUNK tile-group columns per chunk; 0 = plain
# grid order): bench.py per config, kernel_ms_grid_order (one launch alone) and the
# pipelined per-frame time.   bash profiles/r04/ab_xcd.sh <out> [chunks...] -- [configs...]
set -o pipefail
O=$1; shift
CH=(); CF=()
seen=0
for a in "$@"; do if [ "$a" = "--" ]; then seen=1; elif [ $seen = 0 ]; then CH+=("$a"); else CF+=("$a"); fi; done
[ ${#CH[@]} -eq 0 ] && CH=(0 2 4 8)
[ ${#CF[@]} -eq 0 ] && CF=(C2 C3 C4 C5)
mkdir -p $O
for C in "${CF[@]}"; do
  for w in "${CH[@]}"; do
    VR_XCD_CHUNK=$w timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > $O/ab_${C}_w$w.json 2> $O/ab_${C}_w$w.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/ab_${C}_w$w.json').read().strip().splitlines()[-1]); print('$C', 'w=$w', 'grid_ms', d['kernel_ms_grid_order'], 'learned_ms', d['kernel_ms'], 'frame_ms', d['ms_per_step'])" | tee -a $O/ab_xcd.txt
  done
done
