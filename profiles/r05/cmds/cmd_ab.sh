#!/bin/bash
# Heaviest-first work order with frames in flight (VR_INFLIGHT_HEAVY=1) vs grid order (AUTO's
# choice), now that the lane order is on.
set -o pipefail
O=${1:-gpurun_out/r05ab}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
for C in C2 C3 C4 C5; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L $L:VR_INFLIGHT_HEAVY=1 --rounds 2 > $O/ab_$C.txt 2>&1 || { tail -5 $O/ab_$C.txt; exit 1; }
  cat $O/ab_$C.txt
done
