#!/bin/bash
# Lane order: why is the lone heaviest-first launch slower?  Order refresh every launch, no
# work order, vs the default.
set -o pipefail
O=${1:-gpurun_out/r05i}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
for C in C2 C3; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L $L:VR_ORDER_REFRESH=1 $L:VR_ORDER=0 $L:VR_ORDER_REFRESH=1,VR_LANE_ORDER=0 --rounds 1 > $O/ab_lane_order_$C.txt 2>&1 || { tail -5 $O/ab_lane_order_$C.txt; exit 1; }
  cat $O/ab_lane_order_$C.txt
done
