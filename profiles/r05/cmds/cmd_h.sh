#!/bin/bash
# Learned per-pixel lane order (16x16 blocks, vr_march.hip lane_pixel): parity with it on
# (the default), then A/B against VR_LANE_ORDER=0 on the same library.
set -o pipefail
O=${1:-gpurun_out/r05h}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_slots.py tests/test_gpu_tiles_deal.py tests/test_gpu_occupancy.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in C2 C3 C4 C5; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L:VR_LANE_ORDER=0 $L --rounds 2 > $O/ab_lane_$C.txt 2>&1 || { tail -5 $O/ab_lane_$C.txt; exit 1; }
  cat $O/ab_lane_$C.txt
done
