#!/bin/bash
# Lane order, rank-count perm_kernel: parity (order, parity, fuzz, slots, tiles, occupancy,
# multirank), A/B vs VR_LANE_ORDER=0 on C2-C5, and a kernel trace with both orders remade
# every launch (perm_kernel's duration).
set -o pipefail
O=${1:-gpurun_out/r05k}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_slots.py tests/test_gpu_tiles_deal.py tests/test_gpu_occupancy.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in C2 C3 C4 C5; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L:VR_LANE_ORDER=0 $L --rounds 2 > $O/ab_lane_$C.txt 2>&1 || { tail -5 $O/ab_lane_$C.txt; exit 1; }
  cat $O/ab_lane_$C.txt
done
VR_ORDER_REFRESH=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_refresh1 -o run -- python3 bench.py --config C2 --no-cpu-baseline --steps 50 > $O/prof_refresh1.log 2>&1 || { tail -5 $O/prof_refresh1.log; exit 1; }
find $O/prof_refresh1 -name '*kernel_stats.csv' -exec head -6 {} \; | cut -c1-60,190-260
