#!/bin/bash
# perm_kernel as per-wave shuffle sort + merge rank: parity, A/B on C2/C4, kernel trace.
set -o pipefail
O=${1:-gpurun_out/r05l}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_slots.py tests/test_gpu_tiles_deal.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VR_ORDER_REFRESH=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_refresh1 -o run -- python3 bench.py --config C2 --no-cpu-baseline --steps 50 > $O/prof_refresh1.log 2>&1 || { tail -5 $O/prof_refresh1.log; exit 1; }
python3 -c "
import csv
for r in list(csv.reader(open('$O/prof_refresh1/run_kernel_stats.csv')))[:6]: print(r[0][:60], r[1:4])"
for C in C2 C4; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L:VR_LANE_ORDER=0 $L --rounds 2 > $O/ab_lane_$C.txt 2>&1 || { tail -5 $O/ab_lane_$C.txt; exit 1; }
  cat $O/ab_lane_$C.txt
done
