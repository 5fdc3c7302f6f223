#!/bin/bash
# Lane-order blocks of 16x16 (default build) vs 32x32 (VR_LANE_BLOCK=32 variant): parity for
# both, A/B on C2-C5, perm_kernel duration of the 32x32 build.
set -o pipefail
O=${1:-gpurun_out/r05n}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
P=voxelraymarcher_amd/ab/libvr_lane32.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_tiles_deal.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests16.log 2>&1 || { tail -40 $O/tests16.log; exit 1; }
tail -1 $O/tests16.log
VR_LIBRARY=$PWD/$P timeout -k 10 600 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_tiles_deal.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests32.log 2>&1 || { tail -40 $O/tests32.log; exit 1; }
tail -1 $O/tests32.log
for C in C2 C3 C4 C5; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L $P --rounds 2 > $O/ab_block_$C.txt 2>&1 || { tail -5 $O/ab_block_$C.txt; exit 1; }
  cat $O/ab_block_$C.txt
done
VR_LIBRARY=$PWD/$P VR_ORDER_REFRESH=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof32 -o run -- python3 bench.py --config C2 --no-cpu-baseline --steps 50 > $O/prof32.log 2>&1 || { tail -5 $O/prof32.log; exit 1; }
python3 -c "
import csv
for r in list(csv.reader(open('$O/prof32/run_kernel_stats.csv')))[:6]: print(r[0][:60], r[1:4])"
