#!/bin/bash
# Orders made once per slot and view (no periodic remake): parity, A/B against the remake
# every 16 uses (VR_ORDER_REFRESH=16) on C2-C5.
set -o pipefail
O=${1:-gpurun_out/r05r}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_slots.py tests/test_gpu_tiles_deal.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in C2 C3 C4 C5; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L:VR_ORDER_REFRESH=16 $L --rounds 2 > $O/ab_$C.txt 2>&1 || { tail -5 $O/ab_$C.txt; exit 1; }
  cat $O/ab_$C.txt
done
