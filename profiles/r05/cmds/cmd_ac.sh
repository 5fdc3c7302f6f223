#!/bin/bash
# Primary-ray reciprocals in LDS for the VCS tile pass (the library) vs made per region walk
# (VR_LDS_RCP=0 build): parity on the library, A/B on C2, C5, C3.
set -o pipefail
O=${1:-gpurun_out/r05ac}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
B=voxelraymarcher_amd/ab/libvr_nolds.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_order.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in C2 C5 C3; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $B $L --rounds 2 > $O/ab_$C.txt 2>&1 || { tail -5 $O/ab_$C.txt; exit 1; }
  cat $O/ab_$C.txt
done
