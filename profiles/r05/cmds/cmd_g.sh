#!/bin/bash
# Predicted all-skip planes (VR_UNIFORM_SKIP=2 build, voxelraymarcher_amd/ab/libvr_pskip.so):
# parity against it, then A/B against the current library.
set -o pipefail
O=${1:-gpurun_out/r05g}
mkdir -p $O
export TMPDIR=/tmp
P=voxelraymarcher_amd/ab/libvr_pskip.so
L=voxelraymarcher_amd/libvr.so
VR_LIBRARY=$PWD/$P timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_occupancy.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_pskip.log 2>&1 || { tail -40 $O/tests_pskip.log; exit 1; }
tail -1 $O/tests_pskip.log
for C in C5 C2 C3; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L $P --rounds 2 > $O/ab_pskip_$C.txt 2>&1 || { tail -5 $O/ab_pskip_$C.txt; exit 1; }
  cat $O/ab_pskip_$C.txt
done
