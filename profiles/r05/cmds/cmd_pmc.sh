#!/bin/bash
# Round-5 PMC pass at HEAD (separate --pmc runs per counter group, profiles/r05/profile_round.sh):
# FETCH_SIZE / WRITE_SIZE / SQ / GRBM+TCC per config -> traffic.json (copied to profiles/traffic.json).
set -o pipefail
O=${1:-gpurun_out/r05pmc}
bash profiles/r05/profile_round.sh $O C2 C3 C4 C5 || exit 1
cat $O/traffic.json | head -c 3000
# the sign-specialised cuckoo loop (variant build): parity on every hash test, then A/B on C4
H=voxelraymarcher_amd/ab/libvr_hsign.so
VR_LIBRARY=$PWD/$H timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_occupancy.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_hsign.log 2>&1 || { tail -40 $O/tests_hsign.log; exit 1; }
tail -1 $O/tests_hsign.log
timeout -k 10 600 python profiles/r05/ab_bench.py C4 voxelraymarcher_amd/libvr.so $H --rounds 3 > $O/ab_hsign_C4.txt 2>&1 || { tail -5 $O/ab_hsign_C4.txt; exit 1; }
cat $O/ab_hsign_C4.txt
