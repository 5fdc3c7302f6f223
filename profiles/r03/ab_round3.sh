# A/B of the round-2 library (voxelraymarcher_amd/ab/libvr_r02.so, built from commit 236bce1's
# csrc + include with `make ../libvr.so`) against the current one, two frames in flight and
# one alone (profiles/inflight_probe.py), then the GPU tests.
#   bash profiles/r03/ab_round3.sh <out dir>
set -o pipefail
O=${1:-gpurun_out/r03}
mkdir -p $O
L="voxelraymarcher_amd/ab/libvr_r02.so voxelraymarcher_amd/libvr.so"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python profiles/ab_inflight.py C2 400 $L --rounds 2 > $O/ab_C2.txt 2>&1 &&
timeout -k 10 300 python profiles/ab_inflight.py C3 200 $L --rounds 2 > $O/ab_C3.txt 2>&1 &&
timeout -k 10 300 python profiles/ab_inflight.py C4 400 $L --rounds 2 > $O/ab_C4.txt 2>&1 &&
timeout -k 10 300 python profiles/ab_inflight.py C5 100 $L --rounds 1 > $O/ab_C5.txt 2>&1
