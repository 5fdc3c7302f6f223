set -o pipefail
O=gpurun_out/ab1; mkdir -p $O
VR_LIBRARY=$PWD/voxelraymarcher_amd/ab/libvr_la1.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests_la1.log 2>&1 &&
timeout -k 10 400 python profiles/ab_inflight.py C3 200 voxelraymarcher_amd/ab/libvr_base.so voxelraymarcher_amd/ab/libvr_la1.so voxelraymarcher_amd/ab/libvr_la1noeq.so --rounds 2 > $O/ab_C3.txt 2>&1
