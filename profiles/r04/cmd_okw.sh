set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash profiles/r04/ab_libs.sh $O/ab 2 C2,C4,C3,C5 voxelraymarcher_amd/ab/libvr_base.so voxelraymarcher_amd/libvr.so
