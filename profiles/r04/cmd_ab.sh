# A/B call: the GPU suite on the new libvr.so, then ab_libs.sh base vs new
#   bash profiles/r04/cmd_ab.sh <out> <rounds> <configs>
set -o pipefail
O=$1; R=${2:-2}; CF=${3:-C2,C4,C3,C5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash profiles/r04/ab_libs.sh $O/ab $R $CF voxelraymarcher_amd/ab/libvr_base.so voxelraymarcher_amd/libvr.so
