#!/bin/bash
# GPU suite (sparse existence test covered in both modes), then A/Bs: issue priority for heavy
# waves (VR_PRIO_HEAD_DIV / VR_PRIO_ESC), the sparse existence test (VR_SPARSE) on C5 and C2,
# then the C5 projection sweep (cmd_d).
set -o pipefail
O=${1:-gpurun_out/r05e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L=voxelraymarcher_amd/libvr.so
timeout -k 10 600 python profiles/r05/ab_bench.py C5 $L:VR_SPARSE=0 $L:VR_SPARSE=1 --rounds 2 --steps 100 > $O/ab_sparse_C5.txt 2>&1 || { tail -5 $O/ab_sparse_C5.txt; exit 1; }
cat $O/ab_sparse_C5.txt
timeout -k 10 600 python profiles/r05/ab_bench.py C2 $L $L:VR_SPARSE=1 $L:VR_PRIO_HEAD_DIV=32 $L:VR_PRIO_HEAD_DIV=8 $L:VR_PRIO_ESC=64 $L:VR_PRIO_ESC=128 --rounds 2 > $O/ab_prio_C2.txt 2>&1 || { tail -5 $O/ab_prio_C2.txt; exit 1; }
cat $O/ab_prio_C2.txt
bash profiles/r05/cmds/cmd_d.sh $O/d
