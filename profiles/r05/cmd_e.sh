#!/bin/bash
# A/B of issue priority for heavy waves (VR_PRIO_HEAD_DIV: the head of a heaviest-first
# order at s_setprio 3; VR_PRIO_ESC: raise priority after a long primary walk) on C2 and C5,
# then the C5 projection sweep (cmd_d).
set -o pipefail
O=${1:-gpurun_out/r05e}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
timeout -k 10 600 python profiles/r05/ab_bench.py C2 $L $L:VR_PRIO_HEAD_DIV=32 $L:VR_PRIO_HEAD_DIV=8 $L:VR_PRIO_ESC=64 $L:VR_PRIO_ESC=128 --rounds 2 > $O/ab_prio_C2.txt 2>&1 || { tail -5 $O/ab_prio_C2.txt; exit 1; }
cat $O/ab_prio_C2.txt
timeout -k 10 600 python profiles/r05/ab_bench.py C5 $L $L:VR_PRIO_HEAD_DIV=16 $L:VR_PRIO_ESC=256 --rounds 1 --steps 100 > $O/ab_prio_C5.txt 2>&1 || { tail -5 $O/ab_prio_C5.txt; exit 1; }
cat $O/ab_prio_C5.txt
bash profiles/r05/cmd_d.sh $O/d
