#!/bin/bash
# C5: which kernels are running over a rank's pipelined frames vs the one-GPU frame's
# (profiles/r05/rank_trace_split.py "active kinds").
set -o pipefail
O=${1:-gpurun_out/r05t}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/tr_r1 -o run -- python3 profiles/r05/rank_trace.py --rank 1 > $O/tr_r1.log 2>&1 || { tail -5 $O/tr_r1.log; exit 1; }
python3 profiles/r05/rank_trace_split.py $(ls $O/tr_r1/*kernel_trace.csv | head -1) > $O/split_r1.txt || exit 1
echo "rank 1 of 8:"; cat $O/split_r1.txt
timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/tr_w1 -o run -- python3 profiles/r05/rank_trace.py --world 1 --rank 0 --steps 40 --lone 10 > $O/tr_w1.log 2>&1 || { tail -5 $O/tr_w1.log; exit 1; }
python3 profiles/r05/rank_trace_split.py $(ls $O/tr_w1/*kernel_trace.csv | head -1) 40 20 10 > $O/split_w1.txt || exit 1
echo "one GPU:"; cat $O/split_w1.txt
