#!/bin/bash
# Where a C5 rank's frame goes (2-D tile deal): kernel traces of one rank's pipelined and
# lone frames (profiles/r05/rank_trace.py), the one-GPU frame for comparison, and the
# 8-rank projection with 1 crawl record per wave and with 12 frames in flight.
set -o pipefail
O=${1:-gpurun_out/r05b}
mkdir -p $O
export TMPDIR=/tmp
for R in 1 0; do
  timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/tr_r$R -o run -- python3 profiles/r05/rank_trace.py --rank $R > $O/tr_r$R.log 2>&1 || { tail -5 $O/tr_r$R.log; exit 1; }
  python3 profiles/r05/rank_trace_split.py $(ls $O/tr_r$R/*kernel_trace.csv | head -1) > $O/split_r$R.txt || exit 1
  echo "rank $R of 8:"; cat $O/split_r$R.txt
done
timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/tr_w1 -o run -- python3 profiles/r05/rank_trace.py --world 1 --rank 0 --steps 40 --lone 10 > $O/tr_w1.log 2>&1 || { tail -5 $O/tr_w1.log; exit 1; }
python3 profiles/r05/rank_trace_split.py $(ls $O/tr_w1/*kernel_trace.csv | head -1) 40 20 10 > $O/split_w1.txt || exit 1
echo "one GPU:"; cat $O/split_w1.txt
VR_CRAWL_RPW=1 timeout -k 10 500 python profiles/rank_projection.py --config C5 --world 8 > $O/proj_rpw1.jsonl 2> $O/proj_rpw1.err || { tail -5 $O/proj_rpw1.err; exit 1; }
echo "rpw1: $(tail -1 $O/proj_rpw1.jsonl)"
timeout -k 10 500 python profiles/rank_projection.py --config C5 --world 8 --frames-in-flight 12 > $O/proj_d12.jsonl 2> $O/proj_d12.err || { tail -5 $O/proj_d12.err; exit 1; }
echo "depth12: $(tail -1 $O/proj_d12.jsonl)"
