#!/bin/bash
# C5 8-rank projection: tile-deal block width sweep (16/32/64/128 columns), 1 crawl record
# per wave, 12 frames in flight; one-GPU and rank-0 kernel traces.
set -o pipefail
O=${1:-gpurun_out/r05d}
mkdir -p $O
export TMPDIR=/tmp
for T in 32 64 128; do
  timeout -k 10 400 python profiles/rank_projection.py --config C5 --world 8 --tile-cols $T --latency-reps 15 > $O/proj_T$T.jsonl 2> $O/proj_T$T.err || { tail -5 $O/proj_T$T.err; exit 1; }
  echo "T$T: $(tail -1 $O/proj_T$T.jsonl | head -c 600)"
done
VR_CRAWL_RPW=1 timeout -k 10 400 python profiles/rank_projection.py --config C5 --world 8 --latency-reps 15 > $O/proj_rpw1.jsonl 2> $O/proj_rpw1.err || { tail -5 $O/proj_rpw1.err; exit 1; }
echo "rpw1: $(tail -1 $O/proj_rpw1.jsonl | head -c 600)"
timeout -k 10 400 python profiles/rank_projection.py --config C5 --world 8 --frames-in-flight 12 --latency-reps 15 > $O/proj_d12.jsonl 2> $O/proj_d12.err || { tail -5 $O/proj_d12.err; exit 1; }
echo "depth12: $(tail -1 $O/proj_d12.jsonl | head -c 600)"
timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/tr_w1 -o run -- python3 profiles/r05/rank_trace.py --world 1 --rank 0 --steps 40 --lone 10 > $O/tr_w1.log 2>&1 || { tail -5 $O/tr_w1.log; exit 1; }
python3 profiles/r05/rank_trace_split.py $O/tr_w1/run_kernel_trace.csv 40 20 10 > $O/split_w1.txt || exit 1
echo "one GPU:"; cat $O/split_w1.txt
