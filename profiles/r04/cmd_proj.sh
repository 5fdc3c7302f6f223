# fixed-tiling C5 projection over N ranks from one GPU, pipelined and single-frame latency
set -o pipefail
O=${1:-gpurun_out/r04proj}
mkdir -p $O
for N in 2 4 8; do
  timeout -k 10 400 python profiles/rank_projection.py --config C5 --world $N > $O/proj_C5_w$N.jsonl 2> $O/proj_C5_w$N.err || { tail -5 $O/proj_C5_w$N.err; exit 1; }
  tail -1 $O/proj_C5_w$N.jsonl
done
