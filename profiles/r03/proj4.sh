# Fixed-tiled C5 over 8 ranks, projected (profiles/rank_projection.py): frames in flight
# 3..8 with 4 (the box default) and 8 / 16 hardware queues per process
set -o pipefail
O=gpurun_out/proj4; mkdir -p $O
for q in 8 16; do
  for d in 4 6 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python -u profiles/rank_projection.py --config C5 --world 8 --ranks 0,2,7 --frames-in-flight $d > $O/C5_w8_q${q}_d$d.jsonl 2>>$O/err || exit 1
  done
done
