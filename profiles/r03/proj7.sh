# Fixed-tiled C5 over 8 ranks (projection): band height 8 / 4 / 2 rows (crawl rows 680-719 spread
# over 5 ranks at 8, all 8 below), 8 frames in flight, 16 hardware queues
set -o pipefail
O=gpurun_out/proj7; mkdir -p $O
for b in 8 4 2; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 150 python -u profiles/rank_projection.py --config C5 --world 8 --frames-in-flight 8 --band-rows $b > $O/C5_w8_b$b.jsonl 2>>$O/err || exit 1
done
