# bench.py's own pipeline policy (tiles.pipeline_depth / pipeline_hw_queues, set inside bench.py)
# for C5 and the driver's C2 line, then the fixed-tiling C5 projection over 2/4/8 ranks under it
set -o pipefail
O=gpurun_out/proj5; mkdir -p $O
timeout -k 10 150 python bench.py --config C5 --no-cpu-baseline --steps 100 > $O/bench_C5.json 2>>$O/err || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.json 2>>$O/err || exit 1
for w in 2 4 8; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 150 python -u profiles/rank_projection.py --config C5 --world $w --frames-in-flight 8 > $O/C5_w${w}_q16_d8.jsonl 2>>$O/err || exit 1
done
