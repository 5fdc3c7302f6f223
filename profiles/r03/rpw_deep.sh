# Crawl records per wave (VR_CRAWL_RPW 4 in-tree, 8, 16 A/B builds) with C5's deep pipeline:
# bench.py C5 (8 frames in flight, 16 queues) and the 8-rank projection's crawl-row ranks
set -o pipefail
O=gpurun_out/rpw_deep; mkdir -p $O
for L in voxelraymarcher_amd/libvr.so voxelraymarcher_amd/ab/libvr_rpw8.so voxelraymarcher_amd/ab/libvr_rpw16.so; do
  n=$(basename $L .so)
  VR_LIBRARY=$PWD/$L timeout -k 10 150 python bench.py --config C5 --no-cpu-baseline --steps 100 > $O/bench_C5_$n.json 2>>$O/err || exit 1
  VR_LIBRARY=$PWD/$L GPU_MAX_HW_QUEUES=16 timeout -k 10 150 python -u profiles/rank_projection.py --config C5 --world 8 --ranks 0,7,2 --frames-in-flight 8 > $O/proj_$n.jsonl 2>>$O/err || exit 1
done
