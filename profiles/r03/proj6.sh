# bench.py's pipeline policy for C5 (8 frames in flight, GPU_MAX_HW_QUEUES raised to 16 inside bench.py)
set -o pipefail
O=gpurun_out/proj6; mkdir -p $O
timeout -k 10 150 python bench.py --config C5 --no-cpu-baseline --steps 100 > $O/bench_C5.json 2>>$O/err || exit 1
timeout -k 10 150 python bench.py --config C5 --no-cpu-baseline --steps 100 --frames-in-flight 3 > $O/bench_C5_d3.json 2>>$O/err || exit 1
