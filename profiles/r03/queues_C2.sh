# bench.py C2 (N = 1): hardware queues per process (GPU_MAX_HW_QUEUES; box default 4) x frames in flight
set -o pipefail
O=gpurun_out/queues; mkdir -p $O
for q in 4 8 16; do
  for d in 2 3 4; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --config C2 --frames-in-flight $d --no-cpu-baseline --steps 200 > $O/C2_q${q}_d$d.json 2>>$O/err || exit 1
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --config C2 --frames-in-flight $d --no-cpu-baseline --steps 20 --warmup 5 > $O/C2_q${q}_d${d}_s20.json 2>>$O/err || exit 1
  done
done
