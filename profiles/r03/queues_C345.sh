# bench.py C3/C4/C5 (N = 1): hardware queues per process x frames in flight
set -o pipefail
O=gpurun_out/queues2; mkdir -p $O
for C in C3 C4; do
  for qd in 4:2 16:3 16:4; do
    q=${qd%:*}; d=${qd#*:}
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --config $C --frames-in-flight $d --no-cpu-baseline --steps 200 > $O/${C}_q${q}_d$d.json 2>>$O/err || exit 1
  done
done
for qd in 4:3 16:4 16:6 16:8 8:6; do
  q=${qd%:*}; d=${qd#*:}
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --config C5 --frames-in-flight $d --no-cpu-baseline --steps 100 > $O/C5_q${q}_d$d.json 2>>$O/err || exit 1
done
