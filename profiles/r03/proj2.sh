set -o pipefail
O=gpurun_out/proj2; mkdir -p $O
for d in 3 4 6 8; do
  timeout -k 10 120 python -u profiles/rank_projection.py --config C5 --world 8 --ranks 0,2,7 --frames-in-flight $d > $O/C5_d$d.jsonl 2>>$O/err || exit 1
done
timeout -k 10 120 python -u profiles/rank_projection.py --config C2 --world 8 --ranks 1,0,0,2 > $O/C2_order.jsonl 2>>$O/err || exit 1
