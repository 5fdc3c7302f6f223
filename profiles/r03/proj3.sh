# Projected fixed-tiling frame time over N ranks (profiles/rank_projection.py), 3 vs 4 frames in flight
set -o pipefail
O=gpurun_out/proj3; mkdir -p $O
for d in 3 4; do
  for w in 2 4 8; do
    timeout -k 10 150 python -u profiles/rank_projection.py --config C5 --world $w --frames-in-flight $d > $O/C5_w${w}_d$d.jsonl 2>>$O/err || exit 1
  done
done
timeout -k 10 150 python -u profiles/rank_projection.py --config C2 --world 8 > $O/C2_w8_d2.jsonl 2>>$O/err || exit 1
