# The driver's bench line (C2, --steps 20 --warmup 5) five times on one box: its spread
set -o pipefail
O=${1:-gpurun_out/driver_rep}; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_$i.json 2>>$O/err || exit 1
done
