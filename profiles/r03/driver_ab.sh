# The driver's bench line (C2, --steps 20 --warmup 5), two bench.py layouts alternated on one box
set -o pipefail
O=${1:-gpurun_out/driver_ab}; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 120 python bench_old.py --steps 20 --warmup 5 --no-cpu-baseline > $O/old_$i.json 2>>$O/err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/new_$i.json 2>>$O/err || exit 1
done
