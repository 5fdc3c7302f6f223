set -o pipefail
O=gpurun_out/h13
mkdir -p $O
for r in 1 2; do for d in 2 3 4; do
timeout -k 10 200 python bench.py --no-cpu-baseline --frames-in-flight $d > $O/bench_d${d}_$r.json 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --frames-in-flight $d --steps 20 --warmup 5 > $O/bench20_d${d}_$r.json 2>&1 || exit 1
done; done
