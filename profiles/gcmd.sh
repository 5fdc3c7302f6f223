set -o pipefail
O=gpurun_out/h9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/sched -o bench -- python3 bench.py --no-cpu-baseline --steps 50 > $O/log.txt 2>&1 &&
for r in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_sched_$r.json 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-schedule > $O/bench_plain_$r.json 2>&1 || exit 1
done &&
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_sched_20.json 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --no-schedule > $O/bench_plain_20.json 2>&1
