# round-end evidence at HEAD: parity suite, smoke, round profile, bench lines, per-config frame times
set -o pipefail
O=gpurun_out/h11
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
bash profiles/run_round.sh r02c C2 > $O/run_round.txt 2>&1 &&
cp gpurun_out/r02c/traffic.json profiles/traffic.json &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2>&1 &&
for c in C3 C4 C5; do timeout -k 10 200 python profiles/inflight_probe.py $c 60 > $O/inflight_$c.txt 2>&1 || exit 1; done
