# one GPU call's steps: parity suite, round profile (rocprofv3 trace + PMC passes), bench lines
set -o pipefail
O=gpurun_out/h4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 &&
bash profiles/run_round.sh r02b C2 > $O/run_round.txt 2>&1 &&
cp gpurun_out/r02b/traffic.json profiles/traffic.json &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2>&1
