# Verification call (GPU box): the GPU parity suite, smoke, the driver's bench line (C2) and
# one bench line per config, then A/B of the in-tree library against earlier builds.
#   bash profiles/r03/cmd_check.sh <out> [lib ...]
set -o pipefail
O=$1; shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
for C in C2 C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $C > $O/bench_$C.json 2> $O/bench_$C.err || exit 1
done
if [ $# -gt 0 ]; then
  for C in C2 C3 C4 C5; do
    timeout -k 10 400 python profiles/ab_inflight.py $C 200 "$@" --rounds 1 > $O/ab_$C.txt 2>&1 || exit 1
  done
fi
