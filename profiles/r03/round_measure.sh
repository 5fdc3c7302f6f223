#!/bin/bash
# The round's measurement call (GPU box): parity suite, the per-config profile, and
# one bench line per BASELINE config (profiles/traffic.json as written by this
# round's profile, so each line carries its measured HBM bytes and VALU issue).
#   bash profiles/r03/round_measure.sh <out dir>
set -o pipefail
O=${1:-gpurun_out/r03m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
bash profiles/r03/profile_round.sh $O/prof C2 C3 C4 C5 > $O/profile.log 2>&1 &&
cp $O/prof/traffic.json $O/traffic.json &&
for C in C2 C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $C --traffic-json $O/traffic.json > $O/bench_$C.json 2> $O/bench_$C.err || exit 1
done &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --traffic-json $O/traffic.json > $O/bench_driver.json 2> $O/bench_driver.err
