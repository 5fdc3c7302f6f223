#!/bin/bash
# The driver's 20-step C2 line under a kernel trace: the timed phase's kernel span vs the
# line's wall-clock ms_per_step (what the fill, drain and host ends of the timed region cost).
set -o pipefail
O=${1:-gpurun_out/r05ae}
mkdir -p $O
export TMPDIR=/tmp
for K in 20 200; do
  timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/prof_s$K -o run -- python3 bench.py --steps $K --warmup 5 --no-cpu-baseline > $O/bench_s$K.json 2> $O/bench_s$K.err || { tail -5 $O/bench_s$K.err; exit 1; }
  python3 profiles/roofline_phases.py $O/prof_s$K/run_kernel_trace.csv $O/bench_s$K.json $O/prof_s$K > $O/phases_s$K.txt || exit 1
  echo "steps $K: ms_per_step $(python3 -c "import json; print(json.loads(open('$O/bench_s$K.json').read().strip().splitlines()[-1])['ms_per_step'])")"; grep timed $O/phases_s$K.txt
  gzip -f $O/prof_s$K/run_kernel_trace.csv
done
