#!/bin/bash
# Round-6 verification call (GPU box): the GPU suite, smoke, the driver's bench line, then
# per config a rocprofv3 kernel trace of ONE bench.py run whose JSON line it splits into
# the run's dispatch phases (profiles/roofline_phases.py: every roofline fraction of the
# line recomputed from the trace).
#   bash profiles/r06/run_check.sh <out> [configs...] [--no-tests] [--cpu]
# (--cpu: also each config's bench line with its CPU baseline, without rocprofv3; C2's is the
# driver line's)
set -o pipefail
O=$1; shift
TESTS=1
CPU=0
CFGS=()
for a in "$@"; do
  if [ "$a" = "--no-tests" ]; then TESTS=0; elif [ "$a" = "--cpu" ]; then CPU=1; else CFGS+=("$a"); fi
done
[ ${#CFGS[@]} -eq 0 ] && CFGS=(C2 C3 C4 C5)
mkdir -p $O
export TMPDIR=/tmp
if [ $TESTS = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
  echo "driver: $(head -c 300 $O/bench_driver.json)"
fi
for C in "${CFGS[@]}"; do
  mkdir -p $O/prof_$C
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$C -o run -- python3 bench.py --config $C --no-cpu-baseline > $O/bench_$C.json 2> $O/bench_$C.err || { tail -5 $O/bench_$C.err; exit 1; }
  python3 profiles/roofline_phases.py $O/prof_$C/run_kernel_trace.csv $O/bench_$C.json $O/prof_$C > $O/phases_$C.txt || exit 1
  echo "$C: $(python3 -c "import json,sys; d=json.loads(open('$O/bench_$C.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], d.get('value_moving_view'), d.get('ms_per_step_moving_view'), d['kernel_ms'], d['kernel_ms_grid_order'], d.get('kernel_ms_first_render'), r['frac'], r.get('frac_grid_order'), r['frac_learned_order'], r['frac_pipelined'], r['crawl_iterations_fast_forwarded'])")"
  cat $O/phases_$C.txt
  rm -f $O/prof_$C/run_kernel_trace.csv.gz; gzip -f $O/prof_$C/run_kernel_trace.csv
done
# the CPU baseline per config (the driver line carries C2's): bench.py without rocprofv3
if [ $CPU = 1 ]; then
  for C in "${CFGS[@]}"; do
    [ $C = C2 ] && continue
    timeout -k 10 400 python bench.py --config $C > $O/bench_cpu_$C.json 2> $O/bench_cpu_$C.err || { tail -5 $O/bench_cpu_$C.err; exit 1; }
    echo "$C cpu: $(python3 -c "import json; d=json.loads(open('$O/bench_cpu_$C.json').read().strip().splitlines()[-1]); print(d['value'], d['cpu_baseline'])")"
  done
fi
