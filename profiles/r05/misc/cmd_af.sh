#!/bin/bash
# The driver's 20-step line: where the ~7 us per step outside the kernels' span go.  Three
# runs each as is and with HSA_ENABLE_INTERRUPT=0 (the runtime polls for completion instead
# of waiting for an interrupt: the end-of-region synchronize returns sooner).
set -o pipefail
O=${1:-gpurun_out/r05af}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for M in default poll; do
    if [ $M = poll ]; then export HSA_ENABLE_INTERRUPT=0; else unset HSA_ENABLE_INTERRUPT; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${M}_$i.json 2> $O/b_${M}_$i.err || { tail -5 $O/b_${M}_$i.err; exit 1; }
    echo "$M $i: $(python3 -c "import json; d=json.loads(open('$O/b_${M}_$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms'], d['host_enqueue_ms_per_step'])")"
  done
done
unset HSA_ENABLE_INTERRUPT
