#!/bin/bash
# Transient per-pixel walk-length buffer: the order / parity / slot / deal tests and C2, C5 lines.
set -o pipefail
O=${1:-gpurun_out/r05aa}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_slots.py tests/test_gpu_tiles_deal.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in C2 C5; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C voxelraymarcher_amd/libvr.so --rounds 1 > $O/ab_$C.txt 2>&1 || { tail -5 $O/ab_$C.txt; exit 1; }
  cat $O/ab_$C.txt
done
for D in 2 3 4; do
  timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --frames-in-flight $D > $O/bench_C2_d$D.json 2> $O/bench_C2_d$D.err || { tail -5 $O/bench_C2_d$D.err; exit 1; }
  echo "C2 depth $D: $(python3 -c "import json; d=json.loads(open('$O/bench_C2_d$D.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms'])")"
done
