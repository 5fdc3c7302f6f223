#!/bin/bash
# Orders keyed by view + vr_forget_orders + the bench's first-render phase: parity, the C2
# bench line, and the 8-rank C5 projection (each emulated rank learns its own orders).
set -o pipefail
O=${1:-gpurun_out/r05q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_slots.py tests/test_gpu_tiles_deal.py tests/test_gpu_occupancy.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline --steps 200 > $O/bench_C2.json 2> $O/bench_C2.err || { tail -5 $O/bench_C2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_C2.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['ms_per_step'], d['kernel_ms'], d['kernel_ms_grid_order'], d['kernel_ms_first_render'], r['frac'], r['frac_grid_order'], r['frac_learned_order'], r['frac_pipelined'])"
timeout -k 10 900 python profiles/rank_projection.py --config C5 --world 8 > $O/proj_C5_w8.jsonl 2> $O/proj.err || { tail -20 $O/proj.err; exit 1; }
tail -1 $O/proj_C5_w8.jsonl
