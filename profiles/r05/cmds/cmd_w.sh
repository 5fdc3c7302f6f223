#!/bin/bash
# 2-D tile deal with 16-row bands (bench.py's default now): deal tests, C5 8-rank emulation
# parity, the full 8-rank projection.
set -o pipefail
O=${1:-gpurun_out/r05w}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tiles_deal.py tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python profiles/rank_projection.py --config C5 --world 8 > $O/proj_C5_w8_b16.jsonl 2> $O/proj.err || { tail -20 $O/proj.err; exit 1; }
cat $O/proj_C5_w8_b16.jsonl | cut -c1-600
