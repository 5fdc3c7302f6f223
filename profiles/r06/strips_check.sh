#!/bin/bash
# The learned strip deal: its GPU tests (multi-rank bench path, C5 eight-rank emulation), the
# C5 8-rank projection with bench.py's calibration settings, and a C2 8-rank projection (weak).
set -u
O=${1:-gpurun_out/r06strips}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py "tests/test_gpu_parity.py::test_c5_eight_rank_emulation" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u profiles/rank_projection.py --config C5 --world 8 --layout strips > $O/proj_C5_w8_strips.jsonl 2> $O/proj.err || { tail -5 $O/proj.err; exit 1; }
tail -1 $O/proj_C5_w8_strips.jsonl
