#!/bin/bash
# GPU suite with the cuckoo key-presence filter; C4 A/B against the round-5 build without it;
# then the C5 per-rank traces (cmd_b).
set -o pipefail
O=${1:-gpurun_out/r05c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python profiles/r05/ab_bench.py C4 voxelraymarcher_amd/libvr.so voxelraymarcher_amd/ab/libvr_nofilter.so --rounds 2 > $O/ab_filter_C4.txt 2>&1 || { tail -5 $O/ab_filter_C4.txt; exit 1; }
cat $O/ab_filter_C4.txt
bash profiles/r05/cmds/cmd_b.sh $O/b
