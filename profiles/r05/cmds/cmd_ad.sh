#!/bin/bash
# Grid order dealt to the XCDs in contiguous stripes (VR_XCD=1) vs round robin: parity with it,
# C5 / C2 / C4 lines, and C5 ranks 1, 2 of 8.
set -o pipefail
O=${1:-gpurun_out/r05ad}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
VR_XCD=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_tiles_deal.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in C5 C2 C4; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L $L:VR_XCD=1 --rounds 2 > $O/ab_$C.txt 2>&1 || { tail -5 $O/ab_$C.txt; exit 1; }
  cat $O/ab_$C.txt
done
run() { local n=$1; shift; timeout -k 10 600 "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; echo "$n: $(head -2 $O/$n.jsonl | tr '\n' ' ')"; }
run c5_rr python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2
VR_XCD=1 run c5_xcd python profiles/rank_projection.py --config C5 --world 8 --ranks 1,2
