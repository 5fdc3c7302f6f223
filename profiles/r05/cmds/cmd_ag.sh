#!/bin/bash
# Crawl pass skipped for views a slot has seen defer nothing (records tagged with their
# launch): the whole GPU suite, then A/B against VR_CRAWL_SKIP=0 on C2-C5.
set -o pipefail
O=${1:-gpurun_out/r05ag}
mkdir -p $O
export TMPDIR=/tmp
L=voxelraymarcher_amd/libvr.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in C2 C4 C3 C5; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C $L:VR_CRAWL_SKIP=0 $L --rounds 2 > $O/ab_$C.txt 2>&1 || { tail -5 $O/ab_$C.txt; exit 1; }
  cat $O/ab_$C.txt
done
