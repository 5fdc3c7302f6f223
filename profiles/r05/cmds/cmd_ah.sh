#!/bin/bash
# Crawl skip with vr_forget_orders resetting it: the GPU suite and the C2 / C3 lines.
set -o pipefail
O=${1:-gpurun_out/r05ah}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
for C in C2 C3; do
  timeout -k 10 600 python profiles/r05/ab_bench.py $C voxelraymarcher_amd/libvr.so:VR_CRAWL_SKIP=0 voxelraymarcher_amd/libvr.so --rounds 1 > $O/ab_$C.txt 2>&1 || { tail -5 $O/ab_$C.txt; exit 1; }
  cat $O/ab_$C.txt
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
echo "driver: $(head -c 200 $O/bench_driver.json)"
