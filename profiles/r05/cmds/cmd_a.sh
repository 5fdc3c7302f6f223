#!/bin/bash
# Round-5 first GPU call: the GPU suite (new: forced occupancy variants, 2-D tile deal, RCCL
# one-rank exchange), smoke, the driver's bench line, the forced in-flight tests under a
# rocprofv3 kernel trace (the <..., true> kernel names), and the 8-rank C5 projection with
# the 2-D tile deal.
set -o pipefail
O=${1:-gpurun_out/r05a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -5 $O/bench_driver.err; exit 1; }
echo "driver: $(head -c 400 $O/bench_driver.json)"
mkdir -p $O/prof_occ
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_occ -o occ -- python3 -m pytest tests/test_gpu_occupancy.py -q -p no:cacheprovider > $O/occ.log 2>&1 || { tail -20 $O/occ.log; exit 1; }
tail -2 $O/occ.log
timeout -k 10 500 python profiles/rank_projection.py --config C5 --world 8 --layout tiles > $O/proj_C5_w8_tiles.jsonl 2> $O/proj_C5_w8_tiles.err || { tail -5 $O/proj_C5_w8_tiles.err; exit 1; }
tail -1 $O/proj_C5_w8_tiles.jsonl
