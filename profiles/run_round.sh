#!/bin/bash
# Round profile of the bench command (run on the GPU box):
#   bash profiles/run_round.sh r01 [C2]
# 1. rocprofv3 --kernel-trace --stats of `bench.py` (its averages must agree with bench's HIP events)
# 2. separate --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ) -- never combined with -s/-r
# 3. profiles/collect_traffic.py -> gpurun_out/<tag>/traffic.json (HBM bytes per launch)
set -u
TAG=${1:-r01}; CFG=${2:-C2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --config $CFG --no-cpu-baseline"
# counter passes: one frame at a time, so every dispatch's counters are its own
PMCB="$BENCH --frames-in-flight 1"
run() { timeout -k 10 400 "$@" >> "$OUT/log.txt" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bench_trace" -o bench -- $BENCH
run rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc_fetch" -o bench -- $PMCB --steps 3 --warmup 1
run rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc_write" -o bench -- $PMCB --steps 3 --warmup 1
run rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -f csv -d "$OUT/pmc_sq" -o bench -- $PMCB --steps 3 --warmup 1
run rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$OUT/pmc_tcc" -o bench -- $PMCB --steps 3 --warmup 1
python3 profiles/collect_traffic.py "$OUT" "$CFG" > "$OUT/traffic.json" || exit 1
cat "$OUT/traffic.json"
