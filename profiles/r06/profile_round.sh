#!/bin/bash
# Round profile of the ray march (run on the GPU box), per config:
#   bash profiles/r06/profile_round.sh <out dir> C2 [C3 C4 C5 ...]
# 1. rocprofv3 --kernel-trace --stats of profiles/profile_kernel.py (tile and crawl
#    pass durations, isolated launches)
# 2. separate --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ; GRBM+TCC), never combined
#    with -s/-r, each under its own time limit
# 3. profiles/collect_traffic.py -> <out>/traffic.json, keyed by config
set -u
OUT=${1:-gpurun_out/r06prof}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for CFG in "$@"; do
  D="$OUT/$CFG"
  mkdir -p "$D"
  DRV="python3 profiles/profile_kernel.py --config $CFG --iters 20"
  run() { timeout -s KILL 120 "$@" >> "$D/log.txt" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
  run rocprofv3 --kernel-trace --stats -f csv -d "$D/trace" -o run -- $DRV
  # the timed (last 20) launches: heaviest-first order in every slot after the warmup
  python3 profiles/trace_avg.py "$D/trace/run_kernel_trace.csv" 20 > "$D/kernel_timed.txt" || exit 1
  run rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$D/pmc_fetch" -o run -- $DRV
  run rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$D/pmc_write" -o run -- $DRV
  run rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-trace -f csv -d "$D/pmc_sq" -o run -- $DRV
  run rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace -f csv -d "$D/pmc_clk" -o run -- $DRV
  python3 profiles/collect_traffic.py "$D" "$CFG" "$OUT/traffic.json" > "$D/traffic.json" || exit 1
  echo "$CFG done"
done
