#!/bin/bash
# Separate rocprofv3 --pmc passes (never with -s/-r) over profile_kernel.py for one
# config: issue, stall, lane-utilisation and vector-memory-pipe counters.
#   bash profiles/pmc_deep.sh <tag> [config]
set -u
TAG=${1:-deep}; CFG=${2:-C2}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
DRV="python3 profiles/profile_kernel.py --config $CFG --kernel tile --iters 3"
run() { timeout -s KILL 90 "$@" > /dev/null 2>>"$OUT/errors.log"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD --kernel-trace -f csv -d "$OUT/a" -o run -- $DRV
run rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_WAVES SQ_LEVEL_WAVES --kernel-trace -f csv -d "$OUT/b" -o run -- $DRV
run rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$OUT/c" -o run -- $DRV
run rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCC_HIT_sum TCC_MISS_sum TD_TD_BUSY_sum GRBM_COUNT --kernel-trace -f csv -d "$OUT/d" -o run -- $DRV
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "march_kernel" in n and "true>" not in n:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    print(f"{k:36s} {sum(agg[k]) / len(agg[k]):.6g}")
PY
