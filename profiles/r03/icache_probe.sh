#!/bin/bash
# Instruction-cache counters of the tile pass (separate --pmc passes), per config:
#   bash profiles/r03/icache_probe.sh <out dir> C2 C3 ...
set -u
OUT=${1:-gpurun_out/icache}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
for CFG in "$@"; do
  DRV="python3 profiles/profile_kernel.py --config $CFG --kernel tile --iters 3"
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --kernel-trace -f csv -d "$OUT/$CFG/a" -o run -- $DRV > "$OUT/$CFG.log" 2>&1 || { echo "pmc a failed $CFG"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH_LEVEL SQ_INSTS_VALU --kernel-trace -f csv -d "$OUT/$CFG/b" -o run -- $DRV >> "$OUT/$CFG.log" 2>&1 || { echo "pmc b failed $CFG"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, os
for d in sorted(glob.glob(sys.argv[1] + "/C*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "march_kernel" in r["Kernel_Name"] and "true>" not in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")))
    for k in sorted(agg):
        print(f"  {k:32s} {sum(agg[k]) / len(agg[k]):.6g}")
PY
