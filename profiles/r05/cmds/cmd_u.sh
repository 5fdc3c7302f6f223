#!/bin/bash
# C5 one rank of 8 vs the whole frame, lone launches under PMC: VALU instructions, waves,
# L2 hits/misses per launch (x8 for the rank).
set -o pipefail
O=${1:-gpurun_out/r05u}
mkdir -p $O
export TMPDIR=/tmp
for W in 1 8; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD --kernel-trace -f csv -d $O/sq_w$W -o run -- python3 profiles/profile_kernel.py --config C5 --iters 20 --world $W --rank 1 > $O/sq_w$W.log 2>&1 || { tail -5 $O/sq_w$W.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/tcc_w$W -o run -- python3 profiles/profile_kernel.py --config C5 --iters 20 --world $W --rank 1 > $O/tcc_w$W.log 2>&1 || { tail -5 $O/tcc_w$W.log; exit 1; }
  python3 - <<PY
import csv, collections
acc = collections.defaultdict(list)
for d in ("$O/sq_w$W", "$O/tcc_w$W"):
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        k = "march" if "march_kernel" in r["Kernel_Name"] else ("crawl" if "crawl_kernel" in r["Kernel_Name"] else None)
        if k:
            acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for key in sorted(acc):
    v = acc[key][-20:]
    print("world $W", key, f"{sum(v) / len(v):.4g}")
PY
done
