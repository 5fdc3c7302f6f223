#!/bin/bash
# PMC pass with the lane order (HEAD), per config, and C2 with VR_LANE_ORDER=0 for comparison.
set -o pipefail
O=${1:-gpurun_out/r05pmc2}
bash profiles/r05/profile_round.sh $O C2 C3 C4 C5 || exit 1
VR_LANE_ORDER=0 bash profiles/r05/profile_round.sh $O/lane_off C2 C3 || exit 1
python3 - <<PY
import json
for f in ("$O/traffic.json", "$O/lane_off/traffic.json"):
    d = json.load(open(f))
    for c, v in d.items():
        if isinstance(v, dict):
            print(f, c, {k: v[k] for k in ("hbm_bytes_per_launch", "rocprof_avg_ns", "valu_insts_per_launch", "lane_util", "l2_hit_rate", "write_kib_raw") if k in v})
PY
# vector-L1 behaviour with and without the lane order (C2): accesses vs L2 read requests
for LO in 1 0; do
  VR_LANE_ORDER=$LO timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -f csv -d $O/tcp_lane$LO -o run -- python3 profiles/profile_kernel.py --config C2 --iters 20 > $O/tcp_lane$LO.log 2>&1 || { tail -5 $O/tcp_lane$LO.log; exit 1; }
  python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$O/tcp_lane$LO/run_counter_collection.csv")))
acc = collections.defaultdict(list)
for r in rows:
    if "march_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("lane order $LO", {k: sum(v[-20:]) / 20 for k, v in acc.items()})
PY
done
