#!/bin/bash
# PMC pass at HEAD (lane order, view keys, 16-row bands): per config -> traffic.json.
set -o pipefail
O=${1:-gpurun_out/r05pmc3}
bash profiles/r05/profile_round.sh $O C2 C3 C4 C5 || exit 1
python3 - <<PY
import json
d = json.load(open("$O/traffic.json"))
for c, v in d.items():
    if isinstance(v, dict):
        print(c, {k: v[k] for k in ("hbm_bytes_per_launch", "rocprof_avg_ns", "valu_insts_per_launch", "lane_util", "l2_hit_rate", "write_kib_raw") if k in v})
PY
