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
