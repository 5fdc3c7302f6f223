#!/usr/bin/env python3
"""Per-kernel mean duration of the LAST n dispatches of each kernel in a rocprofv3
kernel trace (run_kernel_trace.csv): the timed launches of profiles/profile_kernel.py,
after its warmup.
  python profiles/trace_avg.py <trace.csv> [n]"""
import collections
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
per = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for k, v in sorted(per.items()):
    if "vr::" not in k:      # the library's kernels only
        continue
    v.sort()
    last = [d for _, d in v[-n:]]
    print(f"{len(v):5d} dispatches, last {len(last):3d}: mean {sum(last) / len(last) / 1e3:9.2f} us  "
          f"min {min(last) / 1e3:9.2f}  max {max(last) / 1e3:9.2f}  {k}")
