#!/usr/bin/env python3
"""Summarize a run_rocprof.sh output directory: per-kernel mean duration and
per-dispatch mean of every PMC counter (march kernels only)."""
import collections
import csv
import glob
import os
import sys


def summarize(d):
    out = {}
    for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            out.setdefault("kernels", {})[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                                        "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "march_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                out["vgpr"] = r.get("VGPR_Count")
                out["sgpr"] = r.get("SGPR_Count")
    out["counters"] = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
    return out


if __name__ == "__main__":
    import json
    for d in sys.argv[1:]:
        s = summarize(d)
        print(d)
        for k, v in s.get("kernels", {}).items():
            print(f"  {v['avg_ns'] / 1e3:9.1f} us avg  ({v['calls']} calls)  {k[:90]}")
        print(f"  VGPR {s.get('vgpr')} SGPR {s.get('sgpr')}")
        for k, v in s["counters"].items():
            print(f"  {k:30s} {v:14.4g}")
