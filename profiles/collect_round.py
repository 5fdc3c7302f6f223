#!/usr/bin/env python3
"""Copy one round's profiling evidence from a GPU run directory into the
tracked profiles/<tag>/ (gpurun_out/ is scratch):
  python3 profiles/collect_round.py gpurun_out/r01 r01 [bench_line.json]
  - bench_kernel_stats.csv : rocprofv3 --kernel-trace --stats of bench.py
  - pmc_bench_<cfg>.txt    : per-dispatch mean of every --pmc counter for the timed kernel
  - traffic.json           : HBM bytes per launch (also installed as profiles/traffic.json,
                             which bench.py reads for roofline.traffic)
  - bench.json             : the bench line of that round (if given)"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    run, tag = sys.argv[1], sys.argv[2]
    dst = os.path.join(HERE, tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(run, "bench_trace", "bench_kernel_stats.csv"), os.path.join(dst, "bench_kernel_stats.csv"))
    tj = json.load(open(os.path.join(run, "traffic.json")))
    for p in (os.path.join(dst, "traffic.json"), os.path.join(HERE, "traffic.json")):
        json.dump(tj, open(p, "w"), indent=1)
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(run, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] == tj["kernel"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    with open(os.path.join(dst, f"pmc_bench_{tj['config']}.txt"), "w") as f:
        f.write(f"bench.py {tj['config']} timed kernel {tj['kernel']}: per-dispatch mean of separate "
                f"rocprofv3 --pmc passes (rocprof avg duration {tj['rocprof_avg_ns'] / 1e3:.1f} us)\n")
        for k in sorted(agg):
            f.write(f"{k:32s} {sum(agg[k]) / len(agg[k]):.6g}\n")
    if len(sys.argv) > 3:
        line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
        json.dump(json.loads(line), open(os.path.join(dst, "bench.json"), "w"), indent=1)
    print(open(os.path.join(dst, f"pmc_bench_{tj['config']}.txt")).read())


if __name__ == "__main__":
    main()
