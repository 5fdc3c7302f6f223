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
    bench = None
    if len(sys.argv) > 3:
        line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
        bench = json.loads(line)
        json.dump(bench, open(os.path.join(dst, "bench.json"), "w"), indent=1)
    # bench.py's phases in the kernel trace: warmup (pipelined), the isolated
    # event loop, the timed loop (frames in flight).  Per-dispatch durations of
    # the isolated phase vs the timed phase's dispatch throughput (span / count).
    trace = os.path.join(run, "bench_trace", "bench_kernel_trace.csv")
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace))
                  if r["Kernel_Name"] == tj["kernel"])
    steps = int(bench["steps"]) if bench else 20
    if len(rows) >= 2 * steps:
        iso = rows[-2 * steps:-steps]
        timed = rows[-steps:]
        iso_us = sum(e - b for b, e in iso) / len(iso) / 1e3
        span_us = (max(e for _, e in timed) - timed[0][0]) / len(timed) / 1e3
        dur_us = sum(e - b for b, e in timed) / len(timed) / 1e3
        overlap = sum(1 for (b1, e1), (b2, e2) in zip(timed, timed[1:]) if b2 < e1)
        with open(os.path.join(dst, "dispatch_throughput.txt"), "w") as f:
            f.write(f"rocprofv3 kernel trace of bench.py, kernel {tj['kernel']}\n"
                    f"isolated phase ({len(iso)} dispatches, one at a time): mean duration {iso_us:.1f} us\n"
                    f"timed phase ({len(timed)} dispatches, frames in flight): span / dispatches {span_us:.1f} us, "
                    f"mean duration {dur_us:.1f} us, {overlap} of {len(timed) - 1} consecutive pairs overlap\n")
            if bench:
                f.write(f"bench.py: kernel_ms {bench['kernel_ms'] * 1e3:.1f} us (isolated), "
                        f"ms_per_step {bench['ms_per_step'] * 1e3:.1f} us (timed loop, wall clock)\n")
        print(open(os.path.join(dst, "dispatch_throughput.txt")).read())
    print(open(os.path.join(dst, f"pmc_bench_{tj['config']}.txt")).read())


if __name__ == "__main__":
    main()
