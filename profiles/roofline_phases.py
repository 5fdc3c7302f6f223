#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of ONE bench.py run into the run's dispatch phases and
recompute every roofline fraction of its JSON line from the trace alone.

  python profiles/roofline_phases.py <run_kernel_trace.csv> <bench_line.json> [out_dir]

bench.py prints `dispatch_phases` -- the number of non-instrumented launches per phase, in
submission order: warmup, iso_first, untimed, iso_grid, iso_learned, latency (N > 1), timed,
moving (the pipelined loop with a view that changes every frame).
Every launch is one tile-pass dispatch (`march_kernel<S, A, false[, HI]>`) followed by one
crawl-pass dispatch (`crawl_kernel<S, A, false>`) on the same stream, sometimes plus the
learned orders' builds (`perm_kernel`, `order_kernel`: about every 16th launch of a slot).  Dispatches are taken in
Dispatch_Id order (submission order); the instrumented launch (`<..., true>`) is not counted.

For each phase it writes `kernel_stats_<phase>.csv` (rocprofv3's kernel_stats.csv columns,
over that phase's dispatches only) and reports
  period  = (last dispatch end - first dispatch start) / launches: what bench.py's one HIP
            event pair around the phase measures per launch (kernel_ms*),
  kernels = the sum of the phase's per-kernel mean durations (tile + crawl + order builds
            per launch): the kernel_stats figure, without the dispatch gaps,
and the fraction algorithmic_bytes_issued_per_launch / duration / 8 TB/s for both, next
to the bench's own figure for that phase: frac (iso_first: one launch alone as a first
render), frac_grid_order (iso_grid: grid order, learned lane order), frac_learned_order
(iso_learned) and frac_pipelined (timed: per frame).
Results: <out_dir>/roofline_phases.json.
"""
from __future__ import annotations

import collections
import csv
import json
import os
import re
import sys

PEAK_GBS = 8000.0


def load_line(path: str) -> dict:
    text = open(path).read()
    for ln in reversed(text.strip().splitlines()):
        ln = ln.strip()
        if ln.startswith("{"):
            return json.loads(ln)
    raise SystemExit(f"{path}: no JSON line")


def main():
    trace, line_path = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.dirname(os.path.abspath(trace))
    line = load_line(line_path)
    phases = line["dispatch_phases"]
    roof = line["roofline"]
    issued = roof["algorithmic_bytes_issued_per_launch"]
    rows = []
    for r in csv.DictReader(open(trace)):
        name = r["Kernel_Name"]
        if "vr::" not in name:
            continue
        kind = ("tile" if "march_kernel" in name else "crawl" if "crawl_kernel" in name else
                "order" if ("order_kernel" in name or "perm_kernel" in name) else None)
        if kind is None or re.search(r"kernel<\d+, \d+, true[,>]", name):
            continue
        rows.append((int(r["Dispatch_Id"]), kind, name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    launches = []                      # [tile row, crawl row or None, [order rows]]
    for row in rows:
        if row[1] == "tile":
            launches.append([row, None, []])
        elif launches:
            if row[1] == "crawl" and launches[-1][1] is None:
                launches[-1][1] = row
            else:
                launches[-1][2].append(row)
    want = sum(phases.values())
    if len(launches) != want:
        raise SystemExit(f"trace has {len(launches)} launches, dispatch_phases says {want}")
    res = {"trace": os.path.basename(trace), "issued_bytes_per_launch": issued, "phases": {}}
    k = 0
    for ph, n in phases.items():
        part = launches[k:k + n]
        k += n
        if not n:
            continue
        per = collections.defaultdict(list)
        spans = []
        for t, c, od in part:
            per[t[2]].append(t[4] - t[3])
            end = t[4]
            if c is not None:
                per[c[2]].append(c[4] - c[3])
                end = max(end, c[4])
            for o in od:
                per[o[2]].append(o[4] - o[3])
            spans.append(end - t[3])
        with open(os.path.join(out, f"kernel_stats_{ph}.csv"), "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            tot = sum(sum(v) for v in per.values())
            for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 2), min(v), max(v)])
        first = min(t[3] for t, _, _ in part)
        last = max(max([t[4]] + ([c[4]] if c else []) + [o[4] for o in od]) for t, c, od in part)
        period_ns = (last - first) / n
        kern_ns = sum(sum(v) for v in per.values()) / n
        frac = lambda ns: round(issued / (ns * 1e-9) / 1e9 / PEAK_GBS, 4)  # noqa: E731
        res["phases"][ph] = {
            "launches": n,
            "period_us": round(period_ns / 1e3, 3),
            "kernels_us": round(kern_ns / 1e3, 3),
            "span_us": round(sum(spans) / len(spans) / 1e3, 3),
            "kernel_mean_us": {name: round(sum(v) / len(v) / 1e3, 3) for name, v in per.items()},
            "kernel_dispatches": {name: len(v) for name, v in per.items()},
            "frac_from_trace": frac(period_ns),
            "frac_from_kernel_means": frac(kern_ns),
        }
    bench = {"iso_first": roof.get("frac"), "iso_grid": roof.get("frac_grid_order"),
             "iso_learned": roof.get("frac_learned_order"),
             "timed": roof.get("frac_pipelined"), "moving": roof.get("frac_pipelined_moving_view")}
    for ph, fb in bench.items():
        if ph in res["phases"] and fb:
            p = res["phases"][ph]
            p["frac_bench"] = fb
            p["rel_diff"] = round(p["frac_from_trace"] / fb - 1.0, 4)
    with open(os.path.join(out, "roofline_phases.json"), "w") as f:
        json.dump(res, f, indent=1)
    for ph, p in res["phases"].items():
        extra = f"  bench {p['frac_bench']:.4f} ({100 * p['rel_diff']:+.1f} %)" if "frac_bench" in p else ""
        print(f"{ph:12s} {p['launches']:4d} launches  period {p['period_us']:9.3f} us  kernels {p['kernels_us']:9.3f} us  "
              f"frac {p['frac_from_trace']:.4f} (kernel means {p['frac_from_kernel_means']:.4f}){extra}")


if __name__ == "__main__":
    main()
