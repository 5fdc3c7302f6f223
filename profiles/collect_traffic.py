#!/usr/bin/env python3
"""HBM traffic per launch of the bench's timed kernel from separate rocprofv3
--pmc passes (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so the
read side is doubled (an upper estimate for this kernel's dword gathers, whose
width is uncalibrated); WRITE_SIZE is exact for dword stores.
  python3 profiles/collect_traffic.py <round dir> <config>  -> JSON on stdout"""
import csv
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if r["Counter_Name"] != counter or ("march_kernel" not in n and "persist_kernel" not in n):
                continue
            if "true>" in n:          # the COUNT instantiation (bytes counter), not the timed kernel
                continue
            vals.setdefault(n, []).append(float(r["Counter_Value"]))
    return vals


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    fetch = per_dispatch(os.path.join(root, "pmc_fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(root, "pmc_write"), "WRITE_SIZE")
    kern = max(fetch, key=lambda k: len(fetch[k]))
    f_kb = statistics.median(fetch[kern])
    w_kb = statistics.median(write.get(kern, [0.0]))
    stats = {}
    for f in glob.glob(os.path.join(root, "bench_trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    out = {"config": cfg, "world": 1, "kernel": kern, "fetch_kib_raw": f_kb, "write_kib_raw": w_kb,
           "hbm_bytes_per_launch": int((2 * f_kb + w_kb) * 1024),
           "rocprof_avg_ns": stats.get(kern, {}).get("avg_ns")}
    # what does bound the kernel: VALU wave-instructions (2 cycles each on a SIMD-32)
    # and the shader clock cycles (GRBM_GUI_ACTIVE sums the 8 XCDs) per launch
    valu = per_dispatch(os.path.join(root, "pmc_sq"), "SQ_INSTS_VALU").get(kern)
    grbm = per_dispatch(os.path.join(root, "pmc_tcc"), "GRBM_GUI_ACTIVE").get(kern)
    if valu and grbm:
        out["valu_insts_per_launch"] = statistics.median(valu)
        out["grbm_gui_active_per_launch"] = statistics.median(grbm)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
