#!/usr/bin/env python3
"""Per-launch PMC figures of one config's tile-pass kernel from separate rocprofv3
--pmc passes (profiles/r03/profile_round.sh), merged into a JSON keyed by config
(profiles/traffic.json, read by bench.py):
  fetch/write: FETCH_SIZE / WRITE_SIZE in KiB.  They count the L2's memory-side
    requests (MI355X_MICROARCH.md HBM section): Infinity-Cache hits included, so
    they are an upper bound of the HBM bytes.  On gfx950 FETCH_SIZE reports half
    the bytes of wide coalesced reads; the read side is doubled (an upper
    estimate for this kernel's 8-B gathers, whose width is uncalibrated -- see
    profiles/micro/gather_calib.hip for the calibration of random 8-B gathers).
  valu / lane utilisation: SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU.
  clock: GRBM_GUI_ACTIVE (sums the 8 XCDs) over the rocprof kernel duration.
  python3 profiles/collect_traffic.py <profile dir> <config> [merge_into.json]"""
import csv
import hashlib
import re
import glob
import json
import os
import statistics
import sys


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if r["Counter_Name"] != counter or "march_kernel" not in n:
                continue
            if re.search(r"kernel<\d+, \d+, true[,>]", n):   # the COUNT instantiation (bytes counter)
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
    for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    out = {"config": cfg, "world": 1, "kernel": kern, "fetch_kib_raw": f_kb, "write_kib_raw": w_kb,
           "hbm_bytes_per_launch": int((2 * f_kb + w_kb) * 1024),
           "rocprof_avg_ns": stats.get(kern, {}).get("avg_ns"),
           "kernel_stats": stats}
    # the library build the passes ran (bench.py compares it with the one it loads)
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "voxelraymarcher_amd", "libvr.so")
    if os.path.exists(lib):
        out["build"] = "libvr.so sha256:" + hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    valu = per_dispatch(os.path.join(root, "pmc_sq"), "SQ_INSTS_VALU").get(kern)
    thr = per_dispatch(os.path.join(root, "pmc_sq"), "SQ_THREAD_CYCLES_VALU").get(kern)
    salu = per_dispatch(os.path.join(root, "pmc_sq"), "SQ_INSTS_SALU").get(kern)
    grbm = per_dispatch(os.path.join(root, "pmc_clk"), "GRBM_GUI_ACTIVE").get(kern)
    if valu and grbm:
        out["valu_insts_per_launch"] = statistics.median(valu)
        out["grbm_gui_active_per_launch"] = statistics.median(grbm)
    if valu and thr:
        # lane utilisation: in round 2 this ratio reproduced the lane efficiency the oracle's
        # per-pixel iteration counts predict (49 % vs 48 %, profiles/r02/pmc_deep_C2.txt)
        out["thread_cycles_valu_per_launch"] = statistics.median(thr)
        out["lane_util"] = round(statistics.median(thr) / (64.0 * statistics.median(valu)), 4)
    if salu:
        out["salu_insts_per_launch"] = statistics.median(salu)
    tcc_hit = per_dispatch(os.path.join(root, "pmc_clk"), "TCC_HIT_sum").get(kern)
    tcc_miss = per_dispatch(os.path.join(root, "pmc_clk"), "TCC_MISS_sum").get(kern)
    if tcc_hit and tcc_miss:
        out["l2_hit_rate"] = round(statistics.median(tcc_hit) / (statistics.median(tcc_hit) + statistics.median(tcc_miss)), 4)
    if len(sys.argv) > 3:
        path = sys.argv[3]
        try:
            allc = json.load(open(path))
            if "config" in allc:                          # the round-2 single-config form
                allc = {allc["config"]: allc}
        except (OSError, ValueError):
            allc = {}
        allc[cfg] = out
        json.dump(allc, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
