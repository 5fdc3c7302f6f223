#!/usr/bin/env python3
"""Print VGPR/SGPR/scratch/occupancy per kernel from hipcc -Rpass-analysis output files."""
import re
import sys

for f in sys.argv[1:]:
    cur = None
    rows = {}
    for line in open(f):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|SGPRs Spill|VGPRs Spill): (\d+)", line)
        if m and cur:
            key = m.group(1)
            rows[cur][key if "Spill" in key else key.split()[0]] = int(m.group(2))
    for k, v in rows.items():
        name = re.sub(r"_ZN2vr12_GLOBAL__N_1\d+", "", k)[:60]
        print(f"{name:62s} VGPR {v.get('VGPRs', '?'):>4} SGPR {v.get('TotalSGPRs', '?'):>4} scratch {v.get('ScratchSize', '?'):>3} occ {v.get('Occupancy', '?')} "
              f"spill v {v.get('VGPRs Spill', '?')} s {v.get('SGPRs Spill', '?')}")
