#!/bin/bash
# Round-6 A/B 2 (C4): the cuckoo shadow walk's hit answered by the filter alone (no table
# reads) with the in-flight kernel at 7 waves (c4c); + the header requested before the walk
# and 64-bit filter offsets (c4e); against HEAD (base).
set -u
OUT=gpurun_out/r06d; mkdir -p $OUT; export TMPDIR=/tmp
A=voxelraymarcher_amd/ab
run() { timeout -k 10 "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 400 python profiles/r05/ab_bench.py C4 $A/libvr_base.so $A/libvr_c4c.so $A/libvr_c4e.so --rounds 3 > $OUT/ab_C4.txt 2>&1
echo done
