#!/bin/bash
# Round-6 A/B 3: VCS shadow walks answer a hit from the presence bit (no colour read), vs HEAD.
set -u
OUT=gpurun_out/r06f; mkdir -p $OUT; export TMPDIR=/tmp
A=voxelraymarcher_amd/ab
run() { timeout -k 10 "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
for C in C2 C3 C5; do
  run 400 python profiles/r05/ab_bench.py $C $A/libvr_head.so $A/libvr_vs.so --rounds 2 > $OUT/ab_$C.txt 2>&1
done
echo done
