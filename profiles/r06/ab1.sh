#!/bin/bash
# Round-6 A/B 1: cuckoo shadow-hit reads skipped + header hoisted (c4a), + 64-bit filter
# addressing (c4b), + the longest-axis direction rematerialised per region round and 32-bit
# mask offsets in the slow paths (c3b), against HEAD's library (base).
set -u
OUT=gpurun_out/r06c; mkdir -p $OUT; export TMPDIR=/tmp
A=voxelraymarcher_amd/ab
run() { timeout -k 10 "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 400 python profiles/r05/ab_bench.py C4 $A/libvr_base.so $A/libvr_c4a.so $A/libvr_c4b.so $A/libvr_c3b.so --rounds 2 > $OUT/ab_C4.txt 2>&1
run 300 python profiles/r05/ab_bench.py C3 $A/libvr_base.so $A/libvr_c3b.so --rounds 2 > $OUT/ab_C3.txt 2>&1
run 300 python profiles/r05/ab_bench.py C2 $A/libvr_base.so $A/libvr_c3b.so --rounds 2 > $OUT/ab_C2.txt 2>&1
for L in base c3b; do
  export VR_LIBRARY=$PWD/$A/libvr_$L.so
  run 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/pmc_w_$L -o run -- python3 profiles/profile_kernel.py --config C3 --iters 20 > $OUT/pmc_w_$L.log 2>&1
done
unset VR_LIBRARY
echo done
