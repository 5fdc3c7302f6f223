#!/bin/bash
# Kernel trace + stats and separate PMC passes (never combined with -s/-r).
# Usage (on the GPU box): bash profiles/run_rocprof.sh <tag> [config] [kernel] [extra profile_kernel args]
set -u
TAG=${1:-r01}; CFG=${2:-C2}; KER=${3:-persistent}; shift 3 2>/dev/null; EXTRA="$*"
OUT=gpurun_out/prof_${TAG}_${CFG}_${KER}
mkdir -p "$OUT"
export TMPDIR=/tmp
DRV="python3 profiles/profile_kernel.py --config $CFG --kernel $KER $EXTRA"
run() { timeout -k 10 300 "$@" > /dev/null 2>>"$OUT/errors.log"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- $DRV --iters 20
run rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -f csv -d "$OUT/pmc_sq" -o run -- $DRV --iters 3
run rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE SQ_INSTS_FLAT --kernel-trace -f csv -d "$OUT/pmc_sq2" -o run -- $DRV --iters 3
run rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc_fetch" -o run -- $DRV --iters 3
run rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc_write" -o run -- $DRV --iters 3
run rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace -f csv -d "$OUT/pmc_tcc" -o run -- $DRV --iters 3
echo "profile done: $OUT"
