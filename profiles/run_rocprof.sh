#!/bin/bash
# Kernel trace + stats and separate PMC passes (never combined with -s/-r).
# Usage (on the GPU box): bash profiles/run_rocprof.sh <tag> [config]
set -u
TAG=${1:-r01}; CFG=${2:-C2}
OUT=gpurun_out/prof_${TAG}_${CFG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { timeout -k 10 300 "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 profiles/profile_kernel.py --config "$CFG" --iters 20
run rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -f csv -d "$OUT/pmc_sq" -o run -- python3 profiles/profile_kernel.py --config "$CFG" --iters 3
run rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -f csv -d "$OUT/pmc_sq2" -o run -- python3 profiles/profile_kernel.py --config "$CFG" --iters 3
run rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc_fetch" -o run -- python3 profiles/profile_kernel.py --config "$CFG" --iters 3
run rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc_write" -o run -- python3 profiles/profile_kernel.py --config "$CFG" --iters 3
run rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace -f csv -d "$OUT/pmc_tcc" -o run -- python3 profiles/profile_kernel.py --config "$CFG" --iters 3
echo "profile done: $OUT"
