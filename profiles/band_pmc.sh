set -u
export TMPDIR=/tmp
OUT=gpurun_out/bandpmc; mkdir -p $OUT
D="python3 profiles/band_latency.py 352"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -f csv -d $OUT/a -o b -- $D > /dev/null 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --kernel-trace -f csv -d $OUT/b -o b -- $D > /dev/null 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum --kernel-trace -f csv -d $OUT/c -o b -- $D > /dev/null 2>&1 || exit 1
