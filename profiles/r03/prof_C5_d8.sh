# rocprofv3 kernel trace + stats of the C5 bench line under its pipeline policy (8 frames in
# flight, 16 hardware queues: exported here, since the profiler starts the HIP runtime first)
set -o pipefail
O=gpurun_out/prof_C5_d8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
GPU_MAX_HW_QUEUES=16 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config C5 --steps 100 --no-cpu-baseline > $O/bench_C5.json 2> $O/err
