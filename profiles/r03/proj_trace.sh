# Kernel trace of one rank of fixed-tiled C5 over 8 ranks (rank 0 holds crawl rows),
# four frames in flight: the crawl pass's duration per launch.
set -o pipefail
O=gpurun_out/proj_trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/r0 -o run -- python3 profiles/rank_projection.py --config C5 --world 8 --ranks 0 --frames-in-flight 4 --steps 50 > $O/r0.log 2>&1
