# GPU suite, then the in-flight occupancy variants on (default) vs off (VR_INFLIGHT_WAVES=0),
# same library, alternated
set -o pipefail
O=$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for C in C4 C3 C2; do
  for E in 0 1; do
    VR_INFLIGHT_WAVES=$E timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > $O/${C}_w${E}_$r.json 2> $O/${C}_w${E}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/${C}_w${E}_$r.json').read().strip().splitlines()[-1]); print('$C', 'inflight_waves $E', 'grid_ms', d['kernel_ms_grid_order'], 'learned_ms', d['kernel_ms'], 'frame_ms', d['ms_per_step'])" | tee -a $O/ab.txt
  done
done
done
