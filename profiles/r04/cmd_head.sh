# head-only heaviest-first order (VR_ORDER_HEAD) vs the full order, same library; order
# permutation check and the order tests under the head order; then the rpw A/B
set -o pipefail
O=$1
mkdir -p $O
VR_ORDER_HEAD=0.25 timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > $O/tests_head.log 2>&1 || { tail -30 $O/tests_head.log; exit 1; }
tail -1 $O/tests_head.log
VR_ORDER_HEAD=0.25 VR_ORDER_CHECK=1 timeout -k 10 120 python bench.py --config C2 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/check.err || exit 1
grep "\[order\]" $O/check.err | head -3
for r in 1 2; do
for C in C4 C2 C3; do
  for H in 0 0.1 0.25 0.5; do
    VR_ORDER_HEAD=$H timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > $O/${C}_h${H}_$r.json 2> $O/${C}_h${H}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/${C}_h${H}_$r.json').read().strip().splitlines()[-1]); print('$C', 'head $H', 'grid_ms', d['kernel_ms_grid_order'], 'learned_ms', d['kernel_ms'], 'frame_ms', d['ms_per_step'])" | tee -a $O/ab.txt
  done
done
done
