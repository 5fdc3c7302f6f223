# banded work order (VR_ORDER_MODE=bands) vs the 128-class order: parity, permutation
# check, lone-frame A/B per config, C4 L2 hit rate (PMC) under both orders
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
VR_ORDER_MODE=bands timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "order or slots" > $O/tests_bands.log 2>&1 || { tail -20 $O/tests_bands.log; exit 1; }
tail -1 $O/tests_bands.log
VR_ORDER_MODE=bands VR_ORDER_CHECK=1 timeout -k 10 120 python profiles/profile_kernel.py --config C4 --iters 4 --warmup 20 > $O/order_check.log 2>&1 || exit 1
grep -c "bad 0" $O/order_check.log; grep "\[order\]" $O/order_check.log | grep -v "bad 0" | head -3
for r in 1 2; do for C in C4 C2 C3 C5; do for m in classes bands; do
  VR_ORDER_MODE=$m timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > $O/${C}_${m}_$r.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$O/${C}_${m}_$r.json').read().strip().splitlines()[-1]); print('$C', '$m', 'round $r', 'grid_ms', d['kernel_ms_grid_order'], 'learned_ms', d['kernel_ms'], 'frame_ms', d['ms_per_step'])" | tee -a $O/ab.txt
done; done; done
for m in classes bands; do
  VR_ORDER_MODE=$m timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace -f csv -d $O/pmc_$m -o run -- python3 profiles/profile_kernel.py --config C4 --iters 20 > $O/pmc_$m.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for m in ("classes", "bands"):
    f = glob.glob(f"gpurun_out/r04i/pmc_{m}/**/run_counter_collection.csv", recursive=True)
    if not f: print(m, "no counter file"); continue
    rows = [r for r in csv.DictReader(open(f[0])) if "march_kernel<1, 1, false>" in r.get("Kernel_Name", "")]
    rows = rows[-20:]
    tot = {}
    for r in rows:
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    hit, miss = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
    print(m, "C4 tile pass L2 hit rate", round(hit / max(1, hit + miss), 4), {k: v / max(1, len(rows) / 3) for k, v in tot.items()})
PY
