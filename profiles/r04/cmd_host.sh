# host-overhead probe, the band tests, then the driver's 20-step C2 line: previous bench.py
# (render_bands per frame) vs the current one (BandRenderer), alternated
set -o pipefail
O=$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "band_partition" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u profiles/host_overhead_probe.py > $O/host_probe.txt 2>&1 || { cat $O/host_probe.txt; exit 1; }
tail -1 $O/host_probe.txt
for r in 1 2 3 4; do
  for B in bench_prev.py bench.py; do
    timeout -k 10 200 python $B --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$(basename $B .py)_$r.json 2> $O/b_$(basename $B .py)_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/b_$(basename $B .py)_$r.json').read().strip().splitlines()[-1]); print('$B', $r, d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'))" | tee -a $O/ab.txt
  done
done
