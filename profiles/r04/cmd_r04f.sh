set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "c5 or crawl or slots or fuzz or order or tiles" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash profiles/r04/cmd_crawlprof.sh $O && bash profiles/r04/run_check.sh $O C5 --no-tests
for r in 1 2 4 8; do VR_CRAWL_RPW=$r timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > $O/rpw_$r.json 2>/dev/null || exit 1; python3 -c "import json; d=json.loads(open('$O/rpw_$r.json').read().strip().splitlines()[-1]); print('rpw $r', 'grid_ms', d['kernel_ms_grid_order'], 'learned_ms', d['kernel_ms'], 'frame_ms', d['ms_per_step'])"; done
