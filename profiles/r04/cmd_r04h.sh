set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "c5 or crawl or slots or fuzz or never or degenerate or alias" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash profiles/r04/cmd_crawlprof.sh $O > /dev/null && head -16 $O/crawl_prof_C5.txt
for m in 1 0; do for r in 2 4 8; do VR_CRAWL_SCENE_LDS=$m VR_CRAWL_RPW=$r timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > $O/c5_m${m}_r$r.json 2>/dev/null || exit 1; python3 -c "import json; d=json.loads(open('$O/c5_m${m}_r$r.json').read().strip().splitlines()[-1]); print('scene_lds $m rpw $r', 'grid_ms', d['kernel_ms_grid_order'], 'learned_ms', d['kernel_ms'], 'frame_ms', d['ms_per_step'])"; done; done
