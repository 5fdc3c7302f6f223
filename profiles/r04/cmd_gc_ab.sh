# the driver's 20-step C2 line with Python's GC paused in the timed loop (bench.py) vs on
# (bench_gc_on.py, the previous bench.py), alternated on one box
set -o pipefail
O=$1
mkdir -p $O
for r in 1 2 3 4 5; do
  for B in bench_gc_on.py bench.py; do
    timeout -k 10 200 python $B --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$(basename $B .py)_$r.json 2> $O/b_$(basename $B .py)_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/b_$(basename $B .py)_$r.json').read().strip().splitlines()[-1]); print('$B', $r, d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'))" | tee -a $O/ab.txt
  done
done
