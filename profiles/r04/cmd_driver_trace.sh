# the driver's 20-step C2 line under rocprofv3 --kernel-trace, 4 runs: the timed phase's
# kernel span from the trace vs the line's wall-clock ms_per_step
set -o pipefail
O=$1
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3 4 5 6; do
  timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/t$r -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b$r.json 2> $O/b$r.err || { tail -5 $O/b$r.err; exit 1; }
  python3 profiles/roofline_phases.py $O/t$r/run_kernel_trace.csv $O/b$r.json $O/t$r > $O/phases$r.txt || exit 1
  python3 -c "import json; d=json.loads(open('$O/b$r.json').read().strip().splitlines()[-1]); print('run $r', d['ms_per_step'])"
  grep timed $O/phases$r.txt
  python3 - $O/t$r/run_kernel_trace.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'march_kernel' in r['Kernel_Name'] or 'crawl_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t = rows[-40:]
s0 = int(t[0]['Start_Timestamp']); e = max(int(r['End_Timestamp']) for r in t)
ms = [r for r in t if 'march' in r['Kernel_Name']]
print('timed span us %.1f' % ((e - s0) / 1e3), 'first march dur %.1f' % ((int(ms[0]['End_Timestamp']) - int(ms[0]['Start_Timestamp'])) / 1e3),
      'last march dur %.1f' % ((int(ms[-1]['End_Timestamp']) - int(ms[-1]['Start_Timestamp'])) / 1e3),
      'starts', ' '.join('%.0f' % ((int(r['Start_Timestamp']) - s0) / 1e3) for r in ms))
PY
  rm -f $O/t$r/run_kernel_trace.csv
done
