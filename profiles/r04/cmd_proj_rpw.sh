# GPU suite, then the 8-rank fixed C5 projection with the default crawl records per wave
# (2 alone / 8 in flight) and with every launch at 4 and 16 (VR_CRAWL_RPW)
set -o pipefail
O=${1:-gpurun_out/r04projrpw}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python profiles/rank_projection.py --config C5 --world 8 > $O/proj_C5_w8.jsonl 2> $O/proj_C5_w8.err || { tail -5 $O/proj_C5_w8.err; exit 1; }
tail -1 $O/proj_C5_w8.jsonl
for R in 4 16; do
  VR_CRAWL_RPW=$R timeout -k 10 400 python profiles/rank_projection.py --config C5 --world 8 > $O/proj_C5_w8_rpw$R.jsonl 2> $O/proj_C5_w8_rpw$R.err || { tail -5 $O/proj_C5_w8_rpw$R.err; exit 1; }
  tail -1 $O/proj_C5_w8_rpw$R.jsonl
done
