# A/B call (GPU box): full parity suite on the in-tree library, then ab_inflight on several configs.
#   bash profiles/r03/cmd_ab2.sh <out> <steps> "<configs>" lib1 lib2 ...
set -o pipefail
O=$1; K=$2; CFGS=$3; shift 3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for C in $CFGS; do
  timeout -k 10 400 python profiles/ab_inflight.py $C $K "$@" --rounds 2 > $O/ab_$C.txt 2>&1 || exit 1
done
