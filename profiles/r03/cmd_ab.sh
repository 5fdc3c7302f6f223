# A/B call (GPU box): parity of the first library under test, then ab_inflight over all of them.
#   bash profiles/r03/cmd_ab.sh <out> <config> <steps> lib1 lib2 ...
set -o pipefail
O=$1; C=$2; K=$3; shift 3
mkdir -p $O
VR_LIBRARY=$PWD/$1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 500 python profiles/ab_inflight.py $C $K "$@" --rounds 2 > $O/ab_$C.txt 2>&1
