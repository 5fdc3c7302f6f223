# A/B call with the crawl-pass profile: GPU suite, C5 per-record crawl profile of the
# VR_CRAWL_PROF build, then ab_libs.sh base vs new
#   bash profiles/r04/cmd_ab_cprof.sh <out> <rounds> <configs>
set -o pipefail
O=$1; R=${2:-2}; CF=${3:-C5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VR_LIBRARY=voxelraymarcher_amd/ab/libvr_cprof.so timeout -k 10 120 python profiles/crawl_prof.py C5 > $O/crawl_prof_C5.txt 2>&1 || { cat $O/crawl_prof_C5.txt; exit 1; }
sed -n 2,13p $O/crawl_prof_C5.txt
bash profiles/r04/ab_libs.sh $O/ab $R $CF voxelraymarcher_amd/ab/libvr_base.so voxelraymarcher_amd/libvr.so
