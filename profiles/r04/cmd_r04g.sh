set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
VR_LIBRARY=voxelraymarcher_amd/ab/libvr_lfd.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "LONGEST or longest or fuzz or c3 or C3" > $O/tests_lfd.log 2>&1 || { tail -30 $O/tests_lfd.log; exit 1; }
tail -1 $O/tests_lfd.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "c5 or crawl or slots" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash profiles/r04/cmd_crawlprof.sh $O > /dev/null && head -14 $O/crawl_prof_C5.txt
bash profiles/r04/ab_libs.sh $O/ab 2 C3 voxelraymarcher_amd/libvr.so voxelraymarcher_amd/ab/libvr_lfd.so
bash profiles/r04/ab_libs.sh $O/ab 2 C5 voxelraymarcher_amd/libvr.so voxelraymarcher_amd/ab/libvr_rolled.so
