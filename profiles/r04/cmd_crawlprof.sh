# crawl-pass profile (C5, both algorithms) from the VR_CRAWL_PROF build
set -o pipefail
O=${1:-gpurun_out/r04e}
mkdir -p $O
VR_LIBRARY=voxelraymarcher_amd/ab/libvr_cprof.so timeout -k 10 120 python profiles/crawl_prof.py C5 > $O/crawl_prof_C5.txt 2>&1 || { cat $O/crawl_prof_C5.txt; exit 1; }
VR_LIBRARY=voxelraymarcher_amd/ab/libvr_cprof.so timeout -k 10 120 python profiles/crawl_prof.py C5 LONGEST_AXIS > $O/crawl_prof_C5_long.txt 2>&1 || exit 1
cat $O/crawl_prof_C5*.txt
