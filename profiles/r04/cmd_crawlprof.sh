set -o pipefail
mkdir -p gpurun_out/r04b
VR_LIBRARY=voxelraymarcher_amd/ab/libvr_diag.so timeout -k 10 120 python profiles/crawl_prof.py C5 > gpurun_out/r04b/crawl_prof_C5.txt 2>&1 || exit 1
VR_LIBRARY=voxelraymarcher_amd/ab/libvr_diag.so timeout -k 10 120 python profiles/crawl_prof.py C5 LONGEST_AXIS > gpurun_out/r04b/crawl_prof_C5_long.txt 2>&1 || exit 1
cat gpurun_out/r04b/crawl_prof_C5*.txt
bash profiles/r04/run_check.sh gpurun_out/r04b C2 C5 --no-tests
