set -o pipefail
bash profiles/r04/run_check.sh gpurun_out/r04d C5 && bash profiles/r04/ab_xcd.sh gpurun_out/r04d 0 2 4 8
