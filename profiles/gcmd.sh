set -o pipefail
O=gpurun_out/h15
mkdir -p $O
A=voxelraymarcher_amd/ab
timeout -k 10 600 python profiles/ab_inflight.py C3 100 $A/libvr_lw6.so $A/libvr_lw5.so $A/libvr_lw4.so --rounds 2 > $O/ab_C3.txt 2>&1
