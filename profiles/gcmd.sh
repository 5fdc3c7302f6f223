set -o pipefail
O=gpurun_out/h14
mkdir -p $O
A=voxelraymarcher_amd/ab
timeout -k 10 500 python profiles/ab_inflight.py C3 100 $A/libvr_jf0.so $A/libvr_jf1.so --rounds 3 > $O/ab_C3.txt 2>&1
