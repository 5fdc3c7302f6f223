set -o pipefail
O=gpurun_out/h17
mkdir -p $O
A=voxelraymarcher_amd/ab
timeout -k 10 600 python profiles/ab_inflight.py C2 400 $A/libvr_t21.so $A/libvr_t12.so $A/libvr_t41.so --rounds 2 > $O/ab_C2.txt 2>&1
