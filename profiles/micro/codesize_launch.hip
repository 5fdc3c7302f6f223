// Does a kernel's launch cost grow with its code size?  Kernels that exit at
// once but carry N KiB of unreachable code, each launched after a busy kernel
// (to mimic the render -> crawl-pass boundary) and alone; HIP-event timed.
#include <hip/hip_runtime.h>
#include <cstdio>

#define NOP16 "v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n v_mov_b32 v1, v2\n v_mov_b32 v2, v1\n"
#define NOP256 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16
#define KB1 NOP256                     /* 256 x 4 B = 1 KiB */
#define KB8 KB1 KB1 KB1 KB1 KB1 KB1 KB1 KB1

__global__ void busy(float* p, int n) {
    float a = p[threadIdx.x];
    for (int i = 0; i < n; ++i) a = a * 1.0001f + 0.5f;
    p[threadIdx.x + blockIdx.x * blockDim.x] = a;
}
template <int K8>
__global__ void dead(const int* flag) {
    if (*flag != 12345) return;
    if (K8 >= 1) asm volatile(KB8 ::: "v1", "v2");
    if (K8 >= 2) asm volatile(KB8 ::: "v1", "v2");
    if (K8 >= 4) { asm volatile(KB8 ::: "v1", "v2"); asm volatile(KB8 ::: "v1", "v2"); }
    if (K8 >= 8) { asm volatile(KB8 KB8 ::: "v1", "v2"); asm volatile(KB8 KB8 ::: "v1", "v2"); }
    if (K8 >= 16) { asm volatile(KB8 KB8 KB8 KB8 ::: "v1", "v2"); asm volatile(KB8 KB8 KB8 KB8 ::: "v1", "v2"); }
}

template <int K8>
void run(float* p, int* flag, hipEvent_t a, hipEvent_t b, hipEvent_t c) {
    float t1 = 0, t2 = 0;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(busy, dim3(4096), dim3(256), 0, 0, p, 20000);
        hipEventRecord(a);
        hipLaunchKernelGGL(dead<K8>, dim3(64), dim3(256), 0, 0, flag);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (r) t1 += ms;
        hipEventRecord(a);
        hipLaunchKernelGGL(dead<K8>, dim3(64), dim3(256), 0, 0, flag);
        hipEventRecord(c);
        hipEventSynchronize(c);
        hipEventElapsedTime(&ms, a, c);
        if (r) t2 += ms;
    }
    printf("dead code %3d KiB: after busy kernel %.1f us, idle %.1f us\n", K8 * 8, t1 / (reps - 1) * 1e3, t2 / (reps - 1) * 1e3);
}

int main() {
    float* p; int* flag;
    if (hipMalloc(&p, 4096 * 256 * 4) != hipSuccess || hipMalloc(&flag, 4) != hipSuccess) return 1;
    if (hipMemset(flag, 0, 4) != hipSuccess || hipMemset(p, 0, 4096 * 256 * 4) != hipSuccess) return 1;
    hipEvent_t a, b, c;
    hipEventCreate(&a); hipEventCreate(&b); hipEventCreate(&c);
    run<0>(p, flag, a, b, c);
    run<1>(p, flag, a, b, c);
    run<2>(p, flag, a, b, c);
    run<4>(p, flag, a, b, c);
    run<8>(p, flag, a, b, c);
    run<16>(p, flag, a, b, c);
    run<0>(p, flag, a, b, c);
    return 0;
}
