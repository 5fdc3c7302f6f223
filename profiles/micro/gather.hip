// Gather-throughput microbenchmark: every lane walks a dependent chain of
// scattered loads inside a small (L1/L2-resident) table, the access pattern
// of the VCS walk (neighbouring lanes in nearby, not identical, lines).  Compares
// 4-B (global_load_dword) and 8-B (global_load_dwordx2) gathers at the same
// addresses: if the vector-memory pipe's cost is per lane, both take the same time.
//   gather [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int W>
__global__ __launch_bounds__(128) void chase(const uint32_t* __restrict__ t, uint32_t mask, int iters, uint32_t* out) {
    uint32_t i = (blockIdx.x * 128u + threadIdx.x) * 2654435761u;
    uint32_t acc = 0;
    for (int k = 0; k < iters; ++k) {
        // neighbouring lanes: nearby words (a tile's rays in nearby cells)
        const uint32_t idx = ((i >> 7) & mask & ~63u) + (threadIdx.x & 63u) * 3u;
        if (W == 1) {
            const uint32_t v = t[idx & mask];
            acc += v;
            i = i * 1664525u + v;
        } else {
            const uint2 v = reinterpret_cast<const uint2*>(t)[(idx & mask) >> 1];
            acc += v.x ^ v.y;
            i = i * 1664525u + v.x + v.y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 256;
    const uint32_t words = 1u << 20;                 // 4 MB
    std::vector<uint32_t> h(words);
    for (uint32_t k = 0; k < words; ++k) h[k] = k * 2246822519u;
    uint32_t *t, *o;
    hipMalloc(&t, words * 4);
    hipMalloc(&o, 4);
    hipMemcpy(t, h.data(), words * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * 4 * 7 * 2;              // ~7 waves per SIMD, twice over
    for (int rep = 0; rep < 3; ++rep) {
        for (int w = 1; w <= 2; ++w) {
            hipEventRecord(a);
            if (w == 1) hipLaunchKernelGGL(chase<1>, dim3(blocks), dim3(128), 0, 0, t, words - 1, iters, o);
            else hipLaunchKernelGGL(chase<2>, dim3(blocks), dim3(128), 0, 0, t, words - 1, iters, o);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double loads = (double)blocks * 2 * iters;  // wave-level load instructions
            printf("rep %d %s: %.3f ms, %.2f ns per wave-load, %.1f wave-loads per CU per us\n", rep,
                   w == 1 ? "dword  " : "dwordx2", ms, ms * 1e6 / loads, loads / 256 / (ms * 1e3));
        }
    }
    return 0;
}
