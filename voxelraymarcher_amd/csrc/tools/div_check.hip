// div_check -- exhaustive device check of vr::div_fast (vr_device.h) against
// the correctly rounded division the kernels otherwise use, for every float
// numerator n with 2^-90 <= |n| < 2^20 (both signs, ~1.85e9 values) and a list
// of divisors (edge cases + pseudo-random ones over [2^-64, 2^20]).  Built with
// the library's flags, so `n / d` is hipcc's IEEE division.  Prints one JSON
// line; exit 0 iff there is no mismatch.
//   div_check [n_random_divisors] [seed]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../vr_device.h"

namespace {

constexpr int kExpLo = -90, kExpHi = 20;                     // |n| in [2^-90, 2^20)
constexpr unsigned long long kCount = 2ull * (kExpHi - kExpLo) << 23;

__global__ void check(const float* ds, int nd, unsigned long long* bad, unsigned int* first) {
    extern __shared__ float sd[];
    for (int i = threadIdx.x; i < nd; i += blockDim.x) sd[i] = ds[i];
    __syncthreads();
    unsigned long long local = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < kCount; i += stride) {
        const unsigned int sign = (unsigned int)(i & 1u);
        const unsigned long long k = i >> 1;
        const unsigned int e = (unsigned int)(k >> 23), m = (unsigned int)(k & 0x7FFFFFu);
        const float n = __uint_as_float((sign << 31) | ((unsigned int)(e + kExpLo + 127) << 23) | m);
        for (int j = 0; j < nd; ++j) {
            const float d = sd[j];
            const vr::Rcp c = vr::rcp_setup(d);
            const float a = vr::div_fast(n, c), b = n / d;
            if (!vr::div_fast_ok(n, c) || __float_as_uint(a) != __float_as_uint(b)) {
                ++local;
                if (atomicCAS(first, 0xFFFFFFFFu, __float_as_uint(n)) == 0xFFFFFFFFu) first[1] = __float_as_uint(d);
            }
        }
    }
    if (local) atomicAdd(bad, local);
}

}  // namespace

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 2; } } while (0)

int main(int argc, char** argv) {
    const int nrand = argc > 1 ? atoi(argv[1]) : 48;
    unsigned long long seed = argc > 2 ? strtoull(argv[2], nullptr, 0) : 0x9E3779B97F4A7C15ull;
    std::vector<float> ds = {1.0f, -1.0f, 0x1p-64f, -0x1p-64f, 0x1p+20f, 0x1.fffffep-1f, -0x1.fffffep-1f,
                             0x1.000002p+0f, 0.57735026f, -0.57735026f, 0.70710677f, 1e-3f, -3e-7f, 0x1.fffffep-64f * 2.0f,
                             0x1.0p-32f, 0x1.800000p-1f, 0x1.555556p-2f, 0x1.99999ap-4f};
    for (int i = 0; i < nrand; ++i) {      // splitmix64: half unit-vector-like, half log-uniform
        seed += 0x9E3779B97F4A7C15ull;
        unsigned long long z = seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        unsigned int mant = (unsigned int)(z & 0x7FFFFFu), sgn = (unsigned int)((z >> 23) & 1u);
        int ex = (i & 1) ? -64 + (int)((z >> 24) % 84u) : -1 - (int)((z >> 24) % 12u);
        unsigned int bits = (sgn << 31) | ((unsigned int)(ex + 127) << 23) | mant;
        float f;
        memcpy(&f, &bits, 4);
        ds.push_back(f);
    }
    float* dd = nullptr;
    unsigned long long* dbad = nullptr;
    unsigned int* dfirst = nullptr;
    CK(hipMalloc(&dd, ds.size() * 4));
    CK(hipMalloc(&dbad, 8));
    CK(hipMalloc(&dfirst, 8));
    CK(hipMemcpy(dd, ds.data(), ds.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dbad, 0, 8));
    CK(hipMemset(dfirst, 0xFF, 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), ds.size() * 4, 0, dd, (int)ds.size(), dbad, dfirst);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    unsigned long long bad = 0;
    unsigned int first[2];
    CK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(first, dfirst, 8, hipMemcpyDeviceToHost));
    printf("{\"divisors\": %zu, \"numerators\": %llu, \"pairs\": %llu, \"mismatches\": %llu, \"first_n\": \"0x%08x\", "
           "\"first_d\": \"0x%08x\", \"ms\": %.1f}\n",
           ds.size(), kCount, kCount * ds.size(), bad, first[0], first[1], ms);
    return bad ? 1 : 0;
}
