// div_proof -- exhaustive device proof that a 3-operation division with a
// hoisted reciprocal equals hipcc's IEEE f32 division:
//
//   r = RN(1 / d), or the Newton-refined v_rcp_f32 of vr_device.h rcp_setup  (once per walk)
//   q = RN(n * r); e = fma(-d, q, n); q' = fma(e, r, q)      == RN(n / d) ?
//
// For normal n, d whose intermediates stay normal (no overflow/underflow) every
// step scales exactly with the exponents of n and d, so the outcome depends
// only on the two significands: checking every pair of significands in [1, 2)
// (2^23 x 2^23 = 7.0e13 pairs) covers the whole domain the kernels use it on.
// The kernels' domain guard (vr_device.h: div_fast_ok) keeps |d| in [2^-64, 2^20],
// |n| in [2^-90, 2^20], so r, q, e and e * r are normal floats.
//
// Also counts the same sequence with hipcc's Newton-refined reciprocal (the
// r of rcp_setup, which the kernels use), and checks that this reciprocal scales
// exactly with the divisor's exponent (recip_scaling).  Progress on stderr, one
// JSON line on stdout; exit 0 iff there is no mismatch of any kind.
//   div_proof [first_divisor_block last_divisor_block]   (blocks of 2^16 divisors, 0..127)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "vr_device.h"   // the rcp_setup / div_fast the kernels use: proven as written there

namespace {

constexpr unsigned kDivPerLaunch = 1u << 16;       // divisors per launch
constexpr unsigned kSplit = 64;                    // threads per divisor
constexpr unsigned kPerThread = (1u << 23) / kSplit;   // numerators per thread

__global__ __launch_bounds__(256) void prove(unsigned d0, unsigned long long* bad, unsigned* first) {
    const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned dm = d0 + gid / kSplit;
    const unsigned n0 = (gid % kSplit) * kPerThread;
    const float d = __uint_as_float(0x3F800000u | dm);
    const float ra = 1.0f / d;                                        // RN(1/d)
    const vr::Rcp rc = vr::rcp_setup(d);                              // rcp_setup's r
    unsigned long long la = 0, lb = 0;
    for (unsigned k = 0; k < kPerThread; ++k) {
        const float n = __uint_as_float(0x3F800000u | (n0 + k));
        const float want = n / d;
        float q = n * ra;
        q = __builtin_fmaf(__builtin_fmaf(-d, q, n), ra, q);
        const float p = vr::div_fast(n, rc);
        const bool ba = __float_as_uint(q) != __float_as_uint(want);
        la += ba;
        lb += __float_as_uint(p) != __float_as_uint(want);
        if (ba && atomicCAS(first, 0xFFFFFFFFu, __float_as_uint(n)) == 0xFFFFFFFFu) first[1] = __float_as_uint(d);
    }
    if (la) atomicAdd(&bad[0], la);
    if (lb) atomicAdd(&bad[1], lb);
}

// The Newton-refined reciprocal r(d) = fma(fma(-d, r0, 1), r0, r0), r0 = v_rcp_f32(d)
// (vr_device.h rcp_setup) scales exactly with d's exponent and sign over the
// kernels' divisor domain: r(+-m * 2^e) == +-r(m) * 2^-e for every significand m
// and every e in [-64, 20] -- so the significand proof above covers it as well.
__global__ __launch_bounds__(256) void recip_scaling(unsigned long long* bad) {
    const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;       // significand bits
    if (m >= (1u << 23)) return;
    auto rn = [](float d) { return vr::rcp_setup(d).r; };
    const float r1 = rn(__uint_as_float(0x3F800000u | m));
    unsigned long long local = 0;
    for (int e = -64; e <= 20; ++e) {
        const float d = __uint_as_float((unsigned)(e + 127) << 23 | m);
        const float want = r1 * __uint_as_float((unsigned)(127 - e) << 23);   // exact: 2^-e
        local += __float_as_uint(rn(d)) != __float_as_uint(want);
        local += __float_as_uint(rn(-d)) != __float_as_uint(-want);
    }
    if (local) atomicAdd(bad, local);
}

}  // namespace

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 2; } } while (0)

int main(int argc, char** argv) {
    const unsigned blk_lo = argc > 2 ? (unsigned)atoi(argv[1]) : 0u;
    const unsigned blk_hi = argc > 2 ? (unsigned)atoi(argv[2]) : 127u;
    if (blk_lo > blk_hi || blk_hi > 127u) { fprintf(stderr, "bad block range\n"); return 2; }
    unsigned long long* dbad = nullptr;
    unsigned* dfirst = nullptr;
    CK(hipMalloc(&dbad, 16));
    CK(hipMalloc(&dfirst, 8));
    CK(hipMemset(dbad, 0, 16));
    CK(hipMemset(dfirst, 0xFF, 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    const unsigned threads = kDivPerLaunch * kSplit;
    for (unsigned blk = blk_lo; blk <= blk_hi; ++blk) {
        hipLaunchKernelGGL(prove, dim3(threads / 256u), dim3(256), 0, 0, blk * kDivPerLaunch, dbad, dfirst);
        CK(hipGetLastError());
        if ((blk & 7u) == 7u) {
            CK(hipDeviceSynchronize());
            fprintf(stderr, "divisor block %u done\n", blk);
        }
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    unsigned long long* dscal = nullptr;
    CK(hipMalloc(&dscal, 8));
    CK(hipMemset(dscal, 0, 8));
    hipLaunchKernelGGL(recip_scaling, dim3((1u << 23) / 256u), dim3(256), 0, 0, dscal);
    CK(hipGetLastError());
    unsigned long long scal = 0;
    CK(hipMemcpy(&scal, dscal, 8, hipMemcpyDeviceToHost));
    unsigned long long bad[2];
    unsigned first[2];
    CK(hipMemcpy(bad, dbad, 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(first, dfirst, 8, hipMemcpyDeviceToHost));
    const unsigned long long pairs = (unsigned long long)(blk_hi - blk_lo + 1) * kDivPerLaunch * (1ull << 23);
    printf("{\"divisor_blocks\": [%u, %u], \"pairs\": %llu, \"mismatches_rn_recip\": %llu, "
           "\"mismatches_newton_recip\": %llu, \"newton_recip_scaling_mismatches\": %llu, \"first_n\": \"0x%08x\", "
           "\"first_d\": \"0x%08x\", \"ms\": %.1f}\n",
           blk_lo, blk_hi, pairs, bad[0], bad[1], scal, first[0], first[1], ms);
    return (bad[0] || bad[1] || scal) ? 1 : 0;
}
