// din_common.h -- definitions shared by the DIN kernels: shapes, fragment
// types, the split-fp16 helpers and the prep header's scale record.
#pragma once

#include "nrk_common.h"

namespace nrk {

constexpr int DIN_E = 32;   // embedding dim (din_embedding_dim, config.py:115)
constexpr int DIN_H = 36;   // ActivationUnit hidden (default [36], DIN.py:188)

typedef _Float16 din_half8 __attribute__((ext_vector_type(8)));
typedef float din_f4 __attribute__((ext_vector_type(4)));
typedef uint32_t din_u4 __attribute__((ext_vector_type(4)));  // native vector: promotable to VGPRs

// scales of the round-3 attention prep (nrk_din_prepare): s_k puts
// max |table| at <= 2^14 in fp16
struct DinScales {
    float s_k, s_m, inv, pad;
};

// the power of two that puts mx in [2^13, 2^14) (fp16 range with headroom)
__device__ __forceinline__ float pow2_scale(float mx) {
    if (!(mx > 0.0f)) return 1.0f;
    int e;
    frexpf(mx, &e);  // mx in [2^(e-1), 2^e)
    return ldexpf(1.0f, 14 - e);
}

// x * s = hi + lo, both fp16 (exact when x * s is; else ~2^-22 relative)
__device__ __forceinline__ void split8(const float (&x)[8], float s, din_half8& hi, din_half8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float v = x[e] * s;
        const _Float16 h = (_Float16)v;
        hi[e] = h;
        lo[e] = (_Float16)(v - (float)h);
    }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS traffic
// (lgkmcnt) but not for its outstanding global loads, which __syncthreads()
// (a workgroup release fence: vmcnt(0) on gfx9) would drain -- prefetched
// gathers stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// W slice staging: every thread moves CPT 16-B chunks (clamped, so the
// loads are unconditional; the stores past the slice are skipped)
template <int CPT, int CH>
__device__ __forceinline__ void stage_load(din_u4 (&stg)[CPT], const din_u4* __restrict__ src, int tid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) stg[i] = src[min(tid + 256 * i, CH - 1)];
}
template <int CPT, int CH>
__device__ __forceinline__ void stage_store(const din_u4 (&stg)[CPT], din_u4* dst, int tid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i)
        if (tid + 256 * i < CH) dst[tid + 256 * i] = stg[i];
}

// the value of lane l ^ 16 / l ^ 32 (v_permlane16_swap / v_permlane32_swap
// with vdst = src = v: r[0] holds the lower row's value in the upper row,
// r[1] the upper row's in the lower one) -- VALU, no LDS round trip
__device__ __forceinline__ uint32_t xor16u(uint32_t v, int lane) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((lane >> 4) & 1) ? (uint32_t)r[0] : (uint32_t)r[1];
}
__device__ __forceinline__ uint32_t xor32u(uint32_t v, int lane) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane >> 5) ? (uint32_t)r[0] : (uint32_t)r[1];
}
__device__ __forceinline__ double xor16d(double v, int lane) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double((long long)((uint64_t)xor16u((uint32_t)b, lane) |
                                            ((uint64_t)xor16u((uint32_t)(b >> 32), lane) << 32)));
}
__device__ __forceinline__ double xor32d(double v, int lane) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double((long long)((uint64_t)xor32u((uint32_t)b, lane) |
                                            ((uint64_t)xor32u((uint32_t)(b >> 32), lane) << 32)));
}

}  // namespace nrk
