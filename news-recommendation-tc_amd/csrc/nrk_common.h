// nrk_common.h -- shared device/host helpers for libnrk (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/nrk.h"

namespace nrk {

// ----------------------------------------------------------------- errors --
void set_error(const std::string& msg);
void clear_error();

#define NRK_REQUIRE(cond, msg)                                  \
    do {                                                        \
        if (!(cond)) {                                          \
            ::nrk::set_error(std::string(__func__) + ": " + (msg)); \
            return NRK_EINVAL;                                  \
        }                                                       \
    } while (0)

#define NRK_UNSUPPORTED(msg)                                    \
    do {                                                        \
        ::nrk::set_error(std::string(__func__) + ": " + (msg)); \
        return NRK_EUNSUPPORTED;                                \
    } while (0)

#define NRK_CHECK_LAUNCH()                                                          \
    do {                                                                            \
        hipError_t e_ = hipGetLastError();                                          \
        if (e_ != hipSuccess) {                                                     \
            ::nrk::set_error(std::string(__func__) + ": " + hipGetErrorString(e_)); \
            return NRK_EHIP;                                                        \
        }                                                                           \
    } while (0)

inline hipStream_t as_stream(nrk_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int WAVE = 64;

// ------------------------------------------------------------- bf16 bits --
// Round-to-nearest-even fp32 -> bf16 (finite inputs; NaN is not produced by
// the hot path).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// ---------------------------------------------------------- ordered keys --
// (score desc, row asc) -- "better" first.  Exact scores are fp64.
struct Cand {
    double s;
    int32_t row;
};

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
    return a.s > b.s || (a.s == b.s && a.row < b.row);
}

__device__ __forceinline__ Cand shfl_xor_cand(const Cand& c, int m) {
    Cand o;
    o.s = __shfl_xor(c.s, m, WAVE);
    o.row = __shfl_xor(c.row, m, WAVE);
    return o;
}

// Wave-wide bitonic sort of E*64 candidates, best first.  Element index
// i = e*64 + lane.  E is a compile-time power of two; every loop has a
// compile-time trip count so x[] stays in registers.
template <int E>
__device__ __forceinline__ void wave_bitonic_sort(Cand (&x)[E]) {
    const int lane = threadIdx.x & (WAVE - 1);
    // fully unrolled: E = 8 already costs minutes of compile time per
    // instantiation, so larger sorts go through wave_lds_sort
    static_assert(E == 1 || E == 2 || E == 4, "E must be 1, 2 or 4 (wave_lds_sort beyond)");
    constexpr int LOGN = (E == 1 ? 6 : E == 2 ? 7 : 8);
#pragma unroll
    for (int kl = 1; kl <= LOGN; ++kl) {
        const int k = 1 << kl;
#pragma unroll
        for (int jl = kl - 1; jl >= 0; --jl) {
            const int j = 1 << jl;
            if (jl >= 6) {
                const int jj = j >> 6;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if ((e & jj) == 0) {
                        const int p = e | jj;
                        const bool up = (((e * WAVE + lane) & k) == 0);
                        const bool sw = up ? better(x[p], x[e]) : better(x[e], x[p]);
                        const double as = x[e].s, bs = x[p].s;
                        const int32_t ar = x[e].row, br = x[p].row;
                        x[e].s = sw ? bs : as;
                        x[e].row = sw ? br : ar;
                        x[p].s = sw ? as : bs;
                        x[p].row = sw ? ar : br;
                    }
                }
            } else {
                const bool lower = (lane & j) == 0;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const double ys = __shfl_xor(x[e].s, j, WAVE);
                    const int32_t yr = __shfl_xor(x[e].row, j, WAVE);
                    const bool up = (((e * WAVE + lane) & k) == 0);
                    const bool keep_better = (lower == up);
                    const bool xb = x[e].s > ys || (x[e].s == ys && x[e].row < yr);
                    const bool take = keep_better != xb;
                    x[e].s = take ? ys : x[e].s;
                    x[e].row = take ? yr : x[e].row;
                }
            }
        }
    }
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-cooperative bitonic sort of n candidates (a power of two) held in
// this wave's LDS region, best first.  Run-time loops (nothing unrolled):
// the large-list path of the merge / bound / fusion kernels.
__device__ inline void wave_lds_sort(Cand* x, int n) {
    const int lane = threadIdx.x & (WAVE - 1);
    wave_sync_lds();
    for (int sz = 2; sz <= n; sz <<= 1) {
        for (int st = sz >> 1; st > 0; st >>= 1) {
            for (int i = lane; i < n / 2; i += WAVE) {
                const int lo = 2 * st * (i / st) + (i % st), hi = lo + st;
                const bool up = (lo & sz) == 0;
                const Cand a = x[lo], b = x[hi];
                if (up ? better(b, a) : better(a, b)) {
                    x[lo] = b;
                    x[hi] = a;
                }
            }
            wave_sync_lds();
        }
    }
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, WAVE);
    return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, WAVE);
    return v;
}

}  // namespace nrk
