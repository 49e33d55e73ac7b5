// nrk_common.h -- shared device/host helpers for libnrk (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>
#include <type_traits>
#include <utility>

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

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): unrolled
// with the index usable as a constant expression (asm / DPP operands)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// value of lane ^ J (J < 64) without ds_bpermute's address VGPR: DPP
// quad_perm for J = 1, 2; ds_swizzle's xor mode (within 32 lanes) for 4, 8;
// the gfx950 row / half swaps for 16, 32 (vdst = src = v: one result holds
// the even rows' / lower half's values in both, the other the odd / upper)
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
    static_assert(J == 1 || J == 2 || J == 4 || J == 8 || J == 16 || J == 32, "lane_xor");
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (J == 4 || J == 8) {
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (J << 10) | 0x1F);  // and 0x1F, xor J
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? (uint32_t)r[0] : (uint32_t)r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? (uint32_t)r[0] : (uint32_t)r[1];
    }
}
template <int J>
__device__ __forceinline__ double lane_xor_f64(double d) {
    const uint64_t b = (uint64_t)__double_as_longlong(d);
    const uint32_t lo = lane_xor<J>((uint32_t)b), hi = lane_xor<J>((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Wave-wide bitonic sort of E*64 candidates, best first.  Element index
// i = e*64 + lane.  E is a compile-time power of two; every stage is
// unrolled at compile time (lane_xor needs constant distances), so x[]
// stays in registers.
template <int E>
__device__ __forceinline__ void wave_bitonic_sort(Cand (&x)[E]) {
    const int lane = threadIdx.x & (WAVE - 1);
    // E = 8 already costs minutes of compile time per instantiation, so
    // larger sorts go through wave_lds_sort
    static_assert(E == 1 || E == 2 || E == 4, "E must be 1, 2 or 4 (wave_lds_sort beyond)");
    constexpr int LOGN = (E == 1 ? 6 : E == 2 ? 7 : 8);
    static_for<LOGN>([&](auto klc) {
        constexpr int kl = decltype(klc)::value + 1, k = 1 << kl;
        static_for<kl>([&](auto jc) {
            constexpr int jl = kl - 1 - decltype(jc)::value, j = 1 << jl;
            if constexpr (jl >= 6) {
                constexpr int jj = j >> 6;
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
                    const double ys = lane_xor_f64<j>(x[e].s);
                    const int32_t yr = (int32_t)lane_xor<j>((uint32_t)x[e].row);
                    const bool up = (((e * WAVE + lane) & k) == 0);
                    const bool keep_better = (lower == up);
                    const bool xb = x[e].s > ys || (x[e].s == ys && x[e].row < yr);
                    const bool take = keep_better != xb;
                    x[e].s = take ? ys : x[e].s;
                    x[e].row = take ? yr : x[e].row;
                }
            }
        });
    });
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
