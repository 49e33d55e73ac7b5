// ip_topk.hip -- brute-force user x item inner-product top-K on gfx950.
//
// Replaces faiss.IndexFlatIP.add/.search (src/recall/youtubednn_recaller.py
// :493-494, :520; the second Faiss site src/similarity/embedding.py:46-50).
// Contract (= IndexFlatIP): exact inner product, score desc, ties -> lower
// row, -1 / -FLT_MAX padding when k exceeds the catalog.  "Exact" is the fp64
// sum of the fp32 products accumulated in dimension order (the oracle's
// definition, oracle/nrk_oracle.c).  Any k >= 1 up to IP_KMAX.
//
// Design (MI355X-first):
//   1. ip_scan    -- the one dense contraction on MFMA: fp16 32x32x16 tiles
//      (power-of-two scaled, so the only error is fp16 rounding), items
//      (A operand) streamed through an LDS ring by LDS-DMA, UG x 32 users per
//      wave (B operands) in registers, so one LDS fragment read feeds UG
//      MFMAs.  Each lane owns one 16-item half of every 32-item block for
//      each of its users and takes the half-block max.  A half-block max that
//      reaches the lane's cut tau is appended (score, half-block id) to the
//      user's list in HBM; tau = theta - 2 eps, theta = the smaller of the two
//      lanes' j-th largest maxima (2(j+1) >= k, so k distinct half-blocks each
//      hold an item >= theta: a lower bound of the k-th score), kept as a
//      sorted register list per lane.  No per-user lists in LDS and no list
//      compaction in the scan: the LDS holds only the catalog ring.
//   2. ip_select  -- one wave per user: theta = the exact k-th largest
//      appended maximum (bit-wise radix select), the band = appended entries
//      >= theta - 2 eps (every half-block that can hold a top-k item).
//   3. ip_refine  -- one wave per user: fp64 exact rescoring of every item of
//      the band (fp16 prefilter first), keep items with exact score >=
//      cut + eps, wave bitonic sort on (score desc, row asc).
//   4. ip_fallback -- users whose lists or band overflowed (dense exact or
//      near ties, e.g. duplicated catalog rows), and every user when k >
//      IP_KFAST: exact fp64 radix-select over the whole catalog, then a
//      workgroup bitonic sort of the k winners.
#include "nrk_common.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <utility>

namespace nrk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int IP_KFAST = 128;   // largest k on the screen path
constexpr int IP_KMAX = 2048;   // largest k at all (exact path above IP_KFAST)
// screen tile: one LDS ring slot, one barrier (dev builds may try NRK_SCAN_TILE = 16384)
#ifndef NRK_SCAN_TILE
#define NRK_SCAN_TILE 8192
#endif
constexpr int SCAN_TILE = NRK_SCAN_TILE;
// dim 128 (BASELINE config 5): blocks per tile -- a 32-item block is already
// 8 KB there; 4 blocks (32-KB tiles): one barrier / DMA wait per four blocks
// and the next block's fragments read under the current block's MFMAs (see
// ip_scan_kernel's PF2).  250k users x 5M items, one box (tools/scan128.py,
// rows identical): 275.6 ms at 1 block, 254.3 at 2, 245.1 at 4
#ifndef NRK_SCAN_TB128
#define NRK_SCAN_TB128 4
#endif
// 32-item blocks per screen tile (one LDS ring slot, one barrier) at padded dim dp
__host__ __device__ constexpr int scan_tb(int dp) {
    return dp == 128 ? NRK_SCAN_TB128 : (64 * dp >= SCAN_TILE ? 1 : SCAN_TILE / (64 * dp));
}
constexpr int IP_SEL = 512;     // appended maxima >= theta_lb held by the select
constexpr int IP_BQ = 288;      // largest band (k = 128); the refine holds SV + 32 entries
constexpr int IP_KRING = 256;   // prefilter-kept rows awaiting an exact round (ring, power of two)
constexpr size_t CATALOG_HDR = 256;

__host__ __device__ static inline int pad_dim(int d) {
    return d <= 16 ? 16 : d <= 32 ? 32 : d <= 64 ? 64 : d <= 128 ? 128 : 256;
}
__host__ __device__ static inline int64_t n_blocks_of(int64_t n_items) { return (n_items + 31) / 32; }

// Catalog header (after the packed blocks).
struct CatalogHdr {
    float max_norm;  // max_j ||v_j||_2 (fp32)
    float max_abs;   // max_j,d |v_jd|
    float scale;     // power of two applied before the fp16 conversion
    int32_t dim;
    int32_t dp;
    float max_dnorm;  // max_j ||fp16(v_j * scale) / scale - v_j||_2 (rounded up)
};

// 2^(14 - e) where m = f * 2^e, f in [0.5, 1): maps max |x| into [2^13, 2^14)
__device__ __forceinline__ float pow2_scale(float maxabs) {
    if (!(maxabs > 0.0f)) return 1.0f;
    int e;
    (void)frexpf(maxabs, &e);
    return ldexpf(1.0f, 14 - e);
}

static inline size_t catalog_body_bytes(int64_t n_items, int dp) {
    return (size_t)n_blocks_of(n_items) * 64u * (size_t)dp;
}
// dims <= 64: a second fp16 copy after the header, half-block major (the
// refine's prefilter): half-block q = 2 b + h holds the 16 items
// 32 b + (r & 3) + 8 (r >> 2) + 4 h, r = 0..15, each as dp contiguous fp16 --
// one 16 dp-B run per half-block instead of half of every 128-B line of the
// fragment-ordered body
__host__ __device__ static inline bool catalog_has_hb(int dp) { return dp <= 64; }
__host__ __device__ static inline size_t catalog_hb_offset(int64_t n_items, int dp) {
    return (size_t)n_blocks_of(n_items) * 64u * (size_t)dp + CATALOG_HDR;
}

// --------------------------------------------------------- catalog build --
// Thread -> one 16-byte fragment: block b, k-step s, lane l:
//   8 fp16 of item 32b + (l & 31), dims 16s + 8(l >> 5) + [0, 8).
__global__ void catalog_pack_kernel(const float* __restrict__ items, int64_t n_items, int dim,
                                    int dp, const CatalogHdr* __restrict__ hdr,
                                    uint4* __restrict__ out) {
    const int ds = dp / 16;
    const float scale = hdr->scale;
    const int64_t total = n_blocks_of(n_items) * ds * 64;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(t & 63);
        const int s = (int)((t >> 6) % ds);
        const int64_t b = (t >> 6) / ds;
        const int64_t item = b * 32 + (lane & 31);
        const int d0 = 16 * s + 8 * (lane >> 5);
        uint16_t v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int d = d0 + e;
            const float f = (item < n_items && d < dim) ? items[item * dim + d] : 0.0f;
            v[e] = __builtin_bit_cast(uint16_t, (_Float16)(f * scale));
        }
        uint4 o;
        o.x = v[0] | ((uint32_t)v[1] << 16);
        o.y = v[2] | ((uint32_t)v[3] << 16);
        o.z = v[4] | ((uint32_t)v[5] << 16);
        o.w = v[6] | ((uint32_t)v[7] << 16);
        out[t] = o;
    }
}

// Thread -> one 16-byte piece of the half-block-major copy: half-block q,
// item r, dims 8p + [0, 8).
__global__ void catalog_pack_hb_kernel(const float* __restrict__ items, int64_t n_items, int dim,
                                       int dp, const CatalogHdr* __restrict__ hdr,
                                       uint4* __restrict__ out) {
    const int ppr = dp / 8;  // pieces per item row
    const float scale = hdr->scale;
    const int64_t total = n_blocks_of(n_items) * 2 * 16 * ppr;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(t % ppr);
        const int r = (int)((t / ppr) & 15);
        const int64_t q = t / ppr / 16;
        const int64_t item = (q >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (q & 1);
        uint16_t v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int d = 8 * p + e;
            const float f = (item < n_items && d < dim) ? items[item * dim + d] : 0.0f;
            v[e] = __builtin_bit_cast(uint16_t, (_Float16)(f * scale));
        }
        out[t] = make_uint4(v[0] | ((uint32_t)v[1] << 16), v[2] | ((uint32_t)v[3] << 16),
                            v[4] | ((uint32_t)v[5] << 16), v[6] | ((uint32_t)v[7] << 16));
    }
}

// The catalog statistics read the fp32 rows coalesced: L lanes per row (the
// power of two >= dim, at most 64), 64 / L consecutive rows per wave and
// step, lane j of a row holding dims j, j + L, ... (a row-per-lane loop read
// one 4-B word per 128-B line per lane: 1.2 GB fetched per launch for a 47-MB
// config-2 catalog).  The per-row sums then run in a lane tree instead of
// dimension order; max_norm and max_dnorm only enter the screen's error
// bound eps, whose 1.0001 / (1 + 1e-6) margins cover that rounding.
__device__ __forceinline__ int cat_lanes(int dim) { return dim <= 16 ? 16 : dim <= 32 ? 32 : 64; }

__global__ void catalog_norm_kernel(const float* __restrict__ items, int64_t n_items, int dim,
                                    CatalogHdr* hdr) {
    const int lane = threadIdx.x & 63, L = cat_lanes(dim), R = WAVE / L, j = lane & (L - 1);
    const int64_t wid = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    float m = 0.0f, a = 0.0f;
    for (int64_t r0 = wid * R; r0 < n_items; r0 += nw * R) {
        const int64_t r = r0 + lane / L;
        float s = 0.0f;
        if (r < n_items) {
            const float* row = items + r * dim;
            for (int d = j; d < dim; d += L) {
                const float x = row[d];
                s += x * x;
                a = fmaxf(a, fabsf(x));
            }
        }
        for (int o = L >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, WAVE);
        if (r < n_items) m = fmaxf(m, sqrtf(s));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        m = fmaxf(m, __shfl_xor(m, o, WAVE));
        a = fmaxf(a, __shfl_xor(a, o, WAVE));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax((unsigned int*)&hdr->max_norm, __float_as_uint(m));
        atomicMax((unsigned int*)&hdr->max_abs, __float_as_uint(a));
    }
}

// max_j of the fp16 rounding error norm of item j, exactly as catalog_pack
// rounds it (for the screen's error bound eps)
__global__ void catalog_dnorm_kernel(const float* __restrict__ items, int64_t n_items, int dim,
                                     CatalogHdr* hdr) {
    const float scale = hdr->scale;
    const int lane = threadIdx.x & 63, L = cat_lanes(dim), R = WAVE / L, j = lane & (L - 1);
    const int64_t wid = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    double m = 0.0;
    for (int64_t r0 = wid * R; r0 < n_items; r0 += nw * R) {
        const int64_t r = r0 + lane / L;
        double s = 0.0;
        if (r < n_items) {
            const float* row = items + r * dim;
            for (int d = j; d < dim; d += L) {
                const float f = row[d];
                const float x = (float)(_Float16)(f * scale);  // catalog_pack's rounding
                const double e = (double)x / (double)scale - (double)f;
                s += e * e;
            }
        }
        for (int o = L >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, WAVE);
        if (r < n_items) m = fmax(m, sqrt(s));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, WAVE));
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)&hdr->max_dnorm, __float_as_uint((float)(m * (1.0 + 1e-6))));
}

__global__ void catalog_hdr_kernel(CatalogHdr* hdr, int dim, int dp) {
    hdr->dim = dim;
    hdr->dp = dp;
    hdr->scale = pow2_scale(hdr->max_abs);
}

// ------------------------------------------------------------- screening --
// theta - two_eps rounded toward -inf (one ulp below the fp32 result)
__device__ __forceinline__ float round_down_sub(float theta, float two_eps) {
    float c = theta - two_eps;
    return __uint_as_float(c > 0.0f ? __float_as_uint(c) - 1u
                                    : (c == 0.0f ? 0x80000001u : __float_as_uint(c) + 1u));
}

// value of lane l ^ 32 (v_permlane32_swap: lanes 32-63 of vdst <-> lanes
// 0-31 of src; with vdst = src = v, r[0] = [lo, lo], r[1] = [hi, hi])
__device__ __forceinline__ uint32_t partner32(uint32_t v, int h) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return h ? (uint32_t)r[0] : (uint32_t)r[1];
}
__device__ __forceinline__ float partner32f(float v, int h) {
    return __uint_as_float(partner32(__float_as_uint(v), h));
}

// min of v over the lane pair (l, l ^ 32), in both lanes: v_permlane32_swap
// with vdst = src = v leaves the lower half's values in one result and the
// upper half's in the other
__device__ __forceinline__ float pair_min32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fminf(__uint_as_float((uint32_t)r[0]), __uint_as_float((uint32_t)r[1]));
}

// x + (lane bit of m) with the compare's lane mask as the carry-in: one
// v_addc_co_u32 instead of v_cndmask + v_add
__device__ __forceinline__ uint32_t add_if(uint32_t x, uint64_t m) {
    uint32_t r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(x), "s"(m));
    (void)co;
    return r;
}

// Sorted (descending) register list: insert v (v = -inf inserts nothing).
// new[i] = max(t[i], min(t[i-1], v)) -- independent per element.  The scan
// fills the first MT - (jk + 1) slots with +inf, so t[MT - 1] is always the
// (jk + 1)-th largest inserted value (no run-time index into the list).
template <int MT>
__device__ __forceinline__ void top_insert(float (&t)[MT], float v) {
    // t[i - 1] >= t[i], so max(t[i], min(t[i - 1], v)) is their median: one
    // v_med3_f32 per slot instead of a max + min pair
#pragma unroll
    for (int i = MT - 1; i >= 1; --i) t[i] = __builtin_amdgcn_fmed3f(t[i], t[i - 1], v);
    t[0] = fmaxf(t[0], v);
}

// dev-only phase stamps of ip_scan_kernel (make dev DEVFLAGS=-DNRK_SCAN_STAMP=1,
// read by nrk_dev_scan_stamps): waves 0 and NW / 2 of each workgroup (the
// first of each stagger half), shader cycles per phase
#ifndef NRK_SCAN_STAMP
#define NRK_SCAN_STAMP 0
#endif

// list pre-pass of the one-pass scan: n_pre = min(SCAN_PRE_MAX, n / 6) tiles
// of an n-tile range, none below SCAN_PRE_MIN tiles
constexpr int SCAN_PRE_MAX = 64, SCAN_PRE_MIN = 128, SCAN_PRE_DIV = 6, SCAN_SHARD_PRE_DIV = 6;
// (lane bit of m) ? T : F, one v_cndmask_b32 on the compare's SGPR lane mask
// with inline constants (0..64); sel_mask_v: (lane bit of m) ? T : f
template <int F, int T>
__device__ __forceinline__ uint32_t sel_mask_c(uint64_t m) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "n"(F), "n"(T), "s"(m));
    return r;
}
template <int T>
__device__ __forceinline__ uint32_t sel_mask_v(uint64_t m, uint32_t f) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "n"(T), "s"(m));
    return r;
}
// the first b < TB whose lane bit is set in am[b] (TB - 1 if none):
// TB - 1 v_cndmask_b32 on the compare masks
template <int TB>
__device__ __forceinline__ uint32_t first_set_block(const uint64_t (&am)[TB]) {
    if constexpr (TB == 1) {
        return 0u;
    } else {
        uint32_t bs = sel_mask_c<TB - 1, TB - 2>(am[TB - 2]);
        static_for<TB - 2>([&](auto bc) {
            constexpr int b = TB - 3 - decltype(bc)::value;
            bs = sel_mask_v<b>(am[b], bs);
        });
        return bs;
    }
}
#if NRK_SCAN_STAMP
__device__ unsigned long long scan_stamps[1024 * 16];
#define SC_STAMP(k)                                           \
    do {                                                      \
        const uint64_t t_now_ = __builtin_readcyclecounter(); \
        sstp[k] += t_now_ - t_prev;                           \
        t_prev = t_now_;                                      \
    } while (0)
#else
#define SC_STAMP(k) \
    do {            \
    } while (0)
#endif

// Config-4 shard list bound of one user (lane pair (q, h)): the bnd_m largest
// values of its two lanes' final lists (t: descending, +inf placeholders in
// front, jk + 1 real values) as exact lower bounds v / scl - eps (rounded down
// to fp32, descending, -inf padded) -- each list value is a distinct
// half-block's fp16 maximum of this range, so each bounds a distinct item's
// exact score from below.  The pair's lists are merged in registers: A .
// reverse(B) is bitonic, log2(2 MT) half-cleaner stages sort it.  Reads the
// user's record (scl, eps) back from uinfo (written by this lane at setup).
template <int MT>
__device__ __forceinline__ void list_bound_out(const float (&t)[MT], bool live, int h, int user, int n_users, int jk,
                                               float* __restrict__ bnd, int bnd_m, const float4* __restrict__ uinfo) {
    const int nl = jk + 1;  // real list values per lane
    float c[2 * MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        c[i] = t[i];
        c[2 * MT - 1 - i] = partner32f(t[i], h);
    }
#pragma unroll
    for (int d = MT; d >= 1; d >>= 1)
#pragma unroll
        for (int i = 0; i < 2 * MT; ++i)
            if ((i & d) == 0) {
                const float x = c[i], y = c[i + d];
                c[i] = fmaxf(x, y);
                c[i + d] = fminf(x, y);
            }
    if (h == 0 && user < n_users) {
        float* o = bnd + (size_t)user * bnd_m;
        const int p0 = 2 * (MT - nl);  // the placeholders sort to the front
        const float4 ui = uinfo[user];
        const double inv = 1.0 / (double)ui.z;  // exact power of two
#pragma unroll
        for (int j = 0; j < 2 * MT; ++j) {
            const int r = j - p0;
            if (r >= 0 && r < bnd_m) {
                float v = -INFINITY;
                if (live && c[j] != -INFINITY) {
                    const double tv = (double)c[j] * inv - (double)ui.w;
                    v = (float)tv;
                    if ((double)v > tv) v = nextafterf(v, -INFINITY);
                }
                o[r] = v;
            }
        }
        for (int r = 2 * nl; r < bnd_m; ++r) o[r] = -INFINITY;  // fewer values than bnd_m
    }
}

// One user's scan setup (lane pair (q, h) of a 32-user group): the fp16 B
// operand (scaled by a power of two su), and the screen's error bound eps;
// returns the user's scaled record.
//   |fp16 score - exact| = |du.v + u.dv + du.dv + accumulation| with du, dv
//   the actual fp16 rounding errors of this user and of the items:
//     <= ||du|| max||v|| + ||u|| max||dv|| + ||du|| max||dv||
//        + (2^-15 + D 2^-23) ||u|| max||v||  (fp32 accumulation of the exact
//          fp16 products in any order);
//   ||du|| is measured here, max||dv|| by catalog_dnorm_kernel.
template <int DS>
__device__ __forceinline__ void scan_user_setup(const float* __restrict__ users, int n_users, int dim, int user,
                                                int h, float vmax, float dvmax, float sv_scale, f16x8 (&uf)[DS],
                                                float& eps, float& scl, bool& live) {
    constexpr int DP = DS * 16;
    const bool active = user < n_users;
    float uval[DS][8];
    float nrm2 = 0.0f, uabs = 0.0f;
    const float* urow = users + (size_t)(active ? user : 0) * dim;
#pragma unroll
    for (int s = 0; s < DS; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int d = 16 * s + 8 * h + e;
            const float f = (active && d < dim) ? urow[d] : 0.0f;
            uval[s][e] = f;
            nrm2 += f * f;
            uabs = fmaxf(uabs, fabsf(f));
        }
    nrm2 += __shfl_xor(nrm2, 32, WAVE);
    uabs = fmaxf(uabs, __shfl_xor(uabs, 32, WAVE));
    const float su = pow2_scale(uabs);
    float du2 = 0.0f;  // ||fp16(u su) - u su||^2 (scaled units; each difference exact)
#pragma unroll
    for (int s = 0; s < DS; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float a = uval[s][e] * su;
            uf[s][e] = (_Float16)a;
            const float d = (float)uf[s][e] - a;
            du2 += d * d;
        }
    du2 += __shfl_xor(du2, 32, WAVE);
    const float nu = sqrtf(nrm2), ndu = sqrtf(du2) / su;
    const float ceps = 3.0517578e-5f + (float)DP * 1.1920929e-7f;
    eps = (nrm2 == 0.0f) ? 0.0f : (ndu * vmax + nu * dvmax + ndu * dvmax + ceps * nu * vmax) * 1.0001f + 1e-30f;
    scl = su * sv_scale;  // scores are scaled by scl (an exact power of 2)
    // zero users (all scores exactly 0) are answered by the refine directly
    live = active && nrm2 > 0.0f;
}

// Per-user screen record (uinfo): theta_lb (scaled), eps (scaled), the
// exact power-of-two scale scl = su * catalog scale, eps (unscaled).
//
// The scan (every shape but the warp-specialized one below): workgroup ub
// takes user block ub -- NW waves x UG x 32 users -- over the tiles
// [tile_lo, tile_hi); the waves share one NSL-slot LDS ring of catalog tiles
// (8 KB, or one 16-KB block at dim 256).  Per tile every wave reads the tile's
// A fragments and runs TB x DS x UG MFMAs.
template <int DP, int NW, int NSL, int UG, int MT, int WPE>
__global__ __launch_bounds__(NW * 64, WPE) void ip_scan_kernel(
    const float* __restrict__ users, int n_users, const uint8_t* __restrict__ catalog, int n_items, int dim, int k,
    int m2, uint2* __restrict__ app, int32_t* __restrict__ acnt, float4* __restrict__ uinfo, int tile_lo,
    int tile_hi, int n_pre, int pstride, float* __restrict__ bnd, int bnd_m) {
    constexpr int DS = DP / 16;
    constexpr int BLOCK_BYTES = 64 * DP;
    constexpr int TB = scan_tb(DP);
    constexpr int TILE_BYTES = TB * BLOCK_BYTES;
    constexpr int LPT = TILE_BYTES / (NW * 1024);  // 1-KB LDS-DMA pieces per wave per tile
    static_assert(LPT >= 1 && LPT * NW * 1024 == TILE_BYTES, "tile split");
    static_assert(NSL >= 2, "ring");
    __shared__ __attribute__((aligned(16))) uint8_t smem[NSL * TILE_BYTES];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, h = lane >> 5, q = lane & 31;
    const int ub = blockIdx.x;
    const int ubase = ub * (NW * 32 * UG) + wave * (32 * UG);
#if NRK_SCAN_STAMP
    uint64_t sstp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = 0;
#endif

    const int nblk = (n_items + 31) >> 5;
    // tiles [tile_lo, tile_hi) of the catalog (a catalog shard of config 4
    // screens its own range of the shared packed catalog; one GPU: all)
    const int ntile = tile_hi;
    const CatalogHdr* hdr = reinterpret_cast<const CatalogHdr*>(catalog + (size_t)nblk * BLOCK_BYTES);
    const float vmax = hdr->max_norm, sv_scale = hdr->scale, dvmax = hdr->max_dnorm;
    const int jk = (k + 1) / 2 - 1;  // list position whose pair-min bounds the k-th: 2 (jk + 1) >= k

    // B operands: 32 users x DP dims per group, fp16 (scaled by a power of
    // two); lane holds user q of the group, dims 16s + 8h + [0, 8).
    f16x8 ufrag[UG][DS];
    float eps_s[UG], tau[UG];
    float t[UG][MT];
    bool live[UG];
#pragma unroll
    for (int g = 0; g < UG; ++g) {
        const int user = ubase + g * 32 + q;
        float eps, scl;
        scan_user_setup<DS>(users, n_users, dim, user, h, vmax, dvmax, sv_scale, ufrag[g], eps, scl, live[g]);
        eps_s[g] = eps * scl;
        // the user's record now (its list bound .x at the end): scl and eps
        // are not held through the scan
        if (h == 0 && user < n_users) uinfo[user] = make_float4(-INFINITY, eps_s[g], scl, eps);
        tau[g] = live[g] ? -FLT_MAX : INFINITY;
#pragma unroll
        for (int i = 0; i < MT; ++i) t[g][i] = (live[g] && i >= MT - 1 - jk) ? -INFINITY : INFINITY;
    }
    // append lists: the wave's 32 UG users' lists from one wave-uniform base
    // (SGPR address + 32-bit lane offset: 2 * 32 * UG * m2 entries); pos =
    // the lane's next entry, lim = its list's last slot (the count runs past
    // the capacity -- the select then sends the user to the exact fallback
    // -- and extra entries land on the last slot).  Users past n_users are
    // not live: tau = +inf, they never append.
    uint2* const wapp = app + (size_t)(ub * (NW * 32 * UG) + __builtin_amdgcn_readfirstlane(wave) * (32 * UG)) *
                                  2 * (size_t)m2;
    uint32_t pos[UG], lim[UG];
#pragma unroll
    for (int g = 0; g < UG; ++g) {
        pos[g] = (uint32_t)((g * 32 + q) * 2 + h) * (uint32_t)m2;
        lim[g] = pos[g] + (uint32_t)m2 - 1u;
    }
    auto slot = [&](uint32_t x, int g) -> uint32_t { return min(x, lim[g]); };
    // the store from the lanes with a set only, without a branch: the
    // compiler's form (s_and_saveexec, s_cbranch_execz, store, s_or exec per
    // half-block) cost ~55 cycles per (group, block) in the phase stamps,
    // mostly the branch; a store with no lane left is a no-op
    auto app_store_if = [&](uint64_t m, uint32_t e, uint2 v) {
        const uint32_t off = e << 3;
        const uint64_t d = ((uint64_t)v.y << 32) | v.x;
        uint64_t sv;
        asm volatile(
            "s_and_saveexec_b64 %0, %1\n\t"
            "global_store_dwordx2 %2, %3, %4\n\t"
            "s_mov_b64 exec, %0"
            : "=&s"(sv)
            : "s"(m), "v"(off), "v"(d), "s"(wapp)
            : "memory", "scc");  // s_and_saveexec writes SCC
    };

    const uint32_t lds_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(smem);
    const int body_bytes = nblk * BLOCK_BYTES;
    const int tail_blk = n_items >> 5;  // first block holding a row >= n_items
    // Tile t -> ring slot t % NSL by LDS-DMA (global_load_lds_dwordx4: one
    // 1-KB piece per wave-instruction, no VGPR staging); tiles past the end
    // re-load the last piece (keeps the per-wave vmcnt accounting uniform,
    // the data is never used).
    // The prefetches run past the range (the main loop NSL - 1 tiles, the
    // pre-pass (NSL - 1) * pstride): the tile is clamped to the catalog's last
    // one before the 32-bit offset is formed, so a body just under 2 GiB
    // (ip_check's limit) cannot wrap it negative.
    const int last_tile = (nblk - 1) / TB;
    auto issue_tile = [&](int tt, int sl) {
        uint8_t* slot = smem + sl * TILE_BYTES;
        const uint32_t ttc = (uint32_t)min(tt, last_tile);
#pragma unroll
        for (int p = 0; p < LPT; ++p) {
            const int piece = p * NW + wave;
            uint32_t off = ttc * (uint32_t)TILE_BYTES + (uint32_t)piece * 1024u;
            off = off < (uint32_t)body_bytes ? off : (uint32_t)body_bytes - 1024u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(catalog + off + lane * 16),
                (__attribute__((address_space(3))) void*)(slot + piece * 1024), 16, 0, 0);
        }
    };
    const uint32_t lds0 = lds_base + lane * 16;
    // all fragment reads and their wait in inline asm: hipcc's waitcnt pass
    // would otherwise drain the in-flight LDS-DMA (the ring prefetch) in
    // front of a compiler-visible LDS access, and a separate wait statement
    // would let the compiler copy an output before the data landed.
    // One block's DS fragments, one LDS round trip per block:
    auto read_block = [&](int sl, int b, u32x4 (&af)[DS]) {
        const uint32_t base = lds0 + (uint32_t)(sl * TILE_BYTES + b * DS * 1024);
        if constexpr (DS == 1) {
            asm volatile("ds_read_b128 %0, %1 offset:0\n\ts_waitcnt lgkmcnt(0)" : "=&v"(af[0]) : "v"(base) : "memory");
        } else {
#pragma unroll
            for (int s2 = 0; s2 < DS; s2 += 2)
                asm volatile("ds_read_b128 %0, %2 offset:0\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                             : "=&v"(af[s2]), "=&v"(af[s2 + 1])
                             : "v"(base + 1024u * s2)
                             : "memory");
        }
    };
    // DS = 2: block b + 1's fragments are read while block b's MFMAs run --
    // the wait for block b's data and the issue of block b + 1's reads are one
    // asm statement whose operands tie both register sets, so nothing reads
    // (or copies) a fragment before its wait
    constexpr bool PF = DS == 2;
    auto pf_issue = [&](int sl, int b, u32x4 (&af)[DS]) {
        const uint32_t base = lds0 + (uint32_t)(sl * TILE_BYTES + b * DS * 1024);
        asm volatile("ds_read_b128 %0, %2 offset:0\n\tds_read_b128 %1, %2 offset:1024"
                     : "=&v"(af[0]), "=&v"(af[1])
                     : "v"(base)
                     : "memory");
    };
    auto pf_wait_issue = [&](u32x4 (&cur)[DS], int sl, int b, u32x4 (&nxt)[DS]) {
        const uint32_t base = lds0 + (uint32_t)(sl * TILE_BYTES + b * DS * 1024);
        asm volatile("s_waitcnt lgkmcnt(0)\n\tds_read_b128 %0, %4 offset:0\n\tds_read_b128 %1, %4 offset:1024"
                     : "=&v"(nxt[0]), "=&v"(nxt[1]), "+v"(cur[0]), "+v"(cur[1])
                     : "v"(base)
                     : "memory");
    };
    auto pf_wait = [&](u32x4 (&cur)[DS]) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur[0]), "+v"(cur[1])::"memory");
    };
    // DS >= 4 with several blocks per tile (dims 64, 128): two fragment sets
    // by block parity -- block b + 1's DS reads are issued right after block
    // b's have landed, so they fly under block b's UG x DS MFMAs (one LDS
    // round trip per tile exposed instead of one per block)
    constexpr bool PF2 = DS >= 4 && TB >= 2;
    auto blk_issue = [&](int sl, int b, u32x4 (&af)[DS]) {
        const uint32_t base = lds0 + (uint32_t)(sl * TILE_BYTES + b * DS * 1024);
#pragma unroll
        for (int s2 = 0; s2 < DS; s2 += 4)
            asm volatile(
                "ds_read_b128 %0, %4 offset:0\n\tds_read_b128 %1, %4 offset:1024\n\t"
                "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072"
                : "=&v"(af[s2]), "=&v"(af[s2 + 1]), "=&v"(af[s2 + 2]), "=&v"(af[s2 + 3])
                : "v"(base + 1024u * s2)
                : "memory");
    };
    auto blk_wait = [&](u32x4 (&af)[DS]) {
        if constexpr (DS == 4) {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3])::"memory");
        } else {
#pragma unroll
            for (int s2 = 0; s2 < DS; s2 += 8)
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(af[s2]), "+v"(af[s2 + 1]), "+v"(af[s2 + 2]), "+v"(af[s2 + 3]), "+v"(af[s2 + 4]),
                               "+v"(af[s2 + 5]), "+v"(af[s2 + 6]), "+v"(af[s2 + 7])::"memory");
        }
    };
    const int full_tiles = tail_blk / TB;  // tiles whose blocks are all full
    // the tile's MFMAs and half-block maxima (mx); the bookkeeping on them
    // (appends, inserts) is book() below.  Software pipeline over the TB x UG
    // (block, group) steps: step j's DS MFMAs issue while step j - LAG's 16
    // accumulators reduce, so the reduction VALU fills the MFMA shadows
    // instead of waiting on the wave's own MFMA results; LAG + 1 accumulator
    // sets instead of UG (LAG = 2 gives the reduced step's last MFMA a whole
    // step to land before its first reduction VALU reads it).  The reduction
    // is a depth-3 tree of v_max3 (max is order-free: the same maxima as a
    // sequential chain).
    auto tile = [&](int tt, int sl, auto mask_c, float (&mx)[UG][TB]) __attribute__((always_inline)) {
        constexpr bool MASK = decltype(mask_c)::value;
        u32x4 afp[DS];
        if constexpr (PF) pf_issue(sl, 0, afp);
        auto red = [&](const f32x16& a, int bb, int gg) __attribute__((always_inline)) {
            float x[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                x[r] = a[r];
                if constexpr (MASK) {
                    const int row = (tt * TB + bb) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (row >= n_items) x[r] = -INFINITY;
                }
            }
            auto m3 = [](float p, float q, float s) { return fmaxf(fmaxf(p, q), s); };
            const float m0 = m3(x[0], x[1], x[2]), m1 = m3(x[3], x[4], x[5]), m2 = m3(x[6], x[7], x[8]);
            const float m4 = m3(x[9], x[10], x[11]), m5 = m3(x[12], x[13], x[14]);
            mx[gg][bb] = fmaxf(m3(m0, m1, m2), m3(m4, m5, x[15]));
        };
        constexpr int LAG = 2, NACC = LAG + 1, NSTEP = TB * UG;
        f32x16 acc[NACC];
        u32x4 afb[DS];
        u32x4 fb2[PF2 ? 2 : 1][PF2 ? DS : 1];
        if constexpr (PF2) blk_issue(sl, 0, fb2[0]);
        static_for<TB>([&](auto bc) {
            constexpr int b = decltype(bc)::value;
            if constexpr (PF2) {
                blk_wait(fb2[b & 1]);
                if constexpr (b + 1 < TB) blk_issue(sl, b + 1, fb2[(b + 1) & 1]);
#pragma unroll
                for (int s = 0; s < DS; ++s) afb[s] = fb2[b & 1][s];
            } else if constexpr (PF) {
                u32x4 afn[DS];
                if constexpr (b + 1 < TB) pf_wait_issue(afp, sl, b + 1, afn);
                else pf_wait(afp);
#pragma unroll
                for (int s = 0; s < DS; ++s) afb[s] = afp[s];
                if constexpr (b + 1 < TB) {
#pragma unroll
                    for (int s = 0; s < DS; ++s) afp[s] = afn[s];
                }
            } else {
                read_block(sl, b, afb);
            }
            static_for<UG>([&](auto gc) {
                constexpr int g = decltype(gc)::value, j = b * UG + g;
                f32x16& A = acc[j % NACC];
                A = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, afb[0]), ufrag[g][0], f32x16{},
                                                           0, 0, 0);
#pragma unroll
                for (int s = 1; s < DS; ++s)
                    A = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, afb[s]), ufrag[g][s], A, 0,
                                                               0, 0);
                if constexpr (j >= LAG) red(acc[(j - LAG) % NACC], (j - LAG) / UG, (j - LAG) % UG);
                // the order the scheduler must keep: each MFMA of step j
                // followed by its share of step j - LAG's 8 reduction VALU
                if constexpr (!MASK) {
#pragma unroll
                    for (int s = 0; s < DS; ++s) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        if (j >= LAG) __builtin_amdgcn_sched_group_barrier(0x002, (8 + DS - 1) / DS, 0);
                    }
                    // a fence per step: step j - LAG's reduction stays beside step j's MFMAs
                    __builtin_amdgcn_sched_barrier(0);
                }
            });
        });
        // the last LAG steps' reductions (all NSTEP of them when NSTEP < LAG:
        // one block of one group at dim 256)
        constexpr int NTAIL = NSTEP < LAG ? NSTEP : LAG;
        static_for<NTAIL>([&](auto lc) {
            constexpr int j = NSTEP - NTAIL + decltype(lc)::value;
            red(acc[j % NACC], j / UG, j % UG);
        });
    };
    // tau below the exact lb - 2 eps: c = RN(lb - 2 eps) is within half an ulp
    // of it, |c| 2^-22 >= 2 ulp(c) covers that and the fma's own rounding,
    // - 2^-120 covers c = 0 (absorbed for |c| > 2^-96); lb = -inf gives
    // -FLT_MAX (a -inf maximum, rows past the catalog end, is never appended)
    auto retau = [&](int g) {
        const float lb = pair_min32(t[g][MT - 1]);
        const float c = lb - 2.0f * eps_s[g];
        const float tv = fmaxf(__builtin_fmaf(fabsf(c), -0x1p-22f, c) - 0x1p-120f, -FLT_MAX);
        tau[g] = live[g] ? tv : INFINITY;
    };
    auto book = [&](int tt, const float (&mx)[UG][TB], bool ins_ok) __attribute__((always_inline)) {
        // the lane's largest max of the tile, per user group
        float vt[UG];
#pragma unroll
        for (int g = 0; g < UG; ++g) {
            vt[g] = mx[g][0];
#pragma unroll
            for (int b = 1; b < TB; ++b) vt[g] = fmaxf(vt[g], mx[g][b]);
        }
        // appends: every half-block max >= tau reaches the user's HBM list
        // (the count runs past the capacity -- the select then sends the user
        // to the exact fallback -- and extra entries land on the last slots).
        // The lane masks of every half-block max >= tau (compare -> SGPR pair):
        uint64_t am[UG][TB];
        uint64_t any_app = 0;
#pragma unroll
        for (int g = 0; g < UG; ++g)
#pragma unroll
            for (int b = 0; b < TB; ++b) {
                am[g][b] = __builtin_amdgcn_ballot_w64(mx[g][b] >= tau[g]);
                any_app |= am[g][b];
            }
        SC_STAMP(2);
        if (any_app) {
            const uint32_t hb0 = (uint32_t)(tt * TB * 2) + (uint32_t)h;  // id of block 0's half-block
            static_for<UG>([&](auto gc) {
                constexpr int g = decltype(gc)::value;
                if constexpr (TB > 1) {
                    // one store per group: a lane appends 0 or 1 of its TB
                    // half-blocks per tile nearly always, and when it appends
                    // any, its largest (the tile max vt) is among them -- so a
                    // single append IS the tile max's half-block (picked by
                    // v_cndmask on the compare masks); lanes with two or more
                    // redo theirs in block order from the same slot behind a
                    // rare scalar branch
                    uint64_t gm = 0, multi = 0;
#pragma unroll
                    for (int b = 0; b < TB; ++b) {
                        multi |= gm & am[g][b];
                        gm |= am[g][b];
                    }
                    if (gm) {
                        const uint32_t fid = (first_set_block<TB>(am[g]) << 1) + hb0;
                        const uint32_t p0 = pos[g];
                        app_store_if(gm, slot(p0, g), make_uint2(__float_as_uint(vt[g]), fid));
                        uint32_t p = add_if(p0, gm);
                        if (multi) {
                            // p ends at p0 + the lane's append count: the same
                            // as above for the lanes with one or none
                            p = p0;
#pragma unroll
                            for (int b = 0; b < TB; ++b) {
                                app_store_if(am[g][b] & multi, slot(p, g),
                                             make_uint2(__float_as_uint(mx[g][b]), hb0 + 2u * b));
                                p = add_if(p, am[g][b]);
                            }
                        }
                        pos[g] = p;
                    }
                } else {
                    app_store_if(am[g][0], slot(pos[g], g), make_uint2(__float_as_uint(mx[g][0]), hb0));
                    pos[g] = add_if(pos[g], am[g][0]);
                }
            });
        }
        // threshold: maxima enter the lane's top list (a subset of the
        // half-block maxima: the (jk + 1)-th largest stays a lower bound),
        // then tau = (min over the user's two lanes) - 2 eps.  Every inserted
        // value exceeded the lane's list minimum, >= the tau of its tile, so
        // it was appended.  Every tile, per group, the lane's tile max, when
        // some lane of the wave has one that enters (skipped when none does,
        // ~1/4 of the (tile, group)s; -inf inserts nothing).  A pre-pass tile
        // (!ins_ok): its maxima are in the lists already.
        SC_STAMP(3);
        if (ins_ok) {
#pragma unroll
            for (int g = 0; g < UG; ++g) {
                const float v = vt[g];
                const bool in = v > t[g][MT - 1];
                if (!__builtin_amdgcn_ballot_w64(in)) continue;
                top_insert<MT>(t[g], in ? v : -INFINITY);
                retau(g);
            }
        }
    };

    // Stagger: the two waves of a SIMD (w and w + NW/2) run the same tile
    // stream between the same barriers; left in lockstep they reach their
    // MFMAs and their bookkeeping together and the matrix pipe idles during
    // both waves' appends / inserts.  The upper half (LATE) books each tile
    // one tile later, right after the next barrier and before that tile's
    // MFMAs, so one half's bookkeeping VALU runs beside the other half's
    // MFMAs.  The book order per wave is unchanged (tile t's appends use the
    // tau left by tile t - 1's inserts), so the lists are identical.
    // (WPE = 4: two workgroups per CU already interleave on every SIMD)
    const bool late = WPE == 2 && __builtin_amdgcn_readfirstlane(wave) >= NW / 2;
    float mx[UG][TB];  // the LATE half keeps a tile's maxima across the barrier
    int ptt = -1;
    bool pins = true;
    // Pre-pass (n_pre > 0): the tiles tile_lo + i * pstride, i < n_pre, spread
    // over the range, only feed the lists (tile maxima, no appends), so tau
    // starts near its final level instead of at -FLT_MAX: the list warm-up
    // otherwise appends every half-block max of the first tiles and most of
    // the next ones (config 2: 343 -> ~150 appended maxima per user; a
    // config-4 shard of 356 tiles: 265 -> ~90).  The main pass then checks
    // every tile for appends as before but does not insert the sampled tiles
    // again (the list entries stay distinct half-blocks).  Correctness is the
    // one-pass invariant: tau only rises and stays <= lb - 2 eps, every
    // half-block max >= the final tau was appended at its tile, and every
    // final list entry (>= lb) was appended -- a pre-pass entry that is still
    // listed at the end is >= the final lb >= the tau of its main-pass tile.
    int next_s = n_pre > 0 ? tile_lo : INT_MAX, left_s = n_pre;
    auto sampled = [&](int tt) {
        const bool sp = tt == next_s;
        if (sp) {
            next_s = --left_s > 0 ? next_s + pstride : INT_MAX;
        }
        return sp;
    };
    auto step = [&](int tt, int it) {
        // own pieces of tile tt landed (the next NSL-2 tiles' stay in
        // flight; appends issued since only make the wait conservative); the
        // barrier publishes everyone's pieces and retires the previous slot
        SC_STAMP(4);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT * (NSL - 2)) : "memory");
        SC_STAMP(0);
        __builtin_amdgcn_s_barrier();
        SC_STAMP(1);
        issue_tile(tt + NSL - 1, (it + NSL - 1) % NSL);
        if (late && ptt >= 0) book(ptt, mx, pins);
        const int sl = it % NSL;
        if (tt < full_tiles) tile(tt, sl, std::false_type{}, mx);
        else tile(tt, sl, std::true_type{}, mx);
        const bool ins_ok = !sampled(tt);
        if (late) {
            ptt = tt;
            pins = ins_ok;
        } else {
            book(tt, mx, ins_ok);
        }
    };
#if NRK_SCAN_STAMP
    t_prev = __builtin_readcyclecounter();
#endif
    if (n_pre > 0) {
        // the pre-pass over the same ring (its own prologue; the trailing
        // prefetches past the sample are dummies), every wave inserting
        // right after its tile; the MASK body serves every sampled tile
#pragma unroll
        for (int p = 0; p < NSL - 1; ++p) issue_tile(tile_lo + p * pstride, p);
        for (int i = 0; i < n_pre; ++i) {
            const int tt = tile_lo + i * pstride;
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT * (NSL - 2)) : "memory");
            __builtin_amdgcn_s_barrier();
            issue_tile(tt + (NSL - 1) * pstride, (i + NSL - 1) % NSL);
            if (tt < full_tiles) tile(tt, i % NSL, std::false_type{}, mx);
            else tile(tt, i % NSL, std::true_type{}, mx);
#pragma unroll
            for (int g = 0; g < UG; ++g) {
                float v = mx[g][0];
#pragma unroll
                for (int b = 1; b < TB; ++b) v = fmaxf(v, mx[g][b]);
                const bool in = v > t[g][MT - 1];
                if (__builtin_amdgcn_ballot_w64(in)) top_insert<MT>(t[g], in ? v : -INFINITY);
            }
        }
#pragma unroll
        for (int g = 0; g < UG; ++g) retau(g);
        // every piece landed and every wave is done with the ring
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int p = 0; p < NSL - 1; ++p) issue_tile(tile_lo + p, p);
    for (int tt = tile_lo, it = 0; tt < ntile; ++tt, ++it) step(tt, it);
    if (late && ptt >= 0) book(ptt, mx, pins);
#if NRK_SCAN_STAMP
    SC_STAMP(4);
    if ((threadIdx.x == 0 || threadIdx.x == NW / 2 * 64) && blockIdx.x < 1024)
        for (int k = 0; k < 8; ++k) scan_stamps[blockIdx.x * 16 + (threadIdx.x ? 8 : 0) + k] = sstp[k];
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the trailing dummy pieces

#pragma unroll
    for (int g = 0; g < UG; ++g) {
        const float lb = pair_min32(t[g][MT - 1]);
        const int user = ubase + g * 32 + q;
        if (user < n_users) {
            acnt[(size_t)user * 2 + h] = (int)(pos[g] - (lim[g] + 1u - (uint32_t)m2));
            if (h == 0) reinterpret_cast<float*>(uinfo + user)[0] = live[g] ? lb : -INFINITY;
        }
    }
    // Config-4 shard (bnd != nullptr): per user the bnd_m largest list values
    // as exact lower bounds (list_bound_out).  Replaces a pass over the
    // appended maxima (ip_shard_bound_kernel).  Lists of up to 32 (k <= 64;
    // longer ones would spill the merge -- those shards keep the pass).
    if constexpr (MT <= 32) {
        if (bnd != nullptr) {
#pragma unroll
            for (int g = 0; g < UG; ++g)
                list_bound_out<MT>(t[g], live[g], h, ubase + g * 32 + q, n_users, jk, bnd, bnd_m, uinfo);
        }
    }
}

// Warp-specialized scan (WS, round 5; D = 32, k <= 32: config 2 and every
// config-4 shard): the one-pass screen of ip_scan_seg -- same lists, taus,
// append format and list bounds; the appended set differs only by the insert
// period below -- with the work of a SIMD split by role.  12 waves, 1,024
// users per workgroup, one workgroup per CU.  Waves 0-3 (one per SIMD, the
// MFMA waves) hold the fp16 B fragments of 256 users (8 groups), run every
// MFMA of a tile for them, reduce each (block, group) to the lane's half-block
// maximum and write the maxima to LDS; they alone load the ring.  Waves 4-11
// (two book waves per SIMD, 4 groups each) read the maxima one barrier step
// later and do the appends and list inserts, so the matrix pipe never waits
// for bookkeeping and an append store never gates a barrier.  One barrier per
// step of TPS = 2 tiles (the MFMA waves pipeline both tiles as one block
// sequence); main-pass inserts every insp tiles (the largest tile maximum
// since the last insert: the list stays a set of distinct appended
// half-block maxima, so its (jk + 1)-th largest stays a lower bound; only tau
// lags), pre-pass tiles every tile.  LDS: the 4-tile ring (32 KB) + 2 TPS
// maxima slots x 4 pairs x 4 blocks x 2 group quads x 64 lanes x 16 B (128 KB).
// Config 2, one box: 5.08 vs 5.41 ms for ip_scan_kernel.
#ifndef NRK_SCAN_WS
#define NRK_SCAN_WS 1
#endif
#ifndef NRK_SCAN_WS_PRIO
#define NRK_SCAN_WS_PRIO 2
#endif
#ifndef NRK_SCAN_WS_INSP
#define NRK_SCAN_WS_INSP 8
#endif
#ifndef NRK_SCAN_WS_STAMPW
#define NRK_SCAN_WS_STAMPW 4
#endif
#ifndef NRK_SCAN_WS_FLOOR
#define NRK_SCAN_WS_FLOOR 0
#endif
#ifndef NRK_SCAN_WS_TPS
#define NRK_SCAN_WS_TPS 2
#endif
// book waves per MFMA wave (1: 8-wave workgroups, 2: 12)
#ifndef NRK_SCAN_WS_NB
#define NRK_SCAN_WS_NB 2
#endif
constexpr bool SCAN_WS = NRK_SCAN_WS;
constexpr int SCAN_WS_NB = NRK_SCAN_WS_NB;
#ifndef NRK_SCAN_WS_SHARD_INSP
#define NRK_SCAN_WS_SHARD_INSP 4
#endif
constexpr int SCAN_WS_INSP = NRK_SCAN_WS_INSP, SCAN_WS_SHARD_INSP = NRK_SCAN_WS_SHARD_INSP;
static_assert((SCAN_WS_INSP & (SCAN_WS_INSP - 1)) == 0 && SCAN_WS_INSP >= 2 &&
                  (SCAN_WS_SHARD_INSP & (SCAN_WS_SHARD_INSP - 1)) == 0 && SCAN_WS_SHARD_INSP >= 2,
              "insert periods: powers of two >= the two tiles of a step");
template <int DP, int NSL, int MT, int NB>
__global__ __launch_bounds__(64 * 4 * (1 + NB), NB == 1 ? 2 : 1) void ip_scan_ws_kernel(
    const float* __restrict__ users, int n_users, const uint8_t* __restrict__ catalog, int n_items, int dim, int k,
    int m2, uint2* __restrict__ app, int32_t* __restrict__ acnt, float4* __restrict__ uinfo, int tile_lo,
    int tile_hi, int n_pre, int pstride, float* __restrict__ bnd, int bnd_m, int insp) {
    constexpr int NPW = 4, UG = 8, UGB = UG / NB, DS = DP / 16;
    constexpr int BLOCK_BYTES = 64 * DP;
    constexpr int TB = scan_tb(DP);
    constexpr int TILE_BYTES = TB * BLOCK_BYTES;
    constexpr int NPC = TILE_BYTES / 1024;  // 1-KB pieces per tile: waves 0 .. NPC - 1 load one each
    static_assert(TB == 4 && DS == 2 && NPC == 8 && (NB == 1 || NB == 2), "WS scan: 8-KB tiles of four blocks at DP = 32");
    // TPS tiles per barrier step: at step p the MFMA waves run tiles TPS p ..
    // TPS p + TPS - 1 and the book waves book step p - 1's.  Maxima slot:
    // [pair][block][group quad][lane] x 4 floats (the quad's groups); 2 TPS
    // slots.  Only the MFMA waves load the ring (LPW pieces per tile each,
    // DAHEAD steps ahead), so the book waves' appends never gate a barrier.
    constexpr int TPS = NRK_SCAN_WS_TPS, NMX = 2 * TPS, LPW = NPC / NPW, DAHEAD = NSL / TPS - 1;
    static_assert(NSL % TPS == 0 && DAHEAD >= 1, "ring of whole steps, one step ahead at least");
    constexpr int MXP = TB * 2 * 1024, MXS = NPW * MXP;
    __shared__ __attribute__((aligned(16))) uint8_t smem[NSL * TILE_BYTES];
    __shared__ __attribute__((aligned(16))) uint8_t mxb[NMX * MXS];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, h = lane >> 5, q = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const bool mfma_role = wv < NPW;
    const int pw = wv & (NPW - 1);
    const int ubase = (int)blockIdx.x * (NPW * UG * 32) + pw * (UG * 32);
#if NRK_SCAN_STAMP
    // dev stamps (waves 0 and 4): 0 sync; MFMA wave: 1 tile, 7 maxima write
    // + issue, 2 end; book wave: 1 maxima read, 2 appends, 4 inserts, 5 loop
    uint64_t sstp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = __builtin_readcyclecounter();
    auto stamp_out = [&]() {
        if ((threadIdx.x == 0 || threadIdx.x == NRK_SCAN_WS_STAMPW * 64) && blockIdx.x < 1024)
            for (int c = 0; c < 8; ++c) scan_stamps[blockIdx.x * 16 + (threadIdx.x ? 8 : 0) + c] = sstp[c];
    };
#endif

    const int nblk = (n_items + 31) >> 5;
    const CatalogHdr* hdr = reinterpret_cast<const CatalogHdr*>(catalog + (size_t)nblk * BLOCK_BYTES);
    const float vmax = hdr->max_norm, sv_scale = hdr->scale, dvmax = hdr->max_dnorm;
    const int jk = (k + 1) / 2 - 1;
    const int n_main = tile_hi - tile_lo, nseq = n_pre + n_main;
    auto seq = [&](int i) { return i < n_pre ? tile_lo + i * pstride : tile_lo + (i - n_pre); };

    const uint32_t lds_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(smem);
    const uint32_t mx_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(mxb) +
                             (uint32_t)(pw * MXP) + lane * 16;
    const int body_bytes = nblk * BLOCK_BYTES;
    const int tail_blk = n_items >> 5;
    const int full_tiles = tail_blk / TB;
    const int last_tile = (nblk - 1) / TB;
    // MFMA wave wv loads pieces LPW wv .. LPW wv + LPW - 1 of every tile (see
    // ip_scan_seg's issue_tile)
    auto issue_tile = [&](int tt, int sl) {
        const uint32_t ttc = (uint32_t)min(tt, last_tile);
#pragma unroll
        for (int c = 0; c < LPW; ++c) {
            const int piece = wv * LPW + c;
            uint32_t off = ttc * (uint32_t)TILE_BYTES + (uint32_t)piece * 1024u;
            off = off < (uint32_t)body_bytes ? off : (uint32_t)body_bytes - 1024u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(catalog + off + lane * 16),
                (__attribute__((address_space(3))) void*)(smem + sl * TILE_BYTES + piece * 1024), 16, 0, 0);
        }
    };
    auto issue_step = [&](int p) {  // the TPS tiles of step p (past the end: dummies, uniform vmcnt)
#pragma unroll
        for (int t = 0; t < TPS; ++t) {
            const int i = TPS * p + t;
            issue_tile(seq(min(i, nseq - 1)), i % NSL);
        }
    };
    // MFMA waves: own pieces of this step's tiles landed (DAHEAD - 1 steps
    // still in flight), the previous step's maxima written; book waves: their
    // maxima reads done.  Then the barrier publishes both.
    auto sync = [&]() {
        if (mfma_role) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(LPW * TPS * (DAHEAD - 1)) : "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    const int NP = (nseq + TPS - 1) / TPS;  // steps

    if (mfma_role) {
        // ---------------------------------------------------- MFMA waves --
        f16x8 ufrag[UG][DS];
#pragma unroll
        for (int g = 0; g < UG; ++g) {
            float eps, scl;
            bool live;
            scan_user_setup<DS>(users, n_users, dim, ubase + g * 32 + q, h, vmax, dvmax, sv_scale, ufrag[g], eps, scl,
                                live);
        }
#if NRK_SCAN_WS_PRIO
        __builtin_amdgcn_s_setprio(NRK_SCAN_WS_PRIO);
#endif
        const uint32_t lds0 = lds_base + lane * 16;
        auto pf_issue = [&](int sl, int b, u32x4 (&af)[DS]) {
            const uint32_t base = lds0 + (uint32_t)(sl * TILE_BYTES + b * DS * 1024);
            asm volatile("ds_read_b128 %0, %2 offset:0\n\tds_read_b128 %1, %2 offset:1024"
                         : "=&v"(af[0]), "=&v"(af[1])
                         : "v"(base)
                         : "memory");
        };
        auto pf_wait_issue = [&](u32x4 (&cur)[DS], int sl, int b, u32x4 (&nxt)[DS]) {
            const uint32_t base = lds0 + (uint32_t)(sl * TILE_BYTES + b * DS * 1024);
            asm volatile("s_waitcnt lgkmcnt(0)\n\tds_read_b128 %0, %4 offset:0\n\tds_read_b128 %1, %4 offset:1024"
                         : "=&v"(nxt[0]), "=&v"(nxt[1]), "+v"(cur[0]), "+v"(cur[1])
                         : "v"(base)
                         : "memory");
        };
        auto pf_wait = [&](u32x4 (&cur)[DS]) {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur[0]), "+v"(cur[1])::"memory");
        };
        // tile tt in ring slot sl -> the half-block maxima, written to maxima
        // slot ms block by block (software pipeline of ip_scan_seg's tile():
        // step j = (block, group) issues its MFMAs while step j - 2 reduces;
        // block b's maxima are complete after step 8 b + 9)
        // NT tiles (tt[t] in ring slot sl[t], maxima to slot ms[t]) as one
        // software pipeline over their NT TB blocks: no refill between them
        auto tile = [&](auto nt_c, const int (&tt)[TPS], const int (&sl)[TPS], const uint32_t (&ms)[TPS],
                        auto mask_c) __attribute__((always_inline)) {
            constexpr int NT = decltype(nt_c)::value, NBK = NT * TB;
            constexpr bool MASK = decltype(mask_c)::value;
            float mx[2][UG];  // by block parity
            // the half-block max of a step's 16 accumulators in two levels:
            // red1 (6 VALU) folds them into 5 partial maxima, red2 (2 VALU)
            // finishes; step j issues its first MFMA, then step j - 2's red2,
            // its second MFMA, then step j - 1's red1 -- red1 reads an
            // accumulator whose last MFMA is two issue slots back (no hazard
            // wait states), each gap's VALU fits the MFMA's 32 cycles, and only
            // two accumulator sets are live
            using P5 = float[5];
            auto red1 = [&](const f32x16& a, int bb, P5& pm) __attribute__((always_inline)) {
                float x[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    x[r] = a[r];
                    if constexpr (MASK) {
                        const int row = (tt[bb / TB] * TB + bb % TB) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (row >= n_items) x[r] = -INFINITY;
                    }
                }
                auto m3 = [](float p, float s, float u) { return fmaxf(fmaxf(p, s), u); };
                pm[0] = m3(x[0], x[1], x[2]);
                pm[1] = m3(x[3], x[4], x[5]);
                pm[2] = m3(x[6], x[7], x[8]);
                pm[3] = m3(x[9], x[10], x[11]);
                pm[4] = fmaxf(m3(x[12], x[13], x[14]), x[15]);
            };
            auto red2 = [&](const P5& pm, int bb, int gg) __attribute__((always_inline)) {
                mx[bb & 1][gg] = fmaxf(fmaxf(fmaxf(fmaxf(pm[0], pm[1]), pm[2]), pm[3]), pm[4]);  // 2 v_max3
            };
            auto put = [&](int bb) __attribute__((always_inline)) {
                const f32x4 v0 = {mx[bb & 1][0], mx[bb & 1][1], mx[bb & 1][2], mx[bb & 1][3]};
                const f32x4 v1 = {mx[bb & 1][4], mx[bb & 1][5], mx[bb & 1][6], mx[bb & 1][7]};
                asm volatile("ds_write_b128 %0, %1 offset:0\n\tds_write_b128 %0, %2 offset:1024" ::"v"(
                                 ms[bb / TB] + (uint32_t)((bb % TB) * 2048)),
                             "v"(v0), "v"(v1)
                             : "memory");
            };
            auto slb = [&](int bb) { return sl[bb / TB]; };
            constexpr int NSTEP = NBK * UG;
            f32x16 acc[2];
            float pm[2][5];  // partial maxima by step parity
            u32x4 afp[DS], afb[DS];
            pf_issue(slb(0), 0, afp);
            static_for<NBK>([&](auto bc) {
                constexpr int bb = decltype(bc)::value;
                u32x4 afn[DS];
                if constexpr (bb + 1 < NBK) pf_wait_issue(afp, slb(bb + 1), (bb + 1) % TB, afn);
                else pf_wait(afp);
#pragma unroll
                for (int s = 0; s < DS; ++s) afb[s] = afp[s];
                if constexpr (bb + 1 < NBK) {
#pragma unroll
                    for (int s = 0; s < DS; ++s) afp[s] = afn[s];
                }
                static_for<UG>([&](auto gc) {
                    constexpr int g = decltype(gc)::value, j = bb * UG + g;
                    f32x16& A = acc[j & 1];
                    A = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, afb[0]), ufrag[g][0],
                                                               f32x16{}, 0, 0, 0);
                    if constexpr (j >= 2) red2(pm[j & 1], (j - 2) / UG, (j - 2) % UG);
                    if constexpr (!MASK) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        if constexpr (j >= 2) __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                    }
                    A = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, afb[1]), ufrag[g][1], A, 0,
                                                               0, 0);
                    if constexpr (j >= 1) red1(acc[(j - 1) & 1], (j - 1) / UG, pm[(j - 1) & 1]);
                    if constexpr (bb > 0 && g == 2) put(bb - 1);  // block bb - 1 complete (its last red2 at g = 1)
                    if constexpr (!MASK) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        if constexpr (j >= 1) __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                });
            });
            red2(pm[(NSTEP - 2) & 1], (NSTEP - 2) / UG, (NSTEP - 2) % UG);
            red1(acc[(NSTEP - 1) & 1], (NSTEP - 1) / UG, pm[(NSTEP - 1) & 1]);
            red2(pm[(NSTEP - 1) & 1], (NSTEP - 1) / UG, (NSTEP - 1) % UG);
            put(NBK - 1);
        };
#pragma unroll
        for (int p = 0; p < DAHEAD; ++p) issue_step(p);
        for (int p = 0; p <= NP; ++p) {
            SC_STAMP(7);
            sync();
            SC_STAMP(0);
            issue_step(p + DAHEAD);
            int tts[TPS], sls[TPS];
            uint32_t mss[TPS];
#pragma unroll
            for (int t = 0; t < TPS; ++t) {
                const int i = min(TPS * p + t, nseq - 1);
                tts[t] = seq(i);
                sls[t] = (TPS * p + t) % NSL;
                mss[t] = mx_base + (uint32_t)(((p & 1) * TPS + t) * MXS);
            }
            if (TPS * p + TPS <= nseq) {  // a whole step: one pipeline over its TPS tiles
                bool full = true;
#pragma unroll
                for (int t = 0; t < TPS; ++t) full = full && tts[t] < full_tiles;
                if (full) tile(std::integral_constant<int, TPS>{}, tts, sls, mss, std::false_type{});
                else tile(std::integral_constant<int, TPS>{}, tts, sls, mss, std::true_type{});
            } else if (TPS * p < nseq) {  // a short last step: its first tile
                tile(std::integral_constant<int, 1>{}, tts, sls, mss, std::true_type{});
            }
            SC_STAMP(1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if NRK_SCAN_STAMP
        SC_STAMP(2);
        stamp_out();
#endif
        return;
    }

    // --------------------------------------------------------- book waves --
    // book wave wv books groups [gb, gb + UGB) of pair pw
    const int gb = ((wv - NPW) / NPW) * UGB;
    float eps_s[UGB], tau[UGB];
    float t[UGB][MT];
    bool live[UGB];
#pragma unroll
    for (int g = 0; g < UGB; ++g) {
        f16x8 uf[DS];
        float eps, scl;
        const int user = ubase + (gb + g) * 32 + q;
        scan_user_setup<DS>(users, n_users, dim, user, h, vmax, dvmax, sv_scale, uf, eps, scl, live[g]);
        eps_s[g] = eps * scl;
        if (h == 0 && user < n_users) uinfo[user] = make_float4(-INFINITY, eps_s[g], scl, eps);
        tau[g] = live[g] ? -FLT_MAX : INFINITY;
#pragma unroll
        for (int i = 0; i < MT; ++i) t[g][i] = (live[g] && i >= MT - 1 - jk) ? -INFINITY : INFINITY;
    }
    uint2* const wapp = app + (size_t)(ubase + gb * 32) * 2 * (size_t)m2;
    const uint32_t pos0 = (uint32_t)(q * 2 + h) * (uint32_t)m2;  // group 0's first slot
    const uint32_t gstride = 64u * (uint32_t)m2;                  // + g * gstride for group g
    uint32_t pos[UGB];
#pragma unroll
    for (int g = 0; g < UGB; ++g) pos[g] = pos0 + (uint32_t)g * gstride;
    auto slot = [&](uint32_t x, int g) { return min(x, pos0 + (uint32_t)g * gstride + (uint32_t)m2 - 1u); };
    auto app_store_if = [&](uint64_t m, uint32_t e, uint2 v) {
        const uint32_t off = e << 3;
        const uint64_t d = ((uint64_t)v.y << 32) | v.x;
        uint64_t sv;
        asm volatile(
            "s_and_saveexec_b64 %0, %1\n\t"
            "global_store_dwordx2 %2, %3, %4\n\t"
            "s_mov_b64 exec, %0"
            : "=&s"(sv)
            : "s"(m), "v"(off), "v"(d), "s"(wapp)
            : "memory", "scc");
    };
    auto retau = [&](int g) {
        const float lb = pair_min32(t[g][MT - 1]);
        const float c = lb - 2.0f * eps_s[g];
        const float tv = fmaxf(__builtin_fmaf(fabsf(c), -0x1p-22f, c) - 0x1p-120f, -FLT_MAX);
        tau[g] = live[g] ? tv : INFINITY;
    };
    int next_s = n_pre > 0 ? tile_lo : INT_MAX, left_s = n_pre;
#if NRK_SCAN_STAMP
    t_prev = __builtin_readcyclecounter();
#endif
    const uint32_t mq = mx_base + (uint32_t)(gb / 4) * 1024u;  // this wave's first group quad
    // r[b][c]: block b's maxima of group quad c of this wave
    f32x4 rr[TPS][TB][UGB / 4];
    auto read_issue = [&](int t, uint32_t a) {
        if constexpr (NB == 2) {
            asm volatile(
                "ds_read_b128 %0, %4 offset:0\n\tds_read_b128 %1, %4 offset:2048\n\t"
                "ds_read_b128 %2, %4 offset:4096\n\tds_read_b128 %3, %4 offset:6144"
                : "=&v"(rr[t][0][0]), "=&v"(rr[t][1][0]), "=&v"(rr[t][2][0]), "=&v"(rr[t][3][0])
                : "v"(a)
                : "memory");
        } else {
            asm volatile(
                "ds_read_b128 %0, %8 offset:0\n\tds_read_b128 %1, %8 offset:1024\n\t"
                "ds_read_b128 %2, %8 offset:2048\n\tds_read_b128 %3, %8 offset:3072\n\t"
                "ds_read_b128 %4, %8 offset:4096\n\tds_read_b128 %5, %8 offset:5120\n\t"
                "ds_read_b128 %6, %8 offset:6144\n\tds_read_b128 %7, %8 offset:7168"
                : "=&v"(rr[t][0][0]), "=&v"(rr[t][0][1]), "=&v"(rr[t][1][0]), "=&v"(rr[t][1][1]),
                  "=&v"(rr[t][2][0]), "=&v"(rr[t][2][1]), "=&v"(rr[t][3][0]), "=&v"(rr[t][3][1])
                : "v"(a)
                : "memory");
        }
    };
    // tile t's reads landed with `left' later reads still in flight (LDS
    // reads return in order: left = 0 or the reads of one more tile, TPS <= 2);
    // the wait ties rr[t], so nothing copies it earlier
    static_assert(TPS <= 2, "read_wait");
    auto read_wait = [&](int t, bool left) {
        constexpr int L1 = TB * (UGB / 4);
        if constexpr (NB == 2) {
            if (left)
                asm volatile("s_waitcnt lgkmcnt(%4)"
                             : "+v"(rr[t][0][0]), "+v"(rr[t][1][0]), "+v"(rr[t][2][0]), "+v"(rr[t][3][0])
                             : "n"(L1)
                             : "memory");
            else
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(rr[t][0][0]), "+v"(rr[t][1][0]), "+v"(rr[t][2][0]), "+v"(rr[t][3][0])::"memory");
        } else {
            if (left)
                asm volatile("s_waitcnt lgkmcnt(%8)"
                             : "+v"(rr[t][0][0]), "+v"(rr[t][0][1]), "+v"(rr[t][1][0]), "+v"(rr[t][1][1]),
                               "+v"(rr[t][2][0]), "+v"(rr[t][2][1]), "+v"(rr[t][3][0]), "+v"(rr[t][3][1])
                             : "n"(L1)
                             : "memory");
            else
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(rr[t][0][0]), "+v"(rr[t][0][1]), "+v"(rr[t][1][0]), "+v"(rr[t][1][1]),
                               "+v"(rr[t][2][0]), "+v"(rr[t][2][1]), "+v"(rr[t][3][0]), "+v"(rr[t][3][1])::"memory");
        }
    };
    // main-pass inserts every insp tiles (a power of two >= TPS; the host's
    // choice, see launch_scan_v)
    float vtp[UGB];  // INSP > 1: the largest tile maximum since the last insert, per group (-inf: none)
#pragma unroll
    for (int g = 0; g < UGB; ++g) vtp[g] = -INFINITY;
    for (int p = 0; p <= NP; ++p) {
        SC_STAMP(5);
        sync();
        SC_STAMP(0);
        if (p == 0) continue;
        const int p1 = p - 1;
#pragma unroll
        for (int t = 0; t < TPS; ++t)
            if (TPS * p1 + t < nseq) read_issue(t, mq + (uint32_t)(((p1 & 1) * TPS + t) * MXS));
        static_for<TPS>([&](auto tc) {
        constexpr int T = decltype(tc)::value;
        const int j = TPS * p1 + T;
        if (j >= nseq) return;
        read_wait(T, T + 1 < TPS && j + 1 < nseq);  // tile T + 1's reads may stay in flight
        const int tt = seq(j);
        const bool pre = j < n_pre;
        if (j == n_pre) {  // the first main-pass tile: tau from the pre-pass lists
#pragma unroll
            for (int g = 0; g < UGB; ++g) retau(g);
        }
        bool ins_ok = true;
        if (!pre && tt == next_s) {  // a sampled tile: its maxima are in the lists already
            ins_ok = false;
            next_s = --left_s > 0 ? next_s + pstride : INT_MAX;
        }
        const auto& r = rr[T];
        SC_STAMP(1);
#if NRK_SCAN_WS_FLOOR  // dev timing floor: the book waves only read the maxima
        if (r[0][0][0] != 12345.0f) return;
#endif
        const uint32_t hb0 = (uint32_t)(tt * TB * 2) + (uint32_t)h;
        // group g of the tile
        static_for<UGB>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            float mx[TB];
#pragma unroll
            for (int b = 0; b < TB; ++b) mx[b] = r[b][g / 4][g % 4];
            const float vt = fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3]));
            if (!pre) {
                // appends (ip_scan_seg's BSEL form): every half-block max >= tau
                uint64_t am[TB], gm = 0, multi = 0;
#pragma unroll
                for (int b = 0; b < TB; ++b) {
                    am[b] = __builtin_amdgcn_ballot_w64(mx[b] >= tau[g]);
                    multi |= gm & am[b];
                    gm |= am[b];
                }
                if (gm) {
                    const uint32_t fid = (first_set_block<TB>(am) << 1) + hb0;
                    const uint32_t p0 = pos[g];
                    app_store_if(gm, slot(p0, g), make_uint2(__float_as_uint(vt), fid));
                    uint32_t p = add_if(p0, gm);
                    if (multi) {
                        p = p0;
#pragma unroll
                        for (int b = 0; b < TB; ++b) {
                            app_store_if(am[b] & multi, slot(p, g), make_uint2(__float_as_uint(mx[b]), hb0 + 2u * b));
                            p = add_if(p, am[b]);
                        }
                    }
                    pos[g] = p;
                }
            }
            SC_STAMP(2);
            if (pre) {
                // pre-pass tiles insert every tile (they fill the list)
                const bool in = vt > t[g][MT - 1];
                if (__builtin_amdgcn_ballot_w64(in)) top_insert<MT>(t[g], in ? vt : -INFINITY);
            } else {
                // main pass: one insert per INSP tiles, the largest of their
                // tile maxima (a sampled tile's counts as -inf); the list stays
                // a set of distinct appended half-block maxima, so its (jk +
                // 1)-th largest stays a lower bound -- only tau lags by < INSP
                // tiles
                const float vi = fmaxf(ins_ok ? vt : -INFINITY, vtp[g]);
                if (T + 1 < TPS || ((j - n_pre) & (insp - 1)) < insp - TPS) {
                    vtp[g] = vi;
                } else {
                    vtp[g] = -INFINITY;
                    const bool in = vi > t[g][MT - 1];
                    if (__builtin_amdgcn_ballot_w64(in)) {
                        top_insert<MT>(t[g], in ? vi : -INFINITY);
                        if (!pre) retau(g);
                    }
                }
            }
            SC_STAMP(4);
        });
        });
    }
    {  // the maxima since the last insert
#pragma unroll
        for (int g = 0; g < UGB; ++g) {
            const bool in = vtp[g] > t[g][MT - 1];
            top_insert<MT>(t[g], in ? vtp[g] : -INFINITY);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if NRK_SCAN_STAMP
    SC_STAMP(3);
    stamp_out();
#endif
#pragma unroll
    for (int g = 0; g < UGB; ++g) {
        const float lb = pair_min32(t[g][MT - 1]);
        const int user = ubase + (gb + g) * 32 + q;
        if (user < n_users) {
            acnt[(size_t)user * 2 + h] = (int)(pos[g] - (pos0 + (uint32_t)g * gstride));
            if (h == 0) reinterpret_cast<float*>(uinfo + user)[0] = live[g] ? lb : -INFINITY;
        }
    }
    if constexpr (MT <= 32) {
        if (bnd != nullptr) {
#pragma unroll
            for (int g = 0; g < UGB; ++g)
                list_bound_out<MT>(t[g], live[g], h, ubase + (gb + g) * 32 + q, n_users, jk, bnd, bnd_m, uinfo);
        }
    }
}

// ordered uint32 key of a float (monotone; -inf > 0, padding key 0 below all)
__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b >> 31) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
    return __uint_as_float((k >> 31) ? (k & 0x7FFFFFFFu) : ~k);
}

// Descending ranks of the c keys of one wave's LDS row (0 = largest; equal
// keys by position): a lane holds keys at positions pos + 64 e and
// counts, over LDS broadcasts of all c keys (4 per read), the keys above its
// own.  The row must be zero-padded to a multiple of 4.  VALU-only work with
// independent steps -- the bitwise radix select it replaces (32 dependent
// ballot / scalar-count rounds per user) cost 0.2 ms per 250k users.
template <int E>
__device__ __forceinline__ void lds_ranks(const uint32_t* __restrict__ row, int c, const uint32_t (&mine)[E],
                                          int pos, int (&rank)[E]) {
    // pos = the row position of mine[0]; mine[e] sits at pos + 64 e
#pragma unroll
    for (int e = 0; e < E; ++e) rank[e] = 0;
    for (int j0 = 0; j0 < c; j0 += 4) {
        const uint4 q = *reinterpret_cast<const uint4*>(row + j0);
        const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int e = 0; e < E; ++e)
                rank[e] += (qq[t] > mine[e] || (qq[t] == mine[e] && j0 + t < e * WAVE + pos)) ? 1 : 0;
        }
    }
}

// 64 keys, one per lane, sorted descending by a wave bitonic network (21
// exchange stages through lane_xor: DPP / ds_swizzle / permlane swaps, one
// max-or-min each)
__device__ __forceinline__ uint32_t wave_sort_desc_u32(uint32_t x, int lane) {
    static_for<6>([&](auto klc) {
        constexpr int kl = decltype(klc)::value + 1, k = 1 << kl;
        static_for<kl>([&](auto jc) {
            constexpr int j = 1 << (kl - 1 - decltype(jc)::value);
            const uint32_t y = lane_xor<j>(x);
            const bool up = (lane & k) == 0;  // k = 64: every lane (descending overall)
            const bool lower = (lane & j) == 0;
            x = (lower == up) ? max(x, y) : min(x, y);
        });
    });
    return x;
}

// the key of rank r (r < c) of a wave's LDS row of c keys (see lds_ranks):
// up to 64 keys by one wave sort (~21 exchange stages; the rank count costs
// ~5 VALU per key per lane), more 64 at a time (a run-time loop: few
// registers whatever c is)
__device__ __forceinline__ uint32_t lds_select(uint32_t* __restrict__ row, int c, int r, int lane) {
    if (c <= WAVE) {
        wave_sync_lds();
        const uint32_t srt = wave_sort_desc_u32(lane < c ? row[lane] : 0u, lane);
        return (uint32_t)__builtin_amdgcn_readlane((int)srt, r);
    }
    if (lane < 4) row[c + lane] = 0u;  // zero pad (the row has room: c + 4 <= its size)
    wave_sync_lds();
    uint32_t x = 0u;
    for (int b0 = 0; b0 < c; b0 += WAVE) {
        const uint32_t mine[1] = {b0 + lane < c ? row[b0 + lane] : 0u};
        int rank[1];
        lds_ranks<1>(row, c, mine, b0 + lane, rank);
        const unsigned long long b = __ballot(b0 + lane < c && rank[0] == r);
        if (b) {
            x = (uint32_t)__shfl((int)mine[0], __ffsll((long long)b) - 1, WAVE);
            break;
        }
    }
    return x;
}

// The select and the shard kernels run persistent waves (a wave walks users
// wid, wid + nw, ...; the next user's counts / record are loaded during this one) and
// load a user's appended entries 256 at a time, all loads in flight at once:
// one wave per user was bound by per-wave start-up and dependent round trips.
// Workgroups per CU of those persistent grids: every one must be resident,
// or the queued ones run after the first finish (a second, thinner wave of
// work).  Their ~106 SGPRs admit 6 4-wave workgroups per CU, not 8
// (MI355X_MICROARCH.md: floor(800 / (ceil(sgpr / 16) 16 + 16)); the
// occupancy API says 7).  Dev A/B: -DNRK_SH_WG=8 (the round-5 grid).
#ifndef NRK_SH_WG
#define NRK_SH_WG 6
#endif
constexpr int SH_WG_PER_CU = NRK_SH_WG;
constexpr int SH_ENT = 4;  // entries per lane per load batch

__device__ __forceinline__ void sh_load(const uint2* s0, const uint2* s1, int a0, int n, int b0, int lane,
                                        uint2 (&ent)[SH_ENT]) {
#pragma unroll
    for (int j = 0; j < SH_ENT; ++j) {
        const int e = b0 + j * WAVE + lane;
        ent[j] = e < n ? (e < a0 ? s0[e] : s1[e - a0]) : make_uint2(0u, 0u);
    }
}

// Select: one wave per user.  theta = the exact k-th largest appended max:
// the entries >= theta_lb (at least 2 (jk + 1) >= k of them: every value a
// lane's final top list holds entered it at a position <= jk, above the tau
// of that moment, so it was appended) are held one key per lane slot and
// theta is built bit by bit (count of keys >= candidate by ballots).  The
// band = every appended entry >= cut = theta - 2 eps (rounded down); an
// item with exact score >= cut + eps has an fp16 score >= cut, so its
// half-block max was >= every tau of the scan and was appended.
__global__ __launch_bounds__(256) void ip_select_kernel(
    int64_t n_users, int k, int m2, int bandcap, const uint2* __restrict__ app,
    const int32_t* __restrict__ acnt, const float4* __restrict__ uinfo, uint2* __restrict__ cand,
    int32_t* __restrict__ cand_cnt, float2* __restrict__ ucut, int32_t* __restrict__ ovf_flag,
    int32_t* __restrict__ ovf_list, int32_t* __restrict__ ovf_count) {
    __shared__ __attribute__((aligned(16))) uint32_t sel[4][IP_SEL + 4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const unsigned long long lt = (1ull << lane) - 1ull;
    // persistent waves (see the shard kernels): the next user's counts and
    // record load during this one; entries load SH_ENT x 64 at a time (the
    // user's entries: list 0 [0, a0), then list 1 [0, a1))
    int64_t u = (int64_t)blockIdx.x * 4 + wave;
    int2 ac_n = make_int2(0, 0);
    float4 inf_n = make_float4(0.f, 0.f, 0.f, 0.f);
    if (u < n_users) {
        ac_n = reinterpret_cast<const int2*>(acnt)[u];
        inf_n = uinfo[u];
    }
    for (; u < n_users; u += nw) {
        const int a0 = ac_n.x, a1 = ac_n.y;
        const float4 inf = inf_n;
        if (u + nw < n_users) {
            ac_n = reinterpret_cast<const int2*>(acnt)[u + nw];
            inf_n = uinfo[u + nw];
        }
        bool ovf = a0 > m2 || a1 > m2;
        const int n = ovf ? 0 : a0 + a1;
        const uint2* s0 = app + (size_t)(2 * u) * m2;
        const uint2* s1 = s0 + m2;
        auto sh_load = [&](int n_, int b0, int lane_, uint2 (&ent)[SH_ENT]) {
#pragma unroll
            for (int j = 0; j < SH_ENT; ++j) {
                const int e = b0 + j * WAVE + lane_;
                const uint2* src = e < a0 ? s0 + e : s1 + (e - a0);
                ent[j] = e < n_ ? *src : make_uint2(0u, 0u);
            }
        };
        // pass 1: keys of the entries >= theta_lb
        int c = 0;
        uint2 ent[SH_ENT];
        for (int b0 = 0; b0 < n; b0 += SH_ENT * WAVE) {
            sh_load(n, b0, lane, ent);
#pragma unroll
            for (int j = 0; j < SH_ENT; ++j) {
                const int e = b0 + j * WAVE + lane;
                const float v = __uint_as_float(ent[j].x);
                const bool kp = e < n && v >= inf.x;
                const unsigned long long bal = __ballot(kp);
                const int pos = c + __popcll(bal & lt);
                if (kp && pos < IP_SEL) sel[wave][pos] = fkey(v);
                c += __popcll(bal);
            }
        }
        if (c > IP_SEL) ovf = true;
        float theta = -INFINITY;
        wave_sync_lds();
        if (!ovf && c >= k) {
            const uint32_t x = lds_select(sel[wave], c, k - 1, lane);
            theta = fkey_inv(x);
        }
        wave_sync_lds();  // the next user's keys overwrite sel
        float cut = theta;
        if (inf.y != 0.0f && theta != -INFINITY) cut = round_down_sub(theta, 2.0f * inf.y);
        // pass 2: the band (append order); a single batch is still in registers
        int nb = 0;
        uint2* bd = cand + (size_t)u * bandcap;
        for (int b0 = 0; b0 < n; b0 += SH_ENT * WAVE) {
            if (n > SH_ENT * WAVE) sh_load(n, b0, lane, ent);
#pragma unroll
            for (int j = 0; j < SH_ENT; ++j) {
                const int e = b0 + j * WAVE + lane;
                const bool kp = e < n && __uint_as_float(ent[j].x) >= cut;
                const unsigned long long bal = __ballot(kp);
                const int pos = nb + __popcll(bal & lt);
                if (kp && pos < bandcap) bd[pos] = ent[j];
                nb += __popcll(bal);
            }
        }
        if (nb > bandcap) ovf = true;
        if (lane == 0) {
            cand_cnt[u] = ovf ? 0 : nb;
            ucut[u] = make_float2(cut == -INFINITY ? -INFINITY : cut / inf.z, inf.w);
            ovf_flag[u] = ovf ? 1 : 0;
            if (ovf) ovf_list[atomicAdd(ovf_count, 1)] = (int32_t)u;
        }
    }
}

// k > IP_KFAST: every user takes the exact path
__global__ void ip_all_exact_kernel(int64_t n_users, int32_t* __restrict__ cand_cnt,
                                    int32_t* __restrict__ ovf_flag, int32_t* __restrict__ ovf_list,
                                    int32_t* __restrict__ ovf_count) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n_users;
         u += (int64_t)gridDim.x * blockDim.x) {
        cand_cnt[u] = 0;
        ovf_flag[u] = 1;
        ovf_list[u] = (int32_t)u;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *ovf_count = (int32_t)n_users;
}

// ------------------------------------------------------------ refinement --
__device__ __forceinline__ double exact_dot(const float* __restrict__ a, const float* __restrict__ b,
                                            int dim) {
    double s = 0.0;
    if ((dim & 31) == 0) {
        // 8 float4 of both rows in flight per step (a runtime-dim loop
        // otherwise waits on each row piece in turn); same sequential order
        const float4* a4 = reinterpret_cast<const float4*>(a);
        const float4* b4 = reinterpret_cast<const float4*>(b);
        for (int t0 = 0; t0 < dim / 4; t0 += 8) {
            float4 x[8], y[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                x[t] = a4[t0 + t];
                y[t] = b4[t0 + t];
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                s += (double)x[t].x * (double)y[t].x;
                s += (double)x[t].y * (double)y[t].y;
                s += (double)x[t].z * (double)y[t].z;
                s += (double)x[t].w * (double)y[t].w;
            }
        }
    } else if ((dim & 3) == 0) {
        const float4* a4 = reinterpret_cast<const float4*>(a);
        const float4* b4 = reinterpret_cast<const float4*>(b);
        for (int t = 0; t < dim / 4; ++t) {
            const float4 x = a4[t], y = b4[t];
            s += (double)x.x * (double)y.x;
            s += (double)x.y * (double)y.y;
            s += (double)x.z * (double)y.z;
            s += (double)x.w * (double)y.w;
        }
    } else {
        for (int t = 0; t < dim; ++t) s += (double)a[t] * (double)b[t];
    }
    return s + 0.0;
}

// DS4 = dim / 4 when the candidate rows are staged through LDS (dim 16, 32,
// 64): every 64-item round loads the rows with whole-row coalesced float4
// pieces (64 / DS4 rows per instruction) into a padded per-wave LDS stage,
// then each lane sums its own row sequentially (the oracle's order).
// DS4 = 0: the generic per-lane gather.  SV = exact survivors held per user
// (SV / 64 per lane in the final sort).
// the exact rounds' rows read per lane (dims <= 32) instead of staged
#ifndef NRK_REFINE_DIRECT
#define NRK_REFINE_DIRECT 1
#endif
constexpr bool REFINE_DIRECT = NRK_REFINE_DIRECT;
// waves per SIMD the refine's registers are sized for (dim 64's staged
// rounds take 2, the generic dims 4).  Round 6: two prefilter rounds in
// flight (three register slots rotated by unrolling) at 3 waves per SIMD
// measured slower than one round ahead at 4: finish 0.961-0.966 vs
// 0.873-0.884 ms (config 2, one box).  Then the user's fp16 row moved to LDS
// and the direct exact dot to two half-rows: dim 32 needs 80 VGPRs instead of
// 128, and finish went 0.871 -> 0.776 ms at 4 / 0.772 at 6 waves per SIMD
// (one box, two runs each)
#ifndef NRK_REFINE_WPE
#define NRK_REFINE_WPE 6
#endif
template <int DS4, int SV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DS4 == 16 ? 2 : DS4 == 0 ? 4 : NRK_REFINE_WPE))) void ip_refine_kernel(
    const float* __restrict__ users, int64_t n_users, const float* __restrict__ items,
    const uint8_t* __restrict__ catalog, int64_t n_items, int dim, int k, int64_t row_offset,
    const uint2* __restrict__ cand, int bandcap, const int32_t* __restrict__ cand_cnt,
    const float2* __restrict__ ucut, const int32_t* __restrict__ ovf_flag, int32_t* __restrict__ ovf_list,
    int32_t* __restrict__ ovf_count, float* __restrict__ out_s, int32_t* __restrict__ out_r,
    double* __restrict__ out_e, int n_src = 0,
    int64_t src_users = 0, int x_cap = 0, const int32_t* __restrict__ src_cnt = nullptr) {
    constexpr int SE = SV / WAVE;
    __shared__ Cand surv[4][SV];
    __shared__ int32_t krow[4][IP_KRING];
    constexpr int RS = DS4 + 1;  // staged row stride in float4 (one float4 of padding)
    __shared__ float4 stage[DS4 > 0 ? 4 : 1][DS4 > 0 ? 32 * RS : 1];  // half a round (32 rows) at a time
    __shared__ uint32_t bandq[4][SV + 32 > IP_BQ ? SV + 32 : IP_BQ];
    __shared__ __attribute__((aligned(16))) float ushl[4][DS4 > 0 ? 1 : 256];  // DS4 == 0: the user's fp16 values
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    if (u >= n_users) return;
    // one round trip for the per-user state: the overflow flag, the band
    // count and cut, the user's row and (select slots) the first 32 band
    // entries are loaded together before anything branches on them
    const bool slots = n_src == 0;  // kernel argument: uniform
    const float* uv = users + u * dim;
    const int32_t ovf_u = ovf_flag[u];
    const int nbd_slots = slots ? cand_cnt[u] : 0;
    const float2 ce = ucut[u];
    const float uv_r = uv[lane < dim ? lane : 0];  // unconditional (a branch around a load serialises the batch)
    // first 32 band slots (lanes 32-63 re-read slot 0: same line, no traffic)
    const uint2 ent0 = slots ? cand[(size_t)u * bandcap + (lane < 32 ? lane : 0)] : make_uint2(0u, 0u);
    if (ovf_u) return;
    // band: per-user slots of the select (n_src == 0), or the fixed-slot
    // exchange of the catalog-sharded owner protocol (n_src > 0): source s's
    // entries at
    // cand[(s * src_users + u) * x_cap + j], j < src_cnt[s * src_users + u]
    int src_n = 0;  // lane s < n_src: source s's count
    int nsrc_tot = 0;
    if (n_src > 0) {
        for (int s0 = 0; s0 < n_src; s0 += WAVE) {
            const int sl = s0 + lane;
            const int c = sl < n_src ? max(0, src_cnt[(int64_t)sl * src_users + u]) : 0;
            if (s0 == 0) src_n = c;
            nsrc_tot += (int)wave_sum_f32((float)c);
        }
    }
    if (nsrc_tot > IP_BQ) {
        // more than the LDS holds: exact path
        if ((threadIdx.x & 63) == 0) ovf_list[atomicAdd(ovf_count, 1)] = (int32_t)u;
        return;
    }
    // zero user: every score is exactly 0 -> the lowest rows win the ties
    const float uv_l = lane < dim ? uv_r : 0.0f;
    float nz = fabsf(uv_l), uam = fabsf(uv_l);
    for (int d = lane + WAVE; d < dim; d += WAVE) {
        nz += fabsf(uv[d]);
        uam = fmaxf(uam, fabsf(uv[d]));
    }
    nz = wave_sum_f32(nz);
    if (nz == 0.0f) {
        for (int i = lane; i < k; i += WAVE) {
            const bool ok = i < n_items;
            out_s[u * k + i] = ok ? 0.0f : -FLT_MAX;
            out_r[u * k + i] = ok ? (int32_t)(i + row_offset) : -1;
            if (out_e) out_e[u * k + i] = ok ? 0.0 : -INFINITY;
        }
        return;
    }
    const int nbd = n_src > 0 ? 0 : nbd_slots;
    const uint2* bd = cand + (size_t)u * bandcap;
    double thr = -INFINITY;
    if (ce.x != -INFINITY) {
        thr = (double)ce.x + (double)ce.y;
        thr = thr - fabs(thr) * 1e-15 - 1e-300;  // round down
    }
    // The cut in the screen's scaled fp16 units (exact power-of-two rescale):
    // |fp16 score - exact| <= eps, so every item with exact >= cut + eps has
    // an fp16 score >= cut.  Used twice: (a) band entries (half-blocks) whose
    // listed fp16 max is below it are dropped -- none on one GPU (the select
    // kept only entries >= cut), most of the band on a catalog shard after
    // nrk_ip_topk_apply_bound raised the cut to the global bound; (b) the
    // fp16 prefilter (DS4 > 0): every band item's fp16 score recomputed from
    // its 64-B packed row, only items reaching the cut are fetched in fp32
    // for the exact score.
    constexpr int DSK = DS4 / 4;  // 16-dim k-steps of the packed layout
    const bool pre = catalog != nullptr && ce.x != -INFINITY;
    // the user's fp16 values, read 8 at a time by the prefilter (wave-uniform:
    // in registers they held 4 DS4 / 2 VGPRs for the whole kernel)
    __shared__ __attribute__((aligned(16))) _Float16 ushs[4][DS4 > 0 ? 4 * DS4 : 8];
    _Float16* ush = ushs[wave];
    float pcut = 0.0f;
    if (pre) {
        const int dpc = pad_dim(dim);
        const int64_t nblk_c = (n_items + 31) >> 5;
        const CatalogHdr* hdr = reinterpret_cast<const CatalogHdr*>(catalog + (size_t)nblk_c * 64 * dpc);
        float ua = uam;  // max |u_d| (order-free: the same value as a sequential max)
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) ua = fmaxf(ua, __shfl_xor(ua, m, WAVE));
        const float su = pow2_scale(ua);
        if constexpr (DS4 > 0) {
#pragma unroll
            for (int d = lane; d < 4 * DS4; d += WAVE) ush[d] = (_Float16)(uv[d] * su);
            wave_sync_lds();
        }
        pcut = ce.x * (su * hdr->scale);
    }
    // (a) compact the band into LDS (list order kept; sources in rank order)
    int nband = 0;
    auto take_one = [&](uint2 ent, int e, int cnt) {
        const bool kp = e < cnt && (!pre || __uint_as_float(ent.x) >= pcut);
        const unsigned long long bal = __ballot(kp);
        if (kp) bandq[wave][nband + __popcll(bal & ((1ull << lane) - 1ull))] = ent.y;
        nband += __popcll(bal);
    };
    auto take = [&](const uint2* __restrict__ src, int cnt) {
        int b0 = 0;
        if (slots) {  // the first 32 entries were loaded with the user's state
            take_one(ent0, lane < 32 ? lane : cnt, cnt);
            b0 = 32;
        }
        for (; b0 < cnt; b0 += WAVE) {
            const int e = b0 + lane;
            take_one(e < cnt ? src[e] : make_uint2(0u, 0u), e, cnt);
        }
    };
    if (n_src > 0) {
        // the exchange carries bare half-block ids (each source already
        // filtered at its own cut, >= the global bound - eps)
        const uint32_t* ids = reinterpret_cast<const uint32_t*>(cand);
        for (int s2 = 0; s2 < n_src; ++s2) {
            const int c2 = s2 < WAVE ? __shfl(src_n, s2, WAVE) : max(0, src_cnt[(int64_t)s2 * src_users + u]);
            const uint32_t* src = ids + ((size_t)s2 * src_users + u) * x_cap;
            for (int b0 = 0; b0 < c2; b0 += WAVE) {
                const int e = b0 + lane;
                if (e < c2) bandq[wave][nband + e] = src[e];
                nband += min(WAVE, c2 - b0);
            }
        }
    } else {
        take(bd, nbd);
    }
    wave_sync_lds();
    const int nitem = nband * 16;
    int cnt = 0;
    auto push = [&](bool keep, double s, int32_t row) {
        const unsigned long long bal = __ballot(keep);
        const int pos = cnt + __popcll(bal & ((1ull << lane) - 1ull));
        if (keep && pos < SV) surv[wave][pos] = Cand{s, row};
        cnt += __popcll(bal);
    };
    if constexpr (DS4 > 0) {
        // Two phases over the band.  (A) fp16 prefilter in 64-item rounds,
        // software-pipelined: round i+1's packed fp16 pieces are in flight
        // while round i is scored; the kept items' rows go to a per-wave LDS
        // ring.  (B) whenever the ring holds 64 rows (and once at the end),
        // one exact round: the rows staged through LDS with whole-row
        // coalesced float4 pieces, each lane summing its own row sequentially
        // (the oracle's order).
        uint4 pc[DSK > 0 ? 2 * DSK : 1];
        auto band_q = [&](int base) -> uint32_t {
            int idx = base + lane;
            idx = idx < nitem ? idx : nitem - 1;
            return bandq[wave][idx > 0 ? idx >> 4 : 0];
        };
        // the prefilter reads the half-block-major copy: item r of band
        // entry qv is the 8 DS4-B row at ((qv * 16 + r) * 8 DS4), the 16
        // items of a half-block one contiguous run
        const uint8_t* hbc = catalog ? catalog + catalog_hb_offset(n_items, 4 * DS4) : nullptr;
        int64_t hoff = 0;
        auto item_row = [&](int base, uint32_t qv, int32_t& row, bool& inb) {
            const int idx = base + lane, r = idx & 15;
            const int64_t rr = (int64_t)(qv >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (qv & 1);
            inb = idx < nitem && rr < n_items;
            row = inb ? (int32_t)rr : 0;
            hoff = inb ? ((int64_t)qv * 16 + r) * (8 * DS4) : 0;
        };
        auto pieces = [&](int32_t) {
            if (pre) {
                const uint8_t* bp = hbc + hoff;
#pragma unroll
                for (int st = 0; st < DSK; ++st)
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh)
                        pc[2 * st + hh] = *reinterpret_cast<const uint4*>(bp + 32 * st + 16 * hh);
            }
        };
        int kc = 0, ko = 0;  // ring fill / read positions (wave-uniform)
        // rows staged 32 at a time (half the LDS of a whole round: four
        // workgroups per CU instead of three)
        auto exact_round = [&](int m) {
            const int32_t rl = lane < m ? krow[wave][(ko + lane) & (IP_KRING - 1)] : -1;
            double sd = 0.0;
            bool keep = false;
            if constexpr (REFINE_DIRECT && DS4 <= 8) {
                // every lane reads its own row (one 128-B line at D = 32) and
                // sums it: no LDS stage and no half-idle passes (config 2:
                // finish 0.91 -> 0.87 ms).  D = 64 keeps the staged rounds
                // (its 16 float4 per lane spilled)
                if (rl >= 0) {
                    const float4* a4 = reinterpret_cast<const float4*>(uv);
                    const float4* b4 = reinterpret_cast<const float4*>(items + (int64_t)rl * dim);
                    constexpr int YH = DS4 > 4 ? DS4 / 2 : DS4;  // half-rows: fewer live VGPRs
                    double acc = 0.0;
#pragma unroll
                    for (int t0 = 0; t0 < DS4; t0 += YH) {
                        float4 y[YH];
#pragma unroll
                        for (int t = 0; t < YH; ++t) y[t] = b4[t0 + t];
#pragma unroll
                        for (int t = 0; t < YH; ++t) {
                            const float4 x = a4[t0 + t];
                            acc += (double)x.x * (double)y[t].x;
                            acc += (double)x.y * (double)y[t].y;
                            acc += (double)x.z * (double)y[t].z;
                            acc += (double)x.w * (double)y[t].w;
                        }
                    }
                    sd = acc + 0.0;
                    keep = sd >= thr;
                }
                push(keep, sd, rl);
                ko += m;
                return;
            }
#pragma unroll
            for (int hp = 0; hp < 2; ++hp) {
                float4 v[DS4 / 2];
                bool okv[DS4 / 2];
#pragma unroll
                for (int it = 0; it < DS4 / 2; ++it) {
                    const int g = it * 64 + lane, item = 32 * hp + g / DS4, part = g % DS4;
                    const int r_item = __shfl(rl, item, WAVE);
                    okv[it] = r_item >= 0;
                    v[it] = reinterpret_cast<const float4*>(items + (int64_t)(okv[it] ? r_item : 0) * dim)[part];
                }
#pragma unroll
                for (int it = 0; it < DS4 / 2; ++it) {
                    const int g = it * 64 + lane, part = g % DS4;
                    stage[wave][(g / DS4) * RS + part] = okv[it] ? v[it] : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                wave_sync_lds();
                if ((lane >> 5) == hp && rl >= 0) {
                    const float4* a4 = reinterpret_cast<const float4*>(uv);
                    const float4* b4 = &stage[wave][(lane & 31) * RS];
                    double acc = 0.0;
#pragma unroll
                    for (int t = 0; t < DS4; ++t) {
                        const float4 x = a4[t], y = b4[t];
                        acc += (double)x.x * (double)y.x;
                        acc += (double)x.y * (double)y.y;
                        acc += (double)x.z * (double)y.z;
                        acc += (double)x.w * (double)y.w;
                    }
                    sd = acc + 0.0;
                    keep = sd >= thr;
                }
                wave_sync_lds();  // the stage is rewritten next
            }
            push(keep, sd, rl);
            ko += m;
        };
        int32_t row;
        bool inb;
        item_row(0, band_q(0), row, inb);
        pieces(row);
        uint32_t q1 = band_q(WAVE < nitem ? WAVE : 0);
        for (int base = 0; base < nitem; base += WAVE) {
            // (A) fp16 prefilter of this round: every band item's scaled fp16
            // score from its 64-B packed row, kept when it reaches the cut
            // (|fp16 score - exact| <= eps as in the screen)
            bool keep = inb;
            if (pre && inb) {
                float acc = 0.0f;
#pragma unroll
                for (int st = 0; st < DSK; ++st)
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        const f16x8 hv = __builtin_bit_cast(f16x8, pc[2 * st + hh]);
                        const f16x8 uh = *reinterpret_cast<const f16x8*>(&ush[16 * st + 8 * hh]);
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            acc = fmaf((float)hv[e], (float)uh[e], acc);  // exact product: fma_mix
                    }
                keep = acc >= pcut;
            }
            const int32_t row_cur = row;
            // next round's rows and packed pieces, then the band entries of
            // the round after it
            const int nb = base + WAVE;
            if (nb < nitem) {
                item_row(nb, q1, row, inb);
                pieces(row);
                q1 = band_q(nb + WAVE < nitem ? nb + WAVE : nb);
            }
            const unsigned long long bal = __ballot(keep);
            if (keep) krow[wave][(kc + __popcll(bal & ((1ull << lane) - 1ull))) & (IP_KRING - 1)] = row_cur;
            kc += __popcll(bal);
            wave_sync_lds();
            // (B) exact rounds on full 64-row chunks
            while (kc - ko >= WAVE) exact_round(WAVE);
        }
        while (kc > ko) exact_round(kc - ko < WAVE ? kc - ko : WAVE);
    } else {
        // any dim: the fp16 prefilter reads each band item's packed pieces
        // (pad_dim / 16 k-steps of two 16-B pieces) against the user's fp16
        // values held in LDS, and only items reaching the cut get the exact
        // fp64 dot (per lane, the oracle's sequential order)
        const int dpc = pad_dim(dim), dskc = dpc / 16;
        if (pre) {
            float ua = 0.0f;
            for (int d = 0; d < dim; ++d) ua = fmaxf(ua, fabsf(uv[d]));
            const float s2 = pow2_scale(ua);
            for (int d = lane; d < dpc; d += WAVE) ushl[wave][d] = d < dim ? (float)(_Float16)(uv[d] * s2) : 0.0f;
            wave_sync_lds();
        }
        // items reaching the cut wait in the krow ring; whole 64-row exact
        // rounds drain it (round 6: the exact dot ran inside each 64-item
        // prefilter round, so a round with one kept lane paid a whole
        // sequential fp64 row chain -- dim 128's refine: ~8 chains per user)
        int kc = 0, ko = 0;
        auto exact_generic = [&](int m) {
            const int32_t rl = lane < m ? krow[wave][(ko + lane) & (IP_KRING - 1)] : -1;
            double sd = 0.0;
            bool keep = false;
            if (rl >= 0) {
                sd = exact_dot(uv, items + (int64_t)rl * dim, dim);
                keep = sd >= thr;
            }
            push(keep, sd, rl);
            ko += m;
        };
        for (int base = 0; base < nitem; base += WAVE) {
            const int idx = base + lane;
            bool keep = false;
            int32_t row = 0;
            if (idx < nitem) {
                const int bb = idx >> 4, r = idx & 15;
                const uint32_t qv = bandq[wave][bb];
                const int64_t rr = (int64_t)(qv >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (qv & 1);
                if (rr < n_items) row = (int32_t)rr;
                keep = rr < n_items;
                if (keep && pre) {
                    const uint8_t* bp = catalog + (size_t)(rr >> 5) * (64 * dpc);
                    const int il = (int)(rr & 31);
                    float acc = 0.0f;
                    for (int st = 0; st < dskc; ++st) {
                        const f16x8 h0 = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(bp + st * 1024 + il * 16));
                        const f16x8 h1 =
                            __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(bp + st * 1024 + (il + 32) * 16));
                        const float* us = &ushl[wave][16 * st];
#pragma unroll
                        for (int e = 0; e < 8; ++e) acc = fmaf((float)h0[e], us[e], acc);
#pragma unroll
                        for (int e = 0; e < 8; ++e) acc = fmaf((float)h1[e], us[8 + e], acc);
                    }
                    keep = acc >= pcut;
                }
            }
            const unsigned long long bal = __ballot(keep);
            if (keep) krow[wave][(kc + __popcll(bal & ((1ull << lane) - 1ull))) & (IP_KRING - 1)] = row;
            kc += __popcll(bal);
            wave_sync_lds();
            while (kc - ko >= WAVE) exact_generic(WAVE);
        }
        while (kc > ko) exact_generic(kc - ko < WAVE ? kc - ko : WAVE);
    }
    if (cnt > SV) {  // dense exact ties: hand the user to the exact fallback
        if (lane == 0) ovf_list[atomicAdd(ovf_count, 1)] = (int32_t)u;
        return;
    }
    wave_sync_lds();
    // survivors ordered (score desc, row asc); the first k are the output
    auto emit = [&](const Cand* x, int ne) {
        for (int e = 0; e < ne; ++e) {
            const int idx = e * 64 + lane;
            if (idx < k) {
                const bool ok = x[e].row != INT32_MAX;
                out_s[u * k + idx] = ok ? (float)x[e].s : -FLT_MAX;
                out_r[u * k + idx] = ok ? (int32_t)(x[e].row + row_offset) : -1;
                if (out_e) out_e[u * k + idx] = ok ? x[e].s : -INFINITY;
            }
        }
    };
    if (SE > 1 && cnt <= WAVE && k <= WAVE) {
        // up to 64 survivors (nearly every user at config 2): one per lane, a
        // 64-wide sort -- 21 shuffle stages instead of the SV-wide sort's 28 x
        // SE (finish 1.27 -> 0.93 ms; rank counting over LDS broadcasts: 0.94)
        Cand x1[1];
        if (lane < cnt) x1[0] = surv[wave][lane];
        else { x1[0].s = -INFINITY; x1[0].row = INT32_MAX; }
        wave_bitonic_sort<1>(x1);
        emit(x1, 1);
        return;
    }
    Cand x[SE];
#pragma unroll
    for (int e = 0; e < SE; ++e) {
        const int idx = e * 64 + lane;
        if (idx < cnt) x[e] = surv[wave][idx];
        else { x[e].s = -INFINITY; x[e].row = INT32_MAX; }
    }
    wave_bitonic_sort<SE>(x);
    emit(x, SE);
}

// -------------------------------------------------------------- fallback --
__device__ __forceinline__ uint64_t okey(double s) {
    const uint64_t b = (uint64_t)__double_as_longlong(s);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// The exact path (k > 128, overflowed bands, zero-band shards): one
// workgroup per listed user, FB_GRID workgroups, each with its own scratch
// row of n_items keys.  Every exact fp64 score is computed ONCE and stored
// as the ordered key of its fp32 rounding (monotone: a larger fp32 key means
// a larger exact score); a 3-pass radix select (11 / 11 / 10 bits, LDS
// histograms, wave-aggregated counts) finds the kk-th largest key T; every
// item with key >= T is a candidate (the top kk are among them), its exact
// score is recomputed and an LDS bitonic sort on (score desc, row asc)
// picks the kk.  Users with more candidates than the sort holds (many fp32
// ties, e.g. an all-zero user) go to slow_list for ip_fallback_kernel.
constexpr int FB_GRID = 256;

__global__ __launch_bounds__(256) void ip_exact_kernel(
    const float* __restrict__ users, const float* __restrict__ items, int64_t n_items, int dim, int k, int ns,
    int64_t row_offset, const int32_t* __restrict__ ovf_list, const int32_t* __restrict__ ovf_count,
    float* __restrict__ out_s, int32_t* __restrict__ out_r, double* __restrict__ out_e,
    uint32_t* __restrict__ scratch, int32_t* __restrict__ slow_list, int32_t* __restrict__ slow_count) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    Cand* sel = reinterpret_cast<Cand*>(dyn);
    __shared__ unsigned int hist[2048];
    __shared__ unsigned int part[256];
    __shared__ int s_bin, s_krem, s_eq, sel_n;
    const int tid = threadIdx.x, lane = tid & 63;
    const int cnt = *ovf_count;
    const int kk = (int)(n_items < k ? n_items : k);
    uint32_t* key = scratch + (size_t)blockIdx.x * n_items;
    for (int qi = blockIdx.x; qi < cnt; qi += gridDim.x) {
        const int64_t u = ovf_list[qi];
        const float* uv = users + u * dim;
        for (int64_t r = tid; r < n_items; r += 256) key[r] = fkey((float)exact_dot(uv, items + r * dim, dim));
        __syncthreads();
        uint32_t prefix = 0, mask = 0;
        int krem = kk;
        for (int p = 0; p < 3; ++p) {
            const int wbits = p < 2 ? 11 : 10, sh = p == 0 ? 21 : (p == 1 ? 10 : 0);
            const uint32_t nbm = (1u << wbits) - 1u;
            for (int i = tid; i < 2048; i += 256) hist[i] = 0u;
            __syncthreads();
            for (int64_t r0 = 0; r0 < n_items; r0 += 256) {
                const int64_t r = r0 + tid;
                const uint32_t kv = r < n_items ? key[r] : 0u;
                const bool act = r < n_items && (kv & mask) == prefix;
                const uint32_t b = (kv >> sh) & nbm;
                unsigned long long pend = __ballot(act);
                while (pend) {  // one LDS atomic per distinct bin of the wave
                    const int l = __ffsll((long long)pend) - 1;
                    const uint32_t bl = (uint32_t)__shfl((int)b, l, WAVE);
                    const unsigned long long same = __ballot(act && b == bl) & pend;
                    if (lane == l) atomicAdd(&hist[bl], (unsigned int)__popcll(same));
                    pend &= ~same;
                }
            }
            __syncthreads();
            {
                unsigned int sum = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) sum += hist[8 * tid + j];
                part[tid] = sum;
            }
            __syncthreads();
            if (tid == 0) {
                int cum = 0, t = 255;
                for (; t > 0; --t) {
                    if (cum + (int)part[t] >= krem) break;
                    cum += part[t];
                }
                int b = 8 * t + 7;
                for (; b > 8 * t; --b) {
                    if (cum + (int)hist[b] >= krem) break;
                    cum += hist[b];
                }
                s_bin = b;
                s_krem = krem - cum;
                s_eq = (int)hist[b];
            }
            __syncthreads();
            prefix |= (uint32_t)s_bin << sh;
            mask |= nbm << sh;
            krem = s_krem;
        }
        // prefix = T, the kk-th largest key; s_eq = #(key == T)
        const int n_cand = (kk - krem) + s_eq;
        if (n_cand > ns) {
            if (tid == 0) slow_list[atomicAdd(slow_count, 1)] = (int32_t)u;
            __syncthreads();
            continue;
        }
        if (tid == 0) sel_n = 0;
        __syncthreads();
        for (int64_t r = tid; r < n_items; r += 256) {
            if (key[r] >= prefix) {
                const int pos = atomicAdd(&sel_n, 1);
                sel[pos] = Cand{exact_dot(uv, items + r * dim, dim), (int32_t)r};
            }
        }
        __syncthreads();
        for (int i = n_cand + tid; i < ns; i += 256) sel[i] = Cand{-INFINITY, INT32_MAX};
        __syncthreads();
        for (int sz = 2; sz <= ns; sz <<= 1) {
            for (int st = sz >> 1; st > 0; st >>= 1) {
                for (int i = tid; i < ns / 2; i += 256) {
                    const int lo = 2 * st * (i / st) + (i % st), hi = lo + st;
                    const bool up = (lo & sz) == 0;
                    const Cand a = sel[lo], b = sel[hi];
                    if (up ? better(b, a) : better(a, b)) {
                        sel[lo] = b;
                        sel[hi] = a;
                    }
                }
                __syncthreads();
            }
        }
        for (int i = tid; i < k; i += 256) {
            const bool ok = i < kk;
            out_s[u * k + i] = ok ? (float)sel[i].s : -FLT_MAX;
            out_r[u * k + i] = ok ? (int32_t)(sel[i].row + row_offset) : -1;
            if (out_e) out_e[u * k + i] = ok ? sel[i].s : -INFINITY;
        }
        __syncthreads();
    }
}

// One workgroup per listed user: the k-th largest exact key by an 8-bit
// radix select over the whole catalog (8 histogram passes), then the items
// above it plus the first ties in row order (k winners in all), ordered by
// an LDS bitonic sort of ns = next_pow2(max(k, 64)) entries (dynamic LDS).
__global__ __launch_bounds__(256) void ip_fallback_kernel(
    const float* __restrict__ users, const float* __restrict__ items, int64_t n_items, int dim,
    int k, int ns, int64_t row_offset, const int32_t* __restrict__ ovf_list,
    const int32_t* __restrict__ ovf_count, float* __restrict__ out_s, int32_t* __restrict__ out_r,
    double* __restrict__ out_e) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    Cand* sel = reinterpret_cast<Cand*>(dyn);
    __shared__ unsigned int hist[256];
    __shared__ int sel_n;
    __shared__ unsigned long long s_prefix;
    __shared__ int s_krem;
    __shared__ int wcnt[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cnt = *ovf_count;
    const int kk = (int)(n_items < k ? n_items : k);
    for (int qi = blockIdx.x; qi < cnt; qi += gridDim.x) {
        const int64_t u = ovf_list[qi];
        const float* uv = users + u * dim;
        unsigned long long prefix = 0, mask = 0;
        int krem = kk;
        for (int pass = 7; pass >= 0 && kk > 0; --pass) {
            hist[tid] = 0;
            __syncthreads();
            for (int64_t r = tid; r < n_items; r += 256) {
                const uint64_t key = okey(exact_dot(uv, items + r * dim, dim));
                if ((key & mask) == prefix) atomicAdd(&hist[(key >> (8 * pass)) & 255], 1u);
            }
            __syncthreads();
            if (tid == 0) {
                int cum = 0, b = 255;
                for (; b > 0; --b) {
                    if (cum + (int)hist[b] >= krem) break;
                    cum += hist[b];
                }
                s_prefix = prefix | ((unsigned long long)b << (8 * pass));
                s_krem = krem - cum;
            }
            __syncthreads();
            prefix = s_prefix;
            krem = s_krem;
            mask |= 0xFFull << (8 * pass);
        }
        if (tid == 0) sel_n = 0;
        __syncthreads();
        int taken = 0;
        for (int64_t c0 = 0; c0 < n_items && kk > 0; c0 += 256) {
            const int64_t r = c0 + tid;
            double s = 0.0;
            uint64_t key = 0;
            const bool valid = r < n_items;
            if (valid) {
                s = exact_dot(uv, items + r * dim, dim);
                key = okey(s);
            }
            const bool gt = valid && key > prefix;
            const bool eq = valid && key == prefix;
            if (gt) {
                const int pos = atomicAdd(&sel_n, 1);
                sel[pos] = Cand{s, (int32_t)r};
            }
            const unsigned long long bal = __ballot(eq);
            if (lane == 0) wcnt[wave] = __popcll(bal);
            __syncthreads();
            int before = taken;
            for (int w = 0; w < wave; ++w) before += wcnt[w];
            before += __popcll(bal & ((1ull << lane) - 1ull));
            if (eq && before < krem) {
                const int pos = atomicAdd(&sel_n, 1);
                sel[pos] = Cand{s, (int32_t)r};
            }
            taken += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
            __syncthreads();
        }
        __syncthreads();
        const int nsel = sel_n;
        for (int i = nsel + tid; i < ns; i += 256) sel[i] = Cand{-INFINITY, INT32_MAX};
        __syncthreads();
        // bitonic sort of sel[0, ns), best first
        for (int sz = 2; sz <= ns; sz <<= 1) {
            for (int st = sz >> 1; st > 0; st >>= 1) {
                for (int i = tid; i < ns / 2; i += 256) {
                    const int lo = 2 * st * (i / st) + (i % st), hi = lo + st;
                    const bool up = (lo & sz) == 0;
                    const Cand a = sel[lo], b = sel[hi];
                    if (up ? better(b, a) : better(a, b)) {
                        sel[lo] = b;
                        sel[hi] = a;
                    }
                }
                __syncthreads();
            }
        }
        for (int i = tid; i < k; i += 256) {
            const bool ok = i < kk;
            out_s[u * k + i] = ok ? (float)sel[i].s : -FLT_MAX;
            out_r[u * k + i] = ok ? (int32_t)(sel[i].row + row_offset) : -1;
            if (out_e) out_e[u * k + i] = ok ? sel[i].s : -INFINITY;
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------- merge --
// One wave per user.  E = 1, 2, 4: the n_lists * k_in entries in registers
// (E per lane); E = 0: in the wave's dynamic-LDS region of NS entries.
template <int E>
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const double* __restrict__ in_e, const int32_t* __restrict__ in_r, int n_lists,
    int64_t stride, int64_t n_users, int k_in, int k_out, int ns, float* __restrict__ out_s,
    int32_t* __restrict__ out_r, double* __restrict__ out_e) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    if (u >= n_users) return;
    auto load = [&](int idx) -> Cand {
        Cand c{-INFINITY, INT32_MAX};
        const int l = idx / k_in, j = idx - l * k_in;
        if (l < n_lists) {
            const int64_t o = l * stride + u * k_in + j;
            const int32_t r = in_r[o];
            if (r >= 0) c = Cand{in_e[o], r};
        }
        return c;
    };
    auto store = [&](int idx, const Cand& c) {
        const bool ok = c.row != INT32_MAX;
        out_s[u * k_out + idx] = ok ? (float)c.s : -FLT_MAX;
        out_r[u * k_out + idx] = ok ? c.row : -1;
        if (out_e) out_e[u * k_out + idx] = ok ? c.s : -INFINITY;
    };
    if constexpr (E > 0) {
        Cand x[E];
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = load(e * 64 + lane);
        wave_bitonic_sort<E>(x);
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (e * 64 + lane < k_out) store(e * 64 + lane, x[e]);
    } else {
        Cand* x = reinterpret_cast<Cand*>(dyn) + (size_t)wave * ns;
        for (int i = lane; i < ns; i += WAVE) x[i] = load(i);
        wave_lds_sort(x, ns);
        for (int i = lane; i < k_out; i += WAVE) store(i, x[i]);
    }
}

// ------------------------------------------------- catalog-shard bound --
// Per user, the m largest band maxima of this shard as exact lower bounds: a
// half-block whose fp16 max is x (scaled units, scl = su * catalog scale)
// holds an item with exact score >= x / scl - eps.  Distinct half-blocks are
// distinct items, so any k of these values bound k distinct items from
// below.  Descending, -inf padded (fp32, rounded down).  One wave per user;
// E = 1, 2, 4: the band in registers, E = 0: in dynamic LDS (ns per wave).
template <int E>
__global__ __launch_bounds__(256) void ip_bound_kernel(const float* __restrict__ users, int64_t n_users, int dim,
                                                       const CatalogHdr* __restrict__ hdr,
                                                       const uint2* __restrict__ cand, int bandcap,
                                                       const int32_t* __restrict__ cand_cnt,
                                                       const float2* __restrict__ ucut, int m, int ns,
                                                       float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    if (u >= n_users) return;
    const int nb = cand_cnt[u];
    const float* uv = users + u * dim;
    float ua = 0.0f;
    for (int d = lane; d < dim; d += WAVE) ua = fmaxf(ua, fabsf(uv[d]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ua = fmaxf(ua, __shfl_xor(ua, o, WAVE));
    const double inv = 1.0 / ((double)pow2_scale(ua) * (double)hdr->scale);  // exact power of two
    const double eps = (double)ucut[u].y;
    auto load = [&](int i) -> Cand {
        Cand c{-INFINITY, INT32_MAX};
        if (i < nb) {
            const double tv = (double)__uint_as_float(cand[(size_t)u * bandcap + i].x) * inv - eps;
            float v = (float)tv;
            if ((double)v > tv) v = nextafterf(v, -INFINITY);
            c = Cand{(double)v, i};
        }
        return c;
    };
    if constexpr (E > 0) {
        Cand x[E];
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = load(e * 64 + lane);
        wave_bitonic_sort<E>(x);
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (e * 64 + lane < m) out[u * m + e * 64 + lane] = (float)x[e].s;
    } else {
        Cand* x = reinterpret_cast<Cand*>(dyn) + (size_t)wave * ns;
        for (int i = lane; i < ns; i += WAVE) x[i] = load(i);
        wave_lds_sort(x, ns);
        for (int i = lane; i < m; i += WAVE) out[u * m + i] = (float)x[i].s;
    }
}

// G = the k-th largest of the n_lists * m bounds of the user (lists laid out
// [n_lists][n_users][m]; -inf when there are fewer than k finite values) is a
// lower bound of the user's k-th exact score over the whole catalog.  Raise
// the shard's cut to G - eps (rounded down to fp32): the refine then keeps
// exact >= cut + eps <= G, and the band / prefilter tests use the raised cut.
// One wave per user (values in registers for E = 1, 2, 4, in LDS for E = 0).
template <int E>
__global__ __launch_bounds__(256) void ip_apply_bound_kernel(float2* __restrict__ ucut, int64_t n_users,
                                                             const float* __restrict__ vals, int n_lists,
                                                             int m, int k, int ns) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    if (u >= n_users) return;
    auto load = [&](int i) -> Cand {
        Cand c{-(double)INFINITY, i};
        if (i < n_lists * m) {
            const int l = i / m, j = i - l * m;
            c.s = (double)vals[((int64_t)l * n_users + u) * m + j];
        }
        return c;
    };
    double G = -(double)INFINITY;
    if constexpr (E > 0) {
        Cand x[E];
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = load(e * 64 + lane);
        wave_bitonic_sort<E>(x);
#pragma unroll
        for (int e = 0; e < E; ++e)
            if ((k - 1) / 64 == e) G = __shfl(x[e].s, (k - 1) % 64, WAVE);
    } else {
        Cand* x = reinterpret_cast<Cand*>(dyn) + (size_t)wave * ns;
        for (int i = lane; i < ns; i += WAVE) x[i] = load(i);
        wave_lds_sort(x, ns);
        G = x[k - 1].s;
    }
    if (lane != 0 || !(G > -(double)INFINITY)) return;
    float2 c = ucut[u];
    const double tt = G - (double)c.y;
    float f = (float)tt;
    if ((double)f > tt) f = nextafterf(f, -INFINITY);
    if (f > c.x) {
        c.x = f;
        ucut[u] = c;
    }
}

// ------------------------------------ config-4 shard path without a select --
// A catalog shard does not need its own k-th largest maximum: the global
// bound G of the exchange is higher on most users, and the scan's own list
// bound lb (uinfo.x, the smaller of the two lanes' (jk + 1)-th largest
// inserted maxima) is a valid cut on its own: every tau of the scan was
// <= lb - 2 eps, so each half-block whose fp16 max reaches lb - 2 eps was
// appended, and at least 2 (jk + 1) >= k appended half-blocks (distinct
// items) have max >= lb, i.e. an item with exact score >= lb - eps.  So the
// shard runs scan -> shard_bound -> (all_gather) -> shard_band, one pass over
// the appended maxima each, instead of select + bound + apply + pack.
//
// shard_bound: per user the m largest appended maxima (all of them are >= lb
// whenever at least m are) as exact lower bounds v / scl - eps, rounded down
// to fp32, descending, -inf padded; users whose appends overflowed (or that
// hold more than IP_SEL maxima >= lb) are flagged for the exact path.
__global__ __launch_bounds__(256) void ip_shard_bound_kernel(int64_t n_users, int m2, const uint2* __restrict__ app,
                                                             const int32_t* __restrict__ acnt,
                                                             const float4* __restrict__ uinfo, int m,
                                                             float* __restrict__ out, int32_t* __restrict__ ovf_flag,
                                                             int bandcap, uint2* __restrict__ pre,
                                                             int32_t* __restrict__ pre_cnt) {
    __shared__ __attribute__((aligned(16))) uint32_t sel[4][IP_SEL + 4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int64_t u = (int64_t)blockIdx.x * 4 + wave;
    int2 ac_n = make_int2(0, 0);
    float4 inf_n = make_float4(0.f, 0.f, 0.f, 0.f);
    if (u < n_users) {
        ac_n = reinterpret_cast<const int2*>(acnt)[u];
        inf_n = uinfo[u];
    }
    for (; u < n_users; u += nw) {
        const int a0 = ac_n.x, a1 = ac_n.y;
        const float4 inf = inf_n;
        if (u + nw < n_users) {
            ac_n = reinterpret_cast<const int2*>(acnt)[u + nw];
            inf_n = uinfo[u + nw];
        }
        bool ovf = a0 > m2 || a1 > m2;
        const int n = ovf ? 0 : a0 + a1;
        const uint2* s0 = app + (size_t)(2 * u) * m2;
        const uint2* s1 = s0 + m2;
        // the same pass keeps the entries >= the scan's own cut lb - 2 eps (a
        // superset of every later band) in the pre-band, so shard_band reads
        // those few instead of the whole append list
        const float own = inf.x == -INFINITY ? -INFINITY : round_down_sub(inf.x, 2.0f * inf.y);
        uint2* pb = pre + (size_t)u * bandcap;
        int c = 0, cp = 0;
        for (int b0 = 0; b0 < n; b0 += SH_ENT * WAVE) {
            uint2 ent[SH_ENT];
            sh_load(s0, s1, a0, n, b0, lane, ent);
#pragma unroll
            for (int j = 0; j < SH_ENT; ++j) {
                const int e = b0 + j * WAVE + lane;
                const float v = __uint_as_float(ent[j].x);
                const bool kp = e < n && v >= inf.x;
                const unsigned long long bal = __ballot(kp);
                const int pos = c + __popcll(bal & lt);
                if (kp && pos < IP_SEL) sel[wave][pos] = fkey(v);
                c += __popcll(bal);
                const bool kq = e < n && !(v < own);
                const unsigned long long bq = __ballot(kq);
                const int pq = cp + __popcll(bq & lt);
                if (kq && pq < bandcap) pb[pq] = ent[j];
                cp += __popcll(bq);
            }
        }
        if (c > IP_SEL) ovf = true;
        if (lane == 0) pre_cnt[u] = cp > bandcap ? -1 : cp;
        if (ovf) c = 0;
        // the m largest: every key of rank < m goes to out[rank]
        const double inv = inf.z > 0.0f ? 1.0 / (double)inf.z : 0.0;  // exact power of two
        if (lane < 4) sel[wave][c + lane] = 0u;
        wave_sync_lds();
        for (int b0 = 0; b0 < c; b0 += WAVE) {
            const uint32_t mine[1] = {b0 + lane < c ? sel[wave][b0 + lane] : 0u};
            int rank[1];
            lds_ranks<1>(sel[wave], c, mine, b0 + lane, rank);
            if (b0 + lane < c && rank[0] < m) {
                const double tv = (double)fkey_inv(mine[0]) * inv - (double)inf.w;
                float v = (float)tv;
                if ((double)v > tv) v = nextafterf(v, -INFINITY);
                out[u * m + rank[0]] = v;
            }
        }
        for (int i = c + lane; i < m; i += WAVE) out[u * m + i] = -INFINITY;  // fewer than m maxima
        wave_sync_lds();  // the next user's keys overwrite sel
        if (lane == 0) ovf_flag[u] = ovf ? 1 : 0;
    }
}

// shard_band: G = the k-th largest of the user's n_lists * m exchanged bounds
// (-inf with fewer than k values; none without bounds), cut = max(lb - 2 eps,
// G - eps) in the scan's scaled units (both valid: k items have exact >= G,
// and k items have exact >= lb - eps), then the appended entries >= cut
// compacted to out_ent[u * x_cap + j] as GLOBAL half-block ids (-1: more
// than x_cap -> the owner's exact path) and the cut written to ucut for the
// owner's refine.  uinfo.z == 0 marks an empty
// shard: no band, no cut.
__global__ __launch_bounds__(256) void ip_shard_band_kernel(int64_t n_users, int k, int m2,
                                                            const uint2* __restrict__ app,
                                                            const int32_t* __restrict__ acnt,
                                                            const float4* __restrict__ uinfo,
                                                            const float* __restrict__ bounds, int n_lists, int m,
                                                            int bandcap, const int32_t* __restrict__ ovf_flag,
                                                            const uint2* __restrict__ pre,
                                                            const int32_t* __restrict__ pre_cnt,
                                                            float2* __restrict__ ucut, uint32_t* __restrict__ out_ent,
                                                            int32_t* __restrict__ out_cnt, int x_cap) {
    __shared__ __attribute__((aligned(16))) uint32_t pool[4][2 * IP_SEL + 4];  // n_lists * m <= 512
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int tot = bounds ? n_lists * m : 0;
    int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    int2 ac_n = make_int2(0, 0);
    float4 inf_n = make_float4(0.f, 0.f, 0.f, 0.f);
    int ov_n = 0, pc_n = 0;
    // ovf_flag / pre == nullptr (the bounds came from the scan's lists): no
    // pre-band, the whole append list; overflowed lists -> the exact path
    auto ovf_of = [&](int64_t v, int2 ac) { return ovf_flag ? ovf_flag[v] : (ac.x > m2 || ac.y > m2) ? 1 : 0; };
    if (u < n_users) {
        ac_n = reinterpret_cast<const int2*>(acnt)[u];
        inf_n = uinfo[u];
        ov_n = ovf_of(u, ac_n);
        pc_n = pre ? pre_cnt[u] : -1;
    }
    for (; u < n_users; u += nw) {
        const int ov = ov_n, pc = pc_n;
        const float4 inf = inf_n;
        // the pre-band when it fit, else the whole append list
        const uint2* s0 = pc >= 0 ? pre + (size_t)u * bandcap : app + (size_t)(2 * u) * m2;
        const uint2* s1 = app + (size_t)(2 * u) * m2 + m2;
        const int a0 = pc >= 0 ? pc : ac_n.x, n = pc >= 0 ? pc : ac_n.x + ac_n.y;
        if (u + nw < n_users) {
            ac_n = reinterpret_cast<const int2*>(acnt)[u + nw];
            inf_n = uinfo[u + nw];
            ov_n = ovf_of(u + nw, ac_n);
            pc_n = pre ? pre_cnt[u + nw] : -1;
        }
        if (ov || inf.z <= 0.0f) {
            if (lane == 0) {
                out_cnt[u] = ov ? -1 : 0;
                ucut[u] = make_float2(-INFINITY, 0.0f);
            }
            continue;
        }
        uint2 ent[SH_ENT];
        sh_load(s0, s1, a0, n, 0, lane, ent);  // in flight across the bound select
        float G = -INFINITY;
        if (tot >= k) {
            for (int i = lane; i < tot; i += WAVE)
                pool[wave][i] = fkey(bounds[((int64_t)(i / m) * n_users + u) * m + (i % m)]);
            wave_sync_lds();
            G = fkey_inv(lds_select(pool[wave], tot, k - 1, lane));
            wave_sync_lds();
        }
        float cut = inf.x == -INFINITY ? -INFINITY : round_down_sub(inf.x, 2.0f * inf.y);
        if (G > -INFINITY) {
            const double tt = (double)G - (double)inf.w;
            float f = (float)tt;
            if ((double)f > tt) f = nextafterf(f, -INFINITY);
            cut = fmaxf(cut, f * inf.z);  // exact power-of-two rescale
        }
        int c = 0;
        uint32_t* dst = out_ent + (size_t)u * x_cap;
        for (int b0 = 0; b0 < n; b0 += SH_ENT * WAVE) {
            if (b0 > 0) sh_load(s0, s1, a0, n, b0, lane, ent);
#pragma unroll
            for (int j = 0; j < SH_ENT; ++j) {
                const int e = b0 + j * WAVE + lane;
                const bool kp = e < n && !(__uint_as_float(ent[j].x) < cut);
                const unsigned long long bal = __ballot(kp);
                const int pos = c + __popcll(bal & lt);
                if (kp && pos < x_cap) dst[pos] = ent[j].y;
                c += __popcll(bal);
            }
        }
        if (lane == 0) {
            out_cnt[u] = c > x_cap ? -1 : c;
            ucut[u] = make_float2(cut == -INFINITY ? -INFINITY : cut / inf.z, inf.w);
        }
    }
}

// owner side: users flagged for the exact path -> the fallback's list
__global__ void ip_ovf_collect_kernel(int64_t n_users, const int32_t* __restrict__ ovf_in,
                                      int32_t* __restrict__ ovf_flag, int32_t* __restrict__ ovf_list,
                                      int32_t* __restrict__ ovf_count) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n_users;
         u += (int64_t)gridDim.x * blockDim.x) {
        const int f = ovf_in ? ovf_in[u] : 0;
        ovf_flag[u] = f;
        if (f) ovf_list[atomicAdd(ovf_count, 1)] = (int32_t)u;
    }
}

// ------------------------------------------------------------- workspace --
// [hdr 256 B: ovf_count] [ucut f2] [cand_cnt] [ovf_flag] [ovf_list] [uinfo f4]
// [acnt 2 per user] [cand: bandcap per user] [app: 2 x m2 per user]
// ucut .. acnt depend on n_users only (nrk_ip_topk_apply_bound has no k).
struct IpWs {
    int32_t* ovf_count;
    float2* ucut;
    int32_t* cnt;
    int32_t* ovf_flag;
    int32_t* ovf_list;
    float4* uinfo;
    int32_t* acnt;
    uint2* cand;
    uint2* app;
    uint32_t* fbk;      // exact path: FB_GRID scratch rows of n_items keys
    int32_t* slow_list;  // exact path: users with too many fp32 ties (count at ovf_count[1])
    int bandcap, m2;
    int blk_lo, blk_hi;  // block range screened (config-4 shards), set by the caller
    float* bnd = nullptr;  // config-4 shard: the scan's per-user bounds (ip_scan_kernel's bnd)
    int bnd_m = 0;
    size_t bytes;
};

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// band entries kept per user (k + the entries within 2 eps of theta)
static inline int ip_bandcap(int k) {
    const int b = ((2 * k + 32 + 31) / 32) * 32;
    return std::min(IP_BQ, std::max(96, b));
}
// appended maxima per (user, half): about twice the expected record count
// of a lane's top-(jk+1) over its nblk half-blocks (random catalog order),
// never more than nblk (a lane appends at most one entry per block)
// (per half-block appends); the tile-append scan (k <= 32) stores whole
// tiles of TB maxima per passing tile, so there it is TB x the tile count
static inline int ip_m2(int64_t n_items, int k, int dim) {
    if (k > IP_KFAST) return 0;
    const int64_t nblk = std::max<int64_t>(1, n_blocks_of(n_items));
    const double mt = (double)((k + 1) / 2);
    const double est = mt * (1.0 + log(std::max(1.0, (double)nblk / mt)));
    int64_t m2 = (((int64_t)(2.0 * est) + 64 + 63) / 64) * 64;
    m2 = std::min<int64_t>(m2, ((nblk + 63) / 64) * 64);
    if (mt <= 16) {
        const int dp = pad_dim(dim);
        const int64_t tb = scan_tb(dp);
        const int64_t ntile = (nblk + tb - 1) / tb;
        const double et = mt * (1.0 + log(std::max(1.0, (double)ntile / mt)));
        int64_t mt2 = ((tb * ((int64_t)(2.0 * et) + 16) + 63) / 64) * 64;
        mt2 = std::min<int64_t>(mt2, ((ntile * tb + 63) / 64) * 64);
        m2 = std::max(m2, mt2);
    }
    return (int)m2;
}

static IpWs ip_ws_layout(void* base, int64_t n_users, int64_t n_items, int k, int dim) {
    IpWs w;
    w.bandcap = ip_bandcap(k);
    w.m2 = ip_m2(n_items, k, dim);
    w.blk_lo = 0;
    w.blk_hi = (int)n_blocks_of(n_items);
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    size_t off = 0;
    w.ovf_count = reinterpret_cast<int32_t*>(p + off);
    off += 256;
    w.ucut = reinterpret_cast<float2*>(p + off);
    off += align256((size_t)n_users * sizeof(float2));
    w.cnt = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * sizeof(int32_t));
    w.ovf_flag = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * sizeof(int32_t));
    w.ovf_list = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * sizeof(int32_t));
    w.uinfo = reinterpret_cast<float4*>(p + off);
    off += align256((size_t)n_users * sizeof(float4));
    w.acnt = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * 2 * sizeof(int32_t));
    w.cand = reinterpret_cast<uint2*>(p + off);
    off += align256((size_t)n_users * w.bandcap * sizeof(uint2));
    w.app = reinterpret_cast<uint2*>(p + off);
    off += align256((size_t)n_users * 2 * (size_t)w.m2 * sizeof(uint2));
    w.fbk = reinterpret_cast<uint32_t*>(p + off);
    off += align256((size_t)std::min<int64_t>(n_users, FB_GRID) * (size_t)n_items * sizeof(uint32_t));
    w.slow_list = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * sizeof(int32_t));
    w.bytes = off;
    return w;
}

static inline int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

// compute units of the current device (the persistent grids, the FLAT scan)
static int n_cus() {
    static const int n_cu = [] {
        int dev = 0, cu = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
        return cu > 0 ? cu : 256;
    }();
    return n_cu;
}

// scan variants: (DP, waves per workgroup, ring slots, user groups per wave,
// register list length, waves per SIMD)
// ring slots of the UG = 4 scan (config 2): 4 (one more tile in flight
// than round 3's 3) since the bookkeeping got cheaper -- bench context, one
// box, three pairs: scan 5.77 vs 5.80-5.86 ms
constexpr int SCAN_NSL4 = 4;
template <int DP, int NW, int NSL, int UG, int MT, int WPE>
static void launch_scan_v(const float* users, int n_users, const uint8_t* cat, int n_items, int dim, int k,
                          const IpWs& w, hipStream_t s) {
    const int per_wg = NW * 32 * UG;
    constexpr int TB = scan_tb(DP);
    const int nblk = (n_items + 31) / 32;
    const int t_lo = w.blk_lo / TB, t_hi = (std::min(w.blk_hi, nblk) + TB - 1) / TB;
    const unsigned grid = (unsigned)((n_users + per_wg - 1) / per_wg);
    // the list pre-pass: up to 64 tiles spread over the range (+2.2% MFMA at
    // config 2, +17% on a config-4 shard, whose appends it cuts by 2/3)
    const int n = t_hi - t_lo;
    const int pre_div = w.bnd != nullptr ? SCAN_SHARD_PRE_DIV : SCAN_PRE_DIV;  // a catalog shard's own
    const int n_pre = n >= SCAN_PRE_MIN ? std::min(SCAN_PRE_MAX, n / pre_div) : 0;
    const int pstride = n_pre > 0 ? n / n_pre : 1;
    if constexpr (SCAN_WS && DP == 32 && MT == 16 && NW == 8 && UG == 4) {
        // the warp-specialized form of this variant (same users per workgroup)
        // a catalog shard (list bounds) inserts more often: its appended
        // maxima are what the band pass reads
        const int insp = w.bnd != nullptr ? SCAN_WS_SHARD_INSP : SCAN_WS_INSP;
        ip_scan_ws_kernel<DP, NSL, MT, SCAN_WS_NB><<<grid, 256 * (1 + SCAN_WS_NB), 0, s>>>(
            users, n_users, cat, n_items, dim, k, w.m2, w.app, w.acnt, w.uinfo, t_lo, t_hi, n_pre, pstride, w.bnd,
            w.bnd_m, insp);
        return;
    }
    ip_scan_kernel<DP, NW, NSL, UG, MT, WPE><<<grid, NW * 64, 0, s>>>(
        users, n_users, cat, n_items, dim, k, w.m2, w.app, w.acnt, w.uinfo, t_lo, t_hi, n_pre, pstride, w.bnd,
        w.bnd_m);
}

// ring slots of dim 128's 8-wave scan: 4 x 32 KB (tools/scan128.py, 250k x
// 5M, one box, two pairs: 240.2-240.7 vs 241.6-242.8 ms at 3; rows identical)
#ifndef NRK_SCAN128_NSL
#define NRK_SCAN128_NSL 4
#endif
template <int DP, int MT>
static void launch_scan(const float* users, int n_users, const uint8_t* cat, int n_items, int dim, int k,
                        const IpWs& w, hipStream_t s) {
    constexpr int UG = (DP <= 128 && MT <= 32) ? 2 : 1;
    // 2 waves per SIMD everywhere: at 4 (128 VGPRs) the dim-16 / dim-64
    // k <= 32 and the dim-32 k <= 64 variants spilled 42-96 VGPRs to scratch
    constexpr int WPE = 2;
    if constexpr (DP == 32 && MT == 16) {
        // default at D = 32, k <= 32 (BASELINE config 2): 8 waves x 128 users
        // (UG = 4) per workgroup at 2 waves / SIMD -- every LDS fragment read
        // and tile barrier serves twice the MFMAs of the 64-user waves
        // (round 3): config-2 screen 6.8-7.0 vs 7.0-7.2 ms
        launch_scan_v<DP, 8, SCAN_NSL4, 4, MT, 2>(users, n_users, cat, n_items, dim, k, w, s);
        return;
    }
    // 8 waves share a 3-slot ring, 2 workgroups (4 waves / SIMD) per CU; every
    // tile inserts, appends per half-block max >= tau.  Config 2 (round 3,
    // screen = scan + select): 7.1 ms with 343 appended maxima per user;
    // whole-tile appends 7.4-7.5 with 885 (the select reads 2.6x more);
    // 4-wave workgroups 7.9-8.2, 4 / 6 / 8 ring slots 7.3-7.4, alternating
    // inserts 8.1 (the lagging cut doubles the appends)
    // ring slots capped by the CU's 160 KB of LDS (dim 128's 32-KB tiles: 4 -> 3 at UG = 1)
    constexpr int TILE_B = scan_tb(DP) * 64 * DP, NSL_CAP = 163840 / TILE_B;
    constexpr int NW = (UG == 2) ? 8 : 4, NSL0 = (UG == 2) ? (DP == 128 ? NRK_SCAN128_NSL : 3) : 4,
                  NSL = NSL0 < NSL_CAP ? NSL0 : NSL_CAP;
    static_assert(NSL >= 2, "ring");
    launch_scan_v<DP, NW, NSL, UG, MT, WPE>(users, n_users, cat, n_items, dim, k, w, s);
}

template <int DP>
static void launch_scan_k(const float* users, int n_users, const uint8_t* cat, int n_items, int dim, int k,
                          const IpWs& w, hipStream_t s) {
    const int mt = (k + 1) / 2;
    if (mt <= 16) launch_scan<DP, 16>(users, n_users, cat, n_items, dim, k, w, s);
    else if (mt <= 32) launch_scan<DP, 32>(users, n_users, cat, n_items, dim, k, w, s);
    else launch_scan<DP, 64>(users, n_users, cat, n_items, dim, k, w, s);
}

static void scan_dispatch(const float* users, int nu, const uint8_t* cat, int ni, int dim, int k, const IpWs& w,
                          hipStream_t s) {
    switch (pad_dim(dim)) {
        case 16: launch_scan_k<16>(users, nu, cat, ni, dim, k, w, s); break;
        case 32: launch_scan_k<32>(users, nu, cat, ni, dim, k, w, s); break;
        case 64: launch_scan_k<64>(users, nu, cat, ni, dim, k, w, s); break;
        case 128: launch_scan_k<128>(users, nu, cat, ni, dim, k, w, s); break;
        default: launch_scan_k<256>(users, nu, cat, ni, dim, k, w, s); break;
    }
}

// a tile-aligned block range of a shard (config 4), checked
static int ip_range(IpWs& w, int64_t n_items, int dim, int64_t blk_lo, int64_t blk_hi) {
    const int tb = scan_tb(pad_dim(dim));
    NRK_REQUIRE(blk_lo >= 0 && blk_lo <= blk_hi && blk_hi <= n_blocks_of(n_items), "block range out of bounds");
    NRK_REQUIRE(blk_lo == blk_hi || (blk_lo % tb == 0 && (blk_hi % tb == 0 || blk_hi == n_blocks_of(n_items))),
                "block range must start (and end, unless at the catalog end) on a 8-KB tile");
    w.blk_lo = (int)blk_lo;
    w.blk_hi = (int)blk_hi;
    return NRK_OK;
}

// config-4 shard bounds from the scan's register lists (ip_scan_kernel's
// epilogue) instead of a pass over the appended maxima (ip_shard_bound_kernel)
// the scan's epilogue merges lists of up to 32 per lane (k <= 64)
static inline bool shard_listbound(int k) { return (k + 1) / 2 <= 32; }

// persistent grid of the shard kernels: SH_WG_PER_CU 4-wave workgroups per CU
static int sh_grid(int64_t n_users) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n_users + 3) / 4, (int64_t)n_cus() * SH_WG_PER_CU));
}

// empty shard range: no appends, uinfo.z = 0 (shard_band: no band, no cut)
__global__ void ip_empty_range_kernel(int64_t n_users, int32_t* __restrict__ acnt, float4* __restrict__ uinfo) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n_users;
         u += (int64_t)gridDim.x * blockDim.x) {
        acnt[2 * u] = 0;
        acnt[2 * u + 1] = 0;
        uinfo[u] = make_float4(-INFINITY, 0.0f, 0.0f, 0.0f);
    }
}

// the exact path of the users in ovf_list (see ip_exact_kernel)
static void launch_exact(const float* users, int64_t n_users, const float* items, int64_t n_items, int dim, int k,
                         int64_t row_offset, const IpWs& w, float* out_s, int32_t* out_r, double* out_e,
                         hipStream_t s) {
    const int ns = next_pow2(std::max(k, 64));
    const size_t lds = (size_t)ns * sizeof(Cand);
    (void)hipFuncSetAttribute((const void*)ip_exact_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)ip_fallback_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int grid = (int)std::min<int64_t>(n_users, FB_GRID);
    ip_exact_kernel<<<grid, 256, lds, s>>>(users, items, n_items, dim, k, ns, row_offset, w.ovf_list, w.ovf_count,
                                           out_s, out_r, out_e, w.fbk, w.slow_list, w.ovf_count + 1);
    ip_fallback_kernel<<<grid, 256, lds, s>>>(users, items, n_items, dim, k, ns, row_offset, w.slow_list,
                                              w.ovf_count + 1, out_s, out_r, out_e);
}

}  // namespace nrk

using namespace nrk;

extern "C" {

#if NRK_SCAN_STAMP
// dev-only: the phase stamps of the last ip_scan_kernel launch (1024 x 8 u64)
int nrk_dev_scan_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(scan_stamps), sizeof(scan_stamps)) == hipSuccess ? 0 : -1;
}
#endif

int nrk_ip_topk_tile_blocks(int dim) {
    if (dim <= 0 || dim > 256) return 0;
    return scan_tb(pad_dim(dim));
}

size_t nrk_ip_catalog_bytes(int64_t n_items, int dim) {
    if (n_items < 0 || dim <= 0 || dim > 256) return 0;
    const int dp = pad_dim(dim);
    return catalog_body_bytes(n_items, dp) + CATALOG_HDR + (catalog_has_hb(dp) ? catalog_body_bytes(n_items, dp) : 0);
}

int nrk_ip_catalog_build(const float* items, int64_t n_items, int dim, void* catalog,
                         nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(items != nullptr || n_items == 0, "items is null");
    NRK_REQUIRE(catalog != nullptr, "catalog is null");
    NRK_REQUIRE(n_items >= 0 && n_items < INT32_MAX, "n_items out of range");
    NRK_REQUIRE(dim > 0 && dim <= 256, "dim must be in [1, 256]");
    const int dp = pad_dim(dim);
    hipStream_t s = as_stream(stream);
    const size_t body = catalog_body_bytes(n_items, dp);
    CatalogHdr* hdr = reinterpret_cast<CatalogHdr*>(reinterpret_cast<uint8_t*>(catalog) + body);
    if (hipMemsetAsync(hdr, 0, CATALOG_HDR, s) != hipSuccess) {
        set_error("nrk_ip_catalog_build: hipMemsetAsync failed");
        return NRK_EHIP;
    }
    const int64_t total = n_blocks_of(n_items) * (dp / 16) * 64;
    if (total > 0) {
        const int g2 = (int)std::min<int64_t>((n_items + 15) / 16, 2048);  // >= one row group per wave
        catalog_norm_kernel<<<g2, 256, 0, s>>>(items, n_items, dim, hdr);
    }
    catalog_hdr_kernel<<<1, 1, 0, s>>>(hdr, dim, dp);
    if (total > 0) {
        const int g2 = (int)std::min<int64_t>((n_items + 15) / 16, 2048);
        catalog_dnorm_kernel<<<g2, 256, 0, s>>>(items, n_items, dim, hdr);
        const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
        catalog_pack_kernel<<<grid, 256, 0, s>>>(items, n_items, dim, dp, hdr,
                                                 reinterpret_cast<uint4*>(catalog));
        if (catalog_has_hb(dp))
            catalog_pack_hb_kernel<<<grid, 256, 0, s>>>(
                items, n_items, dim, dp, hdr,
                reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(catalog) + catalog_hb_offset(n_items, dp)));
    }
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_ip_topk_workspace_bytes(int64_t n_users, int64_t n_items, int dim, int k) {
    (void)dim;
    if (n_users < 0 || n_items < 0 || k < 1) return 0;
    return ip_ws_layout(nullptr, n_users, n_items, k, dim).bytes;
}

static int ip_check(const float* users, int64_t n_users, const float* items, const void* catalog,
                    int64_t n_items, int dim, int k, void* workspace, size_t workspace_bytes) {
    NRK_REQUIRE(n_users >= 0 && n_items >= 0, "negative sizes");
    NRK_REQUIRE(n_items < (1ll << 30) && n_users < (1ll << 30), "n_items / n_users must be < 2^30");
    NRK_REQUIRE(dim > 0 && dim <= 256, "dim must be in [1, 256]");
    NRK_REQUIRE(k >= 1, "k must be >= 1");
    if (k > IP_KMAX) NRK_UNSUPPORTED("k > 2048 is not compiled");
    // the MFMA scan addresses the packed catalog body with 32-bit offsets
    NRK_REQUIRE(k > IP_KFAST || catalog_body_bytes(n_items, pad_dim(dim)) <= (size_t)INT32_MAX,
                "packed catalog body must be < 2 GiB (n_items * pad_dim(dim) * 2 bytes): split the items");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(users && workspace, "null pointer");
    NRK_REQUIRE(n_items == 0 || (items && catalog), "items/catalog null");
    NRK_REQUIRE(workspace_bytes >= ip_ws_layout(nullptr, n_users, n_items, k, dim).bytes, "workspace too small");
    return NRK_OK;
}

// phases: 1 = the MFMA scan, 2 = the select (or the exact-path / empty
// marking), 3 = both
static int screen_phases(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim, int k,
                         int64_t blk_lo, int64_t blk_hi, void* workspace, size_t workspace_bytes,
                         nrk_stream_t stream, int phases) {
    int rc = ip_check(users, n_users, (const float*)catalog, catalog, n_items, dim, k, workspace,
                      workspace_bytes);
    if (rc != NRK_OK || n_users == 0) return rc;
    IpWs w = ip_ws_layout(workspace, n_users, n_items, k, dim);
    rc = ip_range(w, n_items, dim, blk_lo, blk_hi);
    if (rc != NRK_OK) return rc;
    if (blk_hi == blk_lo) n_items = 0;  // empty range: every output row is padding
    hipStream_t s = as_stream(stream);
    const uint8_t* cat = reinterpret_cast<const uint8_t*>(catalog);
    if ((phases & 1) && n_items > 0 && k <= IP_KFAST) {
        scan_dispatch(users, (int)n_users, cat, (int)n_items, dim, k, w, s);
    }
    if (phases & 2) {
        if (hipMemsetAsync(w.ovf_count, 0, 256, s) != hipSuccess) {
            set_error("nrk_ip_topk_screen: hipMemsetAsync failed");
            return NRK_EHIP;
        }
        if (n_items == 0) {
            // nothing to search: every output row is padding
            (void)hipMemsetAsync(w.cnt, 0, (size_t)n_users * sizeof(int32_t), s);
            (void)hipMemsetAsync(w.ovf_flag, 0, (size_t)n_users * sizeof(int32_t), s);
            (void)hipMemsetAsync(w.ucut, 0xFF, (size_t)n_users * sizeof(float2), s);  // NaN cut: no band
        } else if (k > IP_KFAST) {
            const int grid = (int)std::min<int64_t>((n_users + 255) / 256, 4096);
            ip_all_exact_kernel<<<grid, 256, 0, s>>>(n_users, w.cnt, w.ovf_flag, w.ovf_list, w.ovf_count);
        } else {
            ip_select_kernel<<<sh_grid(n_users), 256, 0, s>>>(n_users, k, w.m2, w.bandcap, w.app, w.acnt, w.uinfo,
                                                              w.cand, w.cnt, w.ucut, w.ovf_flag, w.ovf_list,
                                                              w.ovf_count);
        }
    }
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_ip_topk_scan(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim, int k,
                     void* workspace, size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    return screen_phases(users, n_users, catalog, n_items, dim, k, 0, n_blocks_of(n_items), workspace,
                         workspace_bytes, stream, 1);
}

int nrk_ip_topk_select(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim, int k,
                       void* workspace, size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    return screen_phases(users, n_users, catalog, n_items, dim, k, 0, n_blocks_of(n_items), workspace,
                         workspace_bytes, stream, 2);
}

int nrk_ip_topk_screen(const float* users, int64_t n_users, const void* catalog, int64_t n_items,
                       int dim, int k, void* workspace, size_t workspace_bytes,
                       nrk_stream_t stream) {
    clear_error();
    return screen_phases(users, n_users, catalog, n_items, dim, k, 0, n_blocks_of(n_items), workspace,
                         workspace_bytes, stream, 3);
}

int nrk_ip_topk_finish(const float* users, int64_t n_users, const float* items,
                       const void* catalog, int64_t n_items,
                       int dim, int k, int64_t row_offset, float* out_scores, int32_t* out_rows,
                       double* out_exact, void* workspace, size_t workspace_bytes,
                       nrk_stream_t stream) {
    clear_error();
    int rc = ip_check(users, n_users, items, items, n_items, dim, k, workspace, workspace_bytes);
    if (rc != NRK_OK || n_users == 0) return rc;
    NRK_REQUIRE(out_scores && out_rows, "null output");
    const IpWs w = ip_ws_layout(workspace, n_users, n_items, k, dim);
    hipStream_t s = as_stream(stream);
    const int g2 = (int)((n_users + 3) / 4);
    const uint8_t* cat = reinterpret_cast<const uint8_t*>(catalog);
#define NRK_REFINE(DS4, SV)                                                                                  \
    ip_refine_kernel<DS4, SV><<<g2, 256, 0, s>>>(users, n_users, items, cat, n_items, dim, k, row_offset,   \
                                                 w.cand, w.bandcap, w.cnt, w.ucut, w.ovf_flag, w.ovf_list,   \
                                                 w.ovf_count, out_scores, out_rows, out_exact)
#define NRK_REFINE_SV(DS4)                          \
    do {                                            \
        if (k <= 64) NRK_REFINE(DS4, 128);          \
        else NRK_REFINE(DS4, 256);                  \
    } while (0)
    if (k <= IP_KFAST || n_items == 0) {
        if (dim == 32) NRK_REFINE_SV(8);
        else if (dim == 16) NRK_REFINE_SV(4);
        else if (dim == 64) NRK_REFINE_SV(16);
        else NRK_REFINE_SV(0);
    }
#undef NRK_REFINE_SV
#undef NRK_REFINE
    if (n_items > 0) launch_exact(users, n_users, items, n_items, dim, k, row_offset, w, out_scores, out_rows, out_exact, s);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_ip_topk(const float* users, int64_t n_users, const float* items, const void* catalog,
                int64_t n_items, int dim, int k, int64_t row_offset, float* out_scores,
                int32_t* out_rows, double* out_exact, void* workspace, size_t workspace_bytes,
                nrk_stream_t stream) {
    int rc = nrk_ip_topk_screen(users, n_users, catalog, n_items, dim, k, workspace,
                                workspace_bytes, stream);
    if (rc != NRK_OK) return rc;
    return nrk_ip_topk_finish(users, n_users, items, catalog, n_items, dim, k, row_offset, out_scores,
                              out_rows, out_exact, workspace, workspace_bytes, stream);
}

int nrk_ip_topk_bound(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim,
                      int k, int m, float* out_bound, void* workspace, size_t workspace_bytes,
                      nrk_stream_t stream) {
    clear_error();
    int rc = ip_check(users, n_users, (const float*)catalog, catalog, n_items, dim, k, workspace,
                      workspace_bytes);
    if (rc != NRK_OK) return rc;
    if (k > IP_KFAST) NRK_UNSUPPORTED("the screen bound needs k <= 128");
    NRK_REQUIRE(m >= 1 && m <= 256, "m must be in [1, 256]");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(out_bound != nullptr, "null pointer");
    const IpWs w = ip_ws_layout(workspace, n_users, n_items, k, dim);
    hipStream_t s = as_stream(stream);
    if (n_items == 0) {
        // empty shard: no bound (the screen wrote no band)
        (void)hipMemsetAsync(w.cnt, 0, (size_t)n_users * sizeof(int32_t), s);
    }
    const CatalogHdr* hdr = reinterpret_cast<const CatalogHdr*>(
        reinterpret_cast<const uint8_t*>(catalog) + catalog_body_bytes(n_items, pad_dim(dim)));
    const int grid = (int)((n_users + 3) / 4);
    const int need = std::max(w.bandcap, m);
#define NRK_BOUND(E, NS)                                                                                    \
    ip_bound_kernel<E><<<grid, 256, (E) ? 0 : 4 * (NS) * sizeof(Cand), s>>>(users, n_users, dim, hdr, w.cand, \
                                                                           w.bandcap, w.cnt, w.ucut, m, NS,  \
                                                                           out_bound)
    if (need <= 64) NRK_BOUND(1, 64);
    else if (need <= 128) NRK_BOUND(2, 128);
    else if (need <= 256) NRK_BOUND(4, 256);
    else NRK_BOUND(0, next_pow2(need));
#undef NRK_BOUND
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_ip_topk_apply_bound(int64_t n_users, const float* bounds, int n_lists, int m, int k, void* workspace,
                            size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_users >= 0 && n_users < (1ll << 30), "n_users out of range");
    NRK_REQUIRE(n_lists >= 1 && m >= 1 && n_lists * m <= 512, "need 1 <= n_lists * m <= 512");
    NRK_REQUIRE(k >= 1 && k <= IP_KFAST, "k must be in [1, 128]");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(bounds && workspace, "null pointer");
    // ucut's place depends on n_users only
    NRK_REQUIRE(workspace_bytes >= ip_ws_layout(nullptr, n_users, 0, 1, 1).bytes, "workspace too small");
    const IpWs w = ip_ws_layout(workspace, n_users, 0, 1, 1);
    if (k > n_lists * m) return NRK_OK;  // fewer values than k: no bound, cut unchanged
    const int tot = n_lists * m, grid = (int)((n_users + 3) / 4);
    hipStream_t s = as_stream(stream);
#define NRK_APPLY(E, NS) \
    ip_apply_bound_kernel<E><<<grid, 256, (E) ? 0 : 4 * (NS) * sizeof(Cand), s>>>(w.ucut, n_users, bounds, n_lists, m, k, NS)
    if (tot <= 64) NRK_APPLY(1, 64);
    else if (tot <= 128) NRK_APPLY(2, 128);
    else if (tot <= 256) NRK_APPLY(4, 256);
    else NRK_APPLY(0, next_pow2(tot));
#undef NRK_APPLY
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_ip_topk_shard_screen(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim,
                             int k, int64_t blk_lo, int64_t blk_hi, int m, float* out_bound, void* workspace,
                             size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    int rc = ip_check(users, n_users, (const float*)catalog, catalog, n_items, dim, k, workspace,
                      workspace_bytes);
    if (rc != NRK_OK) return rc;
    if (k > IP_KFAST) NRK_UNSUPPORTED("the shard screen needs k <= 128 (larger k: the merge protocol)");
    NRK_REQUIRE(m >= 1 && m <= IP_SEL, "m must be in [1, 256]");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(out_bound != nullptr, "null pointer");
    IpWs w = ip_ws_layout(workspace, n_users, n_items, k, dim);
    rc = ip_range(w, n_items, dim, blk_lo, blk_hi);
    if (rc != NRK_OK) return rc;
    hipStream_t s = as_stream(stream);
    const bool lbnd = shard_listbound(k);
    if (lbnd) {
        // the bounds come from the scan's own lists (its epilogue); an empty
        // range has none
        w.bnd = out_bound;
        w.bnd_m = m;
    }
    if (blk_lo == blk_hi || n_items == 0) {
        ip_empty_range_kernel<<<(int)std::min<int64_t>((n_users + 255) / 256, 4096), 256, 0, s>>>(n_users, w.acnt,
                                                                                               w.uinfo);
        if (lbnd &&
            hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(out_bound), 0xFF800000u /* -inf */,
                              (size_t)n_users * m, s) != hipSuccess) {
            set_error("nrk_ip_topk_shard_screen: hipMemsetD32Async failed");
            return NRK_EHIP;
        }
    } else {
        scan_dispatch(users, (int)n_users, reinterpret_cast<const uint8_t*>(catalog), (int)n_items, dim, k, w, s);
    }
    if (!lbnd)
        ip_shard_bound_kernel<<<sh_grid(n_users), 256, 0, s>>>(n_users, w.m2, w.app, w.acnt, w.uinfo, m, out_bound,
                                                               w.ovf_flag, w.bandcap, w.cand, w.cnt);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_ip_topk_shard_band(int64_t n_users, int64_t n_items, int dim, int k, const float* bounds, int n_lists,
                           int m, int x_cap, void* workspace, size_t workspace_bytes, void* out_ent,
                           int32_t* out_cnt, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(x_cap >= 1 && x_cap <= IP_BQ, "x_cap must be in [1, 288]");
    NRK_REQUIRE(n_users >= 0 && n_users < (1ll << 30) && n_items >= 0 && dim > 0 && dim <= 256, "bad sizes");
    NRK_REQUIRE(k >= 1 && k <= IP_KFAST, "k must be in [1, 128]");
    NRK_REQUIRE(bounds == nullptr || (n_lists >= 1 && m >= 1 && n_lists * m <= 512),
                "need 1 <= n_lists * m <= 512");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(workspace && out_ent && out_cnt, "null pointer");
    NRK_REQUIRE(workspace_bytes >= ip_ws_layout(nullptr, n_users, n_items, k, dim).bytes, "workspace too small");
    const IpWs w = ip_ws_layout(workspace, n_users, n_items, k, dim);
    ip_shard_band_kernel<<<sh_grid(n_users), 256, 0, as_stream(stream)>>>(
        n_users, k, w.m2, w.app, w.acnt, w.uinfo, bounds, bounds ? n_lists : 0, bounds ? m : 1, w.bandcap,
        shard_listbound(k) ? nullptr : w.ovf_flag, shard_listbound(k) ? nullptr : w.cand,
        shard_listbound(k) ? nullptr : w.cnt, w.ucut, reinterpret_cast<uint32_t*>(out_ent), out_cnt, x_cap);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_ip_topk_refine_x(const float* users, int64_t n_users, const float* items, const void* catalog,
                         int64_t n_items, int dim, int k, int64_t row_offset, const void* band, int n_src,
                         int64_t src_users, int x_cap, const int32_t* src_cnt, const float* ucut,
                         const int32_t* ovf_in, float* out_scores, int32_t* out_rows, double* out_exact,
                         void* workspace, size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    int rc = ip_check(users, n_users, items, items, n_items, dim, k, workspace, workspace_bytes);
    if (rc != NRK_OK || n_users == 0) return rc;
    NRK_REQUIRE(out_scores && out_rows && band && src_cnt && ucut, "null pointer");
    NRK_REQUIRE(n_src >= 1 && x_cap >= 1 && src_users >= n_users, "need n_src >= 1, x_cap >= 1, src_users >= n_users");
    if (k > IP_KFAST) NRK_UNSUPPORTED("the band refine needs k <= 128 (larger k: exact path, ovf_in = 1)");
    const IpWs w = ip_ws_layout(workspace, n_users, n_items, k, dim);
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(w.ovf_count, 0, 256, s) != hipSuccess) {
        set_error("nrk_ip_topk_refine_x: hipMemsetAsync failed");
        return NRK_EHIP;
    }
    ip_ovf_collect_kernel<<<(int)std::min<int64_t>((n_users + 255) / 256, 4096), 256, 0, s>>>(
        n_users, ovf_in, w.ovf_flag, w.ovf_list, w.ovf_count);
    const int g2 = (int)((n_users + 3) / 4);
    const uint8_t* cat = reinterpret_cast<const uint8_t*>(catalog);
    const uint2* bd = reinterpret_cast<const uint2*>(band);
    const float2* uc = reinterpret_cast<const float2*>(ucut);
#define NRK_REFINE(DS4, SV)                                                                                   \
    ip_refine_kernel<DS4, SV><<<g2, 256, 0, s>>>(users, n_users, items, cat, n_items, dim, k, row_offset, bd, 0, \
                                                 nullptr, uc, w.ovf_flag, w.ovf_list, w.ovf_count, out_scores,   \
                                                 out_rows, out_exact, n_src, src_users, x_cap, src_cnt)
#define NRK_REFINE_SV(DS4)                 \
    do {                                   \
        if (k <= 64) NRK_REFINE(DS4, 128); \
        else NRK_REFINE(DS4, 256);         \
    } while (0)
    if (dim == 32) NRK_REFINE_SV(8);
    else if (dim == 16) NRK_REFINE_SV(4);
    else if (dim == 64) NRK_REFINE_SV(16);
    else NRK_REFINE_SV(0);
#undef NRK_REFINE_SV
#undef NRK_REFINE
    if (n_items > 0) launch_exact(users, n_users, items, n_items, dim, k, row_offset, w, out_scores, out_rows, out_exact, s);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_topk_merge(const double* in_exact, const int32_t* in_rows, int n_lists, int64_t list_stride,
                   int64_t n_users, int k_in, int k_out, float* out_scores, int32_t* out_rows,
                   double* out_exact, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_lists >= 1 && k_in >= 1 && k_out >= 1 && n_users >= 0, "bad sizes");
    NRK_REQUIRE(list_stride >= n_users * (int64_t)k_in, "list_stride too small");
    const int tot = n_lists * k_in;
    if (tot > 1024) NRK_UNSUPPORTED("n_lists * k_in > 1024");
    NRK_REQUIRE(k_out <= tot, "k_out > n_lists * k_in");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(in_exact && in_rows && out_scores && out_rows, "null pointer");
    hipStream_t s = as_stream(stream);
    const int grid = (int)((n_users + 3) / 4);
#define NRK_MERGE(E, NS)                                                                                    \
    topk_merge_kernel<E><<<grid, 256, (E) ? 0 : 4 * (NS) * sizeof(Cand), s>>>(in_exact, in_rows, n_lists,      \
                                                                              list_stride, n_users, k_in, k_out, \
                                                                              NS, out_scores, out_rows, out_exact)
    if (tot <= 64) NRK_MERGE(1, 64);
    else if (tot <= 128) NRK_MERGE(2, 128);
    else if (tot <= 256) NRK_MERGE(4, 256);
    else NRK_MERGE(0, next_pow2(tot));
#undef NRK_MERGE
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
