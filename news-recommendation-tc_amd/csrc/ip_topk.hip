// ip_topk.hip -- brute-force user x item inner-product top-K on gfx950.
//
// Replaces faiss.IndexFlatIP.add/.search (src/recall/youtubednn_recaller.py
// :493-494, :520).  Contract (= IndexFlatIP): exact inner product, score desc,
// ties -> lower row.  "Exact" is the fp64 sum of the fp32 products,
// accumulated in dimension order (the oracle's definition, oracle/nrk_oracle.c).
//
// Design (MI355X-first, see DESIGN.md "ip_topk"):
//   1. ip_screen   -- the one dense contraction on MFMA: fp16 32x32x16 tiles
//      (power-of-two scaled, so the only error is fp16 rounding), items
//      (A operand) streamed through LDS from a catalog pre-packed in
//      fragment order, 32 users per wave (B operand) held in registers.
//      Each lane owns one user x one 16-item half of every 32-item block.
//      Per block the lane takes the max of its 16 scores and appends
//      (half-block max, half-block id) to its LDS list, branch-free: the
//      entry is always written and kept only if it beats the lane threshold
//      tau = theta - 2*eps, theta = K-th largest listed half-block max (a
//      lower bound of the K-th largest score: K distinct half-blocks each
//      hold an item >= theta), eps bounds |fp16 score - exact|
//      (eps = c(D) * ||u|| * max_j ||v_j||).  A full list is compacted by a
//      register bitonic sort (all lanes at once, no serial LDS chains).
//   2. ip_refine   -- one wave per user: fp64 exact rescoring of every item
//      of the flagged half-blocks, keep items with exact score >= cut + eps
//      (typically K + a few), wave bitonic sort on (score desc, row asc).
//   3. ip_fallback -- users whose candidate band overflowed (dense exact or
//      near ties, e.g. duplicated catalog rows): exact fp64 radix-select over
//      the whole catalog.  Never taken on non-degenerate data.
#include "nrk_common.h"

#include <float.h>
#include <stdlib.h>

#include <type_traits>

namespace nrk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int IP_CW = 48;  // candidate entries per (user, half) slot of the workspace
constexpr int IP_KMAX = 32;
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

// --------------------------------------------------------- catalog build --
// Thread -> one 16-byte fragment: block b, k-step s, lane l:
//   8 bf16 of item 32b + (l & 31), dims 16s + 8(l >> 5) + [0, 8).
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

__global__ void catalog_norm_kernel(const float* __restrict__ items, int64_t n_items, int dim,
                                    CatalogHdr* hdr) {
    float m = 0.0f, a = 0.0f;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_items;
         r += (int64_t)gridDim.x * blockDim.x) {
        float s = 0.0f;
        for (int d = 0; d < dim; ++d) {
            const float x = items[r * dim + d];
            s += x * x;
            a = fmaxf(a, fabsf(x));
        }
        m = fmaxf(m, sqrtf(s));
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
    double m = 0.0;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_items;
         r += (int64_t)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int d = 0; d < dim; ++d) {
            const float f = items[r * dim + d];
            const float x = (float)(_Float16)(f * scale);  // catalog_pack's rounding
            const double e = (double)x / (double)scale - (double)f;
            s += e * e;
        }
        m = fmax(m, sqrt(s));
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
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float round_down_sub(float theta, float two_eps) {
    float c = theta - two_eps;
    return __uint_as_float(c > 0.0f ? __float_as_uint(c) - 1u
                                    : (c == 0.0f ? 0x80000001u : __float_as_uint(c) + 1u));
}

// ---- per-user candidate lists ---------------------------------------------
// Each wave owns 32 users; user q's list lives in LDS as two SoA planes
// (scores f32, half-block ids u32), entry j at plane + (j * 32 + q) * 4, so
// the 32 lanes of a half-wave touch 128 consecutive bytes.  Both lanes of a
// user (h = 0, 1: the two 16-item halves of every 32-item block) append to
// the same list and keep identical copies of its count n, cut tau and theta.
constexpr int SC_CL = 64;  // entries per user list (default variant)

__device__ __forceinline__ float lds_rd(uint32_t a) {
    float v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}
__device__ __forceinline__ void lds_wr(uint32_t a, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
// v0 at a, v1 at a + OFF (one address register)
template <int OFF>
__device__ __forceinline__ void lds_wr_pair(uint32_t a, uint32_t v0, uint32_t v1) {
    asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %0, %2 offset:%c3" ::"v"(a), "v"(v0), "v"(v1), "n"(OFF)
                 : "memory");
}
// 16 dwords at a + i * stride (i = 0..15), one wait for all of them.  Inline
// asm: hipcc's waitcnt pass would drain the in-flight LDS-DMA (the ring
// prefetch) in front of any compiler-visible LDS access.
template <int STRIDE>
__device__ __forceinline__ void lds_rd16(uint32_t a, uint32_t (&o)[16]) {
    asm volatile(
        "ds_read_b32 %0, %16 offset:%c17*0\n\tds_read_b32 %1, %16 offset:%c17*1\n\t"
        "ds_read_b32 %2, %16 offset:%c17*2\n\tds_read_b32 %3, %16 offset:%c17*3\n\t"
        "ds_read_b32 %4, %16 offset:%c17*4\n\tds_read_b32 %5, %16 offset:%c17*5\n\t"
        "ds_read_b32 %6, %16 offset:%c17*6\n\tds_read_b32 %7, %16 offset:%c17*7\n\t"
        "ds_read_b32 %8, %16 offset:%c17*8\n\tds_read_b32 %9, %16 offset:%c17*9\n\t"
        "ds_read_b32 %10, %16 offset:%c17*10\n\tds_read_b32 %11, %16 offset:%c17*11\n\t"
        "ds_read_b32 %12, %16 offset:%c17*12\n\tds_read_b32 %13, %16 offset:%c17*13\n\t"
        "ds_read_b32 %14, %16 offset:%c17*14\n\tds_read_b32 %15, %16 offset:%c17*15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]),
          "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]),
          "=&v"(o[12]), "=&v"(o[13]), "=&v"(o[14]), "=&v"(o[15])
        : "v"(a), "n"(STRIDE)
        : "memory");
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

// Register bitonic sort of 32 floats, descending (per lane).
__device__ __forceinline__ void sort32_desc(float (&x)[32]) {
#pragma unroll
    for (int kl = 1; kl <= 5; ++kl) {
#pragma unroll
        for (int jl = kl - 1; jl >= 0; --jl) {
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                const int p = i ^ (1 << jl);
                if (p > i) {
                    const bool desc = ((i >> kl) & 1) == 0;
                    const float a = x[i], b = x[p];
                    const float hi = fmaxf(a, b), lo = fminf(a, b);
                    x[i] = desc ? hi : lo;
                    x[p] = desc ? lo : hi;
                }
            }
        }
    }
}

// Compact user q's list (both lanes of the user run this in lock step):
// theta = k-th largest listed half-block max (a lower bound of the user's
// k-th largest score: k distinct half-blocks each hold an item with
// fp16 score >= theta), keep the entries >= cut = theta - 2 eps.  Lane h
// sorts entries [32h, 32h + 32); the top 32 of the union is max(own[i],
// partner[31 - i]) (one bitonic merge step), sorted again to read the k-th.
// A user whose kept band does not leave room for the next tile's appends
// (dense exact ties) stops appending and is redone by the exact fallback.
template <int CL>
__device__ __forceinline__ void user_flush(uint32_t ls, uint32_t li, int h, int& n, float& tau,
                                           float& theta, bool& ovf, int k, float eps, int cap) {
    const uint32_t as = ls + (uint32_t)h * (32u * 32u * 4u), ai = li + (uint32_t)h * (32u * 32u * 4u);
    uint32_t raw[16];
    float x[32];
    const int nv = n - 32 * h;  // valid entries in this lane's half
    lds_rd16<128>(as, raw);
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = i < nv ? __uint_as_float(raw[i]) : -INFINITY;
    lds_rd16<128>(as + 16 * 128, raw);
#pragma unroll
    for (int i = 0; i < 16; ++i) x[16 + i] = 16 + i < nv ? __uint_as_float(raw[i]) : -INFINITY;
    sort32_desc(x);
    float z[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) z[i] = fmaxf(x[i], partner32f(x[31 - i], h));
    // z is bitonic: merge it descending
#pragma unroll
    for (int jl = 4; jl >= 0; --jl) {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int p = i ^ (1 << jl);
            if (p > i) {
                const float a = z[i], b = z[p];
                z[i] = fmaxf(a, b);
                z[p] = fminf(a, b);
            }
        }
    }
    float th = z[0];
#pragma unroll
    for (int j = 1; j < 32; ++j) th = (j == k - 1) ? z[j] : th;
    const float cut = (th == -INFINITY) ? -INFINITY : round_down_sub(th, 2.0f * eps);
    // re-read (score, id) in list order and compact: lane 0's kept entries go
    // to [0, c0), lane 1's to [c0, c0 + c1); a dropped entry is written to
    // slot SC_CL - 1, which no kept entry reaches unless the user overflows.
    uint32_t s[32], id[32];
    lds_rd16<128>(as, raw);
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = raw[i];
    lds_rd16<128>(as + 16 * 128, raw);
#pragma unroll
    for (int i = 0; i < 16; ++i) s[16 + i] = raw[i];
    lds_rd16<128>(ai, raw);
#pragma unroll
    for (int i = 0; i < 16; ++i) id[i] = raw[i];
    lds_rd16<128>(ai + 16 * 128, raw);
#pragma unroll
    for (int i = 0; i < 16; ++i) id[16 + i] = raw[i];
    uint32_t keepm = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i)
        keepm |= (i < nv && __uint_as_float(s[i]) >= cut) ? (1u << i) : 0u;
    const int c_own = __popc(keepm);
    const int c_par = (int)partner32((uint32_t)c_own, h);
    int pos = h ? c_par : 0;
    const uint32_t ls0 = ls - (uint32_t)0, dump = (uint32_t)(CL - 1) * 128u;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const bool kp = (keepm >> i) & 1u;
        const uint32_t off = kp ? (uint32_t)pos * 128u : dump;
        lds_wr(ls0 + off, s[i]);
        lds_wr(li + off, id[i]);
        pos += kp ? 1 : 0;
    }
    const int nn = c_own + c_par;
    theta = th;
    if (nn > cap) {
        ovf = true;
        tau = INFINITY;
        n = 0;
    } else {
        n = nn;
        tau = fmaxf(tau, cut);
    }
}

// Screen: 8 waves (2 per SIMD) x 32 users per workgroup share one LDS ring of
// catalog tiles.  Per tile every wave runs TB x DS MFMAs, takes each lane's
// half-block max and, when any lane beats its user's cut, appends those
// maxima to the user lists (branch per tile).  Lists are compacted when one
// is nearly full; a flush requested by any wave is joined by the others at
// the same tile (they all meet at the per-tile barrier anyway), through an
// LDS hint word.
template <int DP, int NW, int NSL = 3, int CL = SC_CL>
__global__ __launch_bounds__(NW * 64, (NW == 4 && CL < 64) ? 2 : NW / 4) void ip_screen_kernel(
    const float* __restrict__ users, int n_users, const uint8_t* __restrict__ catalog,
    int n_items, int dim, int k, uint2* __restrict__ cand, int32_t* __restrict__ cand_cnt,
    float2* __restrict__ ucut, int32_t* __restrict__ ovf_flag, int32_t* __restrict__ ovf_list,
    int32_t* __restrict__ ovf_count) {
    constexpr int DS = DP / 16;
    constexpr int BLOCK_BYTES = 64 * DP;
    constexpr int TB = BLOCK_BYTES >= 8192 ? 1 : 8192 / BLOCK_BYTES;
    constexpr int TILE_BYTES = TB * BLOCK_BYTES;
    constexpr int LPT = TILE_BYTES / (NW * 64 * 16);  // 1-KB LDS-DMA pieces per wave per tile
    static_assert(LPT >= 1 && LPT * NW * 1024 == TILE_BYTES, "tile split");
    constexpr int NSLOT = NSL;
    constexpr int WLIST = 2 * CL * 32 * 4;  // one wave's score + id planes
    constexpr int CAP = CL - 2 * TB;        // list size that still takes one tile of appends
    constexpr int LDS = NSLOT * TILE_BYTES + NW * WLIST + 16;
    static_assert(LDS <= 163840, "LDS budget");
    __shared__ __attribute__((aligned(16))) uint8_t smem[LDS];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, h = lane >> 5, q = lane & 31;
    const int user = blockIdx.x * (NW * 32) + wave * 32 + q;
    const bool active = user < n_users;

    const int nblk = (n_items + 31) >> 5;
    const int ntile = (nblk + TB - 1) / TB;
    const CatalogHdr* hdr = reinterpret_cast<const CatalogHdr*>(catalog + (size_t)nblk * BLOCK_BYTES);
    const float vmax = hdr->max_norm;
    const float sv_scale = hdr->scale;

    // B operand: 32 users x DP dims, fp16 (scaled by a power of two); lane
    // holds user q, dims 16s + 8h + [0, 8) for k-step s.
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
    f16x8 ufrag[DS];
    float du2 = 0.0f;  // ||fp16(u su) - u su||^2 (scaled units; each difference exact)
#pragma unroll
    for (int s = 0; s < DS; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float a = uval[s][e] * su;
            ufrag[s][e] = (_Float16)a;
            const float d = (float)ufrag[s][e] - a;
            du2 += d * d;
        }
    du2 += __shfl_xor(du2, 32, WAVE);
    // |fp16 score - exact| = |du.v + u.dv + du.dv + accumulation| with du, dv
    // the actual fp16 rounding errors of this user and of the items:
    //   <= ||du|| max||v|| + ||u|| max||dv|| + ||du|| max||dv||
    //      + (2^-15 + D 2^-23) ||u|| max||v||  (fp32 accumulation of the exact
    //        fp16 products in any order, with the round-1 bound's margins);
    // ||du|| is measured here, max||dv|| by catalog_dnorm_kernel -- about
    // 0.65x of round 1's worst case 2^-10 ||u|| max||v||.
    const float nu = sqrtf(nrm2), ndu = sqrtf(du2) / su, dvmax = hdr->max_dnorm;
    const float ceps = 3.0517578e-5f + (float)DP * 1.1920929e-7f;
    const float eps = (nrm2 == 0.0f) ? 0.0f
                                     : (ndu * vmax + nu * dvmax + ndu * dvmax + ceps * nu * vmax) * 1.0001f + 1e-30f;
    const float scl = su * sv_scale;  // scores below are scaled by scl (exact power of 2)
    const float eps_s = eps * scl;

    // zero users (all scores exactly 0) are answered by the refine directly
    const bool live = active && nrm2 > 0.0f;
    int n = 0;
    float tau = live ? -INFINITY : INFINITY, theta = -INFINITY;
    bool ovf = false;

    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t lds_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(smem);
    const uint32_t lst = lds_base + NSLOT * TILE_BYTES + wave * WLIST;
    const uint32_t ls = lst + q * 4;                       // score plane, entry j at + j * 128
    const uint32_t li = lst + CL * 32 * 4 + q * 4;      // id plane
    const uint32_t hint = lds_base + NSLOT * TILE_BYTES + NW * WLIST;
    if (tid == 0) lds_wr(hint, 0xFFFFFFFFu);

    const int body_bytes = nblk * BLOCK_BYTES;
    const int tail_blk = n_items >> 5;  // first block holding a row >= n_items
    // Tile t -> ring slot t % NSLOT by LDS-DMA (global_load_lds_dwordx4: one
    // 1-KB piece per wave-instruction, no VGPR staging); tiles past the end
    // re-load the last piece (keeps the per-wave vmcnt accounting uniform,
    // the data is never used).
    auto issue_tile = [&](int t) {
        uint8_t* slot = smem + (t % NSLOT) * TILE_BYTES;
#pragma unroll
        for (int p = 0; p < LPT; ++p) {
            const int piece = p * NW + wave;
            int off = t * TILE_BYTES + piece * 1024;
            off = off < body_bytes ? off : body_bytes - 1024;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(catalog + off + lane * 16),
                (__attribute__((address_space(3))) void*)(slot + piece * 1024), 16, 0, 0);
        }
    };
    const uint32_t lds0 = lds_base + lane * 16;
    // all fragment reads (and the flush-hint word) and their wait in ONE asm
    // statement: one LDS round trip per tile, and a separate wait statement
    // would let the compiler copy an output before the data landed
    static_assert((TB * DS) % 8 == 0, "fragment groups of 8");
    auto read_frags = [&](int t, u32x4 (&afr)[TB * DS], uint32_t& hraw) {
        const uint32_t base = lds0 + (uint32_t)((t % NSLOT) * TILE_BYTES);
        u32x4* f = &afr[0];
        asm volatile(
            "ds_read_b32 %8, %10\n\t"
            "ds_read_b128 %0, %9 offset:0\n\tds_read_b128 %1, %9 offset:1024\n\t"
            "ds_read_b128 %2, %9 offset:2048\n\tds_read_b128 %3, %9 offset:3072\n\t"
            "ds_read_b128 %4, %9 offset:4096\n\tds_read_b128 %5, %9 offset:5120\n\t"
            "ds_read_b128 %6, %9 offset:6144\n\tds_read_b128 %7, %9 offset:7168\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]), "=&v"(f[5]),
              "=&v"(f[6]), "=&v"(f[7]), "=&v"(hraw)
            : "v"(base), "v"(hint)
            : "memory");
#pragma unroll
        for (int g = 8; g < TB * DS; g += 8) {
            f = &afr[g];
            asm volatile(
                "ds_read_b128 %0, %8 offset:0\n\tds_read_b128 %1, %8 offset:1024\n\t"
                "ds_read_b128 %2, %8 offset:2048\n\tds_read_b128 %3, %8 offset:3072\n\t"
                "ds_read_b128 %4, %8 offset:4096\n\tds_read_b128 %5, %8 offset:5120\n\t"
                "ds_read_b128 %6, %8 offset:6144\n\tds_read_b128 %7, %8 offset:7168\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]), "=&v"(f[5]),
                  "=&v"(f[6]), "=&v"(f[7])
                : "v"(base + 1024u * g)
                : "memory");
        }
    };
    const int full_tiles = tail_blk / TB;  // tiles whose blocks are all full
    auto tile = [&](int t, const u32x4 (&afr)[TB * DS], auto mask_c) {
        constexpr bool MASK = decltype(mask_c)::value;
        float m[TB];
#pragma unroll
        for (int b = 0; b < TB; ++b) {
            f32x16 acc = f32x16{};
#pragma unroll
            for (int s = 0; s < DS; ++s)
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, afr[b * DS + s]),
                                                             ufrag[s], acc, 0, 0, 0);
            if constexpr (MASK) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = (t * TB + b) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (row >= n_items) acc[r] = -INFINITY;
                }
            }
            float v = fmaxf(fmaxf(acc[0], acc[1]), acc[2]);
#pragma unroll
            for (int r = 3; r < 15; r += 2) v = fmaxf(fmaxf(v, acc[r]), acc[r + 1]);
            m[b] = fmaxf(v, acc[15]);
        }
        uint32_t cm = 0;
#pragma unroll
        for (int b = 0; b < TB; ++b) cm |= m[b] > tau ? (1u << b) : 0u;
        if (__builtin_amdgcn_ballot_w64(cm != 0)) {
            // both lanes of a user append in one go, branch-free: lane 0's
            // entries at n + [0, c0), lane 1's at n + c0 + [0, c1); a block
            // not taken is written to slot CL - 1, which a kept entry reaches
            // only when all 2 TB blocks of the user are taken (no dump then)
            const uint32_t pm = partner32(cm, h);
            const int c_own = __popc(cm), c_par = __popc(pm);
            const uint32_t base = (uint32_t)(n + (h ? c_par : 0));
            constexpr uint32_t dump = (uint32_t)(CL - 1) * 128u;
#pragma unroll
            for (int b = 0; b < TB; ++b) {
                const uint32_t off = ((cm >> b) & 1u) ? (base + (uint32_t)__popc(cm & ((1u << b) - 1u))) * 128u
                                                      : dump;
                lds_wr_pair<CL * 32 * 4>(ls + off, __float_as_uint(m[b]), (uint32_t)((t * TB + b) * 2 + h));
            }
            n += c_own + c_par;
        }
    };

#pragma unroll
    for (int p = 0; p < NSLOT - 1; ++p) issue_tile(p);
    for (int t = 0; t < ntile; ++t) {
        // own pieces of tile t landed (the next NSLOT-2 tiles' stay in
        // flight), list appends done; the barrier publishes everyone's
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(LPT * (NSLOT - 2)) : "memory");
        __builtin_amdgcn_s_barrier();
        issue_tile(t + NSLOT - 1);
        u32x4 afr[TB * DS];
        uint32_t hraw;
        read_frags(t, afr, hraw);
        const int hv = (int)__builtin_amdgcn_readfirstlane((int)hraw);
        if (t < full_tiles) tile(t, afr, std::false_type{});
        else tile(t, afr, std::true_type{});
        // flush when a list cannot take the next tile's appends, or with the
        // other waves when one of them flushes at this tile (hint)
        const bool need = __builtin_amdgcn_ballot_w64(n > CAP) != 0;
        const bool soon = __builtin_amdgcn_ballot_w64(n > CAP - 2 * TB) != 0;
        if (soon && lane == 0) lds_wr(hint, (uint32_t)(t + 1));
        if (need || (hv == t && __builtin_amdgcn_ballot_w64(n > CL / 2) != 0))
            user_flush<CL>(ls, li, h, n, tau, theta, ovf, k, eps_s, CAP);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // drain the trailing dummy pieces
    user_flush<CL>(ls, li, h, n, tau, theta, ovf, k, eps_s, CAP);

    if (!active) return;
    float cut = theta;
    if (eps_s != 0.0f && theta != -INFINITY) cut = round_down_sub(theta, 2.0f * eps_s);
    // lane 0 writes list entries [0, min(n, IP_CW)), lane 1 the rest
    const int j0 = h ? IP_CW : 0, j1 = h ? n : (n < IP_CW ? n : IP_CW);
    uint2* dst = cand + ((size_t)user * 2 + h) * IP_CW;
    for (int j = j0; j < j1; ++j) {
        const float sc = lds_rd(ls + (uint32_t)j * 128u);
        const uint32_t id = __float_as_uint(lds_rd(li + (uint32_t)j * 128u));
        dst[j - j0] = make_uint2(__float_as_uint(sc), id);
    }
    cand_cnt[user * 2 + h] = j1 > j0 ? j1 - j0 : 0;
    if (h == 0) {
        // unscaled cut and eps for the refinement (exact power-of-two rescale)
        ucut[user] = make_float2(cut == -INFINITY ? -INFINITY : cut / scl, eps);
        ovf_flag[user] = ovf ? 1 : 0;
        if (ovf) ovf_list[atomicAdd(ovf_count, 1)] = user;
    }
}

// ------------------------------------------------------------ refinement --
__device__ __forceinline__ double exact_dot(const float* __restrict__ a, const float* __restrict__ b,
                                            int dim) {
    double s = 0.0;
    if ((dim & 3) == 0) {
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

constexpr int IP_SURV = 128;  // exact survivors per user held by the refine
constexpr int IP_KRING = 256; // prefilter-kept rows awaiting an exact round (ring, power of two)

// DS4 = dim / 4 when the candidate rows are staged through LDS (dim 16, 32,
// 64): every 64-item round loads the rows with whole-row coalesced float4
// pieces (64 / DS4 rows per instruction) into a padded per-wave LDS stage,
// then each lane sums its own row sequentially (the oracle's order).
// DS4 = 0: the generic per-lane gather.
template <int DS4>
__global__ __launch_bounds__(256) void ip_refine_kernel(
    const float* __restrict__ users, int64_t n_users, const float* __restrict__ items,
    const uint8_t* __restrict__ catalog, int64_t n_items, int dim, int k, int64_t row_offset,
    const uint2* __restrict__ cand,
    const int32_t* __restrict__ cand_cnt, const float2* __restrict__ ucut,
    const int32_t* __restrict__ ovf_flag, int32_t* __restrict__ ovf_list,
    int32_t* __restrict__ ovf_count, float* __restrict__ out_s, int32_t* __restrict__ out_r,
    double* __restrict__ out_e) {
    __shared__ Cand surv[4][IP_SURV];
    __shared__ int32_t krow[DS4 > 0 ? 4 : 1][DS4 > 0 ? IP_KRING : 1];
    constexpr int RS = DS4 + 1;  // staged row stride in float4 (one float4 of padding)
    __shared__ float4 stage[DS4 > 0 ? 4 : 1][DS4 > 0 ? 64 * RS : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    if (u >= n_users || ovf_flag[u]) return;
    const float* uv = users + u * dim;
    // zero user: every score is exactly 0 -> the lowest rows win the ties
    float nz = 0.0f;
    for (int d = lane; d < dim; d += WAVE) nz += fabsf(uv[d]);
    nz = wave_sum_f32(nz);
    if (nz == 0.0f) {
        if (lane < k) {
            const bool ok = lane < n_items;
            out_s[u * k + lane] = ok ? 0.0f : -FLT_MAX;
            out_r[u * k + lane] = ok ? (int32_t)(lane + row_offset) : -1;
            if (out_e) out_e[u * k + lane] = ok ? 0.0 : -INFINITY;
        }
        return;
    }
    const int n0 = cand_cnt[2 * u], n1 = cand_cnt[2 * u + 1];
    const float2 ce = ucut[u];
    double thr = -INFINITY;
    if (ce.x != -INFINITY) {
        thr = (double)ce.x + (double)ce.y;
        thr = thr - fabs(thr) * 1e-15 - 1e-300;  // round down
    }
    // The screen's cut in its scaled fp16 units (exact power-of-two rescale):
    // |fp16 score - exact| <= eps, so every item with exact >= cut + eps has
    // an fp16 score >= cut.  Used twice: (a) band entries (half-blocks) whose
    // listed fp16 max is below it are dropped -- none on one GPU (the final
    // flush kept only entries >= cut), most of the band on a catalog shard
    // after nrk_ip_topk_apply_bound raised the cut to the global bound; (b)
    // the fp16 prefilter (DS4 > 0): every band item's fp16 score recomputed
    // from its 64-B packed row, only items reaching the cut are fetched in
    // fp32 for the exact score.
    constexpr int DSK = DS4 / 4;  // 16-dim k-steps of the packed layout
    const bool pre = catalog != nullptr && ce.x != -INFINITY;
    float ush[DS4 > 0 ? 4 * DS4 : 1];
    float pcut = 0.0f;
    if (pre) {
        const int dpc = pad_dim(dim);
        const int64_t nblk_c = (n_items + 31) >> 5;
        const CatalogHdr* hdr = reinterpret_cast<const CatalogHdr*>(catalog + (size_t)nblk_c * 64 * dpc);
        float ua = 0.0f;
        for (int d = 0; d < dim; ++d) ua = fmaxf(ua, fabsf(uv[d]));
        const float su = pow2_scale(ua);
        if constexpr (DS4 > 0) {
#pragma unroll
            for (int d = 0; d < 4 * DS4; ++d) ush[d] = (float)(_Float16)(uv[d] * su);
        }
        pcut = ce.x * (su * hdr->scale);
    }
    // (a) compact the band of both halves into LDS (list order kept)
    __shared__ uint32_t bandq[4][2 * IP_CW];
    int nband = 0;
    for (int b0 = 0; b0 < n0 + n1; b0 += WAVE) {
        const int e = b0 + lane;
        uint2 ent = make_uint2(0u, 0u);
        if (e < n0 + n1)
            ent = e < n0 ? cand[(size_t)(2 * u) * IP_CW + e] : cand[(size_t)(2 * u + 1) * IP_CW + (e - n0)];
        const bool kp = e < n0 + n1 && (!pre || __uint_as_float(ent.x) >= pcut);
        const unsigned long long bal = __ballot(kp);
        if (kp) bandq[wave][nband + __popcll(bal & ((1ull << lane) - 1ull))] = ent.y;
        nband += __popcll(bal);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nitem = nband * 16;
    int cnt = 0;
    auto push = [&](bool keep, double s, int32_t row) {
        const unsigned long long bal = __ballot(keep);
        const int pos = cnt + __popcll(bal & ((1ull << lane) - 1ull));
        if (keep && pos < IP_SURV) surv[wave][pos] = Cand{s, row};
        cnt += __popcll(bal);
    };
    if constexpr (DS4 > 0) {
        // Two phases over the band.  (A) fp16 prefilter in 64-item rounds,
        // software-pipelined: round i+1's packed fp16 pieces are in flight
        // while round i is scored; the kept items' rows go to a per-wave LDS
        // ring.  (B) whenever the ring holds 64 rows (and once at the end),
        // one exact round: the rows staged through LDS with whole-row
        // coalesced float4 pieces, each lane summing its own row sequentially
        // (the oracle's order).  Most band items fail the prefilter, so the
        // exact rounds (the expensive part) run on full 64-row chunks instead
        // of once per prefilter round.
        uint4 pc[DSK > 0 ? 2 * DSK : 1];
        auto band_q = [&](int base) -> uint32_t {
            int idx = base + lane;
            idx = idx < nitem ? idx : nitem - 1;
            return bandq[wave][idx > 0 ? idx >> 4 : 0];
        };
        auto item_row = [&](int base, uint32_t qv, int32_t& row, bool& inb) {
            const int idx = base + lane, r = idx & 15;
            const int64_t rr = (int64_t)(qv >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (qv & 1);
            inb = idx < nitem && rr < n_items;
            row = inb ? (int32_t)rr : 0;
        };
        auto pieces = [&](int32_t row) {
            if (pre) {
                const int blk = row >> 5, il = row & 31;
                const uint8_t* bp = catalog + (size_t)blk * (64 * 4 * DS4);
#pragma unroll
                for (int st = 0; st < DSK; ++st)
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh)
                        pc[2 * st + hh] = *reinterpret_cast<const uint4*>(bp + st * 1024 + (il + 32 * hh) * 16);
            }
        };
        int kc = 0, ko = 0;  // ring fill / read positions (wave-uniform)
        auto exact_round = [&](int m) {
            const int32_t rl = lane < m ? krow[wave][(ko + lane) & (IP_KRING - 1)] : -1;
            float4 v[DS4];
            bool okv[DS4];
#pragma unroll
            for (int it = 0; it < DS4; ++it) {
                const int g = it * 64 + lane, item = g / DS4, part = g % DS4;
                const int r_item = __shfl(rl, item, WAVE);
                okv[it] = r_item >= 0;
                v[it] = reinterpret_cast<const float4*>(items + (int64_t)(okv[it] ? r_item : 0) * dim)[part];
            }
#pragma unroll
            for (int it = 0; it < DS4; ++it) {
                const int g = it * 64 + lane, item = g / DS4, part = g % DS4;
                stage[wave][item * RS + part] = okv[it] ? v[it] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double sd = 0.0;
            bool keep = false;
            if (rl >= 0) {
                const float4* a4 = reinterpret_cast<const float4*>(uv);
                const float4* b4 = &stage[wave][lane * RS];
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
            __builtin_amdgcn_wave_barrier();  // the stage is rewritten next round
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
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            acc = fmaf((float)hv[e], ush[16 * st + 8 * hh + e], acc);
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
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // (B) exact rounds on full 64-row chunks
            while (kc - ko >= WAVE) exact_round(WAVE);
        }
        while (kc > ko) exact_round(kc - ko < WAVE ? kc - ko : WAVE);
    } else {
        for (int base = 0; base < nitem; base += WAVE) {
            const int idx = base + lane;
            bool keep = false;
            double sd = 0.0;
            int32_t row = 0;
            if (idx < nitem) {
                const int bb = idx >> 4, r = idx & 15;
                const uint32_t q = bandq[wave][bb];
                const int64_t rr = (int64_t)(q >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (q & 1);
                if (rr < n_items) row = (int32_t)rr;
                keep = rr < n_items;
                if (keep) {
                    sd = exact_dot(uv, items + (int64_t)row * dim, dim);
                    keep = sd >= thr;
                }
            }
            push(keep, sd, row);
        }
    }
    if (cnt > IP_SURV) {  // dense exact ties: hand the user to the exact fallback
        if (lane == 0) ovf_list[atomicAdd(ovf_count, 1)] = (int32_t)u;
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    Cand x[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int idx = e * 64 + lane;
        if (idx < cnt) x[e] = surv[wave][idx];
        else { x[e].s = -INFINITY; x[e].row = INT32_MAX; }
    }
    wave_bitonic_sort<2>(x);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int idx = e * 64 + lane;
        if (idx < k) {
            const bool ok = x[e].row != INT32_MAX;
            out_s[u * k + idx] = ok ? (float)x[e].s : -FLT_MAX;
            out_r[u * k + idx] = ok ? (int32_t)(x[e].row + row_offset) : -1;
            if (out_e) out_e[u * k + idx] = ok ? x[e].s : -INFINITY;
        }
    }
}

// -------------------------------------------------------------- fallback --
__device__ __forceinline__ uint64_t okey(double s) {
    const uint64_t b = (uint64_t)__double_as_longlong(s);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__global__ __launch_bounds__(256) void ip_fallback_kernel(
    const float* __restrict__ users, const float* __restrict__ items, int64_t n_items, int dim,
    int k, int64_t row_offset, const int32_t* __restrict__ ovf_list,
    const int32_t* __restrict__ ovf_count, float* __restrict__ out_s, int32_t* __restrict__ out_r,
    double* __restrict__ out_e) {
    __shared__ unsigned int hist[256];
    __shared__ Cand sel[64];
    __shared__ int sel_n;
    __shared__ unsigned long long s_prefix;
    __shared__ int s_krem;
    __shared__ int wcnt[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cnt = *ovf_count;
    const int kk = (int)(n_items < k ? n_items : k);
    for (int q = blockIdx.x; q < cnt; q += gridDim.x) {
        const int64_t u = ovf_list[q];
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
        if (wave == 0) {
            Cand x[1];
            if (lane < sel_n) x[0] = sel[lane];
            else { x[0].s = -INFINITY; x[0].row = INT32_MAX; }
            wave_bitonic_sort<1>(x);
            if (lane < k) {
                const bool ok = lane < kk;
                out_s[u * k + lane] = ok ? (float)x[0].s : -FLT_MAX;
                out_r[u * k + lane] = ok ? (int32_t)(x[0].row + row_offset) : -1;
                if (out_e) out_e[u * k + lane] = ok ? x[0].s : -INFINITY;
            }
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------- merge --
template <int E>
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const double* __restrict__ in_e, const int32_t* __restrict__ in_r, int n_lists,
    int64_t stride, int64_t n_users, int k_in, int k_out, float* __restrict__ out_s,
    int32_t* __restrict__ out_r, double* __restrict__ out_e) {
    const int lane = threadIdx.x & 63;
    const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u >= n_users) return;
    Cand x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int idx = e * 64 + lane;
        const int l = idx / k_in, j = idx - l * k_in;
        x[e].s = -INFINITY;
        x[e].row = INT32_MAX;
        if (l < n_lists) {
            const int64_t o = l * stride + u * k_in + j;
            const int32_t r = in_r[o];
            if (r >= 0) {
                x[e].s = in_e[o];
                x[e].row = r;
            }
        }
    }
    wave_bitonic_sort<E>(x);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int idx = e * 64 + lane;
        if (idx < k_out) {
            const bool ok = x[e].row != INT32_MAX;
            out_s[u * k_out + idx] = ok ? (float)x[e].s : -FLT_MAX;
            out_r[u * k_out + idx] = ok ? x[e].row : -1;
            if (out_e) out_e[u * k_out + idx] = ok ? x[e].s : -INFINITY;
        }
    }
}

// ------------------------------------------------- catalog-shard bound --
constexpr int IP_BOUND_MMAX = 32;

// Per user, the m largest listed half-block maxima of this shard's band as
// exact lower bounds: a half-block whose fp16 max is x (scaled units, scl =
// su * catalog scale) holds an item with exact score >= x / scl - eps.
// Distinct half-blocks are distinct items, so any k of these values bound k
// distinct items from below.  Descending, -inf padded (fp32, rounded down).
template <int MM>
__global__ void ip_bound_kernel(const float* __restrict__ users, int64_t n_users, int dim,
                                const CatalogHdr* __restrict__ hdr, const uint2* __restrict__ cand,
                                const int32_t* __restrict__ cand_cnt, const float2* __restrict__ ucut,
                                int m, float* __restrict__ out) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_users) return;
    float best[MM];
#pragma unroll
    for (int j = 0; j < MM; ++j) best[j] = -INFINITY;
    const int n0 = cand_cnt[2 * u], n1 = cand_cnt[2 * u + 1];
    if (n0 + n1 > 0) {
        const float* uv = users + u * dim;
        float ua = 0.0f;
        for (int d = 0; d < dim; ++d) ua = fmaxf(ua, fabsf(uv[d]));
        const double inv = 1.0 / ((double)pow2_scale(ua) * (double)hdr->scale);  // exact power of two
        const double eps = (double)ucut[u].y;
        for (int e = 0; e < n0 + n1; ++e) {
            const uint2 c = e < n0 ? cand[(size_t)(2 * u) * IP_CW + e] : cand[(size_t)(2 * u + 1) * IP_CW + (e - n0)];
            const double t = (double)__uint_as_float(c.x) * inv - eps;
            float v = (float)t;
            if ((double)v > t) v = nextafterf(v, -INFINITY);
            // insertion into the descending top-m
#pragma unroll
            for (int j = 0; j < MM; ++j) {
                const bool in = j < m && v > best[j];
                const float o = best[j];
                best[j] = in ? v : o;
                v = in ? o : v;
            }
        }
    }
    for (int j = 0; j < m; ++j) out[u * m + j] = best[j];
}

// G = the k-th largest of the n_lists * m bounds of the user (lists laid out
// [n_lists][n_users][m]; -inf when there are fewer than k finite values) is a
// lower bound of the user's k-th exact score over the whole catalog.  Raise
// the shard's cut to G - eps (rounded down to fp32): the refine then keeps
// exact >= cut + eps <= G, and the band / prefilter tests use the raised cut.
// One wave per user: one value per lane, wave bitonic sort (n_lists * m <= 64).
__global__ __launch_bounds__(256) void ip_apply_bound_kernel(float2* __restrict__ ucut, int64_t n_users,
                                                             const float* __restrict__ vals, int n_lists,
                                                             int m, int k) {
    const int lane = threadIdx.x & 63;
    const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u >= n_users) return;
    Cand x[1];
    x[0].row = lane;
    x[0].s = -(double)INFINITY;
    if (lane < n_lists * m) {
        const int l = lane / m, j = lane - l * m;
        x[0].s = (double)vals[((int64_t)l * n_users + u) * m + j];
    }
    wave_bitonic_sort<1>(x);
    const double G = __shfl(x[0].s, k - 1, WAVE);
    if (lane != 0 || !(G > -(double)INFINITY)) return;
    float2 c = ucut[u];
    const double t = G - (double)c.y;
    float f = (float)t;
    if ((double)f > t) f = nextafterf(f, -INFINITY);
    if (f > c.x) {
        c.x = f;
        ucut[u] = c;
    }
}

// ------------------------------------------------------------- workspace --
struct IpWs {
    uint2* cand;
    float2* ucut;
    int32_t* cnt;
    int32_t* ovf_flag;
    int32_t* ovf_list;
    int32_t* ovf_count;
    size_t bytes;
};

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static IpWs ip_ws_layout(void* base, int64_t n_users) {
    IpWs w;
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    size_t off = 0;
    w.ovf_count = reinterpret_cast<int32_t*>(p + off);
    off += 256;
    w.cand = reinterpret_cast<uint2*>(p + off);
    off += align256((size_t)n_users * 2 * IP_CW * sizeof(uint2));
    w.ucut = reinterpret_cast<float2*>(p + off);
    off += align256((size_t)n_users * sizeof(float2));
    w.cnt = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * 2 * sizeof(int32_t));
    w.ovf_flag = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * sizeof(int32_t));
    w.ovf_list = reinterpret_cast<int32_t*>(p + off);
    off += align256((size_t)n_users * sizeof(int32_t));
    w.bytes = off;
    return w;
}

}  // namespace nrk

using namespace nrk;

extern "C" {

size_t nrk_ip_catalog_bytes(int64_t n_items, int dim) {
    if (n_items < 0 || dim <= 0 || dim > 256) return 0;
    return catalog_body_bytes(n_items, pad_dim(dim)) + CATALOG_HDR;
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
        const int g2 = (int)std::min<int64_t>((n_items + 255) / 256, 2048);
        catalog_norm_kernel<<<g2, 256, 0, s>>>(items, n_items, dim, hdr);
    }
    catalog_hdr_kernel<<<1, 1, 0, s>>>(hdr, dim, dp);
    if (total > 0) {
        const int g2 = (int)std::min<int64_t>((n_items + 255) / 256, 2048);
        catalog_dnorm_kernel<<<g2, 256, 0, s>>>(items, n_items, dim, hdr);
        const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
        catalog_pack_kernel<<<grid, 256, 0, s>>>(items, n_items, dim, dp, hdr,
                                                 reinterpret_cast<uint4*>(catalog));
    }
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_ip_topk_workspace_bytes(int64_t n_users, int64_t n_items, int dim, int k) {
    (void)n_items;
    (void)dim;
    (void)k;
    if (n_users < 0) return 0;
    return ip_ws_layout(nullptr, n_users).bytes;
}

static int ip_check(const float* users, int64_t n_users, const float* items, const void* catalog,
                    int64_t n_items, int dim, int k, void* workspace, size_t workspace_bytes) {
    NRK_REQUIRE(n_users >= 0 && n_items >= 0, "negative sizes");
    NRK_REQUIRE(n_items < (1ll << 30) && n_users < (1ll << 30), "n_items / n_users must be < 2^30");
    NRK_REQUIRE(dim > 0 && dim <= 256, "dim must be in [1, 256]");
    NRK_REQUIRE(k >= 1, "k must be >= 1");
    if (k > IP_KMAX) NRK_UNSUPPORTED("k > 32 is not compiled");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(users && workspace, "null pointer");
    NRK_REQUIRE(n_items == 0 || (items && catalog), "items/catalog null");
    NRK_REQUIRE(workspace_bytes >= ip_ws_layout(nullptr, n_users).bytes, "workspace too small");
    return NRK_OK;
}

int nrk_ip_topk_screen(const float* users, int64_t n_users, const void* catalog, int64_t n_items,
                       int dim, int k, void* workspace, size_t workspace_bytes,
                       nrk_stream_t stream) {
    clear_error();
    int rc = ip_check(users, n_users, (const float*)catalog, catalog, n_items, dim, k, workspace,
                      workspace_bytes);
    if (rc != NRK_OK || n_users == 0) return rc;
    const IpWs w = ip_ws_layout(workspace, n_users);
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(w.ovf_count, 0, 256, s) != hipSuccess) {
        set_error("nrk_ip_topk_screen: hipMemsetAsync failed");
        return NRK_EHIP;
    }
    const int dp = pad_dim(dim);
    const uint8_t* cat = reinterpret_cast<const uint8_t*>(catalog);
    if (n_items == 0) {
        // nothing to search: every output row is padding
        (void)hipMemsetAsync(w.cnt, 0, (size_t)n_users * 2 * sizeof(int32_t), s);
        (void)hipMemsetAsync(w.ovf_flag, 0, (size_t)n_users * sizeof(int32_t), s);
    } else {
#define NRK_SCREEN(DPV, NWV)                                                               \
    ip_screen_kernel<DPV, NWV><<<(int)((n_users + 32 * NWV - 1) / (32 * NWV)), 64 * NWV, 0, s>>>( \
        users, (int)n_users, cat, (int)n_items, dim, k, w.cand, w.cnt, w.ucut, w.ovf_flag,       \
        w.ovf_list, w.ovf_count)
        // 4 waves (128 users) per workgroup, a 2-tile LDS-DMA ring and 62-entry
        // lists: 79.9 KB of LDS, so two workgroups share a CU and each one's
        // per-tile barrier / DMA wait is covered by the other (9.5 ms at config
        // 2 against 10.3 ms for one 8-wave workgroup with a 3-tile ring;
        // tools/screen_variants.sh).  NRK_SCREEN_VARIANT=0 selects the latter.
        static const int var = [] { const char* e = getenv("NRK_SCREEN_VARIANT"); return e ? atoi(e) : 1; }();
#define NRK_SCREEN_V(DPV, NWV, NSV, CLV)                                                                   \
    ip_screen_kernel<DPV, NWV, NSV, CLV><<<(int)((n_users + 32 * NWV - 1) / (32 * NWV)), 64 * NWV, 0, s>>>( \
        users, (int)n_users, cat, (int)n_items, dim, k, w.cand, w.cnt, w.ucut, w.ovf_flag, w.ovf_list,        \
        w.ovf_count)
        if (var == 1 && dp <= 64) {  // D = 128 (config 5): the 8-wave form measured 0.8% faster
            switch (dp) {
                case 16: NRK_SCREEN_V(16, 4, 2, 62); break;
                case 32: NRK_SCREEN_V(32, 4, 2, 62); break;
                default: NRK_SCREEN_V(64, 4, 2, 62); break;
            }
        } else switch (dp) {
            case 16: NRK_SCREEN(16, 8); break;
            case 32: NRK_SCREEN(32, 8); break;
            case 64: NRK_SCREEN(64, 8); break;
            case 128: NRK_SCREEN(128, 8); break;
            default: NRK_SCREEN(256, 4); break;
        }
#undef NRK_SCREEN_V
#undef NRK_SCREEN
    }
    NRK_CHECK_LAUNCH();
    return NRK_OK;
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
    const IpWs w = ip_ws_layout(workspace, n_users);
    hipStream_t s = as_stream(stream);
    const int g2 = (int)((n_users + 3) / 4);
#define NRK_REFINE(DS4)                                                                        \
    ip_refine_kernel<DS4><<<g2, 256, 0, s>>>(users, n_users, items,                             \
                                             reinterpret_cast<const uint8_t*>(catalog), n_items, \
                                             dim, k, row_offset,                                 \
                                             w.cand, w.cnt, w.ucut, w.ovf_flag, w.ovf_list,      \
                                             w.ovf_count, out_scores, out_rows, out_exact)
    if (dim == 32) NRK_REFINE(8);
    else if (dim == 16) NRK_REFINE(4);
    else if (dim == 64) NRK_REFINE(16);
    else NRK_REFINE(0);
#undef NRK_REFINE
    if (n_items > 0)
        ip_fallback_kernel<<<256, 256, 0, s>>>(users, items, n_items, dim, k, row_offset, w.ovf_list,
                                               w.ovf_count, out_scores, out_rows, out_exact);
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
                      int m, float* out_bound, void* workspace, size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    int rc = ip_check(users, n_users, (const float*)catalog, catalog, n_items, dim, 1, workspace,
                      workspace_bytes);
    if (rc != NRK_OK) return rc;
    NRK_REQUIRE(m >= 1 && m <= IP_BOUND_MMAX, "m must be in [1, 32]");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(out_bound != nullptr, "null pointer");
    const IpWs w = ip_ws_layout(workspace, n_users);
    hipStream_t s = as_stream(stream);
    if (n_items == 0) {
        // empty shard: no bound (the screen wrote no band)
        (void)hipMemsetAsync(w.cnt, 0, (size_t)n_users * 2 * sizeof(int32_t), s);
    }
    const CatalogHdr* hdr = reinterpret_cast<const CatalogHdr*>(
        reinterpret_cast<const uint8_t*>(catalog) + catalog_body_bytes(n_items, pad_dim(dim)));
    const int grid = (int)((n_users + 255) / 256);
    if (m <= 8)
        ip_bound_kernel<8><<<grid, 256, 0, s>>>(users, n_users, dim, hdr, w.cand, w.cnt, w.ucut, m, out_bound);
    else
        ip_bound_kernel<IP_BOUND_MMAX><<<grid, 256, 0, s>>>(users, n_users, dim, hdr, w.cand, w.cnt, w.ucut, m,
                                                            out_bound);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_ip_topk_apply_bound(int64_t n_users, const float* bounds, int n_lists, int m, int k, void* workspace,
                            size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_users >= 0 && n_users < (1ll << 30), "n_users out of range");
    NRK_REQUIRE(n_lists >= 1 && m >= 1 && n_lists * m <= 64, "need 1 <= n_lists * m <= 64");
    NRK_REQUIRE(k >= 1 && k <= IP_KMAX, "k must be in [1, 32]");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(bounds && workspace, "null pointer");
    NRK_REQUIRE(workspace_bytes >= ip_ws_layout(nullptr, n_users).bytes, "workspace too small");
    const IpWs w = ip_ws_layout(workspace, n_users);
    if (k > n_lists * m) return NRK_OK;  // fewer values than k: no bound, cut unchanged
    ip_apply_bound_kernel<<<(int)((n_users + 3) / 4), 256, 0, as_stream(stream)>>>(w.ucut, n_users, bounds,
                                                                                 n_lists, m, k);
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
    if (tot > 512) NRK_UNSUPPORTED("n_lists * k_in > 512");
    NRK_REQUIRE(k_out <= tot, "k_out > n_lists * k_in");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(in_exact && in_rows && out_scores && out_rows, "null pointer");
    hipStream_t s = as_stream(stream);
    const int grid = (int)((n_users + 3) / 4);
    if (tot <= 64)
        topk_merge_kernel<1><<<grid, 256, 0, s>>>(in_exact, in_rows, n_lists, list_stride, n_users, k_in, k_out, out_scores, out_rows, out_exact);
    else if (tot <= 128)
        topk_merge_kernel<2><<<grid, 256, 0, s>>>(in_exact, in_rows, n_lists, list_stride, n_users, k_in, k_out, out_scores, out_rows, out_exact);
    else if (tot <= 256)
        topk_merge_kernel<4><<<grid, 256, 0, s>>>(in_exact, in_rows, n_lists, list_stride, n_users, k_in, k_out, out_scores, out_rows, out_exact);
    else
        topk_merge_kernel<8><<<grid, 256, 0, s>>>(in_exact, in_rows, n_lists, list_stride, n_users, k_in, k_out, out_scores, out_rows, out_exact);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
