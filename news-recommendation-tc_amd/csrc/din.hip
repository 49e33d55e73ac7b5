// din.hip -- DIN attention-over-history scorer (DINModel.forward, eval) on gfx950.
//
// Reference: src/rank/DIN.py:29-286 (Dice :29-44, ActivationUnit :47-130,
// DINModel.forward :214-286) as DINRanker.predict drives it (:1219-1283).
// All arithmetic is fp32 (parity 1e-5); the embedding tables may be stored as
// bf16 (storage only) or fp32.
//
// Dice normalises with the BATCH mean and unbiased std of every column
// (DIN.py:39-44), so each Dice splits the forward into phases with a
// batch-wide reduction in between.  One call scores every Dice batch of a
// pass (segments of S samples), one launch per phase:
//   1. din_att_h      h[b,t,:] = (Wk - Wd) k_t + (Wq + Wd) q + Wp (q .* k_t) + b0
//                     (= Linear(512->36) on [k, q, q-k, q.*k], DIN.py:105-114,
//                     with the batch-invariant parts folded by nrk_din_prepare);
//                     per-block fp64 column sums of h and h^2.
//   2. col_stats      mean / unbiased std per (t, j) (deterministic, fixed order).
//   3. din_wh         Dice -> Linear(36->1) -> * mask (no softmax, :117-124),
//                     weighted history sum wh (:276).
//   4. din_mlp1       Linear(928->h1) on [user, ctx, cand, wh] (:279-282), the
//                     embedding parts gathered straight from the table; 5. col_stats,
//   6. din_mlp2       Dice-on-load -> Linear(h1->h2); 7. col_stats,
//   8. din_head       Dice -> Linear(h2->1) -> sigmoid (:282-284).
// The general path (T > 64 or h1 > 256) assembles the MLP input with
// din_att_out and runs the f32 MFMA din_gemm instead of 3, 4 and 6.
#include "din_common.h"

namespace nrk {


template <typename TT>
__device__ __forceinline__ float tload(const TT* p);
template <>
__device__ __forceinline__ float tload<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float tload<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
// raw element bits (fp32 bits, or bf16 bits in the low half), for loads whose
// conversion is deferred to the use
__device__ __forceinline__ uint32_t table_bits(const float* p) { return __float_as_uint(*p); }
__device__ __forceinline__ uint32_t table_bits(const uint16_t* p) { return *p; }

// Dice (DIN.py:39-44), fp32 in the reference's operation order.
__device__ __forceinline__ float dice(float x, float mean, float std) {
    const float xn = (x - mean) / (std + 1e-8f);
    const float p = 1.0f / (1.0f + expf(-xn));
    return p * x + ((1.0f - p) * 0.01f) * x;
}

// ------------------------------------------------------------- 1. att h --
// h[b, t, :] = M_b k_t + c_b with M_b = (Wk - Wd) + Wp diag(q_b) [36 x ID]
// and c_b = (Wq + Wd) q_b + b0: per sample a [T x ID] x [ID x 36] product,
// run on the fp16 MFMA (v_mfma_f32_16x16x32_f16) as an exact-f32-class
// split product:
//   * bf16 tables: k is exactly representable in fp16 (scaled by the
//     power-of-two s_k), M_b = M_hi + M_lo (two fp16 terms, scaled by s_m)
//     -> 2 MFMAs per fragment, error ~2^-22 |M| |k| per product + the fp32
//     accumulation (the same class as an f32 GEMM);
//   * fp32 tables: k = k_hi + k_lo too -> 3 MFMAs (k_lo * M_lo dropped).
// The scales live in the prep header (nrk_din_prepare, from the table and
// weight maxima) so that every scaled value is a normal fp16.
// Workgroup = 4 waves; wave w owns t-tiles {w, w+4} (16 rows each) and all
// three 16-column j-tiles (36 -> 48).  M_b's fragments are built once per
// sample into LDS by the whole workgroup; each wave gathers its own k rows
// straight from the table into A fragments.  Column statistics of h
// (fp64 sum / sumsq per (t, j)) stay in registers across the workgroup's
// samples (grid-strided), one partial row per workgroup.

constexpr int DIN_JT = 3;  // 36 columns -> 3 tiles of 16


template <typename TT>
__device__ __forceinline__ void load8(const TT* p, float (&v)[8]);
template <>
__device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <>
__device__ __forceinline__ void load8<uint16_t>(const uint16_t* p, float (&v)[8]) {
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
}


// Segments: the N samples are scored as consecutive Dice batches of S
// (DINRanker.predict's DataLoader batches, DIN.py:1245-1283); workgroup
// blockIdx.x = seg * G + g strides over segment seg's samples, so partial row
// blockIdx.x belongs to segment blockIdx.x / G.
template <typename TT, int NI, int NTW>
__global__ __launch_bounds__(256) void din_att_h_kernel(
    const TT* __restrict__ table, const int64_t* __restrict__ row_base, int n_user,
    const int32_t* __restrict__ item_idx, const int32_t* __restrict__ hist_idx, int64_t N,
    int64_t S, int G, int T, const float* __restrict__ prep, const float* __restrict__ att_b0,
    float* __restrict__ h_out, double* __restrict__ partial) {
    constexpr int ID = NI * DIN_E;
    constexpr bool F32 = sizeof(TT) == 4;
    constexpr int NSLOT = DIN_JT * NI * 64;               // fragment lane-slots per pass
    constexpr int SPT = (NSLOT + 255) / 256;              // slots per thread
    __shared__ __attribute__((aligned(16))) din_half8 mf[2][DIN_JT][NI][64];  // M_b hi / lo
    __shared__ float qs[ID];
    __shared__ float cs[48];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const float* A = prep;
    const float* Bq = prep + DIN_H * ID;
    const float* P = prep + 2 * DIN_H * ID;
    const DinScales sc = *reinterpret_cast<const DinScales*>(prep + 3 * DIN_H * ID);

    // this thread's M slots: fixed (j, k..k+8) -> A, P in registers
    float ra[SPT][8], rp[SPT][8];
#pragma unroll
    for (int m = 0; m < SPT; ++m) {
        const int q = tid + 256 * m;
        const int jt = q / (NI * 64), s = (q / 64) % NI, l = q % 64;
        const int j = 16 * jt + (l & 15), k = 32 * s + 8 * (l >> 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const bool ok = q < NSLOT && j < DIN_H;
            ra[m][e] = ok ? A[j * ID + k + e] : 0.0f;
            rp[m][e] = ok ? P[j * ID + k + e] : 0.0f;
        }
    }
    // c_b partials: thread -> (j = tid / 4, quarter of k)
    constexpr int CQ = ID / 4;
    float rbq[CQ];
    {
        const int j = tid >> 2, k0 = (tid & 3) * CQ;
#pragma unroll
        for (int e = 0; e < CQ; ++e) rbq[e] = j < DIN_H ? Bq[j * ID + k0 + e] : 0.0f;
    }
    double ssum[NTW][DIN_JT][4], ssq[NTW][DIN_JT][4];
#pragma unroll
    for (int a = 0; a < NTW; ++a)
#pragma unroll
        for (int b = 0; b < DIN_JT; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) ssum[a][b][r] = ssq[a][b][r] = 0.0;

    const int64_t seg = blockIdx.x / G;
    const int64_t b_end = (seg + 1) * S < N ? (seg + 1) * S : N;
    // software pipeline over this workgroup's samples b, b + G, ...: the
    // history / candidate indices are loaded two samples ahead and the table
    // rows (k rows, q) one sample ahead, so each sample's gathers overlap the
    // previous sample's M_b build, MFMAs and epilogue
    constexpr int RW = F32 ? 2 : 1;  // 16-B pieces per lane per k row
    typedef uint32_t u4n __attribute__((ext_vector_type(4)));
    // row bases hoisted out of the loop, and q kept as raw bits until use: a
    // gather whose address or conversion depends on another load in flight
    // makes the compiler wait vmcnt(0), draining the prefetched rows with it
    int64_t rbs[NI];
#pragma unroll
    for (int s = 0; s < NI; ++s) rbs[s] = row_base[n_user + s];
    const int64_t qbase = tid < ID ? row_base[n_user + tid / DIN_E] : 0;
    const float b0j = (tid >> 2) < DIN_H ? att_b0[tid >> 2] : 0.0f;
    auto q_of = [&](uint32_t bits) { return F32 ? __uint_as_float(bits) : __uint_as_float(bits << 16); };
    auto idx_of = [&](int64_t bb, int32_t (&hi)[NTW][NI], int32_t& qi) {
#pragma unroll
        for (int a = 0; a < NTW; ++a) {
            const int t = 16 * (wv + 4 * a) + (lane & 15);
#pragma unroll
            for (int s = 0; s < NI; ++s) hi[a][s] = (bb < b_end && t < T) ? hist_idx[(bb * T + t) * NI + s] : -1;
        }
        qi = (bb < b_end && tid < ID) ? item_idx[bb * NI + tid / DIN_E] : -1;
    };
    auto rows_of = [&](const int32_t (&hi)[NTW][NI], int32_t qi, u4n (&raw)[NTW][NI][RW], uint32_t& qv) {
#pragma unroll
        for (int a = 0; a < NTW; ++a)
#pragma unroll
            for (int s = 0; s < NI; ++s) {
#pragma unroll
                for (int w = 0; w < RW; ++w) raw[a][s][w] = u4n{0u, 0u, 0u, 0u};
                if (hi[a][s] >= 0) {
                    const u4n* p = reinterpret_cast<const u4n*>(
                        table + (rbs[s] + hi[a][s]) * DIN_E + 8 * (lane >> 4));
#pragma unroll
                    for (int w = 0; w < RW; ++w) raw[a][s][w] = p[w];
                }
            }
        qv = qi >= 0 ? (uint32_t)table_bits(table + (qbase + qi) * DIN_E + tid % DIN_E) : 0u;
    };
    int32_t nidx[NTW][NI], nqi;
    u4n raw[NTW][NI][RW];
    uint32_t qv;
    {
        int32_t i0[NTW][NI], q0;
        idx_of(seg * S + blockIdx.x % G, i0, q0);
        rows_of(i0, q0, raw, qv);
        idx_of(seg * S + blockIdx.x % G + G, nidx, nqi);
    }
    for (int64_t b = seg * S + blockIdx.x % G; b < b_end; b += G) {
        u4n nraw[NTW][NI][RW];
        uint32_t nqv;
        rows_of(nidx, nqi, nraw, nqv);      // rows of sample b + G
        idx_of(b + 2 * G, nidx, nqi);       // indices of sample b + 2G
        // (1) this wave's k rows -> A fragments
        din_half8 ahi[NTW][NI], alo[NTW][NI];
#pragma unroll
        for (int a = 0; a < NTW; ++a)
#pragma unroll
            for (int s = 0; s < NI; ++s) {
                float v[8];
                if (F32) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[e] = __uint_as_float(raw[a][s][0][e]);
                        v[4 + e] = __uint_as_float(raw[a][s][RW - 1][e]);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        v[2 * i] = __uint_as_float(raw[a][s][0][i] << 16);
                        v[2 * i + 1] = __uint_as_float(raw[a][s][0][i] & 0xFFFF0000u);
                    }
                }
                split8(v, sc.s_k, ahi[a][s], alo[a][s]);
            }
        // (2) query embedding
        if (tid < ID) qs[tid] = q_of(qv);
#pragma unroll
        for (int a = 0; a < NTW; ++a)
#pragma unroll
            for (int s = 0; s < NI; ++s)
#pragma unroll
                for (int w = 0; w < RW; ++w) raw[a][s][w] = nraw[a][s][w];
        qv = nqv;
        lds_barrier();
        // (3) M_b fragments (hi / lo, scaled by s_m) and c_b
#pragma unroll
        for (int m = 0; m < SPT; ++m) {
            const int q = tid + 256 * m;
            if (q < NSLOT) {
                const int jt = q / (NI * 64), s = (q / 64) % NI, l = q % 64;
                const int k = 32 * s + 8 * (l >> 4);
                float mv[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) mv[e] = fmaf(rp[m][e], qs[k + e], ra[m][e]);
                din_half8 hi, lo;
                split8(mv, sc.s_m, hi, lo);
                mf[0][jt][s][l] = hi;
                mf[1][jt][s][l] = lo;
            }
        }
        {
            const int k0 = (tid & 3) * CQ;
            float c = 0.0f;
#pragma unroll
            for (int e = 0; e < CQ; ++e) c = fmaf(rbq[e], qs[k0 + e], c);
            c += __shfl_xor(c, 1, WAVE);
            c += __shfl_xor(c, 2, WAVE);
            const int j = tid >> 2;
            if ((tid & 3) == 0 && j < DIN_H) cs[j] = c + b0j;
        }
        lds_barrier();
        // (4) MFMAs + epilogue
#pragma unroll
        for (int a = 0; a < NTW; ++a) {
            const int tt = wv + 4 * a;
            if (16 * tt >= T) continue;
#pragma unroll
            for (int jt = 0; jt < DIN_JT; ++jt) {
                din_f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int s = 0; s < NI; ++s) {
                    const din_half8 bh = mf[0][jt][s][lane];
                    const din_half8 bl = mf[1][jt][s][lane];
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[a][s], bh, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[a][s], bl, acc, 0, 0, 0);
                    if (F32) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[a][s], bh, acc, 0, 0, 0);
                }
                const int j = 16 * jt + (lane & 15);
                const float cj = j < DIN_H ? cs[j] : 0.0f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = 16 * tt + 4 * (lane >> 4) + r;
                    if (t < T && j < DIN_H) {
                        const float v = acc[r] * sc.inv + cj;
                        h_out[(b * T + t) * DIN_H + j] = v;
                        ssum[a][jt][r] += (double)v;
                        ssq[a][jt][r] += (double)v * (double)v;
                    }
                }
            }
        }
    }
    // per-workgroup partial column sums (every (t, j) is owned by one lane)
    double2* dst = reinterpret_cast<double2*>(partial) + (size_t)blockIdx.x * T * DIN_H;
#pragma unroll
    for (int a = 0; a < NTW; ++a)
#pragma unroll
        for (int jt = 0; jt < DIN_JT; ++jt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int t = 16 * (wv + 4 * a) + 4 * (lane >> 4) + r;
                const int j = 16 * jt + (lane & 15);
                if (t < T && j < DIN_H) dst[t * DIN_H + j] = make_double2(ssum[a][jt][r], ssq[a][jt][r]);
            }
}

// din_att_h2: the T <= 64 path (one t-tile per wave) of din_att_h with a
// two-deep gather pipeline.  gfx9 retires vector memory operations in issue
// order and the compiler can only count them statically when none is
// conditional: one conditional load or store between a prefetch and its use
// makes the wait for ANY older load a vmcnt(0), which drains the prefetch
// (din_att_h pays this at the end of every sample).  Here every vector memory
// operation of the loop is unconditional --
//   * indices and rows are read at clamped addresses (sample min(b, b_end-1),
//     slot 0 for t >= T): real, finite rows whose h lands in padding rows
//     that are never stored;
//   * h is written with buffer stores whose out-of-range offsets the hardware
//     drops (t >= T, j >= 36);
//   * statistics accumulate every (t, j) of the tile; only real ones are
//     written --
// and the k rows / q bits of sample b + 2G are issued into the registers
// sample b just converted (two register sets, the loop unrolled by two: no
// copy of an in-flight register), after the indices of b + 3G.
template <typename TT, int NI>
__global__ __launch_bounds__(256, 2) void din_att_h2_kernel(
    const TT* __restrict__ table, const int64_t* __restrict__ row_base, int n_user,
    const int32_t* __restrict__ item_idx, const int32_t* __restrict__ hist_idx, int64_t N,
    int64_t S, int G, int T, const float* __restrict__ prep, const float* __restrict__ att_b0,
    float* __restrict__ h_out, double* __restrict__ partial) {
    constexpr int ID = NI * DIN_E;
    constexpr bool F32 = sizeof(TT) == 4;
    constexpr int NSLOT = DIN_JT * NI * 64;
    constexpr int SPT = (NSLOT + 255) / 256;
    constexpr int RW = F32 ? 2 : 1;
    typedef uint32_t u4n __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) din_half8 mf[2][DIN_JT][NI][64];
    __shared__ float qs[ID];
    __shared__ float cs[48];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const float* A = prep;
    const float* Bq = prep + DIN_H * ID;
    const float* P = prep + 2 * DIN_H * ID;
    const DinScales sc = *reinterpret_cast<const DinScales*>(prep + 3 * DIN_H * ID);

    float ra[SPT][8], rp[SPT][8];
#pragma unroll
    for (int m = 0; m < SPT; ++m) {
        const int q = tid + 256 * m;
        const int jt = q / (NI * 64), s = (q / 64) % NI, l = q % 64;
        const int j = 16 * jt + (l & 15), k = 32 * s + 8 * (l >> 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const bool ok = q < NSLOT && j < DIN_H;
            ra[m][e] = ok ? A[j * ID + k + e] : 0.0f;
            rp[m][e] = ok ? P[j * ID + k + e] : 0.0f;
        }
    }
    constexpr int CQ = ID / 4;
    float rbq[CQ];
    {
        const int j = tid >> 2, k0 = (tid & 3) * CQ;
#pragma unroll
        for (int e = 0; e < CQ; ++e) rbq[e] = j < DIN_H ? Bq[j * ID + k0 + e] : 0.0f;
    }
    double ssum[DIN_JT][4], ssq[DIN_JT][4];
#pragma unroll
    for (int b = 0; b < DIN_JT; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) ssum[b][r] = ssq[b][r] = 0.0;

    const int64_t seg = blockIdx.x / G;
    const int64_t b_end = (seg + 1) * S < N ? (seg + 1) * S : N;
    const int64_t b0 = seg * S + blockIdx.x % G;
    int64_t rbs[NI];
#pragma unroll
    for (int s = 0; s < NI; ++s) rbs[s] = row_base[n_user + s];
    const int qf = tid < ID ? tid / DIN_E : 0;
    const int64_t qbase = row_base[n_user + qf];
    const float b0j = (tid >> 2) < DIN_H ? att_b0[tid >> 2] : 0.0f;
    const int trow = 16 * wv + (lane & 15);
    const int tg = trow < T ? trow : 0;  // gather slot (padding rows read slot 0)
    auto clampb = [&](int64_t bb) { return bb < b_end ? bb : b_end - 1; };
    auto hidx_of = [&](int64_t bb, int32_t (&hi)[NI]) {
        const int32_t* p = hist_idx + (clampb(bb) * T + tg) * NI;
#pragma unroll
        for (int s = 0; s < NI; ++s) hi[s] = p[s];
    };
    auto qi_of = [&](int64_t bb) -> int32_t { return item_idx[clampb(bb) * NI + qf]; };
    auto rows_of = [&](const int32_t (&hi)[NI], u4n (&raw)[NI][RW]) {
#pragma unroll
        for (int s = 0; s < NI; ++s) {
            const u4n* p = reinterpret_cast<const u4n*>(table + (rbs[s] + hi[s]) * DIN_E + 8 * (lane >> 4));
#pragma unroll
            for (int w = 0; w < RW; ++w) raw[s][w] = p[w];
        }
    };
    auto qbits_of = [&](int32_t qi) -> uint32_t { return table_bits(table + (qbase + qi) * DIN_E + tid % DIN_E); };

    // prologue: every index first, then rows / q of b0 (set A) and b0 + G (set B)
    u4n rawA[NI][RW], rawB[NI][RW];
    uint32_t qvA, qvB;
    int32_t hiA[NI], hiB[NI], qiA, qiB;
    {
        int32_t h0[NI], h1[NI];
        hidx_of(b0, h0);
        const int32_t q0 = qi_of(b0);
        hidx_of(b0 + G, h1);
        const int32_t q1 = qi_of(b0 + G);
        rows_of(h0, rawA);
        qvA = qbits_of(q0);
        rows_of(h1, rawB);
        qvB = qbits_of(q1);
    }
    hidx_of(b0 + 2 * G, hiA);
    qiA = qi_of(b0 + 2 * G);

    // sample b from (raw, qv); then issue b + 3G's indices into (hn, qn) and
    // b + 2G's rows / q (indices hc, qc) into (raw, qv)
    auto step = [&](int64_t b, u4n (&raw)[NI][RW], uint32_t& qv, const int32_t (&hc)[NI], const int32_t& qc,
                    int32_t (&hn)[NI], int32_t& qn) {
        // (1) this wave's k rows -> A fragments; q -> LDS
        din_half8 ahi[NI], alo[NI];
#pragma unroll
        for (int s = 0; s < NI; ++s) {
            float v[8];
            if (F32) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = __uint_as_float(raw[s][0][e]);
                    v[4 + e] = __uint_as_float(raw[s][RW - 1][e]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[2 * i] = __uint_as_float(raw[s][0][i] << 16);
                    v[2 * i + 1] = __uint_as_float(raw[s][0][i] & 0xFFFF0000u);
                }
            }
            split8(v, sc.s_k, ahi[s], alo[s]);
        }
        if (tid < ID) qs[tid] = F32 ? __uint_as_float(qv) : __uint_as_float(qv << 16);
        // (2) prefetch: indices of b + 3G, then rows / q of b + 2G into the
        // registers just consumed
        hidx_of(b + 3 * G, hn);
        qn = qi_of(b + 3 * G);
        rows_of(hc, raw);
        qv = qbits_of(qc);
        lds_barrier();
        // (3) M_b fragments and c_b
#pragma unroll
        for (int m = 0; m < SPT; ++m) {
            const int q = tid + 256 * m;
            if (q < NSLOT) {
                const int jt = q / (NI * 64), s = (q / 64) % NI, l = q % 64;
                const int k = 32 * s + 8 * (l >> 4);
                float mv[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) mv[e] = fmaf(rp[m][e], qs[k + e], ra[m][e]);
                din_half8 hi, lo;
                split8(mv, sc.s_m, hi, lo);
                mf[0][jt][s][l] = hi;
                mf[1][jt][s][l] = lo;
            }
        }
        {
            const int k0 = (tid & 3) * CQ;
            float c = 0.0f;
#pragma unroll
            for (int e = 0; e < CQ; ++e) c = fmaf(rbq[e], qs[k0 + e], c);
            c += __shfl_xor(c, 1, WAVE);
            c += __shfl_xor(c, 2, WAVE);
            const int j = tid >> 2;
            if ((tid & 3) == 0 && j < DIN_H) cs[j] = c + b0j;
        }
        lds_barrier();
        // (4) MFMAs + epilogue: unconditional buffer stores (dropped out of
        // range), statistics of every (t, j) of the tile
        if (16 * wv < T) {
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(h_out + b * T * DIN_H, 0, T * DIN_H * 4, 0x00020000);
#pragma unroll
            for (int jt = 0; jt < DIN_JT; ++jt) {
                din_f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int s = 0; s < NI; ++s) {
                    const din_half8 bh = mf[0][jt][s][lane];
                    const din_half8 bl = mf[1][jt][s][lane];
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[s], bh, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[s], bl, acc, 0, 0, 0);
                    if (F32) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[s], bh, acc, 0, 0, 0);
                }
                const int j = 16 * jt + (lane & 15);
                const float cj = j < DIN_H ? cs[j] : 0.0f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int t = 16 * wv + 4 * (lane >> 4) + r;
                    const float v = acc[r] * sc.inv + cj;
                    const int off = (t < T && j < DIN_H) ? (t * DIN_H + j) * 4 : 0x7FFFFFF0;
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, off, 0, 0);
                    ssum[jt][r] += (double)v;
                    ssq[jt][r] += (double)v * (double)v;
                }
            }
        }
    };
    for (int64_t b = b0; b < b_end; b += 2 * G) {
        step(b, rawA, qvA, hiA, qiA, hiB, qiB);
        if (b + G >= b_end) break;
        step(b + G, rawB, qvB, hiB, qiB, hiA, qiA);
    }
    // per-workgroup partial column sums (every real (t, j) is owned by one lane)
    double2* dst = reinterpret_cast<double2*>(partial) + (size_t)blockIdx.x * T * DIN_H;
#pragma unroll
    for (int jt = 0; jt < DIN_JT; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int t = 16 * wv + 4 * (lane >> 4) + r;
            const int j = 16 * jt + (lane & 15);
            if (t < T && j < DIN_H) dst[t * DIN_H + j] = make_double2(ssum[jt][r], ssq[jt][r]);
        }
}

// Scales for the split-fp16 products: s_k puts max|table| at <= 2^14, s_m
// puts max|M_b| <= max(|A| + |P| max|q|) at <= 2^14 (powers of two, so
// inv = 1 / (s_k s_m) is exact).
__global__ void din_absmax_kernel(const void* __restrict__ table, int dtype, int64_t n,
                                  unsigned int* __restrict__ out) {
    float m = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = dtype == 0 ? reinterpret_cast<const float*>(table)[i]
                                   : bf16_to_f32(reinterpret_cast<const uint16_t*>(table)[i]);
        m = fmaxf(m, fabsf(v));
    }
    m = fmaxf(m, __shfl_xor(m, 32, WAVE));
    m = fmaxf(m, __shfl_xor(m, 16, WAVE));
    m = fmaxf(m, __shfl_xor(m, 8, WAVE));
    m = fmaxf(m, __shfl_xor(m, 4, WAVE));
    m = fmaxf(m, __shfl_xor(m, 2, WAVE));
    m = fmaxf(m, __shfl_xor(m, 1, WAVE));
    // one atomic per workgroup (round 6: one per wave, thousands on one
    // address, made each call ~26 us)
    __shared__ float wm[16];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = fmaxf(m, wm[w]);
        atomicMax(out, __float_as_uint(m));  // m >= 0: bit order == value order
    }
}


__global__ void din_scales_kernel(const float* __restrict__ prep_ap, int ID, const unsigned int* __restrict__ mx,
                                  DinScales* __restrict__ out) {
    const float tmax = __uint_as_float(mx[0]), qmax = tmax;  // q rows come from the same table
    const int n = DIN_H * ID;
    float m = 0.0f;
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        m = fmaxf(m, fabsf(prep_ap[i]) + fabsf(prep_ap[2 * n + i]) * qmax);
    __shared__ float red[256];
    red[threadIdx.x] = m;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + d]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        DinScales s;
        s.s_k = pow2_scale(tmax);
        s.s_m = pow2_scale(red[0] * 1.0001f);
        s.inv = 1.0f / (s.s_k * s.s_m);
        s.pad = 0.0f;
        *out = s;
    }
}

// ------------------------------------------ 1'. att h, position-major --
// din_att_tm_kernel (bf16 tables, T <= 64, 1 / 2 / 4 item features): the
// same h as din_att_h2, computed for the rows that can differ and laid out
// so the MFMA tiles need no per-sample matrix.
//
// * Constant-B formulation: h = (Wk - Wd) k_t + Wp (q .* k_t) + c_b with
//   c_b = (Wq + Wd) q + b0 (DIN.py:105-114 with the batch-invariant parts
//   folded): the weights are the MFMA's B operand, the same for every row, so
//   a 16-row A tile may hold rows of 16 different samples.  Exact-f32-class:
//   k (bf16) is exact in fp16 at the power-of-two scale s; q .* k at scale
//   s^2 is an exact fp32 product of two fp16 values, split as
//   P_hi = fp16(k q) (v_pk_mul_f16) and P_lo = fp16(k q - P_hi)
//   (v_pk_fma_f16: the residual is exact in fp16); W = W_hi + W_lo.
//   5 MFMAs per (16 x 16 tile, k-step): k W1_hi, k W1_lo, P_hi Wp_hi,
//   P_hi Wp_lo, P_lo Wp_hi (the dropped P_lo Wp_lo term is ~2^-22 relative).
// * Only real rows: a row whose mask is 0 and whose indices are all 0 (the
//   collate's padding, DIN.py:476-490) has k_t = the item tables' row 0, so
//   its h is the sample's "pad row" h_pad,b; every row at or past
//   n_b = 1 + the last other row is such a row.  Rows t < n_b are computed
//   and stored; for t >= n_b only h_pad,b is computed, once per sample, and
//   enters the Dice statistics of every column t >= n_b through a
//   difference array (samples sorted by n_b, D(t) = sum of the pad rows of
//   the samples with n_b = t, P(t) = sum_{t' <= t} D(t')).  h rows t >= n_b
//   are left unwritten: their mask is 0, and din_wh2 never reads a masked
//   row's h.  At config 3 (hist_len ~ U[1, 50], 20% empty) that is ~21 of
//   50 rows per sample.
// * Position-major tiles: a workgroup (4 waves, one per SIMD, each holding
//   all weight fragments in registers; ~100 KB of LDS)
//   takes a run of SW = 128 samples of ONE Dice batch, sorts them by n_b
//   (descending, stable), so the samples with a real row at position t are
//   the prefix [0, c_t) -- ceil(c_t / 16) tiles whose rows all share t.  A
//   wave claims positions dynamically (LDS counter, largest first); the
//   column sums of h and h^2 at t (fp64) are a lane-local sum over the
//   tile's rows plus a 4-group butterfly, added once into the workgroup's
//   row R[t] (which starts at P(t)).  Deterministic: every sum's order is
//   fixed by the data, not by which wave ran it.
// * Per tile the k rows of the next two tiles and the indices of the third
//   are in flight (issued before the tile's MFMAs); all loads are unconditional (clamped rows), h goes out through
//   buffer stores whose out-of-range offsets the hardware drops.
// dev-only A/B switch (make devdin DEVFLAGS=-DNRK_TM_DEV=n; the product
// build leaves it 0): 1 skips phase 7, 2 its stores, 3 its MFMAs, 4 phases 4-6
#ifndef NRK_TM_DEV
#define NRK_TM_DEV 0
#endif
constexpr int TM_SW = 128;  // samples per workgroup
// waves per workgroup: 8 (two per SIMD, the weight fragments in LDS, read
// one k-step ahead) or, dev builds only, 4 (one per SIMD, the fragments in
// registers -- issue-bound: ~2.5k cycles per tile against ~1.5k)
#ifndef NRK_TM_NW
#define NRK_TM_NW 8
#endif
constexpr int TM_NW = NRK_TM_NW;
constexpr bool TM_WLDS = TM_NW == 8;
// W fragments from LDS in a 3-slot ring per (k-step, column tile) group (1)
// or double-buffered per k-step (0, round 4)
#ifndef NRK_TM_WRING
#define NRK_TM_WRING 1
#endif
constexpr bool TM_WRING = NRK_TM_WRING;
constexpr int TM_NT = TM_NW * 64;
constexpr int TM_TMAX = 64; // positions (T)

struct DinScalesTM {
    float s;       // table scale: max |table| s <= 2^7, so |q k| s^2 <= 2^14 fits fp16
    float s_w;     // W1 = Wk - Wd at s_w, Wp at s_w / s (both <= 2^14)
    float inv;     // 1 / (s_w s): the accumulator's scale
    float s_qd;    // Wqd = Wq + Wd at s_qd
    float inv_qd;  // 1 / (s_qd s)
    float pad[11];
};

__host__ __device__ constexpr size_t din_tm_base(int n_item) {
    return (((size_t)3 * DIN_H * n_item * DIN_E * 4 + 64) + 255) & ~(size_t)255;
}
// prep layout past the round-3 part: [DinScalesTM, 256 B][wpack: 3 jt x NI
// k-steps x 4 parts x 64 lanes x 16 B][qdpack: 3 x NI x 2 x 64 x 16 B]
// [tab16: the table at scale s as fp16, n_rows x 32, 256-B aligned]
__host__ __device__ constexpr size_t din_tm_bytes(int n_item) { return 256 + (size_t)3 * n_item * 6 * 64 * 16; }
__host__ __device__ constexpr size_t din_tm_tab16_off(int n_item) {
    return (din_tm_base(n_item) + din_tm_bytes(n_item) + 255) & ~(size_t)255;
}

// tab16 = fp16(table * s): bf16 values are exact in fp16 at the power-of-two
// scale s unless they fall below fp16's normal range (|x| < max |table| 2^-21)
__global__ void din_tm_tab16_kernel(const uint16_t* __restrict__ table, int64_t n, const DinScalesTM* __restrict__ sc,
                                    uint32_t* __restrict__ out) {
    const float s = sc->s;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t w = reinterpret_cast<const uint32_t*>(table)[i];
        const _Float16 lo = (_Float16)(__uint_as_float(w << 16) * s);
        const _Float16 hi = (_Float16)(__uint_as_float(w & 0xFFFF0000u) * s);
        out[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
    }
}

__global__ void din_tm_scales_kernel(const float* __restrict__ prep_f, int ID, const unsigned int* __restrict__ tmax,
                                     DinScalesTM* __restrict__ out) {
    const int n = DIN_H * ID;
    float ma = 0.0f, mp = 0.0f, mq = 0.0f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        ma = fmaxf(ma, fabsf(prep_f[i]));
        mq = fmaxf(mq, fabsf(prep_f[n + i]));
        mp = fmaxf(mp, fabsf(prep_f[2 * n + i]));
    }
    __shared__ float red[3][256];
    red[0][threadIdx.x] = ma;
    red[1][threadIdx.x] = mp;
    red[2][threadIdx.x] = mq;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d)
            for (int c = 0; c < 3; ++c) red[c][threadIdx.x] = fmaxf(red[c][threadIdx.x], red[c][threadIdx.x + d]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float tm = __uint_as_float(*tmax);
        float s = tm > 0.0f ? pow2_scale(tm) * 0.0078125f : 1.0f;  // max |table| s in [2^6, 2^7)
        s = fminf(s, 1.0995116e12f);                                  // <= 2^40: s_w s stays finite
        float s_w = pow2_scale(fmaxf(red[0][0], red[1][0] / s));
        s_w = fminf(s_w, 1.1529215e18f);                              // <= 2^60
        DinScalesTM o = {};
        o.s = s;
        o.s_w = s_w;
        o.inv = 1.0f / (s_w * s);
        o.s_qd = fminf(pow2_scale(red[2][0]), 1.1529215e18f);
        o.inv_qd = 1.0f / (o.s_qd * s);
        *out = o;
    }
}

// fragment (jt, s, lane) of a [36 x ID] matrix as the MFMA B operand: 8
// consecutive k of output column 16 jt + (lane & 15), zero past 36
__global__ void din_tm_pack_kernel(const float* __restrict__ prep_f, int NI, const DinScalesTM* __restrict__ sc,
                                   din_half8* __restrict__ wpack, din_half8* __restrict__ qdpack) {
    const int ID = NI * DIN_E, n = DIN_H * ID;
    const int total = 3 * 3 * NI * 64;  // (matrix, jt, s, lane)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int lane = i % 64, s = (i / 64) % NI, jt = (i / (64 * NI)) % 3, m = i / (64 * NI * 3);
        const int j = 16 * jt + (lane & 15), k = DIN_E * s + 8 * (lane >> 4);
        const float* src = m == 0 ? prep_f : m == 1 ? prep_f + 2 * n : prep_f + n;  // W1, Wp, Wqd
        const float scale = m == 0 ? sc->s_w : m == 1 ? sc->s_w / sc->s : sc->s_qd;
        float x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = j < DIN_H ? src[j * ID + k + e] : 0.0f;
        din_half8 hi, lo;
        split8(x, scale, hi, lo);
        if (m < 2) {
            din_half8* o = wpack + ((size_t)(jt * NI + s) * 4 + 2 * m) * 64 + lane;
            o[0] = hi;
            o[64] = lo;
        } else {
            din_half8* o = qdpack + ((size_t)(jt * NI + s) * 2) * 64 + lane;
            o[0] = hi;
            o[64] = lo;
        }
    }
}

typedef uint32_t tm_u4 __attribute__((ext_vector_type(4)));

static inline size_t din_tm_lds(int NI, int T) {
    const int ID = NI * DIN_E;
    return (TM_WLDS ? (size_t)3 * NI * 4 * 1024 : 0)   // W fragments
           + (size_t)TM_SW * (ID * 2 + 16)             // q rows (fp16, padded stride)
           + (size_t)DIN_H * (TM_SW + 4) * 4           // c^T (acc init), padded stride
           + (size_t)TM_SW * DIN_H * 4                 // pad-row h
           + (size_t)T * DIN_H * 16                    // R: (sum, sumsq) per (t, j)
           + (size_t)TM_SW * 12 + (TM_TMAX + 4) * 4;  // perm, perm * T, perm * T * 144, c_t, counter
}


// Dice(x) with the batch (mean, 1 / (std + 1e-8)) of x's column (DIN.py:39-44)
__device__ __forceinline__ float dice_fast(float x, float mean, float inv) {
    const float p = __builtin_amdgcn_rcpf(1.0f + __expf((mean - x) * inv));
    return p * x + ((1.0f - p) * 0.01f) * x;
}

// Plan of a run of TM_SW samples (one Dice batch):
// n_b of every sample (1 + its last row that is not the collate's padding),
// a stable sort by n_b descending (perm: sorted position -> sample) and c_t
// = #{n_b > t}.  plan[blk] = [perm (TM_SW) | c_t (TM_TMAX)]; one 256-thread
// workgroup per run, every (mask, index) row read once, coalesced.  (A
// static longest-first schedule of positions to waves was tried: the waves
// then wait ~10% of the kernel at the end of each run.)
constexpr int TM_PLAN = TM_SW + TM_TMAX;

// dev-only phase stamps (make devdin DEVFLAGS=-DNRK_TM_STAMP=1, read by
// nrk_dev_tm_stamps): per workgroup, shader cycles spent in each phase
#ifndef NRK_TM_STAMP
#define NRK_TM_STAMP 0
#endif
#if NRK_TM_STAMP
__device__ unsigned long long tm_stamps[1024 * 12];
#define TM_STAMP(k)                                           \
    do {                                                      \
        const uint64_t t_now_ = __builtin_readcyclecounter(); \
        stp[k] += t_now_ - t_prev;                            \
        t_prev = t_now_;                                      \
    } while (0)
#else
#define TM_STAMP(k) \
    do {            \
    } while (0)
#endif

template <int NI>
__global__ __launch_bounds__(256) void din_tm_plan_kernel(const int32_t* __restrict__ hist_idx,
                                                          const float* __restrict__ mask, int64_t N, int64_t S,
                                                          int G, int T, int32_t* __restrict__ plan) {
    __shared__ int nbs[TM_SW];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t seg = blockIdx.x / G, g = blockIdx.x % G;
    const int64_t b0 = seg * S + g * TM_SW;
    const int64_t seg_end = (seg + 1) * S < N ? (seg + 1) * S : N;
    const int nw = (int)(seg_end - b0 < TM_SW ? seg_end - b0 : TM_SW);
    int32_t* out = plan + (size_t)blockIdx.x * TM_PLAN;
    if (nw <= 0) return;
    const bool act = lane < T;
    for (int u0 = 0; u0 < TM_SW / 4; u0 += 16) {
        bool nz[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int i = wv * (TM_SW / 4) + u0 + u;
            const int64_t b = b0 + (i < nw ? i : nw - 1);
            const size_t r = (size_t)b * T + (act ? lane : 0);
            const float m = mask[r];
            bool any = m != 0.0f;
            if constexpr (NI == 4) {
                const int4 x = *reinterpret_cast<const int4*>(hist_idx + r * 4);
                any |= (x.x | x.y | x.z | x.w) != 0;
            } else if constexpr (NI == 2) {
                const int2 x = *reinterpret_cast<const int2*>(hist_idx + r * 2);
                any |= (x.x | x.y) != 0;
            } else {
                any |= hist_idx[r] != 0;
            }
            nz[u] = any && act;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint64_t bal = __builtin_amdgcn_ballot_w64(nz[u]);
            const int i = wv * (TM_SW / 4) + u0 + u;
            if (lane == 0) nbs[i] = i < nw ? (bal ? 64 - __builtin_clzll(bal) : 0) : -1;
        }
    }
    __syncthreads();
    if (tid < TM_SW) {
        const int my = nbs[tid];
        int rank = 0;
        for (int j = 0; j < TM_SW; j += 4) {
            const int4 v = *reinterpret_cast<const int4*>(nbs + j);
            rank += (v.x > my || (v.x == my && j < tid)) + (v.y > my || (v.y == my && j + 1 < tid)) +
                    (v.z > my || (v.z == my && j + 2 < tid)) + (v.w > my || (v.w == my && j + 3 < tid));
        }
        out[rank] = tid;
    } else if (tid < TM_SW + T) {
        const int t = tid - TM_SW;
        int c = 0;
        for (int j = 0; j < TM_SW; j += 4) {
            const int4 v = *reinterpret_cast<const int4*>(nbs + j);
            c += (v.x > t) + (v.y > t) + (v.z > t) + (v.w > t);
        }
        out[TM_SW + t] = c;
    }
}

// Persistent: one workgroup per CU walks the runs blk = blockIdx.x,
// blockIdx.x + gridDim.x, ...; the weight fragments are loaded once.
template <int NI>
__global__ __launch_bounds__(TM_NT, 1) __attribute__((amdgpu_waves_per_eu(TM_NW / 4, TM_NW / 4))) void din_att_tm_kernel(
    const din_half8* __restrict__ tab16, const int64_t* __restrict__ row_base, int n_user,
    const int32_t* __restrict__ item_idx, const int32_t* __restrict__ hist_idx, const int32_t* __restrict__ plan,
    int64_t N, int64_t S, int G, int T, const uint8_t* __restrict__ tm, const float* __restrict__ att_b0,
    float* __restrict__ h_out, double* __restrict__ partial) {
    constexpr int ID = NI * DIN_E;
    constexpr int QS = ID * 2 + 16;  // q row stride (bytes): 16-B bank shift per row
    constexpr int CTS = TM_SW + 4;   // c^T row stride (floats)
    extern __shared__ __attribute__((aligned(16))) uint8_t tm_lds[];
    din_half8* wl = reinterpret_cast<din_half8*>(tm_lds);
    uint8_t* ql = tm_lds + (TM_WLDS ? 3 * NI * 4 * 1024 : 0);
    float* ct = reinterpret_cast<float*>(ql + TM_SW * QS);
    float* hp = ct + DIN_H * CTS;
    double2* R = reinterpret_cast<double2*>(hp + TM_SW * DIN_H);
    int* perm = reinterpret_cast<int*>(R + T * DIN_H);
    int* pT = perm + TM_SW;         // perm * T (row of position 0)
    int* pH = pT + TM_SW;           // perm * T * 144 (byte offset of its h row 0)
    int* cnt = pH + TM_SW;          // c_t, t < T
    int* next_t = cnt + TM_TMAX;    // position claim counter

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 15, lg = lane >> 4;
    const DinScalesTM sc = *reinterpret_cast<const DinScalesTM*>(tm);
    const din_half8* wpack = reinterpret_cast<const din_half8*>(tm + 256);
    const din_half8* qdpack = wpack + 3 * NI * 4 * 64;
    // W fragments (12 NI per lane: the B operand of every tile), once per
    // workgroup: to LDS (TM_WLDS; published by the first run's barrier) or
    // to registers
    din_half8 wr[TM_WLDS ? 1 : 3][TM_WLDS ? 1 : NI][4];
    if constexpr (TM_WLDS) {
        const tm_u4* src = reinterpret_cast<const tm_u4*>(wpack);
        tm_u4* d = reinterpret_cast<tm_u4*>(wl);
        for (int c = tid; c < 3 * NI * 4 * 64; c += TM_NT) d[c] = src[c];
    } else {
#pragma unroll
        for (int jt = 0; jt < 3; ++jt)
#pragma unroll
            for (int s = 0; s < NI; ++s)
#pragma unroll
                for (int c = 0; c < 4; ++c) wr[jt][s][c] = wpack[((jt * NI + s) * 4 + c) * 64 + lane];
    }
    const int64_t n_blk = (N + S - 1) / S * G;
#if NRK_TM_STAMP
    uint64_t stp[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = __builtin_readcyclecounter();
#endif
    for (int64_t blk = blockIdx.x; blk < n_blk; blk += gridDim.x) {
    const int64_t seg = blk / G, g = blk % G;
    const int64_t b0 = seg * S + g * TM_SW;
    const int64_t seg_end = (seg + 1) * S < N ? (seg + 1) * S : N;
    const int nw = (int)(seg_end - b0 < TM_SW ? seg_end - b0 : TM_SW);
    double2* dst = reinterpret_cast<double2*>(partial) + (size_t)blk * T * DIN_H;
    if (nw <= 0) {  // a short last batch leaves trailing runs empty: zero partial rows
        for (int e = tid; e < T * DIN_H; e += TM_NT) dst[e] = make_double2(0.0, 0.0);
        continue;
    }
    // ---- phase 1 (din_tm_plan_kernel): perm and c_t -> LDS
    for (int e = tid; e < TM_SW + T; e += TM_NT) {
        const int v = plan[(size_t)blk * TM_PLAN + e];
        if (e < TM_SW) {
            perm[e] = v;
            pT[e] = v * T;
            pH[e] = v * T * (DIN_H * 4);
        } else {
            cnt[e - TM_SW] = v;
        }
    }
    if (tid == 0) *next_t = 0;
    __syncthreads();
    TM_STAMP(0);
    // ---- phase 2: q rows of the sorted samples (fp16 at scale s)
    // (each thread's QT tasks: all index loads in flight, then all row loads)
    {
        constexpr int QT = TM_SW * NI * 4 / TM_NT;
        static_assert(QT * TM_NT == TM_SW * NI * 4, "q tasks");
        int64_t rbq[NI];
#pragma unroll
        for (int f = 0; f < NI; ++f) rbq[f] = row_base[n_user + f];
        int32_t qi[QT];
#pragma unroll
        for (int u = 0; u < QT; ++u) {
            const int task = tid + u * TM_NT, p = task / (NI * 4), f = (task / 4) % NI;
            qi[u] = item_idx[(b0 + perm[p < nw ? p : 0]) * NI + f];
        }
        din_half8 v[QT];
#pragma unroll
        for (int u = 0; u < QT; ++u) {
            const int task = tid + u * TM_NT, f = (task / 4) % NI, c = task % 4;
            v[u] = tab16[(rbq[f] + qi[u]) * 4 + c];
        }
#pragma unroll
        for (int u = 0; u < QT; ++u) {
            const int task = tid + u * TM_NT, p = task / (NI * 4), f = (task / 4) % NI, c = task % 4;
            *reinterpret_cast<din_half8*>(ql + p * QS + (f * DIN_E + 8 * c) * 2) = p < nw ? v[u] : din_half8{};
        }
    }
    __syncthreads();
    TM_STAMP(1);
    // ---- phase 3: c_b = (Wq + Wd) q + b0 for 16 samples per wave (MFMA),
    // stored pre-scaled (x s_w s) and transposed as the accumulator init
    for (int pb = wv; pb < TM_SW / 16; pb += TM_NW) {
        const float b0j[3] = {att_b0[lr], att_b0[16 + lr], 32 + lr < DIN_H ? att_b0[32 + lr] : 0.0f};
        din_f4 acc[3];
#pragma unroll
        for (int jt = 0; jt < 3; ++jt) acc[jt] = din_f4{0.0f, 0.0f, 0.0f, 0.0f};
        const int p = pb * 16 + lr;
#pragma unroll
        for (int s = 0; s < NI; ++s) {
            const din_half8 a = *reinterpret_cast<const din_half8*>(ql + p * QS + (DIN_E * s + 8 * lg) * 2);
#pragma unroll
            for (int jt = 0; jt < 3; ++jt) {
                const din_half8 bh = qdpack[((jt * NI + s) * 2) * 64 + lane];
                const din_half8 bl = qdpack[((jt * NI + s) * 2 + 1) * 64 + lane];
                acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bh, acc[jt], 0, 0, 0);
                acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bl, acc[jt], 0, 0, 0);
            }
        }
        const float to_acc = sc.s_w * sc.s;
#pragma unroll
        for (int jt = 0; jt < 3; ++jt) {
            const int j = 16 * jt + lr;
            if (j < DIN_H) {
                din_f4 c;
#pragma unroll
                for (int r = 0; r < 4; ++r) c[r] = (acc[jt][r] * sc.inv_qd + b0j[jt]) * to_acc;
                *reinterpret_cast<din_f4*>(ct + j * CTS + pb * 16 + 4 * lg) = c;
            }
        }
    }
    __syncthreads();

    // one 16-row tile: rows = sorted positions 16 i + (lane & 15) for the A
    // operand; k fragments kf[s]; accumulator starts at c^T
    auto tile_mfma = [&](int i, const din_half8 (&kf)[NI], int pa, din_f4 (&acc)[3]) {
#pragma unroll
        for (int jt = 0; jt < 3; ++jt) {
            const int j = 16 * jt + lr < DIN_H ? 16 * jt + lr : DIN_H - 1;
            acc[jt] = *reinterpret_cast<const din_f4*>(ct + j * CTS + 16 * i + 4 * lg);
        }
        if constexpr (TM_WLDS && TM_WRING) {
            // the (k-step s, column tile jt) groups' 4 fragments each, read two
            // groups (10 MFMAs) ahead in a 3-slot ring: 12 fragments live
            // instead of a whole k-step double-buffered (24: the NI = 4
            // instantiation spilled 45 VGPRs at 256)
            din_half8 wq[3][4];
            auto wread = [&](int q, din_half8 (&w)[4]) {
                const int s = q / 3, jt = q % 3;
#pragma unroll
                for (int c = 0; c < 4; ++c) w[c] = wl[((jt * NI + s) * 4 + c) * 64 + lane];
            };
            wread(0, wq[0]);
            wread(1, wq[1]);
            din_half8 ph, pl;
            static_for<3 * NI>([&](auto qc) {
                constexpr int q = decltype(qc)::value, s = q / 3, jt = q % 3;
                if constexpr (q + 2 < 3 * NI) wread(q + 2, wq[(q + 2) % 3]);
                if constexpr (jt == 0) {
                    const din_half8 qf = *reinterpret_cast<const din_half8*>(ql + pa * QS + (DIN_E * s + 8 * lg) * 2);
                    __builtin_amdgcn_sched_barrier(0);
                    ph = kf[s] * qf;
                    pl = __builtin_elementwise_fma(kf[s], qf, -ph);
                }
                const din_half8(&w)[4] = wq[q % 3];
                acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], w[0], acc[jt], 0, 0, 0);
                acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], w[1], acc[jt], 0, 0, 0);
                acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, w[2], acc[jt], 0, 0, 0);
                acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, w[3], acc[jt], 0, 0, 0);
                acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl, w[2], acc[jt], 0, 0, 0);
            });
        } else if constexpr (TM_WLDS) {
            // k-step s + 1's 12 fragments are read while k-step s's 15 MFMAs
            // run (two register sets; the barrier keeps the reads ahead)
            din_half8 wb[2][3][4];
            auto wread = [&](int s, din_half8 (&w)[3][4]) {
#pragma unroll
                for (int jt = 0; jt < 3; ++jt)
#pragma unroll
                    for (int c = 0; c < 4; ++c) w[jt][c] = wl[((jt * NI + s) * 4 + c) * 64 + lane];
            };
            wread(0, wb[0]);
#pragma unroll
            for (int s = 0; s < NI; ++s) {
                if (s + 1 < NI) wread(s + 1, wb[(s + 1) & 1]);
                const din_half8 qf = *reinterpret_cast<const din_half8*>(ql + pa * QS + (DIN_E * s + 8 * lg) * 2);
                __builtin_amdgcn_sched_barrier(0);
                const din_half8 ph = kf[s] * qf;
                const din_half8 pl = __builtin_elementwise_fma(kf[s], qf, -ph);
                const din_half8(&w)[3][4] = wb[s & 1];
#pragma unroll
                for (int jt = 0; jt < 3; ++jt) {
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], w[jt][0], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], w[jt][1], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, w[jt][2], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, w[jt][3], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl, w[jt][2], acc[jt], 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int s = 0; s < NI; ++s) {
                const din_half8 qf = *reinterpret_cast<const din_half8*>(ql + pa * QS + (DIN_E * s + 8 * lg) * 2);
                const din_half8 ph = kf[s] * qf;
                const din_half8 pl = __builtin_elementwise_fma(kf[s], qf, -ph);
#pragma unroll
                for (int jt = 0; jt < 3; ++jt) {
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], wr[jt][s][0], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[s], wr[jt][s][1], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, wr[jt][s][2], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, wr[jt][s][3], acc[jt], 0, 0, 0);
                    acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl, wr[jt][s][2], acc[jt], 0, 0, 0);
                }
            }
        }
    };

    TM_STAMP(2);
    // ---- phase 4: pad rows (k = row 0 of every item table) of the samples
    // with n_b < T: sorted positions [c_{T-1}, nw)
    {
        din_half8 k0[NI];
#pragma unroll
        for (int s = 0; s < NI; ++s) k0[s] = tab16[row_base[n_user + s] * 4 + lg];
        const int pad_lo = cnt[T - 1];
        for (int i = pad_lo / 16 + wv; NRK_TM_DEV != 4 && i * 16 < nw; i += TM_NW) {
            const int pa = 16 * i + lr < nw ? 16 * i + lr : nw - 1;
            din_f4 acc[3];
            tile_mfma(i, k0, pa, acc);
#pragma unroll
            for (int jt = 0; jt < 3; ++jt) {
                const int j = 16 * jt + lr;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int p = 16 * i + 4 * lg + r;
                    if (j < DIN_H && p >= pad_lo && p < nw) hp[p * DIN_H + j] = acc[jt][r] * sc.inv;
                }
            }
        }
    }
    __syncthreads();
    TM_STAMP(3);
    // ---- phase 5: D(t) = sum of the pad rows of the samples with n_b = t
    // (sorted positions [c_t, c_{t-1}), c_{-1} = nw), into R
    for (int e = tid; e < T * DIN_H; e += TM_NT) {
        const int t = e / DIN_H, j = e % DIN_H;
        const int lo = cnt[t], hi = NRK_TM_DEV == 4 ? lo : t == 0 ? nw : cnt[t - 1];
        double s = 0.0, ss = 0.0;
        for (int p = lo; p < hi; ++p) {
            const double v = (double)hp[p * DIN_H + j];
            s += v;
            ss += v * v;
        }
        R[e] = make_double2(s, ss);
    }
    __syncthreads();
    TM_STAMP(4);
    // ---- phase 6: P(t) = prefix over t of D, in place (one lane per column,
    // eight positions' loads in flight per step)
    if (tid < DIN_H) {
        double s = 0.0, ss = 0.0;
        for (int t0 = 0; t0 < T; t0 += 8) {
            double2 d[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) d[u] = R[(t0 + u < T ? t0 + u : T - 1) * DIN_H + tid];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s += d[u].x;
                ss += d[u].y;
                if (t0 + u < T) R[(t0 + u) * DIN_H + tid] = make_double2(s, ss);
            }
        }
    }
    __syncthreads();

    TM_STAMP(5);
    // ---- phase 7: real rows, positions claimed dynamically (largest first:
    // c_t is nonincreasing in t); a wave's next claim is issued one claim
    // ahead, so its LDS atomic never sits on the path to the next tile
    int t_eff = 0;  // positions with at least one real row (c_t nonincreasing)
    while (t_eff < T && cnt[t_eff] > 0) ++t_eff;
    int64_t rbs[NI];
#pragma unroll
    for (int s = 0; s < NI; ++s) rbs[s] = row_base[n_user + s] * 4 + lg;  // in 16-B pieces
    // job = (position t, tile i, c = c_t); t >= t_eff: none
    struct Job {
        int t, i, c;
    };
    int pend = lane == 0 ? atomicAdd(next_t, 1) : 0;  // lane 0: the claimed position
    auto claim_job = [&]() -> Job {
        const int t = __builtin_amdgcn_readfirstlane(pend);
        if (t >= t_eff) return Job{t_eff, 0, 0};
        pend = lane == 0 ? atomicAdd(next_t, 1) : 0;
        return Job{t, 0, cnt[t]};
    };
    auto succ = [&](const Job& j) -> Job {
        if (j.t >= t_eff) return j;
        if (16 * (j.i + 1) < j.c) return Job{j.t, j.i + 1, j.c};
        return claim_job();
    };
    // A-row position of a job (clamped into [0, c_t)) and its sample's indices
    auto apos = [&](const Job& j) -> int {
        const int p = 16 * j.i + lr;
        return j.t >= t_eff ? 0 : (p < j.c ? p : j.c - 1);
    };
    // 32-bit offsets from the run's first row (u24 products: sample * T + t
    // < TM_SW * TM_TMAX), so no 64-bit multiply per tile
    const int32_t* hrun = hist_idx + (size_t)b0 * T * NI;
    auto idx_load = [&](const Job& j) -> int4 {
        const int tc = j.t < t_eff ? j.t : 0;
        const int r = (pT[apos(j)] + tc) * NI;
        if constexpr (NI == 4) return *reinterpret_cast<const int4*>(hrun + r);
        else if constexpr (NI == 2) { const int2 x = *reinterpret_cast<const int2*>(hrun + r); return make_int4(x.x, x.y, 0, 0); }
        else return make_int4(hrun[r], 0, 0, 0);
    };
    auto rows_load = [&](const int4& ix, din_half8 (&kf)[NI]) {
        const int32_t iv[4] = {ix.x, ix.y, ix.z, ix.w};
#pragma unroll
        for (int s = 0; s < NI; ++s) kf[s] = tab16[rbs[s] + (int64_t)iv[s] * 4];
    };

    // three slots (k rows + indices) rotate so no register copy waits on a
    // load: in the step of job m, slot m % 3 holds job m's rows and receives
    // job m+3's indices, slot (m+2) % 3 receives job m+2's rows (from the
    // indices it got one step earlier)
    Job j0 = claim_job();
    Job j1 = succ(j0);
    Job j2 = succ(j1);
    din_half8 k_a[NI], k_b[NI], k_c[NI];
    int4 ix_a, ix_b, ix_c;
    ix_a = idx_load(j0);
    ix_b = idx_load(j1);
    rows_load(ix_a, k_a);
    ix_c = idx_load(j2);
    rows_load(ix_b, k_b);
    // h goes out through buffer stores whose out-of-range offsets the
    // hardware drops (unconditional: 3 per step); a step is entered with its
    // far indices followed by 4 row loads and 3 stores, and 3 dropped stores
    // give the loop entry the same shape, so the wait counts merged at the
    // loop head stay those of a steady-state step
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(h_out + b0 * T * DIN_H, 0, nw * T * DIN_H * 4, 0x00020000);
#pragma unroll
    for (int e = 0; e < 3; ++e) __builtin_amdgcn_raw_buffer_store_b128(tm_u4{0u, 0u, 0u, 0u}, rsrc, 0x7FFFF000, 0, 0);
    double ssum[3], ssq[3];
#pragma unroll
    for (int jt = 0; jt < 3; ++jt) ssum[jt] = ssq[jt] = 0.0;
    auto step = [&](din_half8 (&kcur)[NI], int4& ixcur, din_half8 (&kfar)[NI], const int4& ixfar) {
#if NRK_TM_STAMP
        uint64_t t_s = __builtin_readcyclecounter();
#define TM_SSTAMP(k)                                          \
    do {                                                      \
        const uint64_t t_now_ = __builtin_readcyclecounter(); \
        stp[k] += t_now_ - t_s;                               \
        t_s = t_now_;                                         \
    } while (0)
#else
#define TM_SSTAMP(k) \
    do {             \
    } while (0)
#endif
        const Job j3 = succ(j2);
        TM_SSTAMP(8);
        ixcur = idx_load(j3);   // indices three jobs ahead
        rows_load(ixfar, kfar); // rows two jobs ahead
        TM_SSTAMP(9);
        // keep the loads ahead of this tile's MFMAs (the scheduler would sink
        // them past the chain, leaving a load latency exposed per tile)
        __builtin_amdgcn_sched_barrier(0);
        din_f4 acc[3];
        if constexpr (NRK_TM_DEV == 3) {
#pragma unroll
            for (int jt = 0; jt < 3; ++jt)
                acc[jt] = din_f4{kcur[0][0] + kcur[NI - 1][1], 0.0f, 0.0f, 0.0f} * (float)ixfar.x;
        } else {
            tile_mfma(j0.i, kcur, apos(j0), acc);
        }
#if NRK_TM_STAMP
        asm volatile("s_nop 0" ::"v"(acc[0][0]), "v"(acc[1][0]), "v"(acc[2][0]));
#endif
        TM_SSTAMP(10);
        // epilogue: column sums of h and h^2 over the rows < c_t -- the
        // lane's 4 rows in fp32 (relative error ~2^-22, below the reference's
        // own fp32 statistics), then fp64; h of those rows to HBM, transposed
        // through the wave's LDS stage so each lane stores 16 contiguous bytes
        // of a row (3 wide stores per tile instead of 12 scattered ones)
        float* stg = hp + wv * (16 * DIN_H);
        auto epi = [&](auto full_c) {
            constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
            for (int jt = 0; jt < 3; ++jt) {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[jt][r] * sc.inv;
                    if (jt < 2 || lr < DIN_H - 32) stg[(4 * lg + r) * DIN_H + 16 * jt + lr] = v[r];
                    if constexpr (!FULL) v[r] = 16 * j0.i + 4 * lg + r < j0.c ? v[r] : 0.0f;
                }
                const float s4 = (v[0] + v[1]) + (v[2] + v[3]);
                const float q4 = fmaf(v[3], v[3], fmaf(v[2], v[2], fmaf(v[1], v[1], v[0] * v[0])));
                ssum[jt] += (double)s4;
                ssq[jt] += (double)q4;
            }
        };
        if (16 * (j0.i + 1) <= j0.c) epi(std::true_type{});  // uniform: a full tile
        else epi(std::false_type{});
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        {
            // all six LDS reads in flight before the stores (unconditional,
            // clamped rows)
            const int toff = j0.t * (DIN_H * 4);
            tm_u4 x[3];
            int ph[3], c4[3];
            bool ok[3];
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                const int e = lane + 64 * m;  // 16-B piece e = 9 row + c4 of the 16 x 36 tile
                const int row = e / 9;
                c4[m] = e - 9 * row;
                ok[m] = e < 16 * 9 && 16 * j0.i + row < j0.c;
                const int rc = ok[m] ? row : 0;
                x[m] = *reinterpret_cast<const tm_u4*>(stg + rc * DIN_H + 4 * (ok[m] ? c4[m] : 0));
                ph[m] = pH[16 * j0.i + rc];
            }
#pragma unroll
            for (int m = 0; m < 3; ++m)  // past num_records: dropped
                __builtin_amdgcn_raw_buffer_store_b128(x[m], rsrc, ok[m] ? ph[m] + toff + 16 * c4[m] : 0x7FFFF000, 0, 0);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (j1.t != j0.t) {  // last tile of j0.t: combine the 16 rows' lanes, add to R[t]
#pragma unroll
            for (int jt = 0; jt < 3; ++jt) {
                ssum[jt] += xor16d(ssum[jt], lane);
                ssq[jt] += xor16d(ssq[jt], lane);
                ssum[jt] += xor32d(ssum[jt], lane);
                ssq[jt] += xor32d(ssq[jt], lane);
                const int j = 16 * jt + lr;
                if (lane < 16 && j < DIN_H) {
                    double2* rp = R + j0.t * DIN_H + j;
                    const double2 x = *rp;
                    *rp = make_double2(x.x + ssum[jt], x.y + ssq[jt]);
                }
                ssum[jt] = ssq[jt] = 0.0;
            }
        }
        TM_SSTAMP(11);
        j0 = j1;
        j1 = j2;
        j2 = j3;
    };
    while (NRK_TM_DEV != 1 && j0.t < t_eff) {
        step(k_a, ix_a, k_c, ix_c);
        if (j0.t >= t_eff) break;
        step(k_b, ix_b, k_a, ix_a);
        if (j0.t >= t_eff) break;
        step(k_c, ix_c, k_b, ix_b);
    }
    TM_STAMP(6);
    __syncthreads();
    // ---- phase 8: the run's partial row
    for (int e = tid; e < T * DIN_H; e += TM_NT) dst[e] = R[e];
    __syncthreads();  // R, perm and c_t are rewritten by the next run
    TM_STAMP(7);
    }
#if NRK_TM_STAMP
    if (tid == 0 && blockIdx.x < 1024)
        for (int k = 0; k < 12; ++k) tm_stamps[blockIdx.x * 12 + k] = stp[k];
#endif
}

// ---------------------------------------------------------- 2. col stats --
// mean and unbiased std (torch.std default) of each column over one Dice
// batch (segment blockIdx.x), from that segment's per-block fp64 (sum, sumsq)
// partial rows [seg * bps, min((seg + 1) * bps, nblk)).  One wave per
// column: lane l sums partials l, l+64, ... in order, then a fixed butterfly
// -- the same order on every run (bitwise reproducible).  A one-sample
// segment has no std (NaN in the reference); the host marks its output.
__global__ __launch_bounds__(256) void col_stats_kernel(const double* __restrict__ partial, int bps,
                                                        int nblk, int ncol, int64_t N, int64_t S,
                                                        float2* __restrict__ stats,
                                                        float2* __restrict__ stats_inv = nullptr) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int64_t seg = blockIdx.x;
    if (c >= ncol) return;
    const int64_t k1 = (seg + 1) * bps < nblk ? (seg + 1) * bps : nblk;
    const int64_t B = N - seg * S < S ? N - seg * S : S;
    double s = 0.0, ss = 0.0;
    for (int64_t k = seg * bps + lane; k < k1; k += WAVE) {
        const double2 v = *reinterpret_cast<const double2*>(partial + ((size_t)k * ncol + c) * 2);
        s += v.x;
        ss += v.y;
    }
    s = wave_sum_f64(s);
    ss = wave_sum_f64(ss);
    if (lane == 0) {
        const double mean = s / (double)B;
        double var = B > 1 ? (ss - s * mean) / (double)(B - 1) : 0.0;
        if (var < 0.0) var = 0.0;
        const float sd = (float)sqrt(var);
        if (stats) stats[seg * ncol + c] = make_float2((float)mean, sd);
        if (stats_inv) stats_inv[seg * ncol + c] = make_float2((float)mean, 1.0f / (sd + 1e-8f));
    }
}

// --------------------------------------------------------- 3. att out --
// One workgroup per sample (grid-strided): the 36-wide Dice rows of h are
// read coalesced and reduced per history slot in a fixed order
// (w_t = (sum_j w1_j Dice(h_tj) + b1) * mask_t, DIN.py:117-124); then
// thread i < ID forms wh_i = sum_t w_t k_t[i] (t ascending, :276) from the
// re-gathered history rows, and the rest of the workgroup copies the user /
// context / candidate embeddings: MLP input row [user, ctx, cand, wh].
template <typename TT>
__global__ __launch_bounds__(256) void din_att_out_kernel(
    const TT* __restrict__ table, const int64_t* __restrict__ row_base, int n_user, int n_item,
    int n_ctx, const int32_t* __restrict__ user_idx, const int32_t* __restrict__ item_idx,
    const int32_t* __restrict__ hist_idx, const int32_t* __restrict__ ctx_idx,
    const float* __restrict__ mask, int64_t B, int64_t S, int T, const float* __restrict__ h,
    const float2* __restrict__ hstats_all, const float* __restrict__ att_w1,
    const float* __restrict__ att_b1, float* __restrict__ mlp_in) {
    __shared__ float prod[128 * DIN_H];
    __shared__ float wt[128];
    __shared__ int64_t hrow[128 * 8];
    const int tid = threadIdx.x;
    const int ID = n_item * DIN_E;
    const int IN = (n_user + n_ctx + 2 * n_item) * DIN_E;
    const int ncol = T * DIN_H;
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        __syncthreads();
        const float* hb = h + b * ncol;
        const float2* hstats = hstats_all + (b / S) * ncol;
        for (int e = tid; e < ncol; e += 256) {
            const int j = e % DIN_H;
            const float2 st = hstats[e];
            prod[e] = att_w1[j] * dice(hb[e], st.x, st.y);
        }
        for (int e = tid; e < T * n_item; e += 256) {
            const int f = e % n_item;
            hrow[e] = (row_base[n_user + f] + hist_idx[b * T * n_item + e]) * DIN_E;
        }
        __syncthreads();
        if (tid < T) {
            float s = 0.0f;
            for (int j = 0; j < DIN_H; ++j) s += prod[tid * DIN_H + j];
            wt[tid] = (s + att_b1[0]) * mask[b * T + tid];
        }
        __syncthreads();
        float* row = mlp_in + b * IN;
        if (tid < ID) {
            const int f = tid / DIN_E, e = tid % DIN_E;
            float s = 0.0f;
            for (int t = 0; t < T; ++t) s += wt[t] * tload(table + hrow[t * n_item + f] + e);
            row[(n_user + n_ctx + n_item) * DIN_E + tid] = s;
            row[(n_user + n_ctx) * DIN_E + tid] =
                tload(table + (row_base[n_user + f] + item_idx[b * n_item + f]) * DIN_E + e);
        } else {
            for (int i = tid - ID; i < (n_user + n_ctx) * DIN_E; i += 256 - ID) {
                const int f = i / DIN_E, e = i % DIN_E;
                const int64_t r = f < n_user ? row_base[f] + user_idx[b * n_user + f]
                                             : row_base[n_item + f] + ctx_idx[b * n_ctx + (f - n_user)];
                row[i] = tload(table + r * DIN_E + e);
            }
        }
    }
}

// ----------------------------------------------------- 3'. att wh (fast) --
// Fast path (T <= 64, h1 <= 256): only the weighted history sum wh [B, ID]
// is materialised -- GEMM1 (din_mlp1_kernel) gathers the user / context /
// candidate embeddings itself.  One wave per sample.  The sample's h block
// [T x 36] is read as consecutive 16-B chunks (one coalesced 1-KB load per
// 64 chunks; a lane-per-row read touches 64 cache lines per instruction) and
// Dice'd against the batch statistics of the same chunks, held in registers
// per Dice batch; lane t < T then reduces w_t = (sum_j w1_j Dice(h_tj) + b1)
// * mask_t over j ascending from LDS (DIN.py:117-124).  wh = sum_t w_t k_t
// (:276): every lane gathers 16-B pieces of history rows for slots t = tg,
// tg + TG, ... (a round's loads in flight together) and the slot groups are
// combined by an xor tree; slots after the last nonzero weight add exactly
// +0 and are skipped.  Dice uses the hardware exp / reciprocal (~1 ulp each;
// the parity bar is 1e-5), (mean, 1 / (std + 1e-8)) per column from
// col_stats.  The next sample's h block, indices and mask are in flight
// during the gathers.  Each wave owns a contiguous run of samples and
// publishes max |wh| per Dice batch (atomicMax on the float bits) for
// GEMM1's fp16 scale.

// din_wh2: the Dice statistics live in LDS, not registers.  Workgroup
// (seg, g) takes a contiguous run of ONE Dice batch (segment), so its four
// waves share the segment's (mean, 1 / (std + 1e-8)) table, loaded once into
// LDS; the per-wave Dice stage holds T rows (dynamic LDS).  3 waves / SIMD at
// T <= 50 (48 KB of LDS per workgroup) for this latency-bound gather kernel
// (round 2's register-resident variant ran 2 with spills: 1.40 vs 1.10 ms).
// Masked rows (mask_t = 0) never read their h row: the attention kernels may
// leave it unwritten.
template <typename TT, int NI, int NCH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void din_wh2_kernel(
    const TT* __restrict__ table, const int64_t* __restrict__ row_base, int n_user,
    const int32_t* __restrict__ hist_idx, const float* __restrict__ mask, int64_t B, int64_t S,
    int T, int GW, const float* __restrict__ h, const float2* __restrict__ hinv_all,
    const float* __restrict__ att_w1, const float* __restrict__ att_b1, float* __restrict__ wh,
    unsigned int* __restrict__ segmax) {
    constexpr int ID = NI * DIN_E;
    typedef float f4n __attribute__((ext_vector_type(4)));
    typedef uint32_t u4n __attribute__((ext_vector_type(4)));
    constexpr int EPP = 16 / (int)sizeof(TT);
    constexpr int PPR = DIN_E / EPP;
    constexpr int LPT = NI * PPR;
    constexpr int TG = 64 / LPT;
    constexpr int R = 64 / TG < 6 ? 64 / TG : 6;  // loads per lane in flight per round (VGPRs: 3 waves / SIMD)
    constexpr int HQ = DIN_H / 4;
    extern __shared__ __attribute__((aligned(16))) float wh2_lds[];
    const int nq = T * HQ;
    f4n* smean = reinterpret_cast<f4n*>(wh2_lds);       // [nq]
    f4n* sinv = smean + nq;                             // [nq]
    float* dscb = reinterpret_cast<float*>(sinv + nq);  // [4][T * DIN_H]
    int32_t* rrb = reinterpret_cast<int32_t*>(dscb + 4 * T * DIN_H);  // [4][64 * NI]
    float* wsb = reinterpret_cast<float*>(rrb + 4 * 64 * NI);         // [4][64]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* dsc = dscb + wv * T * DIN_H;
    int32_t* rr_s = rrb + wv * 64 * NI;
    float* w_s = wsb + wv * 64;
    const int tg = lane / LPT, gf = (lane / PPR) % NI, gc = lane % PPR;
    const int64_t seg = blockIdx.x / GW, g = blockIdx.x % GW;
    const int64_t s0 = seg * S, s1 = (seg + 1) * S < B ? (seg + 1) * S : B;
    const int64_t cw = (s1 - s0 + GW - 1) / GW;          // samples per workgroup
    const int64_t pw = (cw + 3) / 4;                      // per wave
    const int64_t wb = s0 + g * cw + wv * pw;
    const int64_t wg_end = s0 + (g + 1) * cw < s1 ? s0 + (g + 1) * cw : s1;
    const int64_t b0 = wb;
    const int64_t b1e = wb + pw < wg_end ? wb + pw : wg_end;
    // this segment's statistics -> LDS (chunk q = columns 4q .. 4q + 3)
    {
        const f4n* st = reinterpret_cast<const f4n*>(hinv_all + (size_t)seg * T * DIN_H);
        for (int q = threadIdx.x; q < nq; q += 256) {
            const f4n a = st[2 * q], b = st[2 * q + 1];
            smean[q] = f4n{a.x, a.z, b.x, b.z};
            sinv[q] = f4n{a.y, a.w, b.y, b.w};
        }
    }
    __syncthreads();
    const float ab1 = att_b1[0];
    const bool act = lane < T;
    int64_t rbs[NI];
#pragma unroll
    for (int f = 0; f < NI; ++f) rbs[f] = row_base[n_user + f];
    float mx = 0.0f;
    f4n hq[NCH];
    int32_t ix[NI];
    float mk;
    const f4n* hdummy = reinterpret_cast<const f4n*>(hinv_all);
    auto load_mask = [&](int64_t bb) -> float { return (bb < b1e && act) ? mask[bb * T + lane] : 0.0f; };
    auto fetch = [&](int64_t bb, float mbb) {
        const bool ok = bb < b1e;
        const f4n* hr = reinterpret_cast<const f4n*>(h + (size_t)(ok ? bb : 0) * T * DIN_H);
        const uint64_t live = __builtin_amdgcn_ballot_w64(mbb != 0.0f);
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int q = 64 * i + lane;
            const bool on = ok && q < nq && ((live >> (q / HQ)) & 1ull);
            hq[i] = *(on ? hr + q : hdummy);
        }
#pragma unroll
        for (int f = 0; f < NI; ++f) ix[f] = ok && act ? hist_idx[((size_t)bb * T + lane) * NI + f] : 0;
        mk = mbb;
    };
    float mk_n = load_mask(b0);
    fetch(b0, mk_n);
    mk_n = load_mask(b0 + 1);
    // sample b's wh is stored during sample b + 1, right before its gathers:
    // a store counts in vmcnt, so one issued at the end of a sample made the
    // next sample's first wait a full store round trip; issued before the
    // gathers its acknowledgement overlaps their latency
    float pacc[EPP];
    int64_t pb = -1;
    auto store_wh = [&]() {
        if (pb >= 0 && tg == 0) {
            f4n* o = reinterpret_cast<f4n*>(wh + (size_t)pb * ID + gf * DIN_E + gc * EPP);
#pragma unroll
            for (int v = 0; v < EPP / 4; ++v) o[v] = f4n{pacc[4 * v], pacc[4 * v + 1], pacc[4 * v + 2], pacc[4 * v + 3]};
        }
    };
    for (int64_t b = b0; b < b1e; ++b) {
        // Dice only up to the last live row (rows past it are padding: their
        // weight is 0 whatever Dice gives; ~60% of the rows at config 3)
        const uint64_t lv = __builtin_amdgcn_ballot_w64(act && mk != 0.0f);
        const int tl = lv ? 64 - __builtin_clzll(lv) : 0;
        const int nql = tl * HQ;
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int q = 64 * i + lane;
            if (64 * i >= nql) break;  // uniform
            if (q < nql) {
                const f4n m4 = smean[q], i4 = sinv[q];
                f4n d;
#pragma unroll
                for (int e = 0; e < 4; ++e) d[e] = dice_fast(hq[i][e], m4[e], i4[e]);
                *reinterpret_cast<f4n*>(&dsc[4 * q]) = d;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        float w = 0.0f;
        if (lane < tl && mk != 0.0f) {
            const f4n* dr = reinterpret_cast<const f4n*>(&dsc[lane * DIN_H]);
            float sacc = 0.0f;
#pragma unroll
            for (int c = 0; c < HQ; ++c) {
                const f4n d = dr[c];
#pragma unroll
                for (int e = 0; e < 4; ++e) sacc += att_w1[4 * c + e] * d[e];
            }
            w = (sacc + ab1) * mk;
        }
        w_s[lane] = w;
#pragma unroll
        for (int f = 0; f < NI; ++f) rr_s[lane * NI + f] = act ? (int32_t)(rbs[f] + ix[f]) : 0;
        const uint64_t nz = __builtin_amdgcn_ballot_w64(w != 0.0f);
        const int te = nz ? 64 - __builtin_clzll(nz) : 0;
        asm volatile("" ::: "memory");
        fetch(b + 1, mk_n);
        mk_n = load_mask(b + 2);
        store_wh();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        float acc[EPP];
#pragma unroll
        for (int e = 0; e < EPP; ++e) acc[e] = 0.0f;
        for (int t0 = 0; t0 < te; t0 += TG * R) {
            u4n raw[R];
            float wt[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int t = t0 + TG * u + tg;
                const int tc = t < te ? t : te - 1;
                wt[u] = t < te ? w_s[tc] : 0.0f;
                const int32_t r = rr_s[tc * NI + gf];
                raw[u] = *reinterpret_cast<const u4n*>(table + (int64_t)r * DIN_E + gc * EPP);
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                if constexpr (sizeof(TT) == 4) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[e] = fmaf(wt[u], __uint_as_float(raw[u][e]), acc[e]);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        acc[2 * i] = fmaf(wt[u], __uint_as_float(raw[u][i] << 16), acc[2 * i]);
                        acc[2 * i + 1] = fmaf(wt[u], __uint_as_float(raw[u][i] & 0xFFFF0000u), acc[2 * i + 1]);
                    }
                }
            }
        }
#pragma unroll
        for (int off = LPT; off < 64; off <<= 1)
#pragma unroll
            for (int e = 0; e < EPP; ++e) acc[e] += __shfl_xor(acc[e], off, WAVE);
#pragma unroll
        for (int e = 0; e < EPP; ++e) {
            pacc[e] = acc[e];
            mx = fmaxf(mx, fabsf(acc[e]));
        }
        pb = b;
    }
    store_wh();
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) mx = fmaxf(mx, __shfl_xor(mx, k, WAVE));
    if (lane == 0 && b0 < b1e) atomicMax(segmax + seg, __float_as_uint(mx));
}

static inline size_t din_wh2_lds(int T, int NI) {
    return (size_t)2 * T * (DIN_H / 4) * 16 + (size_t)4 * T * DIN_H * 4 + (size_t)4 * 64 * NI * 4 + 4 * 64 * 4;
}

// ----------------------------------------------------- 4'. mlp1 (fast) --
// z1 = [user | ctx | cand | wh] W0^T + b0 (DIN.py:279-282, Linear(IN -> h1))
// without materialising the MLP input: every 32-wide feature is one k-step
// of v_mfma_f32_16x16x32_f16, its A fragment gathered straight from the
// embedding table (or read from wh).  Exact-f32-class split product, the
// din_att_h scheme:
//   * W0 = W_hi + W_lo (fp16 at scale s_w, packed per call in fragment order
//     by din_w1_pack_kernel);
//   * bf16 table rows are exact in fp16 at scale s_k -> 2 MFMAs per fragment;
//     fp32 rows and wh (scale s_h, per Dice batch) are split too -> 3.
// The embedding k-steps accumulate at scale s_k s_w; the accumulator is then
// rescaled exactly (powers of two) to s_h s_w for the wh k-steps.
// Workgroup = 4 waves x 32 rows (two 16-row A tiles, all NT column tiles per
// wave) = 128 rows.  The W0 slice of k-step s+1 is loaded into registers
// during step s and stored to the other LDS buffer after it (one barrier per
// step); the A rows of step s+1 and the indices of step s+2 are in flight
// during step s.  Per 64-row half: fp64 column sums for the next Dice.
constexpr int MLP1_ROWS = 128;

template <int NT>
__global__ void din_w1_pack_kernel(const float* __restrict__ W, int N, int K,
                                   const unsigned int* __restrict__ wmax, din_half8* __restrict__ out) {
    // out[s][j][v][lane] = 8 halves of (W * s_w) (v = 0: hi, 1: lo) for column
    // n = 16 j + (lane & 15), k = 32 s + 8 (lane >> 4) + [0, 8); zero past N, K
    const float s_w = pow2_scale(__uint_as_float(*wmax));
    const int KS = (K + DIN_E - 1) / DIN_E;
    const int64_t total = (int64_t)KS * NT * 64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(i % 64), j = (int)((i / 64) % NT), s = (int)(i / (64 * NT));
        const int n = 16 * j + (lane & 15), k = DIN_E * s + 8 * (lane >> 4);
        float x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = (n < N && k + e < K) ? W[(size_t)n * K + k + e] : 0.0f;
        din_half8 hi, lo;
        split8(x, s_w, hi, lo);
        out[((int64_t)s * NT + j) * 128 + lane] = hi;
        out[((int64_t)s * NT + j) * 128 + 64 + lane] = lo;
    }
}

// Shared GEMM epilogue of din_mlp1 / din_mlp2 (one 128-row block, 4 waves x
// 32 rows): C = acc * inv + bias, fp64 (sum, sumsq) per column over each
// 64-row half -> partial rows blk0, blk0 + 1 (fixed order: waves 2h, 2h+1),
// and optionally max |C| per Dice batch (atomicMax on the float bits).
template <int NT>
__device__ __forceinline__ void mlp_epilogue(const din_f4 (&acc)[2][NT], float inv, const float* __restrict__ bias,
                                             int N, int64_t M, int64_t m0, int64_t blk0, int64_t S,
                                             double2* cs, float* __restrict__ C, double* __restrict__ partial,
                                             unsigned int* __restrict__ zmax) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4;
    float mx = 0.0f;
    // every bias load before the first store: stores count in vmcnt, so a
    // load issued between (conditional) stores would make its wait a
    // vmcnt(0) that drains the stores already issued -- one store round trip
    // per column tile
    float bns[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int n = 16 * j + (lane & 15);
        bns[j] = bias[n < N ? n : N - 1];
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int n = 16 * j + (lane & 15);
        const float bn = n < N ? bns[j] : 0.0f;
        double su = 0.0, sq = 0.0;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t m = m0 + 16 * a + 4 * q + r;
                const float v = acc[a][j][r] * inv + bn;
                if (n < N && m < M) {
                    C[m * N + n] = v;
                    su += (double)v;
                    sq += (double)v * (double)v;
                    mx = fmaxf(mx, fabsf(v));
                }
            }
        su += __shfl_xor(su, 16, WAVE);
        sq += __shfl_xor(sq, 16, WAVE);
        su += __shfl_xor(su, 32, WAVE);
        sq += __shfl_xor(sq, 32, WAVE);
        if (lane < 16) cs[wv * NT * 16 + n] = make_double2(su, sq);
    }
    if (zmax != nullptr && m0 < M) {
#pragma unroll
        for (int k = 32; k > 0; k >>= 1) mx = fmaxf(mx, __shfl_xor(mx, k, WAVE));
        if (lane == 0) atomicMax(zmax + m0 / S, __float_as_uint(mx));
    }
    __syncthreads();
    for (int e = tid; e < 2 * N; e += 256) {
        const int hf = e / N, n = e % N;
        const int64_t blk = blk0 + hf;
        if (blk * 64 < M) {
            const double2 x = cs[(2 * hf) * NT * 16 + n], y = cs[(2 * hf + 1) * NT * 16 + n];
            partial[((size_t)blk * N + n) * 2] = x.x + y.x;
            partial[((size_t)blk * N + n) * 2 + 1] = x.y + y.y;
        }
    }
    __syncthreads();
}

template <typename TT, int NT>
__global__ __launch_bounds__(256, 2) void din_mlp1_kernel(
    const TT* __restrict__ table, const int64_t* __restrict__ row_base, int n_user, int n_item,
    int n_ctx, const int32_t* __restrict__ user_idx, const int32_t* __restrict__ item_idx,
    const int32_t* __restrict__ ctx_idx, const float* __restrict__ wh,
    const unsigned int* __restrict__ wh_segmax, const float* __restrict__ prep,
    const unsigned int* __restrict__ w1max, const din_u4* __restrict__ w1pack,
    const float* __restrict__ bias, int64_t M, int64_t S, int N, float* __restrict__ C,
    double* __restrict__ partial, unsigned int* __restrict__ zmax) {
    constexpr bool F32 = sizeof(TT) == 4;
    constexpr int CH = NT * 128;               // 16-B chunks per k-step slice
    constexpr int CPT = (CH + 255) / 256;      // chunks per thread
    __shared__ __attribute__((aligned(16))) din_u4 wr[2][CH];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4;
    const int ID = n_item * DIN_E;
    const int KE = n_user + n_ctx + n_item;  // embedding k-steps
    const int KS = KE + n_item;              // + the wh k-steps
    const int64_t m0 = (int64_t)blockIdx.x * MLP1_ROWS + wv * 32;
    int64_t mrow[2];
    bool mok[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        mrow[a] = m0 + 16 * a + (lane & 15);
        mok[a] = mrow[a] < M;
    }
    const int64_t seg = (m0 < M ? m0 : M - 1) / S;  // a wave's 32 rows lie in one Dice batch
    const float s_k = reinterpret_cast<const DinScales*>(prep + 3 * DIN_H * ID)->s_k;
    const float s_w = pow2_scale(__uint_as_float(*w1max));
    const float s_h = pow2_scale(__uint_as_float(wh_segmax[seg]));

    // Loads are unconditional, from a clamped row and a pointer chosen by the
    // (uniform) k-step: a value merged from a conditional load forces a
    // vmcnt(0) at the merge, draining the prefetches in flight.  Rows past M
    // are zeroed at use.
    int64_t mrc[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) mrc[a] = mok[a] ? mrow[a] : M - 1;
    auto idx_load = [&](int s, int a) -> int32_t {
        const int64_t m = mrc[a];
        const int32_t* ip = s < n_user ? user_idx + m * n_user + s
                            : s < n_user + n_ctx ? ctx_idx + m * n_ctx + (s - n_user)
                            : s < KE ? item_idx + m * n_item + (s - n_user - n_ctx)
                                     : item_idx + m * n_item;  // unused (wh k-step)
        return *ip;
    };
    auto data_load = [&](int s, int a, int32_t idx, din_u4 (&raw)[2]) {
        const din_u4* p;
        if (s >= KE) {
            p = reinterpret_cast<const din_u4*>(wh + mrc[a] * ID + (s - KE) * DIN_E + 8 * q);
        } else {
            const int64_t base = s < n_user ? row_base[s]
                                 : s < n_user + n_ctx ? row_base[n_user + n_item + (s - n_user)]
                                                      : row_base[n_user + (s - n_user - n_ctx)];
            p = reinterpret_cast<const din_u4*>(table + (base + idx) * DIN_E + 8 * q);
        }
        // the second piece is read always (a bf16 table row re-reads the
        // first: the row may be the table's last), so no load is conditional
        raw[0] = p[0];
        raw[1] = p[(F32 || s >= KE) ? 1 : 0];
    };
    din_u4 stg[CPT];
    din_f4 acc[2][NT];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[a][j] = din_f4{0.0f, 0.0f, 0.0f, 0.0f};

    din_u4 raw[2][2], nraw[2][2];
    int32_t idx1[2], idx2[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        idx1[a] = idx_load(0, a);
        data_load(0, a, idx1[a], raw[a]);
        idx1[a] = idx_load(1, a);
        idx2[a] = idx_load(2, a);
    }
    stage_load<CPT, CH>(stg, w1pack, tid);
    stage_store<CPT, CH>(stg, wr[0], tid);
    lds_barrier();
    // one k-step: prefetch the next slice / A rows / indices, the MFMAs
    // (A fragments: hi, and lo when split; per column tile its two W
    // fragments), then the slice hand-off.  The split (fp32 tables, the wh
    // steps) is a compile-time parameter: two loops, no branch per MFMA.
    auto kstep = [&](int s, auto split_c) {
        constexpr bool SPLIT = decltype(split_c)::value;
        if (s + 1 < KS) stage_load<CPT, CH>(stg, w1pack + (size_t)(s + 1) * CH, tid);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            if (s + 1 < KS) data_load(s + 1, a, idx1[a], nraw[a]);
            idx1[a] = idx2[a];
            idx2[a] = idx_load(s + 3 < KS ? s + 3 : KS - 1, a);
        }
        const float sc = s >= KE ? s_h : s_k;
        din_half8 ahi[2], alo[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            float v[8];
            if (SPLIT) {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = __uint_as_float(raw[a][e >> 2][e & 3]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[2 * i] = __uint_as_float(raw[a][0][i] << 16);
                    v[2 * i + 1] = __uint_as_float(raw[a][0][i] & 0xFFFF0000u);
                }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = mok[a] ? v[e] : 0.0f;
            split8(v, sc, ahi[a], alo[a]);
        }
        const din_half8* wb = reinterpret_cast<const din_half8*>(wr[s & 1]);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const din_half8 bh = wb[(2 * j) * 64 + lane];
            const din_half8 bl = wb[(2 * j + 1) * 64 + lane];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                acc[a][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[a], bh, acc[a][j], 0, 0, 0);
                acc[a][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[a], bl, acc[a][j], 0, 0, 0);
                if constexpr (SPLIT)
                    acc[a][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[a], bh, acc[a][j], 0, 0, 0);
            }
        }
        if (s + 1 < KS) stage_store<CPT, CH>(stg, wr[(s + 1) & 1], tid);
        lds_barrier();
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            raw[a][0] = nraw[a][0];
            raw[a][1] = nraw[a][1];
        }
    };
    for (int s = 0; s < KE; ++s) {
        if constexpr (F32) kstep(s, std::true_type{});
        else kstep(s, std::false_type{});
    }
    {
        const float r = s_h / s_k;  // exact: both are powers of two
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[a][j] *= r;
    }
    for (int s = KE; s < KS; ++s) kstep(s, std::true_type{});
    // epilogue: scale, bias, store, per-64-row-half fp64 column sums, max |z1|
    lds_barrier();  // (every wave is past its last read of wr)
    double2* cs = reinterpret_cast<double2*>(&wr[0][0]);  // [4 waves][NT * 16]
    static_assert(sizeof(wr) >= 4 * NT * 16 * sizeof(double2), "LDS reuse");
    mlp_epilogue<NT>(acc, 1.0f / (s_h * s_w), bias, N, M, m0, (int64_t)blockIdx.x * 2, S, cs, C, partial, zmax);
}

// ----------------------------------------------------- 6'. mlp2 (fast) --
// z2 = Dice(z1) W1^T + b1 (DIN.py:282-283) on the same split-fp16 MFMA: A =
// Dice-on-load of z1 (batch (mean, 1 / (std + 1e-8)) per column) at scale s_a
// from max |z1| of the Dice batch (|Dice(x)| <= |x|), split hi / lo -> 3 MFMAs
// per fragment.  The whole packed W1 (KS x NT x 2 KB) stays in LDS; each
// workgroup walks 128-row blocks (4 waves x 32 rows), loading the next
// k-step's A while the current one runs.
template <int NT>
__global__ __launch_bounds__(256, 2) void din_mlp2_kernel(
    const float* __restrict__ A, const float2* __restrict__ astats_all,
    const unsigned int* __restrict__ amax, const unsigned int* __restrict__ wmax,
    const din_u4* __restrict__ wpack, const float* __restrict__ bias, int64_t M, int64_t S, int K, int N,
    float* __restrict__ C, double* __restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) din_u4 wl[];
    const int KS = (K + DIN_E - 1) / DIN_E;
    const int CH = KS * NT * 128;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4;
    for (int c = tid; c < CH; c += 256) wl[c] = wpack[c];
    double2* cs = reinterpret_cast<double2*>(wl + CH);
    __syncthreads();
    const din_half8* wb = reinterpret_cast<const din_half8*>(wl);
    const float s_w = pow2_scale(__uint_as_float(*wmax));
    const int64_t nrb = (M + MLP1_ROWS - 1) / MLP1_ROWS;
    typedef float f4n __attribute__((ext_vector_type(4)));
    for (int64_t rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
        const int64_t m0 = rb * MLP1_ROWS + wv * 32;
        const int64_t seg = (m0 < M ? m0 : M - 1) / S;
        const float s_a = pow2_scale(__uint_as_float(amax[seg]));
        const float2* st = astats_all + seg * K;
        int64_t mrow[2];
        bool mok[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            mrow[a] = m0 + 16 * a + (lane & 15);
            mok[a] = mrow[a] < M;
        }
        auto load = [&](int s, int a, f4n (&x)[2]) {
            const int k = DIN_E * s + 8 * q;
            x[0] = x[1] = f4n{0.0f, 0.0f, 0.0f, 0.0f};
            if (!mok[a]) return;
            const float* p = A + mrow[a] * K + k;
            if (k + 8 <= K && (K & 3) == 0) {
                x[0] = *reinterpret_cast<const f4n*>(p);
                x[1] = *reinterpret_cast<const f4n*>(p + 4);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (k + e < K) x[e >> 2][e & 3] = p[e];
            }
        };
        din_f4 acc[2][NT];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[a][j] = din_f4{0.0f, 0.0f, 0.0f, 0.0f};
        f4n cur[2][2], nxt[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a) load(0, a, cur[a]);
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
                if (s + 1 < KS) load(s + 1, a, nxt[a]);
            const int k = DIN_E * s + 8 * q;
            float mu[8], iv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float2 t = k + e < K ? st[k + e] : make_float2(0.0f, 0.0f);
                mu[e] = t.x;
                iv[e] = t.y;
            }
            din_half8 ahi[2], alo[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = k + e < K ? dice_fast(cur[a][e >> 2][e & 3], mu[e], iv[e]) : 0.0f;
                split8(v, s_a, ahi[a], alo[a]);
            }
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const din_half8 bh = wb[((s * NT + j) * 2) * 64 + lane];
                const din_half8 bl = wb[((s * NT + j) * 2 + 1) * 64 + lane];
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    acc[a][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[a], bh, acc[a][j], 0, 0, 0);
                    acc[a][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[a], bl, acc[a][j], 0, 0, 0);
                    acc[a][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[a], bh, acc[a][j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                cur[a][0] = nxt[a][0];
                cur[a][1] = nxt[a][1];
            }
        }
        mlp_epilogue<NT>(acc, 1.0f / (s_a * s_w), bias, N, M, m0, rb * 2, S, cs, C, partial, nullptr);
    }
}

// ---------------------------------------------------------- 4/6. gemm --
// C[M][N] = f(A)[M][K] W[N][K]^T + bias on the f32-input MFMA
// (v_mfma_f32_32x32x2_f32, exact f32 fma chains), f = Dice with per-column
// stats of A (GEMM2, Dice-on-load) or identity (GEMM1).
// Workgroup = 8 waves = 64x64 output tile: waves (wm, wn) own 32x32 blocks,
// kh in {0,1} splits K in two interleaved halves (2 waves / SIMD); the two
// partial accumulators are added in a fixed order through LDS.  Operands go
// global -> registers directly: within an 8-wide k chunk, MFMA step s of
// lane half h uses k = 8h + s, so each lane loads 8 contiguous floats of its
// A row and W row (two float4) -- the k order inside the chunk is permuted
// identically for both operands.  Loads run two chunks ahead.
// Writes per-row-block fp64 column sums (sum, sumsq) of C for the next Dice.
typedef float din_f16v __attribute__((ext_vector_type(16)));

template <bool DICE_A>
__device__ __forceinline__ void gemm_load(const float* __restrict__ A, const float2* __restrict__ astats,
                                          const float* __restrict__ W, int64_t m, bool mok, int n,
                                          bool nok, int K, int k, float (&a)[8], float (&w)[8]) {
    const bool full = k + 8 <= K;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        a[e] = 0.0f;
        w[e] = 0.0f;
    }
    if (full && ((K & 3) == 0)) {
        if (mok) {
            const float4 x = *reinterpret_cast<const float4*>(A + m * K + k);
            const float4 y = *reinterpret_cast<const float4*>(A + m * K + k + 4);
            a[0] = x.x; a[1] = x.y; a[2] = x.z; a[3] = x.w;
            a[4] = y.x; a[5] = y.y; a[6] = y.z; a[7] = y.w;
        }
        if (nok) {
            const float4 x = *reinterpret_cast<const float4*>(W + (int64_t)n * K + k);
            const float4 y = *reinterpret_cast<const float4*>(W + (int64_t)n * K + k + 4);
            w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
            w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
        }
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if (k + e < K) {
                if (mok) a[e] = A[m * K + k + e];
                if (nok) w[e] = W[(int64_t)n * K + k + e];
            }
        }
    }
    if (DICE_A && mok) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (k + e < K) {
                const float2 st = astats[k + e];  // (mean, 1 / (std + 1e-8))
                a[e] = dice_fast(a[e], st.x, st.y);
            }
    }
}

template <bool DICE_A>
__global__ __launch_bounds__(512) void din_gemm_kernel(
    const float* __restrict__ A, const float2* __restrict__ astats_all, const float* __restrict__ W,
    const float* __restrict__ bias, int64_t M, int64_t S, int N, int K, float* __restrict__ C,
    double* __restrict__ partial) {
    __shared__ float red[4][16][64];
    __shared__ double cs[2][2][64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv & 1, wn = (wv >> 1) & 1, kh = wv >> 2;
    const int64_t m = (int64_t)blockIdx.x * 64 + wm * 32 + (lane & 31);
    const int n = blockIdx.y * 64 + wn * 32 + (lane & 31);
    const bool mok = m < M, nok = n < N;
    // Dice statistics of row m's segment (its Dice batch)
    const float2* astats = DICE_A ? astats_all + (mok ? m / S : 0) * K : nullptr;
    const int half = lane >> 5;
    din_f16v acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    // chunks c = kh, kh + 2, kh + 4, ... of 16 k each: lane half h takes k = 16c + 8h + [0, 8)
    const int nch = (K + 15) / 16;
    float a0[8], w0[8], a1[8], w1[8];
    int c = kh;
    if (c < nch) gemm_load<DICE_A>(A, astats, W, m, mok, n, nok, K, 16 * c + 8 * half, a0, w0);
    if (c + 2 < nch) gemm_load<DICE_A>(A, astats, W, m, mok, n, nok, K, 16 * (c + 2) + 8 * half, a1, w1);
    for (; c < nch; c += 4) {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], w0[e], acc, 0, 0, 0);
        if (c + 4 < nch) gemm_load<DICE_A>(A, astats, W, m, mok, n, nok, K, 16 * (c + 4) + 8 * half, a0, w0);
        if (c + 2 < nch) {
#pragma unroll
            for (int e = 0; e < 8; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], w1[e], acc, 0, 0, 0);
            if (c + 6 < nch) gemm_load<DICE_A>(A, astats, W, m, mok, n, nok, K, 16 * (c + 6) + 8 * half, a1, w1);
        }
    }
    // K halves: kh = 1 hands its accumulator to kh = 0 (fixed order)
    if (kh == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) red[wv - 4][r][lane] = acc[r];
    }
    __syncthreads();
    if (kh == 0) {
        const int64_t mrow0 = (int64_t)blockIdx.x * 64 + wm * 32;
        double s = 0.0, ss = 0.0;
        const float bn = nok ? bias[n] : 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t mr = mrow0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            const float v = (acc[r] + red[wv][r][lane]) + bn;
            if (nok && mr < M) {
                C[mr * N + n] = v;
                s += (double)v;
                ss += (double)v * (double)v;
            }
        }
        s += __shfl_xor(s, 32, WAVE);
        ss += __shfl_xor(ss, 32, WAVE);
        if (lane < 32) {
            cs[0][wm][wn * 32 + lane] = s;
            cs[1][wm][wn * 32 + lane] = ss;
        }
    }
    __syncthreads();
    if (tid < 64) {
        const int nn = blockIdx.y * 64 + tid;
        if (nn < N) {
            partial[((size_t)blockIdx.x * N + nn) * 2] = cs[0][0][tid] + cs[0][1][tid];
            partial[((size_t)blockIdx.x * N + nn) * 2 + 1] = cs[1][0][tid] + cs[1][1][tid];
        }
    }
}

// ------------------------------------------------------------ 8. head --
// logit = sum_j w_j Dice(z2_j) + b (DIN.py:283-284), prob = sigmoid.  16
// lanes per sample (4 samples per wave, lane l16 takes j = l16, l16 + 16, ...
// in order), the 16 partial sums combined by a fixed DPP tree within the
// row; grid-strided over the samples.
__device__ __forceinline__ float row16_sum(float x) {
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, false));  // row_half_mirror
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, false));  // row_mirror
    return x;
}

__global__ __launch_bounds__(256) void din_head_kernel(const float* __restrict__ Z, const float2* __restrict__ zstats_all,
                                                       int64_t B, int64_t S, int H, const float* __restrict__ w,
                                                       const float* __restrict__ bias, float* __restrict__ probs,
                                                       float* __restrict__ logits) {
    const int l16 = threadIdx.x & 15;
    const float b0 = bias[0];
    for (int64_t b = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; b < B; b += (int64_t)gridDim.x * 16) {
        const float2* zstats = zstats_all + (b / S) * H;
        const float* zr = Z + b * H;
        float s = 0.0f;
        for (int j = l16; j < H; j += 16) {
            const float2 st = zstats[j];
            s += w[j] * dice_fast(zr[j], st.x, st.y);  // st = (mean, 1 / (std + 1e-8))
        }
        s = row16_sum(s);
        if (l16 == 0) {
            const float lg = s + b0;
            if (logits) logits[b] = lg;
            probs[b] = 1.0f / (1.0f + expf(-lg));
        }
    }
}

// --------------------------------------------------------------- prepare --
__global__ void din_prepare_kernel(const float* __restrict__ w0, int ID, float* __restrict__ prep) {
    // w0 [36][4*ID] = [Wk | Wq | Wd | Wp]
    const int n = DIN_H * ID;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int j = i / ID, c = i % ID;
        const float* row = w0 + (size_t)j * 4 * ID;
        const float wk = row[c], wq = row[ID + c], wd = row[2 * ID + c], wp = row[3 * ID + c];
        prep[i] = wk - wd;
        prep[n + i] = wq + wd;
        prep[2 * n + i] = wp;
    }
}

// ---------------------------------------------------------- index remap --
// The kernels read 32-wide features.  A model with another embedding width D
// (din_embedding_dim, config.py:115) is served as 32-wide VIRTUAL features:
// every table zero-padded to m = ceil(D / 32) * 32 columns and viewed as
// [m * vocab, 32], feature f's index i becoming the m virtual indices
// m i + h; padding features (a shared all-zero row) fill the item features up
// to a supported count.  out[r, j] = map[j] < 0 ? map[2F + j]
//                                                : in[r, map[j]] * map[F + j] + map[2F + j]
// with F = f_out (map: src | mul | add rows).
__global__ void din_remap_kernel(const int32_t* __restrict__ in, int64_t n_rows, int f_in, int f_out,
                                 const int32_t* __restrict__ map, int32_t* __restrict__ out) {
    const int64_t n = n_rows * f_out;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / f_out;
        const int j = (int)(i - r * f_out);
        const int src = map[j];
        out[i] = src < 0 ? map[2 * f_out + j] : in[r * f_in + src] * map[f_out + j] + map[2 * f_out + j];
    }
}

// ------------------------------------------------------------- workspace --
// din_att_h workgroups per segment: about 6144 in the whole grid (24 per CU,
// measured best of 1024...32768 at config 3), at most 512 per segment and
// never more than the segment has samples
static inline int din_att_groups(int64_t N, int64_t S) {
    const int64_t n_seg = (N + S - 1) / S;
    int64_t g = (6144 + n_seg - 1) / n_seg;
    g = g < 8 ? 8 : g > 512 ? 512 : g;
    return (int)(g < S ? g : S);
}

struct DinWs {
    float* h;
    double* hpart;
    int32_t* plan;   // position-major path: per run of TM_SW samples, din_tm_plan_kernel
    float2* hstats;
    float* mlp_in;   // general path only
    float* wh;       // fast path only: [N, ID]
    float2* hinv;    // fast path only: per-segment (mean, 1 / (std + 1e-8)) of h
    unsigned int* whmax;  // fast path: per-segment max |wh| (float bits), then max |W0|
    din_half8* w1pack;    // fast path: packed W0 fragments
    din_half8* w2pack;    // fast path, h2 <= 128: packed W1 fragments
    float* z1;
    double* z1part;
    float2* z1stats;
    float* z2;
    double* z2part;
    float2* z2stats;
    size_t bytes;
};

static inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// fast path: wave-per-sample wh + gather-on-load split-fp16 GEMM1
static inline bool din_fast(int T, int h1) { return T <= 64 && h1 <= 256; }
static inline bool din_fast2(int T, int h1, int h2) { return din_fast(T, h1) && h2 <= 128; }
static inline int din_mlp2_nt(int h2) {
    const int nt = (h2 + 15) / 16;
    return nt <= 2 ? 2 : nt <= 4 ? 4 : nt <= 5 ? 5 : 8;
}
static inline int din_mlp1_nt(int h1) {
    const int nt = (h1 + 15) / 16;
    return nt <= 4 ? 4 : nt <= 8 ? 8 : nt <= 13 ? 13 : 16;
}

// N samples in Dice batches (segments) of S
static DinWs din_ws_layout(void* base, int64_t N, int64_t S, int T, int n_user, int n_item, int n_ctx,
                           int h1, int h2) {
    DinWs w;
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    size_t o = 0;
    const int64_t n_seg = (N + S - 1) / S;
    const int64_t nb_att = n_seg * std::max<int64_t>(din_att_groups(N, S), (S + TM_SW - 1) / TM_SW);
    const int64_t nb_m = (N + 63) / 64;
    const int IN = (n_user + n_ctx + 2 * n_item) * DIN_E;
    const bool fast = din_fast(T, h1);
    auto take = [&](size_t bytes) { uint8_t* r = p + o; o += al(bytes); return r; };
    w.h = (float*)take((size_t)N * T * DIN_H * 4);
    w.hpart = (double*)take((size_t)nb_att * T * DIN_H * 16);
    w.plan = (int32_t*)take((size_t)n_seg * ((S + TM_SW - 1) / TM_SW) * TM_PLAN * 4);
    w.hstats = (float2*)take((size_t)n_seg * T * DIN_H * 8);
    w.mlp_in = fast ? nullptr : (float*)take((size_t)N * IN * 4);
    w.wh = fast ? (float*)take((size_t)N * n_item * DIN_E * 4) : nullptr;
    w.hinv = fast ? (float2*)take((size_t)n_seg * T * DIN_H * 8) : nullptr;
    // [max |wh| per segment][max |W0|][max |z1| per segment][max |W1|]
    w.whmax = fast ? (unsigned int*)take((size_t)(2 * n_seg + 2) * 4) : nullptr;
    w.w2pack = din_fast2(T, h1, h2)
                   ? (din_half8*)take((size_t)((h1 + DIN_E - 1) / DIN_E) * din_mlp2_nt(h2) * 2048)
                   : nullptr;
    w.w1pack = fast ? (din_half8*)take((size_t)(IN / DIN_E) * din_mlp1_nt(h1) * 2048) : nullptr;
    w.z1 = (float*)take((size_t)N * h1 * 4);
    w.z1part = (double*)take((size_t)nb_m * h1 * 16);
    w.z1stats = (float2*)take((size_t)n_seg * h1 * 8);
    w.z2 = (float*)take((size_t)N * h2 * 4);
    w.z2part = (double*)take((size_t)nb_m * h2 * 16);
    w.z2stats = (float2*)take((size_t)n_seg * h2 * 8);
    w.bytes = o;
    return w;
}

}  // namespace nrk

using namespace nrk;

extern "C" {

#if NRK_TM_STAMP
// dev-only: the phase stamps of the last din_att_tm launch (1024 x 8 u64)
int nrk_dev_tm_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tm_stamps), sizeof(tm_stamps)) == hipSuccess ? 0 : -1;
}
#endif

int nrk_din_remap_index(const int32_t* in, int64_t n_rows, int f_in, const int32_t* map, int f_out,
                        int32_t* out, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_rows >= 0 && f_in >= 1 && f_out >= 1, "bad shape");
    if (n_rows == 0) return NRK_OK;
    NRK_REQUIRE(in && map && out, "null pointer");
    hipStream_t s = as_stream(stream);
    const int64_t n = n_rows * f_out;
    din_remap_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 4096), 256, 0, s>>>(in, n_rows, f_in, f_out,
                                                                                        map, out);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_din_prep_bytes(int n_item, int64_t n_table_rows) {
    if (n_item <= 0 || n_table_rows < 0) return 0;
    return din_tm_tab16_off(n_item) + (size_t)n_table_rows * DIN_E * 2;
}

int nrk_din_prepare(const float* att_w0, int n_item, const void* table, int table_dtype,
                    int64_t n_table_rows, void* prep, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(att_w0 && prep && table, "null pointer");
    NRK_REQUIRE(n_item >= 1 && n_item <= 8, "n_item must be in [1, 8]");
    // instantiated for 1, 2, 4 and 8 (32-wide) item features (ops.DinParams pads other counts)
    if (n_item != 8 && n_item != 4 && n_item != 2 && n_item != 1) NRK_UNSUPPORTED("n_item must be 1, 2, 4 or 8");
    NRK_REQUIRE(table_dtype == 0 || table_dtype == 1, "table_dtype must be 0 (f32) or 1 (bf16)");
    NRK_REQUIRE(n_table_rows >= 1, "n_table_rows must be >= 1");
    const int ID = n_item * DIN_E;
    hipStream_t s = as_stream(stream);
    float* pf = reinterpret_cast<float*>(prep);
    DinScales* sc = reinterpret_cast<DinScales*>(pf + 3 * DIN_H * ID);
    unsigned int* mx = reinterpret_cast<unsigned int*>(sc + 1);
    din_prepare_kernel<<<64, 256, 0, s>>>(att_w0, ID, pf);
    (void)hipMemsetAsync(mx, 0, 8, s);
    const int64_t n = n_table_rows * DIN_E;
    const int64_t g = (n + 255) / 256;
    din_absmax_kernel<<<(int)(g < 512 ? g : 512), 256, 0, s>>>(table, table_dtype, n, mx);
    din_scales_kernel<<<1, 256, 0, s>>>(pf, ID, mx, sc);
    // the position-major kernel's scales and packed weight fragments
    uint8_t* tm = reinterpret_cast<uint8_t*>(prep) + din_tm_base(n_item);
    DinScalesTM* tsc = reinterpret_cast<DinScalesTM*>(tm);
    din_half8* wpack = reinterpret_cast<din_half8*>(tm + 256);
    din_tm_scales_kernel<<<1, 256, 0, s>>>(pf, ID, mx, tsc);
    din_tm_pack_kernel<<<(3 * 3 * n_item * 64 + 255) / 256, 256, 0, s>>>(pf, n_item, tsc, wpack,
                                                                            wpack + 3 * n_item * 4 * 64);
    if (table_dtype == 1) {  // the position-major kernel reads the item rows as fp16 (bf16 tables)
        const int64_t nw = n_table_rows * DIN_E / 2;
        din_tm_tab16_kernel<<<(unsigned)std::min<int64_t>((nw + 255) / 256, 4096), 256, 0, s>>>(
            reinterpret_cast<const uint16_t*>(table), n_table_rows * DIN_E, tsc,
            reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(prep) + din_tm_tab16_off(n_item)));
    }
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_din_segments_workspace_bytes(int64_t n_samples, int64_t seg_len, int seq_len, int n_user,
                                        int n_item, int n_ctx, int h1, int h2) {
    if (n_samples < 1 || seg_len < 1 || seq_len < 1) return 0;
    if (seg_len > n_samples) seg_len = n_samples;
    return din_ws_layout(nullptr, n_samples, seg_len, seq_len, n_user, n_item, n_ctx, h1, h2).bytes;
}

size_t nrk_din_workspace_bytes(int64_t batch, int seq_len, int n_user, int n_item, int n_ctx,
                               int h1, int h2) {
    return nrk_din_segments_workspace_bytes(batch, batch, seq_len, n_user, n_item, n_ctx, h1, h2);
}

int nrk_din_forward_segments(const void* table, int table_dtype, const int64_t* row_base, int n_user,
                             int n_item, int n_ctx, const int32_t* user_idx, const int32_t* item_idx,
                             const int32_t* hist_idx, const int32_t* ctx_idx, const float* mask,
                             int64_t n_samples, int64_t seg_len, int seq_len, const void* prep,
                             const float* att_b0, const float* att_w1, const float* att_b1,
                             const float* mlp_w0, const float* mlp_b0, int h1, const float* mlp_w1,
                             const float* mlp_b1, int h2, const float* mlp_w2, const float* mlp_b2,
                             float* out_probs, float* out_logits, void* workspace,
                             size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(table_dtype == 0 || table_dtype == 1, "table_dtype must be 0 (f32) or 1 (bf16)");
    NRK_REQUIRE(n_samples >= 1 && seg_len >= 1, "n_samples and seg_len must be >= 1");
    const int64_t batch = n_samples;
    const int64_t S = seg_len < n_samples ? seg_len : n_samples;
    const int64_t n_seg = (batch + S - 1) / S;
    if (n_seg == 1)
        NRK_REQUIRE(batch >= 2, "batch must be >= 2 (Dice uses the batch std; B = 1 is NaN in the reference)");
    else
        NRK_REQUIRE(S % 64 == 0, "seg_len must be a multiple of 64 when the samples span several segments");
    NRK_REQUIRE(seq_len >= 1 && seq_len <= 128, "seq_len must be in [1, 128]");
    NRK_REQUIRE(n_user >= 1 && n_ctx >= 0 && n_item >= 1, "bad feature counts");
    // instantiated for 1, 2, 4 and 8 (32-wide) item features (ops.DinParams pads other counts)
    if (n_item != 8 && n_item != 4 && n_item != 2 && n_item != 1) NRK_UNSUPPORTED("n_item must be 1, 2, 4 or 8");
    NRK_REQUIRE(h1 >= 1 && h1 <= 1024 && h2 >= 1 && h2 <= 1024, "hidden sizes out of range");
    NRK_REQUIRE(table && row_base && user_idx && item_idx && hist_idx && mask && prep && att_b0 &&
                    att_w1 && att_b1 && mlp_w0 && mlp_b0 && mlp_w1 && mlp_b1 && mlp_w2 && mlp_b2 &&
                    out_probs && workspace,
                "null pointer");
    NRK_REQUIRE(n_ctx == 0 || ctx_idx, "ctx_idx null");
    NRK_REQUIRE(n_seg < (1ll << 31) && batch < (1ll << 40), "too many samples");
    const DinWs w = din_ws_layout(workspace, batch, S, seq_len, n_user, n_item, n_ctx, h1, h2);
    NRK_REQUIRE(workspace_bytes >= w.bytes, "workspace too small");
    hipStream_t s = as_stream(stream);
    const int T = seq_len;
    const int IN = (n_user + n_ctx + 2 * n_item) * DIN_E;
    const int G = din_att_groups(batch, S);
    const int64_t nb_att = n_seg * G;
    NRK_REQUIRE(nb_att < (1ll << 31), "too many segments");
    const float* pf = reinterpret_cast<const float*>(prep);
    // position-major attention (bf16 tables, T <= 64, <= 4 item features,
    // the fast MLP path): plan, then h + its statistics
    const bool tm_path = table_dtype == 1 && T <= TM_TMAX && n_item <= 4 && din_fast(T, h1);
    const int G_tm = (int)((S + TM_SW - 1) / TM_SW);
    // persistent: one workgroup per CU (register- and LDS-bound)
    static const int n_cu = [] {
        int dev = 0, cu = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
        return cu > 0 ? cu : 256;
    }();
    const unsigned tm_grid = (unsigned)std::min<int64_t>(n_seg * G_tm, n_cu);
    const uint8_t* tm = reinterpret_cast<const uint8_t*>(prep) + din_tm_base(n_item);
#define NRK_ATT_TM(NI)                                                                                 \
    do {                                                                                               \
        const size_t lds = din_tm_lds(NI, T);                                                          \
        (void)hipFuncSetAttribute((const void*)din_att_tm_kernel<NI>,                                  \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);               \
        din_att_tm_kernel<NI><<<tm_grid, TM_NT, lds, s>>>(                                             \
            reinterpret_cast<const din_half8*>(reinterpret_cast<const uint8_t*>(prep) +                \
                                               din_tm_tab16_off(n_item)),                               \
            row_base, n_user, item_idx, hist_idx, w.plan, batch, S, G_tm, T, tm, att_b0, w.h, w.hpart); \
    } while (0)
#define NRK_ATT_H(TT, NI)                                                                              \
    do {                                                                                               \
        if (T <= 64 && NI <= 4 && (sizeof(TT) == 2 || NI < 4))                                         \
            din_att_h2_kernel<TT, NI><<<(unsigned)nb_att, 256, 0, s>>>(                                \
                reinterpret_cast<const TT*>(table), row_base, n_user, item_idx, hist_idx, batch, S, G,    \
                T, pf, att_b0, w.h, w.hpart);                                                       \
        else if (T <= 64)                                                                              \
            din_att_h_kernel<TT, NI, 1><<<(unsigned)nb_att, 256, 0, s>>>(                              \
                reinterpret_cast<const TT*>(table), row_base, n_user, item_idx, hist_idx, batch, S, G,    \
                T, pf, att_b0, w.h, w.hpart);                                                       \
        else                                                                                           \
            din_att_h_kernel<TT, NI, 2><<<(unsigned)nb_att, 256, 0, s>>>(                              \
                reinterpret_cast<const TT*>(table), row_base, n_user, item_idx, hist_idx, batch, S, G,    \
                T, pf, att_b0, w.h, w.hpart);                                                       \
    } while (0)
    if (tm_path) {
#define NRK_TM_PLAN(NI) din_tm_plan_kernel<NI><<<(unsigned)(n_seg * G_tm), 256, 0, s>>>(hist_idx, mask, batch, S, G_tm, T, w.plan)
        if (n_item == 4) NRK_TM_PLAN(4); else if (n_item == 2) NRK_TM_PLAN(2); else NRK_TM_PLAN(1);
#undef NRK_TM_PLAN
        if (n_item == 4) NRK_ATT_TM(4); else if (n_item == 2) NRK_ATT_TM(2); else NRK_ATT_TM(1);
    } else if (table_dtype == 0) {
        if (n_item == 8) NRK_ATT_H(float, 8); else if (n_item == 4) NRK_ATT_H(float, 4);
        else if (n_item == 2) NRK_ATT_H(float, 2); else NRK_ATT_H(float, 1);
    } else {
        if (n_item == 8) NRK_ATT_H(uint16_t, 8); else if (n_item == 4) NRK_ATT_H(uint16_t, 4);
        else if (n_item == 2) NRK_ATT_H(uint16_t, 2); else NRK_ATT_H(uint16_t, 1);
    }
#undef NRK_ATT_H
    const int ncol_att = T * DIN_H;
    const unsigned gs = (unsigned)n_seg;
    const int bps_att = tm_path ? G_tm : G;
    col_stats_kernel<<<dim3(gs, (ncol_att + 3) / 4), 256, 0, s>>>(w.hpart, bps_att, (int)(n_seg * bps_att),
                                                                   ncol_att, batch, S, w.hstats, w.hinv);
#undef NRK_ATT_TM
    const int64_t nb_m = (batch + 63) / 64;
    const int bps = n_seg == 1 ? (int)nb_m : (int)(S / 64);  // 64-row GEMM blocks per segment
    if (din_fast(T, h1)) {
        // max |W0| -> packed split-fp16 W0; per-segment max |wh| (zeroed here)
        unsigned int* w1max = w.whmax + n_seg;
        if (hipMemsetAsync(w.whmax, 0, (size_t)(2 * n_seg + 2) * 4, s) != hipSuccess) {
            set_error("nrk_din_forward: hipMemsetAsync failed");
            return NRK_EHIP;
        }
        const int64_t nw = (int64_t)h1 * IN;
        din_absmax_kernel<<<(int)std::min<int64_t>((nw + 255) / 256, 128), 256, 0, s>>>(mlp_w0, 0, nw, w1max);
        const int NT = din_mlp1_nt(h1);
        const int64_t npk = (int64_t)(IN / DIN_E) * NT * 64;
        const int gp = (int)std::min<int64_t>((npk + 255) / 256, 2048);
#define NRK_PACK(NTV) din_w1_pack_kernel<NTV><<<gp, 256, 0, s>>>(mlp_w0, h1, IN, w1max, w.w1pack)
        if (NT == 4) NRK_PACK(4); else if (NT == 8) NRK_PACK(8); else if (NT == 13) NRK_PACK(13); else NRK_PACK(16);
#undef NRK_PACK
        // din_wh2: one wave per sample; workgroups per Dice batch, about 8,192 in all
        const int nch = (T * (DIN_H / 4) + 63) / 64;
        const int gw_seg = (int)std::max<int64_t>(1, std::min<int64_t>(S, (8192 + n_seg - 1) / n_seg));
        const unsigned gw2 = (unsigned)(n_seg * gw_seg);
#define NRK_WH2_K(TT, NI, NCH)                                                                               \
    din_wh2_kernel<TT, NI, NCH><<<gw2, 256, din_wh2_lds(T, NI), s>>>(                                        \
        reinterpret_cast<const TT*>(table), row_base, n_user, hist_idx, mask, batch, S, T, gw_seg, w.h, w.hinv, \
        att_w1, att_b1, w.wh, w.whmax)
#define NRK_WH(TT, NI)                                                                                  \
    do {                                                                                                \
        if (nch <= 4) NRK_WH2_K(TT, NI, 4); else if (nch <= 8) NRK_WH2_K(TT, NI, 8); else NRK_WH2_K(TT, NI, 9); \
    } while (0)
        if (table_dtype == 0) {
            if (n_item == 8) NRK_WH(float, 8); else if (n_item == 4) NRK_WH(float, 4);
            else if (n_item == 2) NRK_WH(float, 2); else NRK_WH(float, 1);
        } else {
            if (n_item == 8) NRK_WH(uint16_t, 8); else if (n_item == 4) NRK_WH(uint16_t, 4);
            else if (n_item == 2) NRK_WH(uint16_t, 2); else NRK_WH(uint16_t, 1);
        }
#undef NRK_WH
#undef NRK_WH2_K
        const unsigned gm = (unsigned)((batch + MLP1_ROWS - 1) / MLP1_ROWS);
#define NRK_MLP1(TT, NTV)                                                                                 \
    din_mlp1_kernel<TT, NTV><<<gm, 256, 0, s>>>(reinterpret_cast<const TT*>(table), row_base, n_user,     \
                                                n_item, n_ctx, user_idx, item_idx, ctx_idx, w.wh, w.whmax, \
                                                pf, w1max,                                                 \
                                                reinterpret_cast<const din_u4*>(w.w1pack), mlp_b0, batch,   \
                                                S, h1, w.z1, w.z1part, w.whmax + n_seg + 1)
        if (table_dtype == 0) {
            if (NT == 4) NRK_MLP1(float, 4); else if (NT == 8) NRK_MLP1(float, 8);
            else if (NT == 13) NRK_MLP1(float, 13); else NRK_MLP1(float, 16);
        } else {
            if (NT == 4) NRK_MLP1(uint16_t, 4); else if (NT == 8) NRK_MLP1(uint16_t, 8);
            else if (NT == 13) NRK_MLP1(uint16_t, 13); else NRK_MLP1(uint16_t, 16);
        }
#undef NRK_MLP1
    } else {
    const int go = (int)(batch < 8192 ? batch : 8192);
    if (table_dtype == 0)
        din_att_out_kernel<float><<<go, 256, 0, s>>>(
            reinterpret_cast<const float*>(table), row_base, n_user, n_item, n_ctx, user_idx,
            item_idx, hist_idx, ctx_idx, mask, batch, S, T, w.h, w.hstats, att_w1, att_b1, w.mlp_in);
    else
        din_att_out_kernel<uint16_t><<<go, 256, 0, s>>>(
            reinterpret_cast<const uint16_t*>(table), row_base, n_user, n_item, n_ctx, user_idx,
            item_idx, hist_idx, ctx_idx, mask, batch, S, T, w.h, w.hstats, att_w1, att_b1, w.mlp_in);
    din_gemm_kernel<false><<<dim3((unsigned)nb_m, (h1 + 63) / 64), 512, 0, s>>>(
        w.mlp_in, nullptr, mlp_w0, mlp_b0, batch, S, h1, IN, w.z1, w.z1part);
    }
    col_stats_kernel<<<dim3(gs, (h1 + 3) / 4), 256, 0, s>>>(w.z1part, bps, (int)nb_m, h1, batch, S,
                                                            nullptr, w.z1stats);
    if (din_fast2(T, h1, h2)) {
        unsigned int* z1max = w.whmax + n_seg + 1;
        unsigned int* w2max = z1max + n_seg;
        const int64_t nw = (int64_t)h2 * h1;
        din_absmax_kernel<<<(int)std::min<int64_t>((nw + 255) / 256, 64), 256, 0, s>>>(mlp_w1, 0, nw, w2max);
        const int NT2 = din_mlp2_nt(h2);
        const int KS2 = (h1 + DIN_E - 1) / DIN_E;
        const int gp = (int)std::min<int64_t>(((int64_t)KS2 * NT2 * 64 + 255) / 256, 512);
        const size_t lds = (size_t)KS2 * NT2 * 2048 + (size_t)4 * NT2 * 16 * 16;
        const unsigned g2 = (unsigned)std::min<int64_t>((batch + MLP1_ROWS - 1) / MLP1_ROWS, 512);
#define NRK_MLP2(NTV)                                                                                   \
    do {                                                                                                \
        din_w1_pack_kernel<NTV><<<gp, 256, 0, s>>>(mlp_w1, h2, h1, w2max, w.w2pack);                     \
        (void)hipFuncSetAttribute((const void*)din_mlp2_kernel<NTV>,                                     \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                 \
        din_mlp2_kernel<NTV><<<g2, 256, lds, s>>>(w.z1, w.z1stats, z1max, w2max,                         \
                                                  reinterpret_cast<const din_u4*>(w.w2pack), mlp_b1,     \
                                                  batch, S, h1, h2, w.z2, w.z2part);                     \
    } while (0)
        if (NT2 == 2) NRK_MLP2(2); else if (NT2 == 4) NRK_MLP2(4); else if (NT2 == 5) NRK_MLP2(5); else NRK_MLP2(8);
#undef NRK_MLP2
    } else {
        din_gemm_kernel<true><<<dim3((unsigned)nb_m, (h2 + 63) / 64), 512, 0, s>>>(
            w.z1, w.z1stats, mlp_w1, mlp_b1, batch, S, h2, h1, w.z2, w.z2part);
    }
    col_stats_kernel<<<dim3(gs, (h2 + 3) / 4), 256, 0, s>>>(w.z2part, bps, (int)nb_m, h2, batch, S,
                                                            nullptr, w.z2stats);
    din_head_kernel<<<(unsigned)std::min<int64_t>((batch + 15) / 16, 8192), 256, 0, s>>>(
        w.z2, w.z2stats, batch, S, h2, mlp_w2, mlp_b2, out_probs, out_logits);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_din_forward(const void* table, int table_dtype, const int64_t* row_base, int n_user,
                    int n_item, int n_ctx, const int32_t* user_idx, const int32_t* item_idx,
                    const int32_t* hist_idx, const int32_t* ctx_idx, const float* mask,
                    int64_t batch, int seq_len, const void* prep, const float* att_b0,
                    const float* att_w1, const float* att_b1, const float* mlp_w0,
                    const float* mlp_b0, int h1, const float* mlp_w1, const float* mlp_b1,
                    int h2, const float* mlp_w2, const float* mlp_b2, float* out_probs,
                    float* out_logits, void* workspace, size_t workspace_bytes,
                    nrk_stream_t stream) {
    if (batch < 2) {
        clear_error();
        NRK_REQUIRE(batch >= 2, "batch must be >= 2 (Dice uses the batch std; B = 1 is NaN in the reference)");
    }
    return nrk_din_forward_segments(table, table_dtype, row_base, n_user, n_item, n_ctx, user_idx,
                                    item_idx, hist_idx, ctx_idx, mask, batch, batch, seq_len, prep,
                                    att_b0, att_w1, att_b1, mlp_w0, mlp_b0, h1, mlp_w1, mlp_b1, h2,
                                    mlp_w2, mlp_b2, out_probs, out_logits, workspace,
                                    workspace_bytes, stream);
}

}  // extern "C"
