// din.hip -- DIN attention-over-history scorer (DINModel.forward, eval) on gfx950.
//
// Reference: src/rank/DIN.py:29-286 (Dice :29-44, ActivationUnit :47-130,
// DINModel.forward :214-286) as DINRanker.predict drives it (:1219-1283).
// All arithmetic is fp32 (parity 1e-5); the embedding tables may be stored as
// bf16 (storage only) or fp32.
//
// Dice normalises with the BATCH mean and unbiased std of every column
// (DIN.py:39-44), so each Dice splits the forward into phases with a
// batch-wide reduction in between:
//   1. din_att_h      h[b,t,:] = (Wk - Wd) k_t + (Wq + Wd) q + Wp (q .* k_t) + b0
//                     (= Linear(512->36) on [k, q, q-k, q.*k], DIN.py:105-114,
//                     with the batch-invariant parts folded by nrk_din_prepare);
//                     per-block fp64 column sums of h and h^2.
//   2. col_stats      mean / unbiased std per (t, j) (deterministic, fixed order).
//   3. din_att_out    Dice -> Linear(36->1) -> * mask (no softmax, :117-124),
//                     weighted history sum (:276), assemble the MLP input
//                     [user, ctx, cand, wh] (:279-281).
//   4. din_gemm       Linear(928->h1) (+ column sums), 5. col_stats,
//   6. din_gemm       Dice-on-load -> Linear(h1->h2) (+ column sums), 7. col_stats,
//   8. din_head       Dice -> Linear(h2->1) -> sigmoid (:282-284).
#include "nrk_common.h"

namespace nrk {

constexpr int DIN_E = 32;   // embedding dim (din_embedding_dim, config.py:115)
constexpr int DIN_H = 36;   // ActivationUnit hidden (default [36], DIN.py:188)

template <typename TT>
__device__ __forceinline__ float tload(const TT* p);
template <>
__device__ __forceinline__ float tload<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float tload<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }

// Dice (DIN.py:39-44), fp32 in the reference's operation order.
__device__ __forceinline__ float dice(float x, float mean, float std) {
    const float xn = (x - mean) / (std + 1e-8f);
    const float p = 1.0f / (1.0f + expf(-xn));
    return p * x + ((1.0f - p) * 0.01f) * x;
}

// ------------------------------------------------------------- 1. att h --
// One workgroup processes SPB samples in turn.  LDS: M_b [36][ID], keys
// [T][ID], query [ID], c [36], and the block's fp64 column sums [T*36][2].
template <typename TT, int ID>
__global__ __launch_bounds__(256) void din_att_h_kernel(
    const TT* __restrict__ table, const int64_t* __restrict__ row_base, int n_user, int n_item,
    const int32_t* __restrict__ item_idx, const int32_t* __restrict__ hist_idx, int64_t B, int T,
    const float* __restrict__ prep, const float* __restrict__ att_b0, int spb,
    float* __restrict__ h_out, double* __restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* M = lds;                       // [36][ID]
    float* Kt = M + DIN_H * ID;           // [T][ID]
    float* q = Kt + (size_t)T * ID;       // [ID]
    float* c = q + ID;                    // [36] (+ pad)
    double* acc = reinterpret_cast<double*>(c + 48);  // [T*36][2]
    const float* A = prep;                // (Wk - Wd)   [36][ID]
    const float* Bq = prep + DIN_H * ID;  // (Wq + Wd)   [36][ID]
    const float* P = prep + 2 * DIN_H * ID;  // Wp       [36][ID]
    const int tid = threadIdx.x;
    const int ncol = T * DIN_H;
    for (int i = tid; i < 2 * ncol; i += 256) acc[i] = 0.0;
    const int64_t b0 = (int64_t)blockIdx.x * spb;
    const int64_t b1 = b0 + spb < B ? b0 + spb : B;
    for (int64_t b = b0; b < b1; ++b) {
        __syncthreads();
        // gather the candidate (query) and the history keys
        for (int i = tid; i < ID; i += 256) {
            const int f = i / DIN_E, e = i % DIN_E;
            const int64_t r = row_base[n_user + f] + item_idx[b * n_item + f];
            q[i] = tload(table + r * DIN_E + e);
        }
        for (int i = tid; i < T * ID; i += 256) {
            const int t = i / ID, f = (i % ID) / DIN_E, e = i % DIN_E;
            const int64_t r = row_base[n_user + f] + hist_idx[(b * T + t) * n_item + f];
            Kt[i] = tload(table + r * DIN_E + e);
        }
        __syncthreads();
        for (int i = tid; i < DIN_H * ID; i += 256) M[i] = A[i] + P[i] * q[i % ID];
        if (tid < DIN_H) {
            float s = att_b0[tid];
            for (int i = 0; i < ID; ++i) s += Bq[tid * ID + i] * q[i];
            c[tid] = s;
        }
        __syncthreads();
        // h[t][j] = sum_i Kt[t][i] M[j][i] + c[j]; thread tile 2 t x 4 j
        const int ntj = ((T + 1) / 2) * (DIN_H / 4);
        for (int w = tid; w < ntj; w += 256) {
            const int t0 = (w / (DIN_H / 4)) * 2, j0 = (w % (DIN_H / 4)) * 4;
            const bool t1ok = t0 + 1 < T;
            float s[2][4] = {};
            const float4* k0 = reinterpret_cast<const float4*>(Kt + t0 * ID);
            const float4* k1 = reinterpret_cast<const float4*>(Kt + (t1ok ? t0 + 1 : t0) * ID);
#pragma unroll 4
            for (int i4 = 0; i4 < ID / 4; ++i4) {
                const float4 a0 = k0[i4], a1 = k1[i4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const float4 m = reinterpret_cast<const float4*>(M + (j0 + jj) * ID)[i4];
                    s[0][jj] += a0.x * m.x + a0.y * m.y + a0.z * m.z + a0.w * m.w;
                    s[1][jj] += a1.x * m.x + a1.y * m.y + a1.z * m.z + a1.w * m.w;
                }
            }
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) {
                if (tt == 1 && !t1ok) break;
                const int t = t0 + tt;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const float v = s[tt][jj] + c[j0 + jj];
                    h_out[(b * T + t) * DIN_H + j0 + jj] = v;
                    const int col = t * DIN_H + j0 + jj;
                    acc[2 * col] += (double)v;
                    acc[2 * col + 1] += (double)v * (double)v;
                }
            }
        }
    }
    __syncthreads();
    double* dst = partial + (size_t)blockIdx.x * 2 * ncol;
    for (int i = tid; i < 2 * ncol; i += 256) dst[i] = acc[i];
}

// ---------------------------------------------------------- 2. col stats --
// mean and unbiased std (torch.std default) of each column over the batch,
// from per-block fp64 (sum, sumsq) partials.  One wave per column: lane l
// sums partials l, l+64, ... in order, then a fixed butterfly -- the same
// order on every run (bitwise reproducible).
__global__ __launch_bounds__(256) void col_stats_kernel(const double* __restrict__ partial, int nblk,
                                                        int ncol, int64_t B, float2* __restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= ncol) return;
    double s = 0.0, ss = 0.0;
    for (int k = lane; k < nblk; k += WAVE) {
        const double2 v = *reinterpret_cast<const double2*>(partial + ((size_t)k * ncol + c) * 2);
        s += v.x;
        ss += v.y;
    }
    s = wave_sum_f64(s);
    ss = wave_sum_f64(ss);
    if (lane == 0) {
        const double mean = s / (double)B;
        double var = (ss - s * mean) / (double)(B - 1);
        if (var < 0.0) var = 0.0;
        stats[c] = make_float2((float)mean, (float)sqrt(var));
    }
}

// --------------------------------------------------------- 3. att out --
// One wave per sample: lane t < T computes the attention weight of history
// position t; lanes then split the item dim for the weighted sum.  Writes the
// MLP input row [user, ctx, cand, wh].
template <typename TT>
__global__ __launch_bounds__(256) void din_att_out_kernel(
    const TT* __restrict__ table, const int64_t* __restrict__ row_base, int n_user, int n_item,
    int n_ctx, const int32_t* __restrict__ user_idx, const int32_t* __restrict__ item_idx,
    const int32_t* __restrict__ hist_idx, const int32_t* __restrict__ ctx_idx,
    const float* __restrict__ mask, int64_t B, int T, const float* __restrict__ h,
    const float2* __restrict__ hstats, const float* __restrict__ att_w1,
    const float* __restrict__ att_b1, float* __restrict__ mlp_in) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const int ID = n_item * DIN_E;
    const int IN = (n_user + n_ctx + 2 * n_item) * DIN_E;
    float* row = mlp_in + b * IN;
    // attention weight of history slot t (lanes t and t + 64 for T <= 128)
    float w0 = 0.0f, w1 = 0.0f;
    for (int half = 0; half < 2; ++half) {
        const int t = lane + 64 * half;
        if (t < T) {
            const float* hr = h + (b * T + t) * DIN_H;
            float s = 0.0f;
            for (int j = 0; j < DIN_H; ++j) {
                const float2 st = hstats[t * DIN_H + j];
                s += att_w1[j] * dice(hr[j], st.x, st.y);
            }
            s = (s + att_b1[0]) * mask[b * T + t];
            if (half == 0) w0 = s; else w1 = s;
        }
    }
    // weighted history sum: lane owns dims lane, lane + 64 (ID <= 128 per pass)
    for (int i = lane; i < ID; i += 64) {
        const int f = i / DIN_E, e = i % DIN_E;
        const int64_t base = row_base[n_user + f];
        float s = 0.0f;
        for (int t = 0; t < T; ++t) {
            const float wt = __shfl(t < 64 ? w0 : w1, t & 63, 64);
            const int64_t r = base + hist_idx[(b * T + t) * n_item + f];
            s += wt * tload(table + r * DIN_E + e);
        }
        row[(n_user + n_ctx + n_item) * DIN_E + i] = s;
        // candidate embedding
        row[(n_user + n_ctx) * DIN_E + i] = tload(table + (row_base[n_user + f] + item_idx[b * n_item + f]) * DIN_E + e);
    }
    for (int i = lane; i < n_user * DIN_E; i += 64) {
        const int f = i / DIN_E, e = i % DIN_E;
        row[i] = tload(table + (row_base[f] + user_idx[b * n_user + f]) * DIN_E + e);
    }
    for (int i = lane; i < n_ctx * DIN_E; i += 64) {
        const int f = i / DIN_E, e = i % DIN_E;
        row[n_user * DIN_E + i] = tload(table + (row_base[n_user + n_item + f] + ctx_idx[b * n_ctx + f]) * DIN_E + e);
    }
}

// ---------------------------------------------------------- 4/6. gemm --
// C[M][N] = f(A)[M][K] W[N][K]^T + bias, f = Dice with per-column stats of A
// (or identity).  64x64 output tile per 256-thread block, 4x4 per thread,
// K staged through LDS 32 at a time.  Writes per-row-block fp64 column sums
// (sum, sumsq) of C for the next Dice.
template <bool DICE_A>
__global__ __launch_bounds__(256) void din_gemm_kernel(
    const float* __restrict__ A, const float2* __restrict__ astats, const float* __restrict__ W,
    const float* __restrict__ bias, int64_t M, int N, int K, float* __restrict__ C,
    double* __restrict__ partial) {
    __shared__ float As[32][64 + 4];
    __shared__ float Ws[32][64 + 4];
    __shared__ double cs[2][16][64];
    const int tid = threadIdx.x;
    const int tx = tid & 15, ty = tid >> 4;  // 16 x 16 threads
    const int64_t m0 = (int64_t)blockIdx.x * 64;
    const int n0 = blockIdx.y * 64;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += 32) {
        // load A tile [64 rows][32 k] transposed into As[k][m]
        for (int i = tid; i < 64 * 32; i += 256) {
            const int r = i / 32, kk = i % 32;
            const int64_t m = m0 + r;
            const int k = k0 + kk;
            float v = 0.0f;
            if (m < M && k < K) {
                v = A[m * K + k];
                if (DICE_A) {
                    const float2 st = astats[k];
                    v = dice(v, st.x, st.y);
                }
            }
            As[kk][r] = v;
        }
        for (int i = tid; i < 64 * 32; i += 256) {
            const int r = i / 32, kk = i % 32;
            const int n = n0 + r;
            const int k = k0 + kk;
            Ws[kk][r] = (n < N && k < K) ? W[(int64_t)n * K + k] : 0.0f;
        }
        __syncthreads();
#pragma unroll 8
        for (int kk = 0; kk < 32; ++kk) {
            float a[4], w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a[i] = As[kk][ty * 4 + i];
                w[i] = Ws[kk][tx * 4 + i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * w[j];
        }
        __syncthreads();
    }
    double csum[4] = {}, csq[4] = {};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t m = m0 + ty * 4 + i;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx * 4 + j;
            if (m < M && n < N) {
                const float v = acc[i][j] + bias[n];
                C[m * N + n] = v;
                csum[j] += (double)v;
                csq[j] += (double)v * (double)v;
            }
        }
    }
    // column sums over the block's 64 rows, in a fixed order
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        cs[0][ty][tx * 4 + j] = csum[j];
        cs[1][ty][tx * 4 + j] = csq[j];
    }
    __syncthreads();
    if (tid < 64) {
        const int n = n0 + tid;
        double s = 0.0, ss = 0.0;
        for (int r = 0; r < 16; ++r) {
            s += cs[0][r][tid];
            ss += cs[1][r][tid];
        }
        if (n < N) {
            partial[((size_t)blockIdx.x * N + n) * 2] = s;
            partial[((size_t)blockIdx.x * N + n) * 2 + 1] = ss;
        }
    }
}

// ------------------------------------------------------------ 8. head --
__global__ void din_head_kernel(const float* __restrict__ Z, const float2* __restrict__ zstats,
                                int64_t B, int H, const float* __restrict__ w,
                                const float* __restrict__ bias, float* __restrict__ probs,
                                float* __restrict__ logits) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    float s = 0.0f;
    for (int j = lane; j < H; j += 64) {
        const float2 st = zstats[j];
        s += w[j] * dice(Z[b * H + j], st.x, st.y);
    }
    s = wave_sum_f32(s);
    if (lane == 0) {
        const float lg = s + bias[0];
        if (logits) logits[b] = lg;
        probs[b] = 1.0f / (1.0f + expf(-lg));
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

// ------------------------------------------------------------- workspace --
constexpr int DIN_SPB = 16;  // samples per block in din_att_h

struct DinWs {
    float* h;
    double* hpart;
    float2* hstats;
    float* mlp_in;
    float* z1;
    double* z1part;
    float2* z1stats;
    float* z2;
    double* z2part;
    float2* z2stats;
    size_t bytes;
};

static inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

static DinWs din_ws_layout(void* base, int64_t B, int T, int n_user, int n_item, int n_ctx, int h1,
                           int h2) {
    DinWs w;
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    size_t o = 0;
    const int64_t nb_att = (B + DIN_SPB - 1) / DIN_SPB;
    const int64_t nb_m = (B + 63) / 64;
    const int IN = (n_user + n_ctx + 2 * n_item) * DIN_E;
    auto take = [&](size_t bytes) { uint8_t* r = p + o; o += al(bytes); return r; };
    w.h = (float*)take((size_t)B * T * DIN_H * 4);
    w.hpart = (double*)take((size_t)nb_att * T * DIN_H * 16);
    w.hstats = (float2*)take((size_t)T * DIN_H * 8);
    w.mlp_in = (float*)take((size_t)B * IN * 4);
    w.z1 = (float*)take((size_t)B * h1 * 4);
    w.z1part = (double*)take((size_t)nb_m * h1 * 16);
    w.z1stats = (float2*)take((size_t)h1 * 8);
    w.z2 = (float*)take((size_t)B * h2 * 4);
    w.z2part = (double*)take((size_t)nb_m * h2 * 16);
    w.z2stats = (float2*)take((size_t)h2 * 8);
    w.bytes = o;
    return w;
}

}  // namespace nrk

using namespace nrk;

extern "C" {

size_t nrk_din_prep_bytes(int n_item) {
    if (n_item <= 0) return 0;
    return (size_t)3 * DIN_H * n_item * DIN_E * sizeof(float);
}

int nrk_din_prepare(const float* att_w0, int n_item, void* prep, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(att_w0 && prep, "null pointer");
    NRK_REQUIRE(n_item >= 1 && n_item <= 8, "n_item must be in [1, 8]");
    const int ID = n_item * DIN_E;
    din_prepare_kernel<<<64, 256, 0, as_stream(stream)>>>(att_w0, ID, reinterpret_cast<float*>(prep));
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_din_workspace_bytes(int64_t batch, int seq_len, int n_user, int n_item, int n_ctx,
                               int h1, int h2) {
    if (batch < 0 || seq_len < 1) return 0;
    return din_ws_layout(nullptr, batch, seq_len, n_user, n_item, n_ctx, h1, h2).bytes;
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
    clear_error();
    NRK_REQUIRE(table_dtype == 0 || table_dtype == 1, "table_dtype must be 0 (f32) or 1 (bf16)");
    NRK_REQUIRE(batch >= 2, "batch must be >= 2 (Dice uses the batch std; B = 1 is NaN in the reference)");
    NRK_REQUIRE(seq_len >= 1 && seq_len <= 128, "seq_len must be in [1, 128]");
    NRK_REQUIRE(n_user >= 1 && n_ctx >= 0 && n_item >= 1, "bad feature counts");
    if (n_item != 4 && n_item != 2 && n_item != 1) NRK_UNSUPPORTED("n_item must be 1, 2 or 4");
    NRK_REQUIRE(h1 >= 1 && h1 <= 1024 && h2 >= 1 && h2 <= 1024, "hidden sizes out of range");
    NRK_REQUIRE(table && row_base && user_idx && item_idx && hist_idx && mask && prep && att_b0 &&
                    att_w1 && att_b1 && mlp_w0 && mlp_b0 && mlp_w1 && mlp_b1 && mlp_w2 && mlp_b2 &&
                    out_probs && workspace,
                "null pointer");
    NRK_REQUIRE(n_ctx == 0 || ctx_idx, "ctx_idx null");
    const DinWs w = din_ws_layout(workspace, batch, seq_len, n_user, n_item, n_ctx, h1, h2);
    NRK_REQUIRE(workspace_bytes >= w.bytes, "workspace too small");
    hipStream_t s = as_stream(stream);
    const int T = seq_len;
    const int ID = n_item * DIN_E;
    const int IN = (n_user + n_ctx + 2 * n_item) * DIN_E;
    const int nb_att = (int)((batch + DIN_SPB - 1) / DIN_SPB);
    const size_t lds_att = sizeof(float) * ((size_t)DIN_H * ID + (size_t)T * ID + ID + 48) +
                           sizeof(double) * 2 * (size_t)T * DIN_H;
    const float* pf = reinterpret_cast<const float*>(prep);
#define NRK_ATT_H(TT, IDV)                                                                          \
    do {                                                                                            \
        (void)hipFuncSetAttribute((const void*)din_att_h_kernel<TT, IDV>,                           \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_att);        \
        din_att_h_kernel<TT, IDV><<<nb_att, 256, lds_att, s>>>(                                     \
            reinterpret_cast<const TT*>(table), row_base, n_user, n_item, item_idx, hist_idx,       \
            batch, T, pf, att_b0, DIN_SPB, w.h, w.hpart);                                           \
    } while (0)
    if (table_dtype == 0) {
        if (ID == 128) NRK_ATT_H(float, 128); else if (ID == 64) NRK_ATT_H(float, 64); else NRK_ATT_H(float, 32);
    } else {
        if (ID == 128) NRK_ATT_H(uint16_t, 128); else if (ID == 64) NRK_ATT_H(uint16_t, 64); else NRK_ATT_H(uint16_t, 32);
    }
#undef NRK_ATT_H
    const int ncol_att = T * DIN_H;
    col_stats_kernel<<<(ncol_att + 3) / 4, 256, 0, s>>>(w.hpart, nb_att, ncol_att, batch, w.hstats);
    const int gb = (int)((batch + 3) / 4);
    if (table_dtype == 0)
        din_att_out_kernel<float><<<gb, 256, 0, s>>>(
            reinterpret_cast<const float*>(table), row_base, n_user, n_item, n_ctx, user_idx,
            item_idx, hist_idx, ctx_idx, mask, batch, T, w.h, w.hstats, att_w1, att_b1, w.mlp_in);
    else
        din_att_out_kernel<uint16_t><<<gb, 256, 0, s>>>(
            reinterpret_cast<const uint16_t*>(table), row_base, n_user, n_item, n_ctx, user_idx,
            item_idx, hist_idx, ctx_idx, mask, batch, T, w.h, w.hstats, att_w1, att_b1, w.mlp_in);
    const int nb_m = (int)((batch + 63) / 64);
    din_gemm_kernel<false><<<dim3(nb_m, (h1 + 63) / 64), 256, 0, s>>>(
        w.mlp_in, nullptr, mlp_w0, mlp_b0, batch, h1, IN, w.z1, w.z1part);
    col_stats_kernel<<<(h1 + 3) / 4, 256, 0, s>>>(w.z1part, nb_m, h1, batch, w.z1stats);
    din_gemm_kernel<true><<<dim3(nb_m, (h2 + 63) / 64), 256, 0, s>>>(
        w.z1, w.z1stats, mlp_w1, mlp_b1, batch, h2, h1, w.z2, w.z2part);
    col_stats_kernel<<<(h2 + 3) / 4, 256, 0, s>>>(w.z2part, nb_m, h2, batch, w.z2stats);
    din_head_kernel<<<gb, 256, 0, s>>>(w.z2, w.z2stats, batch, h2, mlp_w2, mlp_b2, out_probs,
                                       out_logits);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
