// tower.hip -- YouTubeDNN two-tower forward (eval) on gfx950.
//
// User tower: YoutubeDNN.forward (src/recall/youtubednn_recaller.py:129-178)
// as _extract_embeddings drives it (:425-470), fused with the numpy
// re-normalisation of :467-470.  Item tower: get_item_embedding (:184-188)
// fused with :485-489.  Memory-bound gathers (1 + T rows of D fp32 per user)
// feeding a 2-layer MLP that fits in LDS; one wave per user.
#include "nrk_common.h"

namespace nrk {

#ifndef NRK_TT_CH
#define NRK_TT_CH 8
#endif

template <int D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void tt_user_kernel(
    const float* __restrict__ user_table, const float* __restrict__ item_table,
    const int32_t* __restrict__ uid, const int32_t* __restrict__ hist,
    const int32_t* __restrict__ hist_len, int64_t n, int T, const float* __restrict__ w0,
    const float* __restrict__ b0, int h0, const float* __restrict__ w1,
    const float* __restrict__ b1, int h1, float* __restrict__ out) {
    // the 4-wide reads of sx / the weight rows below stay 16-B aligned and
    // inside their own row only while 2D is a multiple of 4 (the host allows
    // D = 16, 32, 64 only)
    static_assert(D % 2 == 0 && D >= 16 && D <= 64 && (D & (D - 1)) == 0, "tt_user_kernel: D in {16, 32, 64}");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    // weight rows padded to a multiple of 4 floats + 4: lane o reads row o, so
    // an unpadded power-of-two row stride would put all 64 lanes on one LDS
    // bank; with the padding the rows are 16-B aligned for the 4-wide reads
    // and lane o's row starts 4 banks after lane o - 1's
    const int S0 = 2 * D + 4, h0p = (h0 + 3) & ~3, S1 = h0p + 4, h1p = (h1 + 3) & ~3;
    float* sw0 = lds;               // [h0][S0]
    float* sb0 = sw0 + h0 * S0;     // [h0] (h0p)
    float* sw1 = sb0 + h0p;         // [h1][S1]
    float* sb1 = sw1 + h1 * S1;     // [h1] (h1p)
    // per-wave broadcast rows for the two matvecs: [x (2D) | y0 (h0)]; every
    // lane reads the same word (LDS broadcast) instead of a v_readlane per term
    float* sx = sb1 + h1p + (threadIdx.x >> 6) * (2 * D + 128);
    for (int i = threadIdx.x; i < h0 * 2 * D; i += blockDim.x) sw0[(i / (2 * D)) * S0 + i % (2 * D)] = w0[i];
    for (int i = threadIdx.x; i < h0; i += blockDim.x) sb0[i] = b0[i];
    for (int i = threadIdx.x; i < h1 * h0; i += blockDim.x) sw1[(i / h0) * S1 + i % h0] = w1[i];
    for (int i = threadIdx.x; i < h1; i += blockDim.x) sb1[i] = b1[i];
    __syncthreads();  // the only block barrier: the user loop below is per wave

    constexpr int P = WAVE / D;  // history phases per lane group
    // history rows in flight per lane (a config-2 user, T = 30 at D = 32, has
    // up to 15 per lane: two rounds).  All 16 at once measured slower in the
    // bench (tower 0.330-0.334 vs 0.294-0.295 ms, one box, two pairs): a
    // round issues CH unconditional loads per lane, and most histories are
    // short (dev A/B: -DNRK_TT_CH=16)
    constexpr int CH = NRK_TT_CH;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int d = lane % D, ph = lane / D;
    const int64_t wstride = (int64_t)gridDim.x * 4;
    // software pipeline over this wave's users: the next user's length, id and
    // history indices (lane t holds index t; T <= 64) are loaded while this
    // user's rows are summed, and the rows themselves are issued CH at a time
    // (unconditional loads: slots past the length read row 0 and are not
    // added), so no load waits on another in flight.
    auto meta = [&](int64_t uu, int& len, int32_t& uidv, int32_t& hv) {
        const bool ok = uu < n;
        len = ok ? hist_len[uu] : 0;
        uidv = ok ? uid[uu] : 0;
        hv = ok && lane < T ? hist[uu * T + lane] : 0;
    };
    int64_t u = (int64_t)blockIdx.x * 4 + wave;
    int len, uidv;
    int32_t hv;
    meta(u, len, uidv, hv);
    // user u's output row is stored during user u + wstride, after that
    // user's first gathers are issued: a store counts in vmcnt, so one issued
    // at the end of a user made the next user's first wait a full store round
    // trip; issued behind the gathers its acknowledgement overlaps them
    float pout = 0.0f;
    int64_t pu = -1;
    for (; u < n; u += wstride) {
        int nlen, nuid;
        int32_t nhv;
        meta(u + wstride, nlen, nuid, nhv);
        const float xu = user_table[(int64_t)uidv * D + d];
        float sum = 0.0f;
        const int nit = (len + P - 1) / P;  // wave-uniform
        for (int i0 = 0; i0 < nit; i0 += CH) {
            float v[CH];
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                const int t = ph + P * (i0 + e);
                const int32_t r = __shfl(hv, t < T ? t : 0, WAVE);
                v[e] = item_table[(int64_t)(t < len ? r : 0) * D + d];
            }
            if (i0 == 0 && pu >= 0) {
                if (lane < h1) out[pu * h1 + lane] = pout;
                pu = -1;
            }
#pragma unroll
            for (int e = 0; e < CH; ++e)
                if (ph + P * (i0 + e) < len) sum += v[e];  // t ascending, as before
        }
#pragma unroll
        for (int off = D; off < WAVE; off <<= 1) sum += __shfl_xor(sum, off, WAVE);
        // lane q < D holds x[q] = E_u[uid][q] and x[D + q] = mean[q]
        const float xm = sum / ((float)len + 1e-8f);
        // layer 0: lane o (and o + 64) owns output o; same fma order as a
        // q-ascending dot (inputs broadcast from LDS)
        if (lane < D) {
            sx[lane] = xu;
            sx[D + lane] = xm;
        }
        __builtin_amdgcn_wave_barrier();
        float y0 = 0.0f, y1 = 0.0f;
        {
            float z0 = lane < h0 ? sb0[lane] : 0.0f;
            float z1 = lane + WAVE < h0 ? sb0[lane + WAVE] : 0.0f;
            const float* wr0 = sw0 + (lane < h0 ? lane : 0) * S0;
            const float* wr1 = sw0 + (lane + WAVE < h0 ? lane + WAVE : 0) * S0;
            // 4 inputs (broadcast) and 4 weights per LDS read; the fma
            // chain still runs q = 0, 1, 2, ... in order.  Outputs 64 ..
            // only when h0 > 64 (round 6: the second chain ran, on row 0,
            // for every h0)
            if (h0 > WAVE) {
#pragma unroll 2
                for (int q = 0; q < 2 * D; q += 4) {
                    const float4 xq = *reinterpret_cast<const float4*>(sx + q);
                    const float4 a = *reinterpret_cast<const float4*>(wr0 + q);
                    const float4 b = *reinterpret_cast<const float4*>(wr1 + q);
                    z0 += a.x * xq.x;
                    z0 += a.y * xq.y;
                    z0 += a.z * xq.z;
                    z0 += a.w * xq.w;
                    z1 += b.x * xq.x;
                    z1 += b.y * xq.y;
                    z1 += b.z * xq.z;
                    z1 += b.w * xq.w;
                }
            } else {
#pragma unroll 2
                for (int q = 0; q < 2 * D; q += 4) {
                    const float4 xq = *reinterpret_cast<const float4*>(sx + q);
                    const float4 a = *reinterpret_cast<const float4*>(wr0 + q);
                    z0 += a.x * xq.x;
                    z0 += a.y * xq.y;
                    z0 += a.z * xq.z;
                    z0 += a.w * xq.w;
                }
            }
            y0 = fmaxf(z0, 0.0f);
            y1 = fmaxf(z1, 0.0f);
        }
        // layer 1: lane o < h1 owns output o
        float* sy = sx + 2 * D;
        if (lane < h0) sy[lane] = y0;
        if (lane + WAVE < h0) sy[lane + WAVE] = y1;
        __builtin_amdgcn_wave_barrier();
        float v = 0.0f;
        {
            float z = lane < h1 ? sb1[lane] : 0.0f;
            const float* wr = sw1 + (lane < h1 ? lane : 0) * S1;
            int q = 0;
            for (; q + 4 <= h0; q += 4) {
                const float4 yq = *reinterpret_cast<const float4*>(sy + q);
                const float4 a = *reinterpret_cast<const float4*>(wr + q);
                z += a.x * yq.x;
                z += a.y * yq.y;
                z += a.z * yq.z;
                z += a.w * yq.w;
            }
            for (; q < h0; ++q) z += wr[q] * sy[q];
            v = lane < h1 ? fmaxf(z, 0.0f) : 0.0f;
        }
        __builtin_amdgcn_wave_barrier();  // sx / sy are rewritten for the next user
        const float nn = sqrtf(wave_sum_f32(v * v));
        v = v / fmaxf(nn, 1e-12f);
        float n2 = sqrtf(wave_sum_f32(v * v));
        if (n2 == 0.0f) n2 = 1.0f;
        if (pu >= 0 && lane < h1) out[pu * h1 + lane] = pout;  // no gathers this user (len == 0)
        pout = v / n2;
        pu = u;
        len = nlen;
        uidv = nuid;
        hv = nhv;
    }
    if (pu >= 0 && lane < h1) out[pu * h1 + lane] = pout;
}

// Any depth (youtubednn_hidden_units is a list, youtubednn_recaller.py:105-112):
// user_tower = [Linear(in_l, w_l), ReLU, Dropout] per layer.  Same gather
// and re-normalisation as tt_user_kernel; the layers run from one packed
// weight buffer (per layer W_l [w_l, in_l] row-major, then b_l [w_l]) read
// through the caches, lane o owning outputs o, o + 64, ..., inputs broadcast
// from a per-wave LDS row; each output is the same q-ascending fma chain as
// the two-layer kernel.
constexpr int TT_MAXL = 8, TT_MAXW = 256;
struct TtLayers {
    int n;
    int w[TT_MAXL];
};

template <int D>
__global__ __launch_bounds__(256) void tt_user_mlp_kernel(
    const float* __restrict__ user_table, const float* __restrict__ item_table,
    const int32_t* __restrict__ uid, const int32_t* __restrict__ hist,
    const int32_t* __restrict__ hist_len, int64_t n, int T, const float* __restrict__ wts, TtLayers ly,
    float* __restrict__ out) {
    __shared__ float sx[4][2][TT_MAXW > 2 * D ? TT_MAXW : 2 * D];
    constexpr int P = WAVE / D;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int d = lane % D, ph = lane / D;
    const int64_t wstride = (int64_t)gridDim.x * 4;
    for (int64_t u = (int64_t)blockIdx.x * 4 + wave; u < n; u += wstride) {
        const int len = hist_len[u];
        const int32_t hv = lane < T ? hist[u * T + lane] : 0;
        const float xu = user_table[(int64_t)uid[u] * D + d];
        float sum = 0.0f;
        const int nit = (len + P - 1) / P;
        for (int i = 0; i < nit; ++i) {
            const int t = ph + P * i;
            const int32_t r = __shfl(hv, t < T ? t : 0, WAVE);
            const float v = item_table[(int64_t)(t < len ? r : 0) * D + d];
            if (t < len) sum += v;  // t ascending
        }
#pragma unroll
        for (int off = D; off < WAVE; off <<= 1) sum += __shfl_xor(sum, off, WAVE);
        const float xm = sum / ((float)len + 1e-8f);
        if (lane < D) {
            sx[wave][0][lane] = xu;
            sx[wave][0][D + lane] = xm;
        }
        wave_sync_lds();
        int in = 2 * D, cur = 0;
        const float* wl = wts;
        for (int l = 0; l < ly.n; ++l) {
            const int wo = ly.w[l];
            const float* bl = wl + (size_t)wo * in;
            for (int o = lane; o < wo; o += WAVE) {
                float z = bl[o];
                const float* wr = wl + (size_t)o * in;
                for (int qq = 0; qq < in; ++qq) z += wr[qq] * sx[wave][cur][qq];
                sx[wave][cur ^ 1][o] = fmaxf(z, 0.0f);
            }
            wave_sync_lds();
            wl = bl + wo;
            in = wo;
            cur ^= 1;
        }
        const float v = lane < D ? sx[wave][cur][lane] : 0.0f;
        const float nn = sqrtf(wave_sum_f32(v * v));
        const float v1 = v / fmaxf(nn, 1e-12f);
        float n2 = sqrtf(wave_sum_f32(v1 * v1));
        if (n2 == 0.0f) n2 = 1.0f;
        if (lane < D) out[u * D + lane] = v1 / n2;
        wave_sync_lds();  // sx is rewritten for the next user
    }
}

template <int D>
__global__ __launch_bounds__(256) void tt_item_kernel(const float* __restrict__ table,
                                                      const int32_t* __restrict__ ids, int64_t n,
                                                      float* __restrict__ out) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const float* src = table + (int64_t)ids[r] * D;
        float v[D];
        float s = 0.0f;
#pragma unroll
        for (int q = 0; q < D; ++q) {
            v[q] = src[q];
            s += v[q] * v[q];
        }
        const float inv = fmaxf(sqrtf(s), 1e-12f);
        float s2 = 0.0f;
#pragma unroll
        for (int q = 0; q < D; ++q) {
            v[q] = v[q] / inv;
            s2 += v[q] * v[q];
        }
        const float n2 = sqrtf(s2);
#pragma unroll
        for (int q = 0; q < D; ++q) out[r * D + q] = v[q] / n2;
    }
}

}  // namespace nrk

using namespace nrk;

// workgroups of 256 threads resident at once on the device (occupancy API x
// CUs), at most one per 4 users; dev A/B: -DNRK_TT_GRID=2048 (the old fixed grid)
#ifndef NRK_TT_GRID
#define NRK_TT_GRID 0
#endif
static int tt_grid(const void* fn, size_t lds, int64_t n) {
    int per_cu = 0, dev = 0, cus = 256;
    if (NRK_TT_GRID > 0) return (int)std::min<int64_t>((n + 3) / 4, NRK_TT_GRID);
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess || per_cu <= 0) per_cu = 4;
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, (int64_t)per_cu * std::max(cus, 1)));
}

extern "C" {

int nrk_tt_user_fwd(const float* user_table, int64_t n_user_rows, const float* item_table,
                    int64_t n_item_rows, int dim, const int32_t* uid, const int32_t* hist,
                    const int32_t* hist_len, int64_t n, int seq_len, const float* w0,
                    const float* b0, int h0, const float* w1, const float* b1, int h1,
                    float* out, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n >= 0 && seq_len >= 1 && seq_len <= 64, "bad sizes (seq_len must be in [1, 64])");
    NRK_REQUIRE(n_user_rows > 0 && n_item_rows > 0, "empty embedding tables");
    if (!(dim == 16 || dim == 32 || dim == 64)) NRK_UNSUPPORTED("dim must be 16, 32 or 64");
    NRK_REQUIRE(h0 >= 1 && h0 <= 128, "h0 must be in [1, 128]");
    NRK_REQUIRE(h1 == dim, "last hidden width must equal the embedding dim "
                           "(youtubednn_recaller.py:461-465)");
    if (n == 0) return NRK_OK;
    NRK_REQUIRE(user_table && item_table && uid && hist && hist_len && w0 && b0 && w1 && b1 && out,
                "null pointer");
    const size_t h0p = (size_t)((h0 + 3) & ~3), h1p = (size_t)((h1 + 3) & ~3);
    const size_t lds = sizeof(float) * ((size_t)h0 * (2 * dim + 4) + h0p + (size_t)h1 * (h0p + 4) + h1p +
                                        (size_t)4 * (2 * dim + 128));
    hipStream_t s = as_stream(stream);
    // persistent grid of resident workgroups only (the weights' LDS admits ~5
    // per CU): a grid larger than the resident set left the queued
    // workgroups to run after the first ones finished, on a thinner machine
#define NRK_TT_LAUNCH(DD)                                                                      \
    do {                                                                                       \
        (void)hipFuncSetAttribute((const void*)tt_user_kernel<DD>,                                 \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);             \
        const int grid = tt_grid((const void*)tt_user_kernel<DD>, lds, n);                      \
        tt_user_kernel<DD><<<grid, 256, lds, s>>>(user_table, item_table, uid, hist, hist_len, \
                                                  n, seq_len, w0, b0, h0, w1, b1, h1, out);    \
    } while (0)
    if (dim == 16) NRK_TT_LAUNCH(16);
    else if (dim == 32) NRK_TT_LAUNCH(32);
    else NRK_TT_LAUNCH(64);
#undef NRK_TT_LAUNCH
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_tt_user_fwd_layers(const float* user_table, int64_t n_user_rows, const float* item_table,
                           int64_t n_item_rows, int dim, const int32_t* uid, const int32_t* hist,
                           const int32_t* hist_len, int64_t n, int seq_len, const float* weights, int n_layers,
                           const int* widths, float* out, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n >= 0 && seq_len >= 1 && seq_len <= 64, "bad sizes (seq_len must be in [1, 64])");
    NRK_REQUIRE(n_user_rows > 0 && n_item_rows > 0, "empty embedding tables");
    if (!(dim == 16 || dim == 32 || dim == 64)) NRK_UNSUPPORTED("dim must be 16, 32 or 64");
    NRK_REQUIRE(widths != nullptr, "null widths");
    if (n_layers < 1 || n_layers > TT_MAXL) NRK_UNSUPPORTED("1 to 8 hidden layers are compiled");
    TtLayers ly{};
    ly.n = n_layers;
    for (int l = 0; l < n_layers; ++l) {
        if (widths[l] < 1 || widths[l] > TT_MAXW) NRK_UNSUPPORTED("hidden widths must be in [1, 256]");
        ly.w[l] = widths[l];
    }
    NRK_REQUIRE(widths[n_layers - 1] == dim, "last hidden width must equal the embedding dim "
                                             "(youtubednn_recaller.py:461-465)");
    if (n == 0) return NRK_OK;
    NRK_REQUIRE(user_table && item_table && uid && hist && hist_len && weights && out, "null pointer");
    hipStream_t s = as_stream(stream);
    const int grid = (int)std::min<int64_t>((n + 3) / 4, 2048);
    if (dim == 16) tt_user_mlp_kernel<16><<<grid, 256, 0, s>>>(user_table, item_table, uid, hist, hist_len, n, seq_len, weights, ly, out);
    else if (dim == 32) tt_user_mlp_kernel<32><<<grid, 256, 0, s>>>(user_table, item_table, uid, hist, hist_len, n, seq_len, weights, ly, out);
    else tt_user_mlp_kernel<64><<<grid, 256, 0, s>>>(user_table, item_table, uid, hist, hist_len, n, seq_len, weights, ly, out);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_tt_item_fwd(const float* item_table, int64_t n_item_rows, int dim, const int32_t* ids,
                    int64_t n, float* out, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n >= 0 && n_item_rows > 0, "bad sizes");
    if (!(dim == 16 || dim == 32 || dim == 64)) NRK_UNSUPPORTED("dim must be 16, 32 or 64");
    if (n == 0) return NRK_OK;
    NRK_REQUIRE(item_table && ids && out, "null pointer");
    hipStream_t s = as_stream(stream);
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
    if (dim == 16) tt_item_kernel<16><<<grid, 256, 0, s>>>(item_table, ids, n, out);
    else if (dim == 32) tt_item_kernel<32><<<grid, 256, 0, s>>>(item_table, ids, n, out);
    else tt_item_kernel<64><<<grid, 256, 0, s>>>(item_table, ids, n, out);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
