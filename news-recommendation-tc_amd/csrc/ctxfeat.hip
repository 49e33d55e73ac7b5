// ctxfeat.hip -- the ranker's context features on gfx950.
//
// Reference: FeatureExtractor._extract_context_features
// (src/features/feature_extractor.py:440-723), then _apply_binning (:838-898)
// and the context LabelEncoders + DINDataset codes (src/rank/DIN.py:330-353,
// :560-617).  Per (user, recalled item) row, with the user's last N history
// items h_1..h_N (user_history_dict[user][-N:], oldest first):
//   score                      the recall score (float64 column);
//   sim_i       f32  w2v(item) . w2v(h_i)          (0 when h_i has no vector,
//                    a missing item is a zero vector; NaN when i > #history);
//   time_diff_i f32( |f64(f32(created(item))) - created(h_i)| ), 0 when
//                    either is missing (:619-633: f32 array - np.float64);
//   word_diff_i f32( || f64(f32(content(item))) - content(h_i) ||_2 ), numpy's
//                    pairwise float64 sum of squares, 0 when h_i has no
//                    content row or the item's row is all zero (:635-650);
//   sim_max / sim_mean / sim_min / sim_std   nan-statistics of the sims
//                    (float32; mean = f32(f64(sum) / count), std with ddof 0);
//   item_user_sim f32  yt(item) . yt(user) (0 when the user has no vector);
//   recall_in_user_cat  category(item) in the user's history categories.
// Users without a history entry keep the initial values (NaN sims / stats,
// zeros elsewhere) -- the reference skips them (:529-530).
// Then every feature goes through its fitted spec (nrk_ctx_spec): binned
// features fill NaN with the fitted median and take bin = #(inner edges <=
// value) (KBinsDiscretizer.transform: searchsorted(edges[1:-1], side=right))
// -> code = lut[bin]; the others map exact values through a small table
// (str(value) -> LabelEncoder class + 1 for one dtype), 0 when unseen.
//
// One wave per user group: the user's last-N history rows (content, w2v,
// created) are staged in LDS once and every lane takes one of the user's
// recalled rows.  Sequential per-lane sums in the reference's order for the
// float64 norms; the float32 dots use a sequential order (the reference's
// BLAS sgemv order is unspecified; ~1e-7 relative).
#include "nrk_common.h"

namespace nrk {

constexpr int CTX_NMAX = 4;      // last_N
constexpr int CTX_DC_MAX = 256;  // content dim
constexpr int CTX_DW_MAX = 128;  // w2v dim

// numpy float64 pairwise sum (loops_utils.h.src) of squares of
// d_e = f64(f32(r[e])) - h[e]; r from global (f64 table), h from LDS
struct SqDiff {
    const double* r;
    const double* h;
    __device__ double operator()(int e) const {
        const double d = __dsub_rn((double)(float)r[e], h[e]);
        double p = __dmul_rn(d, d);
        asm volatile("" : "+v"(p));  // keep the rounded square (no contraction)
        return p;
    }
};

template <typename F>
__device__ double pw_leaf64(const F& f, int b, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r = __dadd_rn(r, f(b + i));
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f(b + j);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = __dadd_rn(r[j], f(b + i + j));
    }
    double res = __dadd_rn(__dadd_rn(__dadd_rn(r[0], r[1]), __dadd_rn(r[2], r[3])),
                           __dadd_rn(__dadd_rn(r[4], r[5]), __dadd_rn(r[6], r[7])));
    for (; i < n; ++i) res = __dadd_rn(res, f(b + i));
    return res;
}

template <int L, typename F>
__device__ double pw_sum64(const F& f, int b, int n) {
    if (L == 0 || n <= 128) return pw_leaf64(f, b, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return __dadd_rn(pw_sum64<(L > 0 ? L - 1 : 0)>(f, b, n2), pw_sum64<(L > 0 ? L - 1 : 0)>(f, b + n2, n - n2));
}

__device__ __forceinline__ float dot_f32(const float* a, const float* b, int n) {
    float s = 0.0f;
    for (int i = 0; i < n; ++i) s = fmaf(a[i], b[i], s);
    return s;
}

__device__ __forceinline__ int32_t ctx_code(const nrk_ctx_spec& sp, double v) {
    if (sp.kind == 0) {
        if (v != v) v = sp.fill;
        int bin = 0;
        for (int k = 0; k < sp.n_edges; ++k) bin += sp.edges[k] <= v ? 1 : 0;
        return bin < sp.n_lut ? sp.lut[bin] : 0;
    }
    for (int k = 0; k < sp.n_vals; ++k)
        if (sp.vals[k] == v) return sp.codes[k];
    return 0;
}

__global__ __launch_bounds__(256) void ctx_features_kernel(nrk_ctx_tables tb, const nrk_ctx_spec* __restrict__ spec,
                                                           double* __restrict__ out_raw,
                                                           int32_t* __restrict__ out_codes) {
    __shared__ double s_cont[4][CTX_NMAX][CTX_DC_MAX];
    __shared__ float s_w2v[4][CTX_NMAX][CTX_DW_MAX];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t g = (int64_t)blockIdx.x * 4 + wv;
    if (g >= tb.n_groups) return;
    const int N = tb.last_n, F = 1 + 3 * N + 6;
    const int32_t u = tb.group_user[g];
    const int hn = u >= 0 ? tb.hist_n[u] : -1;  // -1: the user has no history entry
    int32_t hrow[CTX_NMAX];
    double hcre[CTX_NMAX];
    bool hw2v[CTX_NMAX], hcont[CTX_NMAX];
    for (int i = 0; i < N; ++i) {
        const int32_t r = i < hn ? tb.hist_last[(int64_t)u * N + i] : -1;
        hrow[i] = r;
        hw2v[i] = r >= 0 && tb.w2v_ok[r];
        hcont[i] = r >= 0 && (tb.content_flags[r] & 1);
        hcre[i] = r >= 0 ? tb.created[r] : (double)NAN;
        for (int e = lane; e < tb.dc; e += 64) s_cont[wv][i][e] = hcont[i] ? tb.content[(int64_t)r * tb.dc + e] : 0.0;
        for (int e = lane; e < tb.dw; e += 64) s_w2v[wv][i][e] = hw2v[i] ? tb.w2v[(int64_t)r * tb.dw + e] : 0.0f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const bool uyt = tb.user_yt != nullptr && u >= 0 && tb.user_yt_ok[u];
    const int64_t p0 = tb.group_off[g], p1 = tb.group_off[g + 1];
    for (int64_t q = p0 + lane; q < p1; q += 64) {
        const int64_t pos = tb.pair_pos ? tb.pair_pos[q] : q;
        const int32_t it = tb.pair_item[pos];
        double f[1 + 3 * CTX_NMAX + 6];
        f[0] = tb.pair_score[pos];
        for (int i = 0; i < N; ++i) {
            f[1 + 3 * i] = NAN;
            f[2 + 3 * i] = 0.0;
            f[3 + 3 * i] = 0.0;
        }
        for (int k = 0; k < 4; ++k) f[1 + 3 * N + k] = NAN;
        f[1 + 3 * N + 4] = 0.0;
        f[1 + 3 * N + 5] = 0.0;
        if (hn >= 0) {
            const bool iw2v = it >= 0 && tb.w2v_ok[it];
            const uint8_t icf = it >= 0 ? tb.content_flags[it] : 0;
            const double icre = it >= 0 ? (double)(float)tb.created[it] : (double)NAN;  // f32 array (:588-594)
            float sims[CTX_NMAX];
            for (int i = 0; i < N; ++i) {
                sims[i] = NAN;
                if (i >= hn) continue;
                // sim_i (:612-615): 0 when h_i has no vector, zero vector for a missing item
                float sv = 0.0f;
                if (hw2v[i] && iw2v) sv = dot_f32(tb.w2v + (int64_t)it * tb.dw, s_w2v[wv][i], tb.dw);
                sims[i] = sv;
                f[1 + 3 * i] = (double)sv;
                // time_diff_i (:617-631)
                double td = 0.0;
                if (hcre[i] == hcre[i]) {
                    const double d = fabs(icre - hcre[i]);
                    td = d == d ? d : 0.0;
                }
                f[2 + 3 * i] = (double)(float)td;
                // word_diff_i (:633-648)
                double wd = 0.0;
                if (hcont[i] && (icf & 2)) {
                    SqDiff sq{tb.content + (int64_t)it * tb.dc, s_cont[wv][i]};
                    wd = sqrt(pw_sum64<2>(sq, 0, tb.dc));
                }
                f[3 + 3 * i] = (double)(float)wd;
            }
            // nan-statistics of the sims (:660-664), float32
            float mx = -INFINITY, mn = INFINITY, tot = 0.0f;
            int cnt = 0;
            for (int i = 0; i < N; ++i) {
                if (sims[i] != sims[i]) continue;
                mx = fmaxf(mx, sims[i]);
                mn = fminf(mn, sims[i]);
                tot = __fadd_rn(tot, sims[i]);
                ++cnt;
            }
            if (cnt > 0) {
                const float mean = (float)((double)tot / (double)cnt);
                float ss = 0.0f;
                for (int i = 0; i < N; ++i) {
                    if (sims[i] != sims[i]) continue;
                    const float d = __fsub_rn(sims[i], mean);
                    float sq = __fmul_rn(d, d);
                    asm volatile("" : "+v"(sq));  // no contraction into the running sum
                    ss = __fadd_rn(ss, sq);
                }
                const float var = (float)((double)ss / (double)cnt);
                f[1 + 3 * N + 0] = (double)mx;
                f[1 + 3 * N + 1] = (double)mean;
                f[1 + 3 * N + 2] = (double)mn;
                f[1 + 3 * N + 3] = (double)(float)sqrt((double)var);  // correctly rounded f32 sqrt
            }
            // item_user_sim (:538-558), zero vector for a missing item
            if (uyt && it >= 0 && tb.item_yt_ok[it])
                f[1 + 3 * N + 4] = (double)dot_f32(tb.item_yt + (int64_t)it * tb.dy, tb.user_yt + (int64_t)u * tb.dy, tb.dy);
            // recall_in_user_cat (:677-690)
            const int32_t c = it >= 0 ? tb.category[it] : -1;
            int inc = 0;
            if (c >= 0)
                for (int64_t k = tb.ucat_off[u]; k < tb.ucat_off[u + 1]; ++k) inc |= tb.ucat[k] == c ? 1 : 0;
            f[1 + 3 * N + 5] = (double)inc;
        }
        if (out_raw)
            for (int k = 0; k < F; ++k) out_raw[pos * F + k] = f[k];
        if (out_codes)
            for (int k = 0; k < F; ++k) out_codes[pos * tb.code_stride + k] = ctx_code(spec[k], f[k]);
    }
}

}  // namespace nrk

using namespace nrk;

extern "C" {

int nrk_ctx_features(const nrk_ctx_tables* tables, const nrk_ctx_spec* spec, double* out_raw, int32_t* out_codes,
                     nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(tables != nullptr, "null tables");
    const nrk_ctx_tables& t = *tables;
    NRK_REQUIRE(t.last_n >= 1 && t.last_n <= CTX_NMAX, "last_n must be in [1, 4]");
    NRK_REQUIRE(t.dc >= 1 && t.dc <= CTX_DC_MAX, "content dim must be in [1, 256]");
    NRK_REQUIRE(t.dw >= 1 && t.dw <= CTX_DW_MAX, "w2v dim must be in [1, 128]");
    NRK_REQUIRE(t.n_groups >= 0, "n_groups must be >= 0");
    NRK_REQUIRE(out_raw || out_codes, "no output");
    NRK_REQUIRE(!out_codes || (spec && t.code_stride >= 1 + 3 * t.last_n + 6), "codes need a spec and a stride");
    if (t.n_groups == 0) return NRK_OK;
    NRK_REQUIRE(t.group_off && t.group_user && t.pair_item && t.pair_score && t.hist_last && t.hist_n &&
                    t.ucat_off && t.ucat && t.w2v && t.w2v_ok && t.content && t.content_flags && t.created &&
                    t.category,
                "null table pointer");
    NRK_REQUIRE(!t.user_yt || (t.user_yt_ok && t.item_yt && t.item_yt_ok && t.dy >= 1), "yt tables incomplete");
    ctx_features_kernel<<<(int)((t.n_groups + 3) / 4), 256, 0, as_stream(stream)>>>(t, spec, out_raw, out_codes);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
