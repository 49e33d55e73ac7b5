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

// numpy's float64 pairwise sum (loops_utils.h.src) of the squares
// d_e^2, d_e = f64(f32(r[e])) - h[e] (r: the item's content row, f64 table;
// h: the history row in LDS) -- restated as pw_sum64<2> below
// The leaves of that sum, pw_sum64<2>(f, 0, n) (numpy's pairwise blocks of <= 128;
// a leaf of n >= 8: 8 strided accumulators, a fixed tree, the tail in order)
// and how they combine: shape 0 = l0; 1 = l0 + l1; 2 = (l0 + l1) + l2;
// 3 = l0 + (l1 + l2); 4 = (l0 + l1) + (l2 + l3).
struct PwPlan {
    int nl, shape;
    int b[4], n[4];
};
__device__ __forceinline__ PwPlan pw_plan(int n) {
    // every store at a constant index (a run-time index puts the plan in scratch)
    PwPlan p{};
    if (n <= 128) {
        p.nl = 1;
        p.b[0] = 0;
        p.n[0] = n;
        return p;
    }
    const int n2 = n / 2 - (n / 2) % 8, r1 = n - n2;  // numpy's halves
    const int m0 = n2 / 2 - (n2 / 2) % 8, m1 = r1 / 2 - (r1 / 2) % 8;
    const bool s0 = n2 > 128, s1 = r1 > 128;  // a half above 128 splits once more
    if (!s0 && !s1) {
        p.nl = 2;
        p.b[0] = 0, p.n[0] = n2;
        p.b[1] = n2, p.n[1] = r1;
        p.shape = 1;
    } else if (s0 && !s1) {
        p.nl = 3;
        p.b[0] = 0, p.n[0] = m0;
        p.b[1] = m0, p.n[1] = n2 - m0;
        p.b[2] = n2, p.n[2] = r1;
        p.shape = 2;
    } else if (!s0 && s1) {
        p.nl = 3;
        p.b[0] = 0, p.n[0] = n2;
        p.b[1] = n2, p.n[1] = m1;
        p.b[2] = n2 + m1, p.n[2] = r1 - m1;
        p.shape = 3;
    } else {
        p.nl = 4;
        p.b[0] = 0, p.n[0] = m0;
        p.b[1] = m0, p.n[1] = n2 - m0;
        p.b[2] = n2, p.n[2] = m1;
        p.b[3] = n2 + m1, p.n[3] = r1 - m1;
        p.shape = 4;
    }
    return p;
}

// xor-1 / xor-2 / xor-4 partner of a double within 8 lanes (DPP quad swaps
// and the half-row mirror: lane j gets 7 - j, whose pair sums equal the
// xor-4 partner's after the first two steps)
__device__ __forceinline__ double dpp_f64(double v, int ctrl) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
    switch (ctrl) {
        case 0xB1: lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false); break;
        case 0x4E: lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false); break;
        default: lo = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xF, 0xF, false); break;
    }
    return __longlong_as_double((long long)((uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32)));
}

// word_diff of one recalled row against all N history items on a half-wave
// (32 lanes): lane (leaf l, j) keeps numpy's j-th leaf accumulator (elements
// b + j, b + j + 8, ...: 8 lanes read 64 consecutive bytes of the item row)
// for every history item, a xor-1/2/4 butterfly is the leaf's
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), lane j = 0 adds the leaf's tail in
// order, and the leaves combine by the plan's shape -- the same operations in
// the same order as numpy's pairwise sum (bit-identical)
__device__ __forceinline__ void coop_word_diff_n(const PwPlan& pl, const double* __restrict__ r,
                                                 const double* __restrict__ hb, int hs, int N, int s,
                                                 double (&out)[CTX_NMAX]) {
    auto h = [&](int i, int e) { return hb[i * hs + e]; };  // history row i, element e (LDS)
    const int l = s >> 3, j = s & 7;
    const bool act = l < pl.nl;
    // the lane's leaf by selects (a run-time index into pl.b / pl.n would put
    // the plan in scratch)
    const int lb = !act ? 0 : l == 0 ? pl.b[0] : l == 1 ? pl.b[1] : l == 2 ? pl.b[2] : pl.b[3];
    const int ln = !act ? 0 : l == 0 ? pl.n[0] : l == 1 ? pl.n[1] : l == 2 ? pl.n[2] : pl.n[3];
    double acc[CTX_NMAX] = {0.0, 0.0, 0.0, 0.0};
    auto fa = [&](int e, bool first) {
        const double re = (double)(float)r[e];
#pragma unroll
        for (int i = 0; i < CTX_NMAX; ++i) {
            if (i >= N) break;
            const double d = __dsub_rn(re, h(i, e));
            double p = __dmul_rn(d, d);
            asm volatile("" : "+v"(p));
            acc[i] = first ? p : __dadd_rn(acc[i], p);
        }
    };
    const int full = ln - ln % 8;
    if (ln >= 8) {
        fa(lb + j, true);
        for (int i = 8; i < full; i += 8) fa(lb + i + j, false);
    }
    const int base = threadIdx.x & 32;  // this half-wave's lane 0
#pragma unroll
    for (int i = 0; i < CTX_NMAX; ++i) {
        if (i >= N) break;
        double a = acc[i];
        a = __dadd_rn(a, dpp_f64(a, 0xB1));
        a = __dadd_rn(a, dpp_f64(a, 0x4E));
        a = __dadd_rn(a, dpp_f64(a, 0x141));
        acc[i] = a;
    }
    if (j == 0 && act) {
        for (int e = ln < 8 ? 0 : full; e < ln; ++e) {
            const double re = (double)(float)r[lb + e];
#pragma unroll
            for (int i = 0; i < CTX_NMAX; ++i) {
                if (i >= N) break;
                const double d = __dsub_rn(re, h(i, lb + e));
                double p = __dmul_rn(d, d);
                asm volatile("" : "+v"(p));
                acc[i] = (ln < 8 && e == 0) ? p : __dadd_rn(acc[i], p);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < CTX_NMAX; ++i) {
        if (i >= N) break;
        const double v0 = __shfl(acc[i], base, WAVE), v1 = __shfl(acc[i], base + 8, WAVE);
        const double v2 = __shfl(acc[i], base + 16, WAVE), v3 = __shfl(acc[i], base + 24, WAVE);
        switch (pl.shape) {
            case 0: out[i] = v0; break;
            case 1: out[i] = __dadd_rn(v0, v1); break;
            case 2: out[i] = __dadd_rn(__dadd_rn(v0, v1), v2); break;
            case 3: out[i] = __dadd_rn(v0, __dadd_rn(v1, v2)); break;
            default: out[i] = __dadd_rn(__dadd_rn(v0, v1), __dadd_rn(v2, v3)); break;
        }
    }
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
    // the history content rows: N x dc doubles per wave (dynamic, sized by
    // the host: 24 KB at N = 3, dc = 250 instead of a 32-KB worst case, so 4
    // workgroups fit a CU instead of 3)
    extern __shared__ double s_dyn[];
    __shared__ __attribute__((aligned(16))) float s_w2v[4][CTX_NMAX][CTX_DW_MAX];
    __shared__ double s_wd[4][64][CTX_NMAX];  // word_diff of this chunk's rows
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t g = (int64_t)blockIdx.x * 4 + wv;
    if (g >= tb.n_groups) return;
    const int N = tb.last_n, F = 1 + 3 * N + 6;
    double* const s_cont = s_dyn + (size_t)wv * N * tb.dc;  // [N][dc]
    const int32_t u = tb.group_user[g];
    const int hn = u >= 0 ? tb.hist_n[u] : -1;  // -1: the user has no history entry
    int32_t hrow[CTX_NMAX];
    double hcre[CTX_NMAX];
    bool hw2v[CTX_NMAX], hcont[CTX_NMAX];
#pragma unroll
    for (int i = 0; i < CTX_NMAX; ++i) {
        if (i >= N) {
            hrow[i] = -1;
            hw2v[i] = hcont[i] = false;
            hcre[i] = (double)NAN;
            continue;
        }
        const int32_t r = i < hn ? tb.hist_last[(int64_t)u * N + i] : -1;
        hrow[i] = r;
        hw2v[i] = r >= 0 && tb.w2v_ok[r];
        hcont[i] = r >= 0 && (tb.content_flags[r] & 1);
        hcre[i] = r >= 0 ? tb.created[r] : (double)NAN;
        for (int e = lane; e < tb.dc; e += 64) s_cont[i * tb.dc + e] = hcont[i] ? tb.content[(int64_t)r * tb.dc + e] : 0.0;
        for (int e = lane; e < tb.dw; e += 64) s_w2v[wv][i][e] = hw2v[i] ? tb.w2v[(int64_t)r * tb.dw + e] : 0.0f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const bool uyt = tb.user_yt != nullptr && u >= 0 && tb.user_yt_ok[u];
    // the user's history categories: up to 64 held one per lane (loaded with
    // every lane active, read back by v_readlane per category); more take the
    // per-row loop below
    const int64_t uk0 = u >= 0 ? tb.ucat_off[u] : 0, uk1 = u >= 0 ? tb.ucat_off[u + 1] : 0;
    const int ncat = (int)(uk1 - uk0);
    const int32_t ucv = (ncat <= 64 && lane < ncat) ? tb.ucat[uk0 + lane] : -1;
    const int64_t p0 = tb.group_off[g], p1 = tb.group_off[g + 1];
    const PwPlan plan = pw_plan(tb.dc);
    for (int64_t c0 = p0; c0 < p1; c0 += 64) {
        // word_diff of the chunk's rows first, two (row, history item)
        // tasks per wave instruction (coalesced item-row reads), into LDS
        const int nr = (int)(p1 - c0 < 64 ? p1 - c0 : 64);
        if (hn > 0) {
            // one row per half-wave, all N history items per pass over the row
            for (int r0 = 0; r0 < nr; r0 += 2) {
                const int qr0 = r0 + (lane >> 5);
                const int qr = qr0 < nr ? qr0 : nr - 1;
                const int64_t pos = tb.pair_pos ? tb.pair_pos[c0 + qr] : c0 + qr;
                const int32_t it = tb.pair_item[pos];
                const bool ion = it >= 0 && (tb.content_flags[it] & 2);
                const double* rrow = tb.content + (int64_t)(ion ? it : 0) * tb.dc;
                // every lane runs the (shuffling) sums; rows that do not count take 0
                double ss[CTX_NMAX];
                coop_word_diff_n(plan, rrow, s_cont, tb.dc, N, lane & 31, ss);
                if ((lane & 31) == 0 && qr0 < nr) {
#pragma unroll
                    for (int i = 0; i < CTX_NMAX; ++i)
                        if (i < N) s_wd[wv][qr][i] = (ion && i < hn && hcont[i]) ? sqrt(ss[i]) : 0.0;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        const int64_t q = c0 + lane;
        if (q >= p1) continue;
        const int64_t pos = tb.pair_pos ? tb.pair_pos[q] : q;
        const int32_t it = tb.pair_item[pos];
        // the row's features in registers: every array below is indexed by
        // compile-time loop indices (a runtime-N index put them in scratch)
        double fs[CTX_NMAX][3];  // sim_i, time_diff_i, word_diff_i
        double st[6];            // sim_max, sim_mean, sim_min, sim_std, item_user_sim, recall_in_user_cat
#pragma unroll
        for (int i = 0; i < CTX_NMAX; ++i) {
            fs[i][0] = NAN;
            fs[i][1] = 0.0;
            fs[i][2] = 0.0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) st[k] = NAN;
        st[4] = 0.0;
        st[5] = 0.0;
        if (hn >= 0) {
            const bool iw2v = it >= 0 && tb.w2v_ok[it];
            const double icre = it >= 0 ? (double)(float)tb.created[it] : (double)NAN;  // f32 array (:588-594)
            float sims[CTX_NMAX];
            // sim_i (:612-615): 0 when h_i has no vector, zero vector for a
            // missing item.  The N dots run interleaved over one pass of the
            // item's row (16-B loads; each dot still sums e = 0, 1, ... in order)
            float dots[CTX_NMAX] = {0.0f, 0.0f, 0.0f, 0.0f};
            if (iw2v && hn > 0) {
                const float* ir = tb.w2v + (int64_t)it * tb.dw;
                if ((tb.dw & 3) == 0) {
                    for (int e = 0; e < tb.dw; e += 4) {
                        const float4 x = *reinterpret_cast<const float4*>(ir + e);
#pragma unroll
                        for (int i = 0; i < CTX_NMAX; ++i) {
                            if (i >= N) break;
                            const float4 y = *reinterpret_cast<const float4*>(&s_w2v[wv][i][e]);
                            dots[i] = fmaf(x.w, y.w, fmaf(x.z, y.z, fmaf(x.y, y.y, fmaf(x.x, y.x, dots[i]))));
                        }
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < CTX_NMAX; ++i) {
                        if (i >= N) break;
                        dots[i] = dot_f32(ir, s_w2v[wv][i], tb.dw);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < CTX_NMAX; ++i) {
                sims[i] = NAN;
                if (i >= N || i >= hn) continue;
                const float sv = hw2v[i] && iw2v ? dots[i] : 0.0f;
                sims[i] = sv;
                fs[i][0] = (double)sv;
                // time_diff_i (:617-631)
                double td = 0.0;
                if (hcre[i] == hcre[i]) {
                    const double d = fabs(icre - hcre[i]);
                    td = d == d ? d : 0.0;
                }
                fs[i][1] = (double)(float)td;
                // word_diff_i (:633-648), computed cooperatively above
                fs[i][2] = (double)(float)s_wd[wv][lane][i];
            }
            // nan-statistics of the sims (:660-664), float32
            float mx = -INFINITY, mn = INFINITY, tot = 0.0f;
            int cnt = 0;
#pragma unroll
            for (int i = 0; i < CTX_NMAX; ++i) {
                if (i >= N || sims[i] != sims[i]) continue;
                mx = fmaxf(mx, sims[i]);
                mn = fminf(mn, sims[i]);
                tot = __fadd_rn(tot, sims[i]);
                ++cnt;
            }
            if (cnt > 0) {
                const float mean = (float)((double)tot / (double)cnt);
                float ss = 0.0f;
#pragma unroll
                for (int i = 0; i < CTX_NMAX; ++i) {
                    if (i >= N || sims[i] != sims[i]) continue;
                    const float d = __fsub_rn(sims[i], mean);
                    float sq = __fmul_rn(d, d);
                    asm volatile("" : "+v"(sq));  // no contraction into the running sum
                    ss = __fadd_rn(ss, sq);
                }
                const float var = (float)((double)ss / (double)cnt);
                st[0] = (double)mx;
                st[1] = (double)mean;
                st[2] = (double)mn;
                st[3] = (double)(float)sqrt((double)var);  // correctly rounded f32 sqrt
            }
            // item_user_sim (:538-558), zero vector for a missing item
            if (uyt && it >= 0 && tb.item_yt_ok[it]) {
                const float* a = tb.item_yt + (int64_t)it * tb.dy;
                const float* b = tb.user_yt + (int64_t)u * tb.dy;
                float d = 0.0f;
                if ((tb.dy & 3) == 0) {
                    for (int e = 0; e < tb.dy; e += 4) {
                        const float4 x = *reinterpret_cast<const float4*>(a + e);
                        const float4 y = *reinterpret_cast<const float4*>(b + e);
                        d = fmaf(x.w, y.w, fmaf(x.z, y.z, fmaf(x.y, y.y, fmaf(x.x, y.x, d))));
                    }
                } else {
                    d = dot_f32(a, b, tb.dy);
                }
                st[4] = (double)d;
            }
            // recall_in_user_cat (:677-690)
            const int32_t c = it >= 0 ? tb.category[it] : -1;
            int inc = 0;
            if (c >= 0) {
                if (ncat <= 64) {
                    for (int kk = 0; kk < ncat; ++kk) inc |= __builtin_amdgcn_readlane(ucv, kk) == c ? 1 : 0;
                } else {
                    for (int64_t k = uk0; k < uk1; ++k) inc |= tb.ucat[k] == c ? 1 : 0;
                }
            }
            st[5] = (double)inc;
        }
        // column order: score, (sim, time_diff, word_diff) per history item,
        // the six row statistics
        auto emit = [&](int col, double v) {
            if (out_raw) out_raw[pos * F + col] = v;
            if (out_codes) out_codes[pos * tb.code_stride + col] = ctx_code(spec[col], v);
        };
        emit(0, tb.pair_score[pos]);
#pragma unroll
        for (int i = 0; i < CTX_NMAX; ++i) {
            if (i >= N) break;
#pragma unroll
            for (int c = 0; c < 3; ++c) emit(1 + 3 * i + c, fs[i][c]);
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) emit(1 + 3 * N + k, st[k]);
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
    const size_t lds = (size_t)4 * t.last_n * t.dc * sizeof(double);
    ctx_features_kernel<<<(int)((t.n_groups + 3) / 4), 256, lds, as_stream(stream)>>>(t, spec, out_raw, out_codes);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
