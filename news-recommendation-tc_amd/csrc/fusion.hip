// fusion.hip -- RecallFusion.fuse on gfx950.
//
// Reference: src/recall/fusion.py:67-342 as RecallPipeline.fusion_recall
// drives it (src/pipeline/recall_pipeline.py:276-288): every recall method's
// per-user lists are score-normalised (global min-max, per-list min-max, or
// per-method z-score + sigmoid, :67-187), merged per user into one score per
// distinct item (six strategies, :189-265), optionally filtered against the
// user's seen items, and the top-k kept by a STABLE descending sort whose tie
// order is the merged dict's insertion order = the item's first appearance
// in (method order, list order) (:327-333).
//
// Layout (built by nrk/recall/fusion.py): every (method, user, position)
// entry of every list, grouped by user in the output's user order; inside a
// user the entries stay in method order, then list order -- the order the
// reference walks them (:205-218), so the per-item sums below run in the
// reference's order and are bit-identical.  Items are dense int32 codes.
//
// One wave per user, up to 256 entries (4 per lane).  Per entry: normalised
// score, then w * s (the term every strategy sums); the first occurrence of
// each item leads its group and accumulates the group's terms in entry order
// from LDS; leaders are ranked by (merged score desc, first occurrence asc)
// with the wave bitonic sort; the top-k are written.  Integer/byte work
// around a few fp64 ops per entry: latency-bound, no MFMA.
#include "nrk_common.h"

namespace nrk {

constexpr int FUSE_E = 4;               // entries per lane
constexpr int FUSE_MAX = FUSE_E * 64;   // entries per user
constexpr int FUSE_WMAX = 2048;         // entries per user on the wide path

enum FuseStrategy { FS_WSUM = 0, FS_WAVG = 1, FS_MAX = 2, FS_HARM = 3, FS_DIV = 4, FS_RRF = 5 };
// FN_PRE: scores already normalised by the caller (the z-score sigmoid on
// the host with numpy's exp, bit-identical to the reference's np.exp)
enum FuseNorm { FN_LOCAL = 0, FN_GLOBAL = 1, FN_ZSCORE = 2, FN_PRE = 3 };

struct FuseParams {
    int strategy, norm, n_methods, topk;
    double gmin, gmax;  // global min / max (FN_GLOBAL)
};

__device__ __forceinline__ double wave_min_f64(double v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v = fmin(v, __shfl_xor(v, m, WAVE));
    return v;
}
__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v = fmax(v, __shfl_xor(v, m, WAVE));
    return v;
}

__global__ __launch_bounds__(256) void fuse_kernel(
    const int64_t* __restrict__ offsets, int64_t n_users, const int32_t* __restrict__ item,
    const double* __restrict__ score, const int32_t* __restrict__ method, const int32_t* __restrict__ rank,
    const double* __restrict__ weight, const double* __restrict__ zmean, const double* __restrict__ zstd,
    const int64_t* __restrict__ seen_off, const int32_t* __restrict__ seen, FuseParams prm,
    int32_t* __restrict__ out_item, double* __restrict__ out_score, int32_t* __restrict__ out_cnt) {
    __shared__ int32_t s_item[4][FUSE_MAX];
    __shared__ double s_term[4][FUSE_MAX];
    __shared__ double s_w[4][FUSE_MAX];
    __shared__ int32_t s_rank[4][FUSE_MAX];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t u = (int64_t)blockIdx.x * 4 + wv;
    if (u >= n_users) return;
    const int64_t b = offsets[u];
    const int n = (int)(offsets[u + 1] - b);
    if (n > FUSE_MAX) {  // not this kernel's job (nrk_fuse_wide): flagged, padded
        for (int i = lane; i < prm.topk; i += WAVE) {
            out_item[u * prm.topk + i] = -1;
            out_score[u * prm.topk + i] = 0.0;
        }
        if (lane == 0) out_cnt[u] = -1;
        return;
    }

    int32_t it[FUSE_E], mt[FUSE_E];
    double sc[FUSE_E];
#pragma unroll
    for (int e = 0; e < FUSE_E; ++e) {
        const int i = e * 64 + lane;
        const bool ok = i < n;
        it[e] = ok ? item[b + i] : -1;
        mt[e] = ok ? method[b + i] : -1;
        sc[e] = ok ? score[b + i] : 0.0;
        s_rank[wv][i] = ok ? rank[b + i] : 0;
    }
    // normalised score of every entry
    double ns[FUSE_E];
    if (prm.norm == FN_GLOBAL) {
        const double span = prm.gmax - prm.gmin;
#pragma unroll
        for (int e = 0; e < FUSE_E; ++e) ns[e] = prm.gmax > prm.gmin ? (sc[e] - prm.gmin) / span : 1.0;
    } else if (prm.norm == FN_PRE) {
#pragma unroll
        for (int e = 0; e < FUSE_E; ++e) ns[e] = sc[e];
    } else if (prm.norm == FN_ZSCORE) {
#pragma unroll
        for (int e = 0; e < FUSE_E; ++e) {
            const int m = mt[e] < 0 ? 0 : mt[e];
            const double sd = zstd[m];
            ns[e] = sd > 0.0 ? 1.0 / (1.0 + exp(-((sc[e] - zmean[m]) / sd))) : 0.5;
        }
    } else {
        // per (method, user) list: min-max; a one-entry list -> 1.0 (:84-93)
#pragma unroll
        for (int e = 0; e < FUSE_E; ++e) ns[e] = 1.0;
        for (int m = 0; m < prm.n_methods; ++m) {
            double mn = INFINITY, mx = -INFINITY;
            int c = 0;
#pragma unroll
            for (int e = 0; e < FUSE_E; ++e) {
                const bool in = mt[e] == m;
                mn = in ? fmin(mn, sc[e]) : mn;
                mx = in ? fmax(mx, sc[e]) : mx;
                c += in ? 1 : 0;
            }
            mn = wave_min_f64(mn);
            mx = wave_max_f64(mx);
            for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, WAVE);
#pragma unroll
            for (int e = 0; e < FUSE_E; ++e)
                if (mt[e] == m) ns[e] = (c > 1 && mx > mn) ? (sc[e] - mn) / (mx - mn) : 1.0;
        }
    }
#pragma unroll
    for (int e = 0; e < FUSE_E; ++e) {
        const int i = e * 64 + lane;
        const double w = mt[e] >= 0 ? weight[mt[e]] : 0.0;
        s_item[wv][i] = it[e];
        s_w[wv][i] = w;
        s_term[wv][i] = w * ns[e];  // s["weight"] * s["score"]
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // group leaders (first occurrence of the item) and their merged score
    const int64_t so = seen_off ? seen_off[u] : 0;
    const int ns_seen = seen_off ? (int)(seen_off[u + 1] - so) : 0;
    Cand x[FUSE_E];
#pragma unroll
    for (int e = 0; e < FUSE_E; ++e) {
        const int i = e * 64 + lane;
        x[e].s = -INFINITY;
        x[e].row = INT32_MAX;
        if (i >= n) continue;
        const int32_t me = it[e];
        bool lead = true;
        for (int j = 0; j < i && lead; ++j) lead = s_item[wv][j] != me;
        if (!lead) continue;
        bool drop = false;
        for (int j = 0; j < ns_seen && !drop; ++j) drop = seen[so + j] == me;
        if (drop) continue;
        double acc = 0.0, tw = 0.0, mxv = -INFINITY, hs = 0.0;
        int cnt = 0;
        for (int j = i; j < n; ++j) {
            if (s_item[wv][j] != me) continue;
            const double t = s_term[wv][j], w = s_w[wv][j];
            ++cnt;
            switch (prm.strategy) {
                case FS_MAX: mxv = cnt == 1 ? t : fmax(mxv, t); break;
                case FS_HARM: hs += 1.0 / (t + 1e-8); break;
                case FS_RRF: acc += w / (double)(60 + s_rank[wv][j]); break;
                case FS_WAVG: tw += w; acc += t; break;
                default: acc += t; break;  // weighted_sum, diversity_weighted
            }
        }
        double merged;
        switch (prm.strategy) {
            case FS_WSUM: merged = acc; break;
            case FS_MAX: merged = mxv; break;
            case FS_HARM: merged = (double)cnt / hs; break;
            case FS_DIV: merged = acc * (1.0 + (double)cnt * 0.1); break;
            case FS_RRF: merged = acc; break;
            default: merged = tw > 0.0 ? acc / tw : 0.0; break;
        }
        x[e].s = merged;
        x[e].row = i;  // insertion order of the merged dict
    }
    wave_bitonic_sort<FUSE_E>(x);
    int kept = 0;
#pragma unroll
    for (int e = 0; e < FUSE_E; ++e) {
        const int i = e * 64 + lane;
        const bool ok = x[e].row != INT32_MAX;
        if (i < prm.topk) {
            out_item[u * prm.topk + i] = ok ? s_item[wv][x[e].row] : -1;
            out_score[u * prm.topk + i] = ok ? x[e].s : 0.0;
        }
        kept += (ok && i < prm.topk) ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o, WAVE);
    if (lane == 0) out_cnt[u] = kept;
}

// Users with more than FUSE_MAX entries (nrk_fuse_wide): the same per-entry
// arithmetic in the same order, one wave per user with every array in
// dynamic LDS (nw = next_pow2(max entries) slots), the leaders ranked by an
// LDS bitonic sort on (merged desc, first occurrence asc).
__global__ __launch_bounds__(64) void fuse_wide_kernel(
    const int64_t* __restrict__ offsets, int64_t n_users, const int32_t* __restrict__ item,
    const double* __restrict__ score, const int32_t* __restrict__ method, const int32_t* __restrict__ rank,
    const double* __restrict__ weight, const double* __restrict__ zmean, const double* __restrict__ zstd,
    const int64_t* __restrict__ seen_off, const int32_t* __restrict__ seen, FuseParams prm, int nw,
    int32_t* __restrict__ out_item, double* __restrict__ out_score, int32_t* __restrict__ out_cnt) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    Cand* x = reinterpret_cast<Cand*>(dyn);                  // [nw]
    double* s_term = reinterpret_cast<double*>(x + nw);      // [nw]
    double* s_w = s_term + nw;                               // [nw]
    int32_t* s_item = reinterpret_cast<int32_t*>(s_w + nw);  // [nw]
    int32_t* s_rank = s_item + nw;                           // [nw]
    int32_t* s_m = s_rank + nw;                              // [nw]
    const int lane = threadIdx.x;
    for (int64_t u = blockIdx.x; u < n_users; u += gridDim.x) {
        const int64_t b = offsets[u];
        const int n = (int)(offsets[u + 1] - b);
        for (int i = lane; i < nw; i += WAVE) {
            const bool ok = i < n;
            s_item[i] = ok ? item[b + i] : -1;
            s_m[i] = ok ? method[b + i] : -1;
            s_term[i] = ok ? score[b + i] : 0.0;  // raw score until normalised below
            s_rank[i] = ok ? rank[b + i] : 0;
        }
        wave_sync_lds();
        // normalised score of every entry, then w * s
        if (prm.norm == FN_LOCAL) {
            // per (method, user) list: min-max over the raw scores of that
            // method's entries, which only this method's pass rewrites
            for (int m = 0; m < prm.n_methods; ++m) {
                double mn = INFINITY, mx = -INFINITY;
                int c = 0;
                for (int i = lane; i < n; i += WAVE)
                    if (s_m[i] == m) {
                        mn = fmin(mn, s_term[i]);
                        mx = fmax(mx, s_term[i]);
                        ++c;
                    }
                mn = wave_min_f64(mn);
                mx = wave_max_f64(mx);
                for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, WAVE);
                for (int i = lane; i < n; i += WAVE)
                    if (s_m[i] == m) s_term[i] = (c > 1 && mx > mn) ? (s_term[i] - mn) / (mx - mn) : 1.0;
            }
        }
        for (int i = lane; i < n; i += WAVE) {
            double ns;
            const double sc = s_term[i];
            const int m = s_m[i];
            if (prm.norm == FN_GLOBAL) {
                ns = prm.gmax > prm.gmin ? (sc - prm.gmin) / (prm.gmax - prm.gmin) : 1.0;
            } else if (prm.norm == FN_PRE) {
                ns = sc;
            } else if (prm.norm == FN_ZSCORE) {
                const double sd = zstd[m];
                ns = sd > 0.0 ? 1.0 / (1.0 + exp(-((sc - zmean[m]) / sd))) : 0.5;
            } else {
                ns = sc;
            }
            const double w = weight[m];
            s_w[i] = w;
            s_term[i] = w * ns;
        }
        wave_sync_lds();
        const int64_t so = seen_off ? seen_off[u] : 0;
        const int ns_seen = seen_off ? (int)(seen_off[u + 1] - so) : 0;
        for (int i = lane; i < nw; i += WAVE) {
            Cand c{-INFINITY, INT32_MAX};
            if (i < n) {
                const int32_t me = s_item[i];
                bool lead = true;
                for (int j = 0; j < i && lead; ++j) lead = s_item[j] != me;
                bool drop = !lead;
                for (int j = 0; j < ns_seen && !drop; ++j) drop = seen[so + j] == me;
                if (!drop) {
                    double acc = 0.0, tw = 0.0, mxv = -INFINITY, hs = 0.0;
                    int cnt = 0;
                    for (int j = i; j < n; ++j) {
                        if (s_item[j] != me) continue;
                        const double t = s_term[j], w = s_w[j];
                        ++cnt;
                        switch (prm.strategy) {
                            case FS_MAX: mxv = cnt == 1 ? t : fmax(mxv, t); break;
                            case FS_HARM: hs += 1.0 / (t + 1e-8); break;
                            case FS_RRF: acc += w / (double)(60 + s_rank[j]); break;
                            case FS_WAVG: tw += w; acc += t; break;
                            default: acc += t; break;
                        }
                    }
                    double merged;
                    switch (prm.strategy) {
                        case FS_WSUM: merged = acc; break;
                        case FS_MAX: merged = mxv; break;
                        case FS_HARM: merged = (double)cnt / hs; break;
                        case FS_DIV: merged = acc * (1.0 + (double)cnt * 0.1); break;
                        case FS_RRF: merged = acc; break;
                        default: merged = tw > 0.0 ? acc / tw : 0.0; break;
                    }
                    c = Cand{merged, i};
                }
            }
            x[i] = c;
        }
        wave_lds_sort(x, nw);
        int kept = 0;
        for (int i = lane; i < prm.topk; i += WAVE) {
            const bool ok = i < nw && x[i].row != INT32_MAX;
            out_item[u * prm.topk + i] = ok ? s_item[x[i].row] : -1;
            out_score[u * prm.topk + i] = ok ? x[i].s : 0.0;
            kept += ok ? 1 : 0;
        }
        for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o, WAVE);
        if (lane == 0) out_cnt[u] = kept;
        wave_sync_lds();
    }
}

__global__ void fuse_minmax_kernel(const double* __restrict__ score, int64_t n, double* __restrict__ out) {
    // out[0] = min, out[1] = max over all entries (one workgroup, fixed order)
    __shared__ double smn[256], smx[256];
    double mn = INFINITY, mx = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        mn = fmin(mn, score[i]);
        mx = fmax(mx, score[i]);
    }
    smn[threadIdx.x] = mn;
    smx[threadIdx.x] = mx;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d) {
            smn[threadIdx.x] = fmin(smn[threadIdx.x], smn[threadIdx.x + d]);
            smx[threadIdx.x] = fmax(smx[threadIdx.x], smx[threadIdx.x + d]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = smn[0];
        out[1] = smx[0];
    }
}

}  // namespace nrk

using namespace nrk;

extern "C" {

int nrk_fuse_minmax(const double* score, int64_t n, double* out_minmax, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n >= 1, "need at least one score");
    NRK_REQUIRE(score && out_minmax, "null pointer");
    fuse_minmax_kernel<<<1, 256, 0, as_stream(stream)>>>(score, n, out_minmax);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_fuse(const int64_t* offsets, int64_t n_users, const int32_t* item, const double* score,
             const int32_t* method, const int32_t* rank, int n_methods, const double* weight, int strategy,
             int norm, double gmin, double gmax, const double* zmean, const double* zstd, const int64_t* seen_off,
             const int32_t* seen, int topk, int32_t* out_item, double* out_score, int32_t* out_cnt,
             nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_users >= 0, "n_users must be >= 0");
    NRK_REQUIRE(n_methods >= 1, "n_methods must be >= 1");
    NRK_REQUIRE(strategy >= 0 && strategy <= 5, "strategy must be in [0, 5]");
    NRK_REQUIRE(norm >= 0 && norm <= 3, "norm must be 0 (local), 1 (global), 2 (z-score) or 3 (pre-normalised)");
    NRK_REQUIRE(topk >= 1 && topk <= FUSE_MAX, "topk must be in [1, 256]");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(offsets && item && score && method && rank && weight && out_item && out_score && out_cnt,
                "null pointer");
    NRK_REQUIRE(norm != 2 || (zmean && zstd), "z-score needs zmean / zstd");
    NRK_REQUIRE((seen_off == nullptr) == (seen == nullptr), "seen_off and seen go together");
    FuseParams p{strategy, norm, n_methods, topk, gmin, gmax};
    fuse_kernel<<<(int)((n_users + 3) / 4), 256, 0, as_stream(stream)>>>(
        offsets, n_users, item, score, method, rank, weight, zmean, zstd, seen_off, seen, p, out_item, out_score,
        out_cnt);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_fuse_wide(const int64_t* offsets, int64_t n_users, const int32_t* item, const double* score,
                  const int32_t* method, const int32_t* rank, int n_methods, const double* weight, int strategy,
                  int norm, double gmin, double gmax, const double* zmean, const double* zstd,
                  const int64_t* seen_off, const int32_t* seen, int max_entries, int topk, int32_t* out_item,
                  double* out_score, int32_t* out_cnt, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_users >= 0, "n_users must be >= 0");
    NRK_REQUIRE(n_methods >= 1, "n_methods must be >= 1");
    NRK_REQUIRE(strategy >= 0 && strategy <= 5, "strategy must be in [0, 5]");
    NRK_REQUIRE(norm >= 0 && norm <= 3, "norm must be 0 (local), 1 (global), 2 (z-score) or 3 (pre-normalised)");
    NRK_REQUIRE(max_entries >= 1, "max_entries must be >= 1");
    if (max_entries > FUSE_WMAX) NRK_UNSUPPORTED("more than 2048 entries for one user");
    NRK_REQUIRE(topk >= 1, "topk must be >= 1");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(offsets && item && score && method && rank && weight && out_item && out_score && out_cnt,
                "null pointer");
    NRK_REQUIRE(norm != 2 || (zmean && zstd), "z-score needs zmean / zstd");
    NRK_REQUIRE((seen_off == nullptr) == (seen == nullptr), "seen_off and seen go together");
    int nw = 64;
    while (nw < max_entries) nw <<= 1;
    const size_t lds = (size_t)nw * (sizeof(Cand) + 2 * sizeof(double) + 3 * sizeof(int32_t));
    (void)hipFuncSetAttribute((const void*)fuse_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    FuseParams p{strategy, norm, n_methods, topk, gmin, gmax};
    fuse_wide_kernel<<<(int)(n_users < 65536 ? n_users : 65536), 64, lds, as_stream(stream)>>>(
        offsets, n_users, item, score, method, rank, weight, zmean, zstd, seen_off, seen, p, nw, out_item,
        out_score, out_cnt);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
