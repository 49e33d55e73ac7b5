// assemble.hip -- recall -> rank hand-off on the device (BASELINE config 5).
//
// The reference builds the DIN inputs of every recalled (user, item) pair
// on the host: FeatureExtractor assembles context features per pair
// (src/features/feature_extractor.py:440-723) and DINDataset / collate_fn
// encode them (src/rank/DIN.py:330-520): user profile indices, candidate
// item indices, the user's last T history items (left-aligned, mask 1 on
// valid slots, index 0 = padding) and 16 binned context features.  For the
// fused pipeline those tensors are built here, straight from the recall
// output in HBM, for a chunk of users:
//   pair p = (u - u0) * k_use + c  <-  recall row c + skip of user u;
//   ctx[0] = the recall score's bin (ctx_bins equal-width bins over
//   [score_lo, score_hi], + 1: 0 stays "unknown"), ctx[f > 0] = a hash bin of
//   (user, item, f, seed) -- the real context features come from host ETL
//   (SURVEY 8f #2), the synthetic ones keep the same shapes and vocabularies.
// One wave per pair (grid-strided); the history block (T x n_item int32) is
// written coalesced.  Pure integer/byte work: HBM-bound, no MFMA.
#include "nrk_common.h"

namespace nrk {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void din_assemble_kernel(
    const int32_t* __restrict__ rec_rows, const float* __restrict__ rec_scores, int k_in, int skip,
    int k_use, const int32_t* __restrict__ user_feat, int n_user, const int32_t* __restrict__ item_feat,
    int n_item, const int32_t* __restrict__ user_hist, const int32_t* __restrict__ hist_len, int T,
    int n_ctx, int ctx_bins, float score_lo, float score_hi, uint32_t seed, int64_t u0, int64_t n_pairs,
    int32_t* __restrict__ out_user, int32_t* __restrict__ out_item, int32_t* __restrict__ out_hist,
    int32_t* __restrict__ out_ctx, float* __restrict__ out_mask, int32_t* __restrict__ out_cand) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const float inv = ctx_bins / (score_hi - score_lo);
    for (int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < n_pairs; p += nw) {
        const int64_t u = u0 + p / k_use;
        const int c = (int)(p % k_use) + skip;
        const int32_t row = rec_rows[u * k_in + c];
        const int32_t item = row >= 0 ? row : 0;
        const int L = hist_len[u];
        if (lane < n_user) out_user[p * n_user + lane] = user_feat[u * n_user + lane];
        if (lane < n_item) out_item[p * n_item + lane] = item_feat[(int64_t)item * n_item + lane];
        if (lane == 0) out_cand[p] = row;
        if (lane < n_ctx) {
            int32_t v;
            if (lane == 0) {
                const float s = rec_scores[u * k_in + c];
                int bin = (int)floorf((s - score_lo) * inv);
                bin = bin < 0 ? 0 : bin >= ctx_bins ? ctx_bins - 1 : bin;
                v = bin + 1;
            } else {
                const uint32_t h = mix32((uint32_t)u * 0x9e3779b9u ^ mix32((uint32_t)item + 0x85ebca6bu * (uint32_t)lane) ^ seed);
                v = (int32_t)(h % (uint32_t)ctx_bins) + 1;
            }
            out_ctx[p * n_ctx + lane] = v;
        }
        for (int t = lane; t < T; t += 64) out_mask[p * T + t] = t < L ? 1.0f : 0.0f;
        const int HN = T * n_item;
        for (int e = lane; e < HN; e += 64) {
            const int t = e / n_item, f = e - t * n_item;
            const int32_t hrow = user_hist[u * T + t];
            out_hist[p * HN + e] = t < L ? item_feat[(int64_t)hrow * n_item + f] : 0;
        }
    }
}

// Row gather of 4-byte words: out[b] = idx[b] in [0, n_rows) ? src[idx[b]] : 0.
// One thread per (row, word), rows of W words contiguous in both buffers:
// consecutive threads write consecutive words (coalesced stores); the reads
// are W-word runs of random rows (the tables are small and cache-resident).
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint32_t* __restrict__ src, int64_t n_rows, int W,
                                                          const int32_t* __restrict__ idx, int64_t n,
                                                          uint32_t* __restrict__ out) {
    const int64_t total = n * W;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / W;
        const int w = (int)(e - b * W);
        const int32_t r = idx[b];
        out[e] = (r >= 0 && r < n_rows) ? src[(int64_t)r * W + w] : 0u;
    }
}

}  // namespace nrk

using namespace nrk;

extern "C" {

int nrk_din_assemble(const int32_t* rec_rows, const float* rec_scores, int64_t n_users, int k_in, int skip,
                     int k_use, const int32_t* user_feat, int n_user, const int32_t* item_feat,
                     int64_t n_items, int n_item, const int32_t* user_hist, const int32_t* hist_len, int T,
                     int n_ctx, int ctx_bins, float score_lo, float score_hi, uint32_t seed, int64_t u0,
                     int64_t nu, int32_t* out_user, int32_t* out_item, int32_t* out_hist, int32_t* out_ctx,
                     float* out_mask, int32_t* out_cand, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_users >= 0 && nu >= 0 && u0 >= 0 && u0 + nu <= n_users, "user range out of bounds");
    NRK_REQUIRE(k_in >= 1 && skip >= 0 && k_use >= 1 && skip + k_use <= k_in, "bad k_in / skip / k_use");
    NRK_REQUIRE(n_user >= 1 && n_user <= 64 && n_item >= 1 && n_item <= 64 && n_ctx >= 0 && n_ctx <= 64,
                "feature counts must be in [1, 64] (ctx [0, 64])");
    NRK_REQUIRE(T >= 1 && n_items >= 1, "T and n_items must be >= 1");
    NRK_REQUIRE(ctx_bins >= 1 && score_hi > score_lo, "bad context bins");
    if (nu == 0) return NRK_OK;
    NRK_REQUIRE(rec_rows && rec_scores && user_feat && item_feat && user_hist && hist_len && out_user &&
                    out_item && out_hist && out_mask && out_cand && (n_ctx == 0 || out_ctx),
                "null pointer");
    const int64_t n_pairs = nu * k_use;
    const int64_t g = (n_pairs + 3) / 4;
    din_assemble_kernel<<<(int)(g < 65536 ? g : 65536), 256, 0, as_stream(stream)>>>(
        rec_rows, rec_scores, k_in, skip, k_use, user_feat, n_user, item_feat, n_item, user_hist, hist_len, T,
        n_ctx, ctx_bins, score_lo, score_hi, seed, u0, n_pairs, out_user, out_item, out_hist, out_ctx,
        out_mask, out_cand);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_gather_rows(const void* src, int64_t n_rows, int row_words, const int32_t* idx, int64_t n, void* out,
                    nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_rows >= 0 && n >= 0 && row_words >= 1, "bad sizes");
    if (n == 0) return NRK_OK;
    NRK_REQUIRE(idx && out && (src || n_rows == 0), "null pointer");
    const int64_t total = n * row_words;
    const int64_t g = (total + 255) / 256;
    gather_rows_kernel<<<(int)(g < 65536 ? g : 65536), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const uint32_t*>(src), n_rows, row_words, idx, n, reinterpret_cast<uint32_t*>(out));
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
