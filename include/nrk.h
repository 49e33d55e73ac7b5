/*
 * nrk.h -- C ABI of libnrk.so, the MI355X-native recall + rank hot path.
 *
 * Every entry point:
 *   - takes caller-owned DEVICE buffers (plain pointers + sizes, row-major,
 *     contiguous) and an explicit HIP stream (hipStream_t passed as void*);
 *   - is asynchronous on that stream, performs no hidden allocation, no host
 *     synchronisation and no hipMalloc/hipMemcpy (graph-capturable); scratch
 *     comes from a caller workspace sized by the matching *_bytes() query;
 *   - returns NRK_OK (0) or an error code; nrk_last_error() gives a
 *     thread-local message.  No C++ exception crosses the ABI.
 *
 * The reference (qiqiqicheng/news-recommendation-tc) is pure Python with no
 * FFI of its own; each function below names the reference call site it
 * replaces (paths relative to the reference root).  The Python plugins in
 * news-recommendation-tc_amd/nrk bind these through ctypes; INTEGRATION.md
 * shows the binding a reference maintainer would add.
 */
#ifndef NRK_H
#define NRK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* nrk_stream_t; /* hipStream_t */

#define NRK_OK 0
#define NRK_EINVAL 1       /* bad argument (shape, null pointer, size)      */
#define NRK_EHIP 2         /* HIP runtime error (launch / device)           */
#define NRK_EUNSUPPORTED 3 /* configuration outside the compiled variants   */

const char* nrk_last_error(void);
/* ABI version 3 (round 5): the round-3 CSR owner protocol
 * (nrk_ip_topk_screen_range, nrk_ip_topk_band_pack, nrk_ip_topk_refine_csr)
 * is gone; config 4 runs shard_screen -> shard_band -> refine_x.
 * Version 2 (round 4): nrk_ip_topk_bound takes k before m (the screen's k, so
 * the bound pass knows the list length); the packed catalog carries a
 * half-block-major fp16 copy after its header (nrk_ip_catalog_bytes grew);
 * nrk_din_remap_index added; DIN item features 1, 2, 4 or 8.  A caller built
 * against an older version must be rebuilt. */
#define NRK_ABI_VERSION 3
int nrk_abi_version(void);

/* ---------------------------------------------------------------------- */
/* YouTubeDNN two-tower forward                                           */
/* ---------------------------------------------------------------------- */

/* User tower, eval mode.  Replaces YoutubeDNN.forward / get_user_embedding
 * (src/recall/youtubednn_recaller.py:129-182) as driven by
 * _extract_embeddings (:425-470), INCLUDING the host-side numpy
 * re-normalisation with zero-norm -> 1 (:467-470):
 *   x   = [E_u[uid] ; sum_{t<len} E_i[hist_t] / (len + 1e-8)]
 *   x   = ReLU(W1 ReLU(W0 x + b0) + b1)          (dropout = identity)
 *   out = renorm(x / max(||x||, 1e-12))
 * dim in {16, 32, 64}; h0 <= 128; h1 == dim.  hist is [n, seq_len]. */
int nrk_tt_user_fwd(const float* user_table, int64_t n_user_rows, const float* item_table,
                    int64_t n_item_rows, int dim, const int32_t* uid, const int32_t* hist,
                    const int32_t* hist_len, int64_t n, int seq_len, const float* w0,
                    const float* b0, int h0, const float* w1, const float* b1, int h1,
                    float* out, nrk_stream_t stream);

/* Item tower.  Replaces get_item_embedding (:184-188) + numpy re-norm
 * (:485-489): out[r] = renorm(normalize(E_i[ids[r]])). */
/* The user tower at any depth (youtubednn_hidden_units of any length,
 * youtubednn_recaller.py:105-112): weights packed per layer as W_l
 * [widths[l], in_l] row-major then b_l [widths[l]] (in_0 = 2 * dim), 1 to 8
 * layers of width <= 256, the last equal to dim.  Same outputs as
 * nrk_tt_user_fwd for two layers. */
int nrk_tt_user_fwd_layers(const float* user_table, int64_t n_user_rows, const float* item_table,
                           int64_t n_item_rows, int dim, const int32_t* uid, const int32_t* hist,
                           const int32_t* hist_len, int64_t n, int seq_len, const float* weights, int n_layers,
                           const int* widths, float* out, nrk_stream_t stream);
int nrk_tt_item_fwd(const float* item_table, int64_t n_item_rows, int dim, const int32_t* ids,
                    int64_t n, float* out, nrk_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Brute-force inner-product top-K (replaces faiss.IndexFlatIP)           */
/* ---------------------------------------------------------------------- */

/* Catalog = the "index": an fp16 copy of the item rows (power-of-two scaled)
 * in MFMA-fragment order, a header (max row norm, scale, max rounding error)
 * and, for dim <= 64, a half-block-major fp16 copy read by the refine's
 * prefilter.  Replaces faiss.IndexFlatIP(d).add(items)
 * (youtubednn_recaller.py:493-494).  items stays the fp32 source of truth
 * for exact rescoring and must outlive the catalog. */
size_t nrk_ip_catalog_bytes(int64_t n_items, int dim);
int nrk_ip_catalog_build(const float* items, int64_t n_items, int dim, void* catalog,
                         nrk_stream_t stream);

/* Exact top-k by inner product for every user row.  Replaces
 * faiss_index.search(user_emb, topk + 1) (youtubednn_recaller.py:520) for a
 * whole user batch at once.  Contract (same as IndexFlatIP): exact score
 * (fp64 accumulation of the fp32 products), sorted by score desc, ties ->
 * lower row; fewer than k items -> rows -1 / scores -FLT_MAX.
 * out_rows are catalog rows + row_offset (global rows of a shard).
 * out_exact (nullable) receives the fp64 scores used for ordering (the
 * merge key for catalog-sharded runs).  1 <= k <= 2048 (the fp16 MFMA screen
 * path up to k = 128, an exact radix-select path above); dim <= 256. */
size_t nrk_ip_topk_workspace_bytes(int64_t n_users, int64_t n_items, int dim, int k);
int nrk_ip_topk(const float* users, int64_t n_users, const float* items, const void* catalog,
                int64_t n_items, int dim, int k, int64_t row_offset, float* out_scores,
                int32_t* out_rows, double* out_exact, void* workspace, size_t workspace_bytes,
                nrk_stream_t stream);

/* The two phases of nrk_ip_topk, for callers that pipeline or time them:
 * screen (fp16 MFMA scan -> per-user candidate band in the workspace) and
 * finish (exact fp64 rescoring + ordering, exact fallback for overflowed
 * users).  finish must follow screen on the same workspace.  finish reads
 * the packed catalog (may be NULL) for an fp16 prefilter of the candidate
 * band before the exact fp32-row rescoring. */
int nrk_ip_topk_screen(const float* users, int64_t n_users, const void* catalog, int64_t n_items,
                       int dim, int k, void* workspace, size_t workspace_bytes,
                       nrk_stream_t stream);
/* nrk_ip_topk_screen in its two launches (timing / profiling of the MFMA
 * scan alone): nrk_ip_topk_scan, then nrk_ip_topk_select, same arguments. */
int nrk_ip_topk_scan(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim, int k,
                     void* workspace, size_t workspace_bytes, nrk_stream_t stream);
int nrk_ip_topk_select(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim, int k,
                       void* workspace, size_t workspace_bytes, nrk_stream_t stream);
int nrk_ip_topk_finish(const float* users, int64_t n_users, const float* items,
                       const void* catalog, int64_t n_items,
                       int dim, int k, int64_t row_offset, float* out_scores, int32_t* out_rows,
                       double* out_exact, void* workspace, size_t workspace_bytes,
                       nrk_stream_t stream);

/* Catalog-sharded runs, between screen and
 * finish:
 *   nrk_ip_topk_bound (same k as the screen) writes, per user, the m
 *   (<= 256) largest exact lower
 *   bounds this shard's screen found, descending, fp32 [n_users, m], -inf
 *   padded: each one bounds a distinct item's exact score from below.
 *   After an all_gather of every shard's [n_users, m] block (layout
 *   [n_lists][n_users][m], n_lists * m <= 512), nrk_ip_topk_apply_bound takes
 *   the k-th largest of the user's n_lists * m values -- a lower bound of
 *   the user's k-th exact score over the WHOLE catalog -- and raises the
 *   shard's refine cut to it, so finish rescores only the candidates that
 *   can still reach the merged top-k (the output then holds the shard's
 *   top-k among items with exact score >= the global bound, -1 padded).
 *   k > n_lists * m leaves the cut unchanged.  New: no reference
 *   counterpart (a Faiss search is single-index). */
int nrk_ip_topk_bound(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim,
                      int k, int m, float* out_bound, void* workspace, size_t workspace_bytes,
                      nrk_stream_t stream);
int nrk_ip_topk_apply_bound(int64_t n_users, const float* bounds, int n_lists, int m, int k, void* workspace,
                            size_t workspace_bytes, nrk_stream_t stream);

/* 32-item blocks per screen tile at this dim (one LDS ring slot of the MFMA
 * scan; 8 KB, or 4 blocks = 32 KB at dims 65..128): catalog shard ranges start
 * on a tile.  0 for dim outside [1, 256].  Host-only, no device work.  New: no
 * reference counterpart (Faiss shards are whole indexes). */
int nrk_ip_topk_tile_blocks(int dim);

/* Config 4 (catalog sharded) with owner refine: every rank
 * holds the SAME packed catalog and fp32 rows (nrk_ip_catalog_build over all
 * items) and screens only its block range [blk_lo, blk_hi) (32-item blocks;
 * blk_lo a multiple of nrk_ip_topk_tile_blocks(dim), blk_hi too unless it is
 * the catalog end) for every user; half-block ids stay global.  No per-shard
 * select:
 *   nrk_ip_topk_shard_screen = the scan of [blk_lo, blk_hi) + per user the m
 *   (1..256) largest appended half-block maxima as exact lower bounds
 *   (out_bound [n_users, m] f32, descending, -inf padded; k <= 128);
 *   nrk_ip_topk_shard_band, after the all_gather of every shard's bounds
 *   (bounds [n_lists][n_users][m], n_lists * m <= 512, or NULL): cut =
 *   max(the scan's own list bound - 2 eps, k-th largest bound - eps), the
 *   appended half-blocks >= cut packed as uint32 global half-block ids to
 *   out_ent[u * x_cap + j] (x_cap in [1, 288]; out_cnt -1 when more: the
 *   user then takes the owner's exact path), and ucut written for the refine.
 * The ids and counts of each user block go to its owner in one fixed-size
 * all_to_all (nrk.dist.catalog_sharded_owner, or nrk_rccl_band_alltoall),
 * and the owner runs nrk_ip_topk_refine_x over its users: source s's ids for
 * user u at band[(s * src_users + u) * x_cap + j], j < src_cnt[s * src_users
 * + u]; ucut [n_users, 2] (cut, eps) = the owner's own shard_band values
 * for its user block (every shard's cut bounds the user's k-th exact score
 * over the whole catalog); ovf_in [n_users] (1 = exact path over the full
 * catalog).  Output = the final top-k (no merge).  New: no reference
 * counterpart. */
int nrk_ip_topk_shard_screen(const float* users, int64_t n_users, const void* catalog, int64_t n_items, int dim,
                             int k, int64_t blk_lo, int64_t blk_hi, int m, float* out_bound, void* workspace,
                             size_t workspace_bytes, nrk_stream_t stream);
int nrk_ip_topk_shard_band(int64_t n_users, int64_t n_items, int dim, int k, const float* bounds, int n_lists,
                           int m, int x_cap, void* workspace, size_t workspace_bytes, void* out_ent,
                           int32_t* out_cnt, nrk_stream_t stream);
int nrk_ip_topk_refine_x(const float* users, int64_t n_users, const float* items, const void* catalog,
                         int64_t n_items, int dim, int k, int64_t row_offset, const void* band, int n_src,
                         int64_t src_users, int x_cap, const int32_t* src_cnt, const float* ucut,
                         const int32_t* ovf_in, float* out_scores, int32_t* out_rows, double* out_exact,
                         void* workspace, size_t workspace_bytes, nrk_stream_t stream);

/* Merge n_lists per-shard top-k_in lists (fp64 exact scores + global rows,
 * list l of user u at [l * list_stride + u * k_in]) into the top-k_out by
 * (score desc, row asc).  New: the catalog-sharded multi-GPU merge
 * (SURVEY.md §8e); n_lists * k_in <= 1024. */
int nrk_topk_merge(const double* in_exact, const int32_t* in_rows, int n_lists,
                   int64_t list_stride, int64_t n_users, int k_in, int k_out, float* out_scores,
                   int32_t* out_rows, double* out_exact, nrk_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Embedding similarity (the second Faiss site)                           */
/* ---------------------------------------------------------------------- */

/* out[r] = x[r] / ||x[r]||, bit-identical to numpy's float32
 *   item_emb_np / np.linalg.norm(item_emb_np, axis=1, keepdims=True)
 * (src/similarity/embedding.py:41; pairwise float32 sum of squares, correctly
 * rounded sqrt and division).  norms (nullable) receives ||x[r]||.  The
 * self-search that follows (embedding.py:46-50) is nrk_ip_topk with
 * users == items == out.  dim <= 256; out may not alias x. */
int nrk_row_normalize(const float* x, int64_t n, int dim, float* out, float* norms,
                      nrk_stream_t stream);

/* ---------------------------------------------------------------------- */
/* ItemCF co-occurrence similarity                                        */
/* ---------------------------------------------------------------------- */

/* Replaces ItemCFSimilarity.calculate (src/similarity/item_cf.py:17-89).
 * Input: user click lists in CSR (users in ascending id order, each list in
 * click-time order = UserFeatureExtractor.get_user_item_time_dict,
 * src/data/extractors.py:10-36), dense item ids, raw ms timestamps, and the
 * MinMax-scaled created time per dense item (float64).
 * Pass 1 (nrk_itemcf_pair_offsets): per-user pair-slot offsets
 * (pair_off[u] = sum_{v<u} L_v^2, pair_off[n_users] = total) -- the caller
 * reads the total to size the workspace and outputs.
 * Pass 2 (nrk_itemcf_sim): one entry per distinct (i, j), sorted by (i, j):
 * normalised similarity (fp64, per-pair weights summed in the reference's
 * order), first-encounter slot (the dict insertion order that the
 * reference's stable sorts use as tie-break) and item_cnt per dense item.
 * *out_n (device int64) receives the number of entries. */
int nrk_itemcf_pair_offsets(const int64_t* offsets, int64_t n_users, int64_t* pair_off,
                            nrk_stream_t stream);
size_t nrk_itemcf_workspace_bytes(int64_t n_pairs, int32_t n_items);
int nrk_itemcf_sim(const int64_t* offsets, int64_t n_users, const int32_t* items,
                   const int64_t* ts, const double* created, int32_t n_items,
                   const int64_t* pair_off, int64_t n_pairs, double loc_alpha,
                   double loc_alpha_rev, double loc_beta, double time_alpha,
                   double created_alpha, int32_t* out_i, int32_t* out_j, double* out_v,
                   int64_t* out_first, int64_t* out_n, int64_t* out_cnt, void* workspace,
                   size_t workspace_bytes, nrk_stream_t stream);

/* Per-row top-n of the similarity CSR by (score desc, first-encounter asc):
 * replaces ItemCFRecaller._precompute_topk_similar_items
 * (src/recall/itemcf_recaller.py:41-54).  row_off has n_rows + 1 entries.
 * Outputs [n_rows, topn] (-1 / 0 padded) and counts. topn <= 64. */
int nrk_itemcf_topn(const int64_t* row_off, int64_t n_rows, const int32_t* cols,
                    const double* vals, const int64_t* first, int topn, int32_t* out_cols,
                    double* out_vals, int32_t* out_cnt, nrk_stream_t stream);

/* Users-sharded ItemCF: each rank owns a contiguous user range
 * and items are owned by contiguous id ranges; one exchange step.
 * nrk_itemcf_pairs: the pair tuples of the rank's users -- key (i << b | j),
 * b = smallest with 2^b > n_items (sentinel for i == j), the pair's GLOBAL
 * slot (slot_base + local slot; the global slot order is the reference's
 * S[i][j] += w order), weight -- as nrk_itemcf_sim computes them, and the
 * rank's click counts (item_cnt += ; caller zeroes).  pair_off from
 * nrk_itemcf_pair_offsets over the rank's users.
 * nrk_itemcf_reduce: the owner's pass over the tuples it received, in global
 * slot order (all_to_all concatenates sources in rank order): one entry per
 * distinct key, (i, j), sum / sqrt(cnt_i cnt_j) with the all-reduced counts,
 * first slot.  Same results as nrk_itemcf_sim on one GPU. */
int nrk_itemcf_pairs(const int64_t* offsets, int64_t n_users, const int32_t* items, const int64_t* ts,
                     const double* created, int32_t n_items, const int64_t* pair_off, int64_t slot_base,
                     double loc_alpha, double loc_alpha_rev, double loc_beta, double time_alpha,
                     double created_alpha, uint64_t* keys, int32_t* slots, double* w, int64_t* item_cnt,
                     nrk_stream_t stream);
size_t nrk_itemcf_reduce_workspace_bytes(int64_t n);
int nrk_itemcf_reduce(const uint64_t* keys, const int32_t* slots, const double* w, int64_t n, int32_t n_items,
                      const int64_t* item_cnt, int32_t* out_i, int32_t* out_j, double* out_v,
                      int64_t* out_first, int64_t* out_n, void* workspace, size_t workspace_bytes,
                      nrk_stream_t stream);

/* CSR row offsets (n_rows + 1) of nrk_itemcf_sim's entries, which are sorted
 * by i: row_off[r] = number of entries with i < r. */
int nrk_itemcf_row_offsets(const int32_t* ei, int64_t n, int64_t n_rows, int64_t* row_off,
                           nrk_stream_t stream);

/* ItemCFRecaller.recall for a batch of query users (replaces the per-user
 * host loop of src/recall/itemcf_recaller.py:56-129).  Dense item ids; the
 * user click lists in CSR (offsets, items; the history order of
 * user_item_time_dict); q_slot[q] = the query's row in that CSR or -1 for an
 * unknown user (cold start, :68-70).  nbr_*: per item its top-n neighbours
 * [n_items, topn] from nrk_itemcf_topn (A9).  emb_* (ke = 0: none): per item
 * up to ke embedding neighbours (EmbeddingSimilarity, the content weight of
 * :98-103).  hot: item_topk_click (dense), the fill order of :116-122.
 * Pass 1 (nrk_itemcf_recall_offsets): cand_off[q] = exclusive prefix of the
 * candidate counts, cand_off[n_query] = n_cand (read it to size the
 * workspace).  Pass 2: per query up to topk (item, score) sorted like
 * sorted(item_rank.items(), key=score, reverse=True)[:topk] -- ties in dict
 * insertion order; out_src = 0 scored candidate, 1 hot fill (-x - 100),
 * 2 cold start (-x), -1 padding.  topk <= 64. */
int nrk_itemcf_recall_offsets(const int64_t* q_slot, int64_t n_query, const int64_t* offsets,
                              const int32_t* items, const int32_t* nbr_cnt, int64_t* cand_off,
                              nrk_stream_t stream);
size_t nrk_itemcf_recall_workspace_bytes(int64_t n_cand);
int nrk_itemcf_recall(const int64_t* q_slot, int64_t n_query, const int64_t* offsets, const int32_t* items,
                      const int32_t* nbr_cols, const double* nbr_vals, const int32_t* nbr_cnt, int topn,
                      const double* created, int32_t n_items, const int32_t* hot, int n_hot,
                      const int32_t* emb_cols, const double* emb_vals, const int32_t* emb_cnt, int ke,
                      double loc_beta, double created_alpha, const int64_t* cand_off, int64_t n_cand,
                      int topk, int32_t* out_items, double* out_scores, int32_t* out_src,
                      int32_t* out_cnt, void* workspace, size_t workspace_bytes, nrk_stream_t stream);

/* ---------------------------------------------------------------------- */
/* DIN attention-over-history scorer                                      */
/* ---------------------------------------------------------------------- */

/* DINModel.forward (src/rank/DIN.py:214-286) in eval mode for one batch,
 * as DINRanker.predict drives it (DIN.py:1219-1283).  Dice uses the batch
 * statistics (mean, unbiased std over the batch, DIN.py:39-44), so a batch
 * is the unit of work and the caller batches exactly like the reference.
 *
 * Embedding tables: all per-feature nn.Embedding(vocab, 32) tables
 * concatenated row-wise into one table (fp32: table_dtype 0, bf16: 1);
 * feature f's row r lives at row_base[f] + r.  Feature order: user features
 * [0, n_user), item features [n_user, n_user + n_item) (shared by the
 * candidate and the history), context features after them.
 * Index tensors are int32: user [B, n_user], item [B, n_item],
 * hist [B, T, n_item], ctx [B, n_ctx]; mask [B, T] float (1 valid, 0 pad).
 * Weights (fp32, the state_dict tensors): att_w0 [36, 4*n_item*32],
 * att_b0 [36], att_w1 [36], att_b1 [1]; mlp_w0 [h1, in], mlp_b0 [h1],
 * mlp_w1 [h2, h1], mlp_b1 [h2], mlp_w2 [h2], mlp_b2 [1]
 * with in = 32 * (n_user + n_ctx + 2 * n_item).
 * nrk_din_prepare derives the batch-invariant attention matrices, the
 * power-of-two scales of the split-fp16 attention products (from max|table|),
 * the packed weight fragments and (bf16 tables) an fp16 copy of the table at
 * that scale, once per weight load into prep (nrk_din_prep_bytes(n_item,
 * n_table_rows)); call it again if the table changes.  B >= 2 (B = 1 is NaN in the
 * reference too). */
/* Embedding widths other than 32 (din_embedding_dim, src/utils/config.py:115,
 * read back by DINRanker.load_model, DIN.py:1371-1379): the kernels read
 * 32-wide VIRTUAL features.  The host zero-pads every table to
 * m = ceil(D / 32) * 32 columns, views it as [m * vocab, 32] (feature f's
 * index i -> virtual indices m i + h, h < m), expands att_w0 / mlp_w0 with
 * zero columns at the padded positions, and pads the item features with a
 * shared all-zero row up to 1, 2, 4 or 8.  nrk_din_remap_index maps caller
 * index rows [n_rows, f_in] to the virtual layout [n_rows, f_out]:
 * out[r, j] = map[j] < 0 ? map[2 f_out + j]
 *                        : in[r, map[j]] * map[f_out + j] + map[2 f_out + j]
 * (map: int32 device array, rows src | mul | add).  Identity when D = 32 and
 * the item-feature count is 1, 2, 4 or 8 (no call needed). */
int nrk_din_remap_index(const int32_t* in, int64_t n_rows, int f_in, const int32_t* map, int f_out,
                        int32_t* out, nrk_stream_t stream);
size_t nrk_din_prep_bytes(int n_item, int64_t n_table_rows);
int nrk_din_prepare(const float* att_w0, int n_item, const void* table, int table_dtype,
                    int64_t n_table_rows, void* prep, nrk_stream_t stream);
size_t nrk_din_workspace_bytes(int64_t batch, int seq_len, int n_user, int n_item, int n_ctx,
                               int h1, int h2);
int nrk_din_forward(const void* table, int table_dtype, const int64_t* row_base, int n_user,
                    int n_item, int n_ctx, const int32_t* user_idx, const int32_t* item_idx,
                    const int32_t* hist_idx, const int32_t* ctx_idx, const float* mask,
                    int64_t batch, int seq_len, const void* prep, const float* att_b0,
                    const float* att_w1, const float* att_b1, const float* mlp_w0,
                    const float* mlp_b0, int h1, const float* mlp_w1, const float* mlp_b1,
                    int h2, const float* mlp_w2, const float* mlp_b2, float* out_probs,
                    float* out_logits, void* workspace, size_t workspace_bytes,
                    nrk_stream_t stream);

/* The whole of DINRanker.predict (DIN.py:1245-1283) in one call: n_samples
 * rows scored as consecutive Dice batches of seg_len (the DataLoader's
 * batch_size, shuffle=False), each batch with its own statistics -- the
 * same result as nrk_din_forward once per batch, with every batch's phases
 * in one launch each.  seg_len >= n_samples is one batch (n_samples >= 2);
 * otherwise seg_len must be a multiple of 64.  A trailing batch of a single
 * row has no std (NaN in the reference): its output is unspecified here and
 * the caller marks it NaN.  Index tensors are [n_samples, ...] as above. */
size_t nrk_din_segments_workspace_bytes(int64_t n_samples, int64_t seg_len, int seq_len, int n_user,
                                        int n_item, int n_ctx, int h1, int h2);
int nrk_din_forward_segments(const void* table, int table_dtype, const int64_t* row_base, int n_user,
                             int n_item, int n_ctx, const int32_t* user_idx, const int32_t* item_idx,
                             const int32_t* hist_idx, const int32_t* ctx_idx, const float* mask,
                             int64_t n_samples, int64_t seg_len, int seq_len, const void* prep,
                             const float* att_b0, const float* att_w1, const float* att_b1,
                             const float* mlp_w0, const float* mlp_b0, int h1, const float* mlp_w1,
                             const float* mlp_b1, int h2, const float* mlp_w2, const float* mlp_b2,
                             float* out_probs, float* out_logits, void* workspace,
                             size_t workspace_bytes, nrk_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Recall -> rank hand-off (fused config 5)                               */
/* ---------------------------------------------------------------------- */

/* Builds the DIN index tensors of the recalled pairs of users [u0, u0 + nu)
 * on the device -- the counterpart of the host feature assembly and
 * encoding (src/features/feature_extractor.py:440-723, src/rank/DIN.py:330-520)
 * for the fused pipeline.  rec_rows / rec_scores [n_users, k_in] from
 * nrk_ip_topk; pair p = (u - u0) * k_use + c uses recall column c + skip
 * (skip = 1 drops rank 0 as youtubednn_recaller.py:524 does).  user_feat
 * [n_users, n_user], item_feat [n_items, n_item] table indices; user_hist
 * [n_users, T] item rows (left-aligned, hist_len valid).  Outputs
 * out_user [P, n_user], out_item [P, n_item], out_hist [P, T, n_item]
 * (0 on padding), out_ctx [P, n_ctx] (ctx 0 = recall-score bin + 1, the
 * rest hash bins + 1), out_mask [P, T], out_cand [P] (candidate item row). */
int nrk_din_assemble(const int32_t* rec_rows, const float* rec_scores, int64_t n_users, int k_in, int skip,
                     int k_use, const int32_t* user_feat, int n_user, const int32_t* item_feat,
                     int64_t n_items, int n_item, const int32_t* user_hist, const int32_t* hist_len, int T,
                     int n_ctx, int ctx_bins, float score_lo, float score_hi, uint32_t seed, int64_t u0,
                     int64_t nu, int32_t* out_user, int32_t* out_item, int32_t* out_hist, int32_t* out_ctx,
                     float* out_mask, int32_t* out_cand, nrk_stream_t stream);

/* Row gather of 4-byte words (int32 codes or f32 mask values): out[b] =
 * src[idx[b]] (row_words words per row), zeros when idx[b] is outside
 * [0, n_rows).  The device half of the vectorised DIN encoder
 * (nrk/rank/encode.py): DINDataset.__getitem__ + collate_fn (src/rank/
 * DIN.py:358-520) look every sample's user profile, candidate item features
 * and last-T history up in per-user / per-item dicts; here those lookups
 * become row indices into encoded tables resident in HBM. */
int nrk_gather_rows(const void* src, int64_t n_rows, int row_words, const int32_t* idx, int64_t n, void* out,
                    nrk_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Recall fusion                                                          */
/* ---------------------------------------------------------------------- */

/* RecallFusion.fuse (src/recall/fusion.py:267-342) for every user at once.
 * Entries of all recall methods' lists grouped by user (offsets [n_users+1]),
 * inside a user in method order then list order: item (dense int32 code),
 * raw score (f64), method index, position in its list.  weight [n_methods].
 * strategy: 0 weighted_sum, 1 weighted_avg, 2 max_score, 3 harmonic_mean,
 * 4 diversity_weighted, 5 rrf (:189-265).  norm: 0 local (per list min-max,
 * :71-98), 1 global (gmin / gmax from nrk_fuse_minmax, :100-134), 2 z-score
 * (zmean / zstd per method, :136-187; device exp), 3 pre-normalised (the
 * caller passes the normalised scores: the Python wrapper computes the
 * z-score sigmoid with numpy exactly as the reference does).  Optional
 * seen_off / seen: per-user item codes removed after the merge (:320-326).
 * Output: the top-k items by (merged score desc, first appearance asc) --
 * the reference's stable sort of its insertion-ordered dict -- -1 padded,
 * and the count per user.  nrk_fuse takes users of at most 256 entries: a
 * user with more gets out_cnt = -1 (padded output); nrk_fuse_wide takes any
 * user of at most max_entries (<= 2048) entries, any topk. */
int nrk_fuse_minmax(const double* score, int64_t n, double* out_minmax, nrk_stream_t stream);
int nrk_fuse(const int64_t* offsets, int64_t n_users, const int32_t* item, const double* score,
             const int32_t* method, const int32_t* rank, int n_methods, const double* weight, int strategy,
             int norm, double gmin, double gmax, const double* zmean, const double* zstd, const int64_t* seen_off,
             const int32_t* seen, int topk, int32_t* out_item, double* out_score, int32_t* out_cnt,
             nrk_stream_t stream);
int nrk_fuse_wide(const int64_t* offsets, int64_t n_users, const int32_t* item, const double* score,
                  const int32_t* method, const int32_t* rank, int n_methods, const double* weight, int strategy,
                  int norm, double gmin, double gmax, const double* zmean, const double* zstd,
                  const int64_t* seen_off, const int32_t* seen, int max_entries, int topk, int32_t* out_item,
                  double* out_score, int32_t* out_cnt, nrk_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Ranker context features                                                */
/* ---------------------------------------------------------------------- */

/* FeatureExtractor._extract_context_features
 * (src/features/feature_extractor.py:440-723) for every (user, recalled
 * item) row, then the fitted binning (_apply_binning :838-898) and context
 * LabelEncoder codes (src/rank/DIN.py:330-353, :560-617).  Features per row,
 * F = 1 + 3 * last_n + 6 (16 at last_n = 3), in feature_lists order:
 *   score, (sim_i, time_diff_i, word_diff_i) i = 1..last_n, sim_max,
 *   sim_mean, sim_min, sim_std, item_user_sim, recall_in_user_cat.
 * Rows are processed in user groups (group_off / pair_pos); tables are
 * indexed by dense user / item rows.  Outputs (either may be NULL):
 * out_raw [n_rows, F] f64 (the reference's column values: float32 features
 * exactly representable, NaN where the reference leaves NaN) and out_codes
 * [n_rows, code_stride] int32 (spec[f] applied to feature f). */
typedef struct {
    int64_t n_groups;           /* user groups                                      */
    const int64_t* group_off;   /* [n_groups + 1] into the grouped pair order       */
    const int32_t* group_user;  /* [n_groups] user row (-1: no such user)           */
    const int64_t* pair_pos;    /* [n_pairs] output row of grouped pair q (NULL: q) */
    const int32_t* pair_item;   /* [n_rows] item row of output row (-1: unknown)    */
    const double* pair_score;   /* [n_rows] recall score                            */
    int32_t last_n;             /* history items used (config.last_N = 3), <= 4     */
    int32_t code_stride;        /* row stride of out_codes (>= F)                   */
    const int32_t* hist_last;   /* [n_users, last_n] last items, oldest first, -1 = unknown item */
    const int32_t* hist_n;      /* [n_users] min(len, last_n); -1 = no history entry */
    const int64_t* ucat_off;    /* [n_users + 1] */
    const int32_t* ucat;        /* distinct categories of each user's whole history */
    const float* user_yt;       /* [n_users, dy] YouTubeDNN user vectors, or NULL   */
    const uint8_t* user_yt_ok;  /* [n_users] */
    int64_t n_items;
    const float* w2v;           /* [n_items, dw] article-id Word2Vec vectors        */
    const uint8_t* w2v_ok;      /* [n_items] */
    int32_t dw;
    const double* content;      /* [n_items, dc] content embeddings (float64)       */
    const uint8_t* content_flags; /* bit 0 row present, bit 1 f32 row not all zero */
    int32_t dc;
    const double* created;      /* [n_items] MinMax created time, NaN = missing     */
    const int32_t* category;    /* [n_items] category, -1 = missing                 */
    const float* item_yt;       /* [n_items, dy] YouTubeDNN item vectors            */
    const uint8_t* item_yt_ok;  /* [n_items] */
    int32_t dy;
} nrk_ctx_tables;

/* One feature's fitted encoding.  kind 0 (KBins-binned): NaN -> fill, bin =
 * #(edges[k] <= value) over the inner edges, code = lut[bin] (0 past n_lut).
 * kind 1 (unbinned): code = codes[k] where vals[k] == value, else 0. */
typedef struct {
    int32_t kind, n_edges, n_lut, n_vals;
    double fill;
    double edges[16];
    double vals[32];
    int32_t lut[32];
    int32_t codes[32];
} nrk_ctx_spec;

int nrk_ctx_features(const nrk_ctx_tables* tables, const nrk_ctx_spec* spec, double* out_raw, int32_t* out_codes,
                     nrk_stream_t stream);

/* ---- multi-GPU exchanges over RCCL --------
 * For a caller binding the C ABI without torch.distributed: one process per
 * GPU; rank 0 makes a unique id (nrk_rccl_unique_id_bytes() bytes), the
 * caller sends it to every rank, each rank calls nrk_rccl_comm_init with its
 * device current.  Communicators are opaque (void*).
 * nrk_rccl_topk_allgather: the merge protocol -- all-gather every shard's
 *   top-k_in of every user (fp64 + global row) into the caller's
 *   gather_exact / gather_rows [n_ranks][n_users][k_in], then nrk_topk_merge.
 *   Replaces: nothing (a Faiss search is single-index).
 * nrk_rccl_bound_allgather / nrk_rccl_band_alltoall: the owner protocol's
 *   two exchanges (bounds [n_users, m] f32; counts [n_ranks * per] and
 *   x_cap ids per user, user block o to rank o), around
 *   nrk_ip_topk_shard_screen / _shard_band / _refine_x. */
int nrk_rccl_unique_id_bytes(void);
int nrk_rccl_get_unique_id(void* out_id);
int nrk_rccl_comm_init(void** out_comm, int n_ranks, const void* id, int rank);
int nrk_rccl_comm_destroy(void* comm);
int nrk_rccl_topk_allgather(void* comm, const double* in_exact, const int32_t* in_rows, int64_t n_users, int k_in,
                            int k_out, double* gather_exact, int32_t* gather_rows, float* out_scores,
                            int32_t* out_rows, double* out_exact, nrk_stream_t stream);
int nrk_rccl_bound_allgather(void* comm, const float* bounds, int64_t n_users, int m, float* out,
                             nrk_stream_t stream);
int nrk_rccl_band_alltoall(void* comm, const int32_t* cnt, const int32_t* ids, int64_t per, int x_cap,
                           int32_t* out_cnt, int32_t* out_ids, nrk_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* NRK_H */
