/*
 * nrk_oracle.c -- CPU restatement of the reference's hot-path arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline) -- never as the thing measured or shipped.
 *
 * Parity pinning: every function here is checked in tests/test_oracle_golden.py
 * against fixtures produced by executing the reference itself
 * (tests/golden/make_golden.py).  At the Faiss boundary the reference's own
 * dependency (faiss-cpu>=1.7.4, pyproject.toml:21) is absent from the image,
 * so oracle_ip_topk restates the IndexFlatIP contract (exact inner product,
 * score desc, ties -> lower row, -1/-FLT_MAX padding) and is pinned through
 * the reference's recall() driven by that restated contract.
 *
 * Build: see oracle/Makefile (gcc -O2 -fopenmp -shared).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* A4: faiss.IndexFlatIP(d).add(items); .search(users, k)                    */
/* youtubednn_recaller.py:493-494 (add), :520 (search).                      */
/* Exact score: fp64, products of the fp32 inputs accumulated sequentially   */
/* over the dimension.  Order: score desc, row asc.                          */
/* ------------------------------------------------------------------------ */
static inline int better(double sa, int64_t ra, double sb, int64_t rb) {
    return sa > sb || (sa == sb && ra < rb);
}

void oracle_ip_topk(const float* users, int64_t nu, const float* items, int64_t ni, int d,
                    int k, float* out_s, int64_t* out_rows, double* out_exact, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        double* hs = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k : 1));
        int64_t* hr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(k > 0 ? k : 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int64_t u = 0; u < nu; ++u) {
            const float* q = users + u * d;
            int n = 0; /* sorted list hs[0..n) best-first */
            for (int64_t r = 0; r < ni; ++r) {
                const float* v = items + r * d;
                double s = 0.0;
                for (int t = 0; t < d; ++t) s += (double)q[t] * (double)v[t];
                s += 0.0; /* canonical +0 */
                if (n == k && !better(s, r, hs[k - 1], hr[k - 1])) continue;
                int pos = (n < k) ? n : k - 1;
                while (pos > 0 && better(s, r, hs[pos - 1], hr[pos - 1])) {
                    hs[pos] = hs[pos - 1];
                    hr[pos] = hr[pos - 1];
                    --pos;
                }
                hs[pos] = s;
                hr[pos] = r;
                if (n < k) ++n;
            }
            for (int i = 0; i < k; ++i) {
                if (i < n) {
                    out_s[u * k + i] = (float)hs[i];
                    out_rows[u * k + i] = hr[i];
                    if (out_exact) out_exact[u * k + i] = hs[i];
                } else {
                    out_s[u * k + i] = -FLT_MAX;
                    out_rows[u * k + i] = -1;
                    if (out_exact) out_exact[u * k + i] = -INFINITY;
                }
            }
        }
        free(hs);
        free(hr);
    }
}

/* ------------------------------------------------------------------------ */
/* A8: ItemCFSimilarity.calculate, item_cf.py:17-89 with WeightCalculator    */
/* weights.py:7-60.  Users in list order (ascending user id, extractors.py    */
/* :25-35), each list in click-time order.  Items are dense indices.          */
/* Output: one entry per distinct (i, j), in global first-insertion order     */
/* (which, restricted to a row, is the dict insertion order the reference's   */
/* stable sorts rely on).  row_rank[i] = order in which row i was created     */
/* (setdefault at item_cf.py:44), -1 if never.  cnt[i] = item_cnt (:43).      */
/* Values are normalised by sqrt(cnt_i * cnt_j) (:81-84).                     */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint64_t key;
    int64_t slot;
} hent_t;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

int64_t oracle_itemcf_sim(int64_t n_users, const int64_t* offsets, const int32_t* items,
                          const int64_t* ts, const double* created, int32_t n_items,
                          double loc_alpha, double loc_alpha_rev, double loc_beta,
                          double time_alpha, double created_alpha, int64_t capacity,
                          int32_t* out_i, int32_t* out_j, double* out_v, int64_t* row_rank,
                          int64_t* cnt) {
    int64_t cap = 1;
    while (cap < 2 * capacity + 16) cap <<= 1;
    hent_t* tab = (hent_t*)malloc(sizeof(hent_t) * (size_t)cap);
    for (int64_t h = 0; h < cap; ++h) tab[h].slot = -1;
    for (int32_t i = 0; i < n_items; ++i) {
        row_rank[i] = -1;
        cnt[i] = 0;
    }
    int64_t n_slots = 0, n_rows = 0;
    for (int64_t u = 0; u < n_users; ++u) {
        const int64_t b = offsets[u], L = offsets[u + 1] - offsets[u];
        const double user_penalty = 1.0 / log((double)(L + 1));
        for (int64_t l1 = 0; l1 < L; ++l1) {
            const int32_t i = items[b + l1];
            const int64_t ti = ts[b + l1];
            cnt[i] += 1;
            if (row_rank[i] < 0) row_rank[i] = n_rows++;
            for (int64_t l2 = 0; l2 < L; ++l2) {
                const int32_t j = items[b + l2];
                if (i == j) continue;
                const int64_t tj = ts[b + l2];
                const double la = (l2 > l1) ? loc_alpha : loc_alpha_rev;
                const int64_t dl = (l2 > l1 ? l2 - l1 : l1 - l2) - 1;
                const double loc_weight = la * pow(loc_beta, (double)dl);
                const int64_t dt = ti > tj ? ti - tj : tj - ti;
                const double click_w = exp(pow(time_alpha, (double)dt));
                const double created_w = exp(pow(created_alpha, fabs(created[i] - created[j])));
                const double w = loc_weight * click_w * created_w * user_penalty;
                const uint64_t key = ((uint64_t)(uint32_t)i << 32) | (uint32_t)j;
                uint64_t h = mix64(key) & (uint64_t)(cap - 1);
                while (tab[h].slot >= 0 && tab[h].key != key) h = (h + 1) & (uint64_t)(cap - 1);
                if (tab[h].slot < 0) {
                    if (n_slots >= capacity) {
                        free(tab);
                        return -1;
                    }
                    tab[h].key = key;
                    tab[h].slot = n_slots;
                    out_i[n_slots] = i;
                    out_j[n_slots] = j;
                    out_v[n_slots] = 0.0;
                    ++n_slots;
                }
                out_v[tab[h].slot] += w;
            }
        }
    }
    for (int64_t s = 0; s < n_slots; ++s)
        out_v[s] = out_v[s] / sqrt((double)(cnt[out_i[s]] * cnt[out_j[s]]));
    free(tab);
    return n_slots;
}

/* The same similarity on T OpenMP threads (a CPU baseline variant for
 * bench.py's ItemCF leg, not a checker).  Thread t owns the rows i with
 * i % T == t: it walks every user list in order but only accumulates the
 * pairs of its own rows, so each (i, j) sum sees its terms in the sequential
 * order and the values are bit-identical to oracle_itemcf_sim's.  Thread t
 * writes its entries (its own first-insertion order) to
 * out[base[t] .. base[t] + n[t]); base[t] is the prefix of the per-thread
 * pair counts (an upper bound on its distinct pairs).  The caller sizes the
 * outputs for sum(L^2) entries.  Returns the total number of entries. */
int64_t oracle_itemcf_sim_omp(int64_t n_users, const int64_t* offsets, const int32_t* items,
                              const int64_t* ts, const double* created, int32_t n_items,
                              double loc_alpha, double loc_alpha_rev, double loc_beta,
                              double time_alpha, double created_alpha, int nthreads,
                              int32_t* out_i, int32_t* out_j, double* out_v, int64_t* base,
                              int64_t* n_out) {
    int T = nthreads > 0 ? nthreads : 1;
    int64_t* cnt = (int64_t*)calloc((size_t)n_items, sizeof(int64_t));
    int64_t* need = (int64_t*)calloc((size_t)T, sizeof(int64_t));
    for (int64_t u = 0; u < n_users; ++u) {
        const int64_t b = offsets[u], L = offsets[u + 1] - b;
        for (int64_t l = 0; l < L; ++l) {
            cnt[items[b + l]] += 1;
            need[items[b + l] % T] += L;
        }
    }
    int64_t acc = 0;
    for (int t = 0; t < T; ++t) {
        base[t] = acc;
        acc += need[t];
    }
#ifdef _OPENMP
#pragma omp parallel num_threads(T)
#endif
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num();
#else
        const int t = 0;
#endif
        int64_t cap = 1;
        while (cap < 2 * need[t] + 16) cap <<= 1;
        hent_t* tab = (hent_t*)malloc(sizeof(hent_t) * (size_t)cap);
        for (int64_t h = 0; h < cap; ++h) tab[h].slot = -1;
        int32_t* oi = out_i + base[t];
        int32_t* oj = out_j + base[t];
        double* ov = out_v + base[t];
        int64_t n = 0;
        for (int64_t u = 0; u < n_users; ++u) {
            const int64_t b = offsets[u], L = offsets[u + 1] - offsets[u];
            const double user_penalty = 1.0 / log((double)(L + 1));
            for (int64_t l1 = 0; l1 < L; ++l1) {
                const int32_t i = items[b + l1];
                if (i % T != t) continue;
                const int64_t ti = ts[b + l1];
                for (int64_t l2 = 0; l2 < L; ++l2) {
                    const int32_t j = items[b + l2];
                    if (i == j) continue;
                    const int64_t tj = ts[b + l2];
                    const double la = (l2 > l1) ? loc_alpha : loc_alpha_rev;
                    const int64_t dl = (l2 > l1 ? l2 - l1 : l1 - l2) - 1;
                    const double loc_weight = la * pow(loc_beta, (double)dl);
                    const int64_t dt = ti > tj ? ti - tj : tj - ti;
                    const double click_w = exp(pow(time_alpha, (double)dt));
                    const double created_w = exp(pow(created_alpha, fabs(created[i] - created[j])));
                    const double w = loc_weight * click_w * created_w * user_penalty;
                    const uint64_t key = ((uint64_t)(uint32_t)i << 32) | (uint32_t)j;
                    uint64_t h = mix64(key) & (uint64_t)(cap - 1);
                    while (tab[h].slot >= 0 && tab[h].key != key) h = (h + 1) & (uint64_t)(cap - 1);
                    if (tab[h].slot < 0) {
                        tab[h].key = key;
                        tab[h].slot = n;
                        oi[n] = i;
                        oj[n] = j;
                        ov[n] = 0.0;
                        ++n;
                    }
                    ov[tab[h].slot] += w;
                }
            }
        }
        for (int64_t s = 0; s < n; ++s) ov[s] = ov[s] / sqrt((double)(cnt[oi[s]] * cnt[oj[s]]));
        n_out[t] = n;
        free(tab);
    }
    int64_t tot = 0;
    for (int t = 0; t < T; ++t) tot += n_out[t];
    free(cnt);
    free(need);
    return tot;
}

/* ------------------------------------------------------------------------ */
/* A9: ItemCFRecaller._precompute_topk_similar_items, itemcf_recaller.py     */
/* :41-54: per row, stable sort by score desc (ties keep insertion order),    */
/* keep the first `topn`.  Input: CSR rows (entries in insertion order).      */
/* ------------------------------------------------------------------------ */
static void stable_sort_desc(double* s, int32_t* it, int64_t n, double* ts, int32_t* ti) {
    /* bottom-up merge sort; stable for equal keys */
    for (int64_t w = 1; w < n; w <<= 1) {
        for (int64_t lo = 0; lo < n; lo += 2 * w) {
            int64_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
            int64_t a = lo, b = mid, o = lo;
            while (a < mid && b < hi) {
                if (s[b] > s[a]) { ts[o] = s[b]; ti[o++] = it[b++]; }
                else { ts[o] = s[a]; ti[o++] = it[a++]; }
            }
            while (a < mid) { ts[o] = s[a]; ti[o++] = it[a++]; }
            while (b < hi) { ts[o] = s[b]; ti[o++] = it[b++]; }
        }
        memcpy(s, ts, sizeof(double) * (size_t)n);
        memcpy(it, ti, sizeof(int32_t) * (size_t)n);
    }
}

void oracle_topn_rows(int64_t n_rows, const int64_t* row_off, const int32_t* cols,
                      const double* vals, int topn, int32_t* out_cols, double* out_vals,
                      int32_t* out_cnt) {
    int64_t maxlen = 0;
    for (int64_t r = 0; r < n_rows; ++r)
        if (row_off[r + 1] - row_off[r] > maxlen) maxlen = row_off[r + 1] - row_off[r];
    double* s = (double*)malloc(sizeof(double) * (size_t)(maxlen + 1));
    double* ts = (double*)malloc(sizeof(double) * (size_t)(maxlen + 1));
    int32_t* it = (int32_t*)malloc(sizeof(int32_t) * (size_t)(maxlen + 1));
    int32_t* ti = (int32_t*)malloc(sizeof(int32_t) * (size_t)(maxlen + 1));
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t n = row_off[r + 1] - row_off[r];
        memcpy(s, vals + row_off[r], sizeof(double) * (size_t)n);
        memcpy(it, cols + row_off[r], sizeof(int32_t) * (size_t)n);
        stable_sort_desc(s, it, n, ts, ti);
        const int64_t m = n < topn ? n : topn;
        for (int64_t q = 0; q < m; ++q) {
            out_cols[r * topn + q] = it[q];
            out_vals[r * topn + q] = s[q];
        }
        out_cnt[r] = (int32_t)m;
    }
    free(s); free(ts); free(it); free(ti);
}

/* ------------------------------------------------------------------------ */
/* A10: ItemCFRecaller.recall, itemcf_recaller.py:56-129 (no embedding        */
/* content weight).  q_slot[q] = index of the user's list in the CSR, or -1   */
/* for an unknown user (cold start :68-70).  nbr: per dense item, its top-N   */
/* (j, w_ij) in stable-sorted order (A9).  Output per query: up to topk       */
/* (item, score), counts in out_cnt.                                          */
/* ------------------------------------------------------------------------ */
void oracle_itemcf_recall(int64_t n_query, const int64_t* q_slot, const int64_t* offsets,
                          const int32_t* items, const int32_t* nbr_cols,
                          const double* nbr_vals, const int32_t* nbr_cnt, int topn,
                          const double* created, const int32_t* hot, int n_hot, int topk,
                          double loc_beta, double created_alpha, int32_t n_items,
                          int32_t* out_items, double* out_scores, int32_t* out_cnt) {
    int32_t* pos = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_items); /* item -> rank idx */
    char* inhist = (char*)calloc((size_t)n_items, 1);
    for (int32_t i = 0; i < n_items; ++i) pos[i] = -1;
    int64_t maxc = 16;
    for (int64_t q = 0; q < n_query; ++q)
        if (q_slot[q] >= 0) {
            int64_t L = offsets[q_slot[q] + 1] - offsets[q_slot[q]];
            if (L * topn + n_hot + 16 > maxc) maxc = L * topn + n_hot + 16;
        }
    int32_t* cj = (int32_t*)malloc(sizeof(int32_t) * (size_t)maxc);
    double* cs = (double*)malloc(sizeof(double) * (size_t)maxc);
    int32_t* tj = (int32_t*)malloc(sizeof(int32_t) * (size_t)maxc);
    double* tsb = (double*)malloc(sizeof(double) * (size_t)maxc);
    for (int64_t q = 0; q < n_query; ++q) {
        int32_t* oi = out_items + q * topk;
        double* os = out_scores + q * topk;
        if (q_slot[q] < 0) {
            int m = n_hot < topk ? n_hot : topk;
            for (int x = 0; x < m; ++x) { oi[x] = hot[x]; os[x] = (double)(-x); }
            out_cnt[q] = m;
            continue;
        }
        const int64_t b = offsets[q_slot[q]], L = offsets[q_slot[q] + 1] - b;
        for (int64_t l = 0; l < L; ++l) inhist[items[b + l]] = 1;
        int64_t n = 0;
        for (int64_t loc = 0; loc < L; ++loc) {
            const int32_t i = items[b + loc];
            for (int x = 0; x < nbr_cnt[i]; ++x) {
                const int32_t j = nbr_cols[(int64_t)i * topn + x];
                const double wij = nbr_vals[(int64_t)i * topn + x];
                if (inhist[j]) continue;
                const double cw = exp(pow(created_alpha, fabs(created[i] - created[j])));
                const double lw = pow(loc_beta, (double)(L - loc));
                const double content = 1.0;
                if (pos[j] < 0) { pos[j] = (int32_t)n; cj[n] = j; cs[n] = 0.0; ++n; }
                cs[pos[j]] += cw * lw * content * wij;
            }
        }
        if (n < topk) {
            for (int x = 0; x < n_hot; ++x) {
                const int32_t it = hot[x];
                if (pos[it] >= 0 || inhist[it]) continue;
                pos[it] = (int32_t)n; cj[n] = it; cs[n] = (double)(-x - 100); ++n;
                if (n == topk) break;
            }
        }
        for (int64_t x = 0; x < n; ++x) pos[cj[x]] = -1;
        stable_sort_desc(cs, cj, n, tsb, tj);
        const int64_t m = n < topk ? n : topk;
        for (int64_t x = 0; x < m; ++x) { oi[x] = cj[x]; os[x] = cs[x]; }
        out_cnt[q] = (int32_t)m;
        for (int64_t l = 0; l < L; ++l) inhist[items[b + l]] = 0;
    }
    free(pos); free(inhist); free(cj); free(cs); free(tj); free(tsb);
}
