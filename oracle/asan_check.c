/*
 * asan_check.c -- drives every entry point of nrk_oracle.c under
 * AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5's optional
 * host sanitizer build; `make -C oracle asan`, run by
 * tests/test_oracle_sanitizers.py).  TEST INFRASTRUCTURE ONLY: a host
 * program, no GPU.
 *
 * Inputs: small random cases plus the edges the reference's paths have
 * (k > n_items padding, all-tie users, empty and one-click users, repeated
 * clicks, unknown / cold-start users, rows shorter than top-n).  Besides
 * running clean, the checks are internal consistency: the OpenMP ItemCF
 * similarity has the sequential one's entry count, oracle_topn_rows is
 * sorted (score desc, insertion order), ip_topk rows are (score desc, row
 * asc) with -1 padding.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_ip_topk(const float* users, int64_t nu, const float* items, int64_t ni, int d, int k, float* out_s,
                    int64_t* out_rows, double* out_exact, int nthreads);
int64_t oracle_itemcf_sim(int64_t n_users, const int64_t* offsets, const int32_t* items, const int64_t* ts,
                          const double* created, int32_t n_items, double loc_alpha, double loc_alpha_rev,
                          double loc_beta, double time_alpha, double created_alpha, int64_t capacity,
                          int32_t* out_i, int32_t* out_j, double* out_v, int64_t* row_rank, int64_t* cnt);
int64_t oracle_itemcf_sim_omp(int64_t n_users, const int64_t* offsets, const int32_t* items, const int64_t* ts,
                              const double* created, int32_t n_items, double loc_alpha, double loc_alpha_rev,
                              double loc_beta, double time_alpha, double created_alpha, int nthreads,
                              int32_t* out_i, int32_t* out_j, double* out_v, int64_t* base, int64_t* n_out);
void oracle_topn_rows(int64_t n_rows, const int64_t* row_off, const int32_t* cols, const double* vals, int topn,
                      int32_t* out_cols, double* out_vals, int32_t* out_cnt);
void oracle_itemcf_recall(int64_t n_query, const int64_t* q_slot, const int64_t* offsets, const int32_t* items,
                          const int32_t* nbr_cols, const double* nbr_vals, const int32_t* nbr_cnt, int topn,
                          const double* created, const int32_t* hot, int n_hot, int topk, double loc_beta,
                          double created_alpha, int32_t n_items, int32_t* out_items, double* out_scores,
                          int32_t* out_cnt);

static uint64_t rs = 88172645463325252ull;
static uint64_t rnd(void) {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}
static double urand(void) { return (double)(rnd() >> 11) / 9007199254740992.0; }

#define FAIL(...)                          \
    do {                                   \
        fprintf(stderr, __VA_ARGS__);      \
        fprintf(stderr, "\n");             \
        exit(1);                           \
    } while (0)

static void check_topk(int64_t nu, int64_t ni, int d, int k, int ties) {
    float* u = malloc(sizeof(float) * (size_t)(nu * d + 1));
    float* it = malloc(sizeof(float) * (size_t)(ni * d + 1));
    for (int64_t i = 0; i < nu * d; ++i) u[i] = (float)(urand() - 0.5);
    for (int64_t i = 0; i < ni * d; ++i) it[i] = ties ? (float)((int)(urand() * 4) - 2) : (float)(urand() - 0.5);
    if (nu > 1)
        for (int e = 0; e < d; ++e) u[d + e] = 0.0f; /* all-tie user */
    float* s = malloc(sizeof(float) * (size_t)(nu * k));
    int64_t* r = malloc(sizeof(int64_t) * (size_t)(nu * k));
    double* x = malloc(sizeof(double) * (size_t)(nu * k));
    oracle_ip_topk(u, nu, it, ni, d, k, s, r, x, 2);
    for (int64_t q = 0; q < nu; ++q)
        for (int j = 0; j < k; ++j) {
            const int64_t row = r[q * k + j];
            if (j >= ni) {
                if (row != -1) FAIL("ip_topk: padding row %lld", (long long)row);
                continue;
            }
            if (row < 0 || row >= ni) FAIL("ip_topk: row out of range");
            if (j > 0) {
                const double a = x[q * k + j - 1], b = x[q * k + j];
                if (a < b || (a == b && r[q * k + j - 1] >= row)) FAIL("ip_topk: order at user %lld", (long long)q);
            }
        }
    free(u); free(it); free(s); free(r); free(x);
}

static void check_itemcf(int64_t n_users, int32_t n_items, int maxlen) {
    int64_t* off = malloc(sizeof(int64_t) * (size_t)(n_users + 1));
    off[0] = 0;
    for (int64_t u = 0; u < n_users; ++u) off[u + 1] = off[u] + (u % 7 == 0 ? 0 : (int64_t)(rnd() % (maxlen + 1)));
    const int64_t n = off[n_users];
    int32_t* items = malloc(sizeof(int32_t) * (size_t)(n + 1));
    int64_t* ts = malloc(sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t i = 0; i < n; ++i) {
        items[i] = (int32_t)(rnd() % (uint64_t)n_items);
        ts[i] = 1500000000000ll + i * (int64_t)(rnd() % 50);
    }
    if (n > 3) items[1] = items[0]; /* repeated click */
    double* created = malloc(sizeof(double) * (size_t)n_items);
    for (int32_t i = 0; i < n_items; ++i) created[i] = urand();
    int64_t pairs = 0;
    for (int64_t u = 0; u < n_users; ++u) pairs += (off[u + 1] - off[u]) * (off[u + 1] - off[u]);
    const int64_t cap = pairs + 1;
    int32_t *oi = malloc(4 * (size_t)cap), *oj = malloc(4 * (size_t)cap);
    double* ov = malloc(8 * (size_t)cap);
    int64_t* rank = malloc(8 * (size_t)n_items);
    int64_t* cnt = malloc(8 * (size_t)n_items);
    const int64_t m = oracle_itemcf_sim(n_users, off, items, ts, created, n_items, 1.0, 0.7, 0.9, 0.7, 0.8, cap,
                                        oi, oj, ov, rank, cnt);
    int32_t *pi = malloc(4 * (size_t)cap), *pj = malloc(4 * (size_t)cap);
    double* pv = malloc(8 * (size_t)cap);
    int64_t* base = malloc(8 * (size_t)(n_items + 1));
    int64_t* nout = malloc(8 * (size_t)(n_items + 1));
    const int64_t m2 = oracle_itemcf_sim_omp(n_users, off, items, ts, created, n_items, 1.0, 0.7, 0.9, 0.7, 0.8, 3,
                                             pi, pj, pv, base, nout);
    if (m2 != m) FAIL("itemcf: omp entries %lld vs %lld", (long long)m2, (long long)m);
    /* per-row CSR of the sequential result (rows by first encounter) for top-n */
    int64_t* row_off = calloc((size_t)n_items + 1, sizeof(int64_t));
    for (int64_t e = 0; e < m; ++e) row_off[oi[e] + 1]++;
    for (int32_t i = 0; i < n_items; ++i) row_off[i + 1] += row_off[i];
    int64_t* fill = calloc((size_t)n_items, sizeof(int64_t));
    int32_t* cols = malloc(4 * (size_t)(m + 1));
    double* vals = malloc(8 * (size_t)(m + 1));
    for (int64_t e = 0; e < m; ++e) {
        const int64_t p = row_off[oi[e]] + fill[oi[e]]++;
        cols[p] = oj[e];
        vals[p] = ov[e];
    }
    const int topn = 5;
    int32_t* tc = malloc(4 * (size_t)n_items * topn);
    double* tv = malloc(8 * (size_t)n_items * topn);
    int32_t* tn = malloc(4 * (size_t)n_items);
    oracle_topn_rows(n_items, row_off, cols, vals, topn, tc, tv, tn);
    for (int32_t i = 0; i < n_items; ++i) {
        const int64_t len = row_off[i + 1] - row_off[i];
        if (tn[i] != (len < topn ? len : topn)) FAIL("topn: count");
        for (int q = 1; q < tn[i]; ++q)
            if (tv[i * topn + q - 1] < tv[i * topn + q]) FAIL("topn: order");
    }
    /* recall: every user + two cold-start users */
    const int64_t nq = n_users + 2;
    int64_t* qs = malloc(8 * (size_t)nq);
    for (int64_t q = 0; q < nq; ++q) qs[q] = q < n_users ? q : -1;
    int32_t hot[7];
    for (int h = 0; h < 7; ++h) hot[h] = (int32_t)(rnd() % (uint64_t)n_items);
    const int topk = 9;
    int32_t* ri = malloc(4 * (size_t)nq * topk);
    double* rsc = malloc(8 * (size_t)nq * topk);
    int32_t* rc = malloc(4 * (size_t)nq);
    oracle_itemcf_recall(nq, qs, off, items, tc, tv, tn, topn, created, hot, 7, topk, 0.9, 0.8, n_items, ri, rsc,
                         rc);
    for (int64_t q = 0; q < nq; ++q) {
        if (rc[q] < 0 || rc[q] > topk) FAIL("recall: count");
        for (int j = 0; j < rc[q]; ++j)
            if (ri[q * topk + j] < 0 || ri[q * topk + j] >= n_items) FAIL("recall: item");
    }
    free(off); free(items); free(ts); free(created); free(oi); free(oj); free(ov); free(rank); free(cnt);
    free(pi); free(pj); free(pv); free(base); free(nout); free(row_off); free(fill); free(cols); free(vals);
    free(tc); free(tv); free(tn); free(qs); free(ri); free(rsc); free(rc);
}

int main(void) {
    check_topk(37, 500, 32, 31, 0);
    check_topk(20, 300, 16, 61, 1);   /* heavy ties */
    check_topk(5, 7, 8, 12, 0);       /* k > n_items: -1 padding */
    check_topk(3, 1000, 250, 21, 0);  /* EmbeddingSimilarity's width */
    check_itemcf(300, 200, 12);
    check_itemcf(50, 20, 40);         /* dense: many repeated pairs */
    check_itemcf(9, 5000, 1);         /* one click per user: no pairs */
    printf("asan_check OK\n");
    return 0;
}
