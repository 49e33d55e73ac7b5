// itemcf.hip -- ItemCF co-occurrence similarity on gfx950.
//
// Reference: ItemCFSimilarity.calculate, src/similarity/item_cf.py:17-89,
// weights from src/utils/weights.py:7-60 (time_decay_weight, log_penalty);
// top-n per item: ItemCFRecaller._precompute_topk_similar_items,
// src/recall/itemcf_recaller.py:41-54.
//
// The reference walks users in dict order, then (loc1, loc2) and does
// S[i][j] += w.  Every ordered position pair (u, loc1, loc2) therefore has a
// global sequence number ("slot") = pair_off[u] + loc1 * L_u + loc2, and the
// reference's fp64 sum for (i, j) is the sum of its pair weights in slot
// order.  The GPU reproduces exactly that order without a hash table:
//   1. cf_pairs_flat   flat over the slots, CF_CHUNK per wave: weight
//                      w[slot] and key (i << b | j) per slot (i == j ->
//                      sentinel); cf_item_count: item_cnt.
//   2. LSD radix sort  of (key, slot) -- stable, so equal keys keep slot
//                      order (rs_upsweep / rs_scan_rows / rs_downsweep,
//                      8 bits per pass, 2b bits total).
//   3. cf_tile_reduce / cf_carry_scan / cf_emit
//                      one entry per distinct key: fp64 sum of w[slot] over
//                      the key's run (slot order within a thread chunk, fixed
//                      segmented-scan association across chunks and tiles),
//                      / sqrt(cnt_i * cnt_j), and the first slot (= dict
//                      insertion order, the reference's stable-sort tie-break).
// Memory-bound integer/byte work: no MFMA; tiles of 4096 keys per 256-thread
// workgroup, coalesced 16-element strips.
#include "nrk_common.h"

#include <climits>
#include <cmath>

namespace nrk {

constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;  // 4096 keys per workgroup
constexpr int CF_WIDE_MAX = 2048;  // largest topn / topk (wide LDS path above 64)
constexpr int64_t CF_HEAVY = 4096;               // top-n rows longer than this get a workgroup
// LDS tile images of 4096 8-byte values read as thread-contiguous chunks of
// 16: one pad slot per 16 keeps the chunk reads free of bank conflicts
__device__ __forceinline__ int cf_pad(int i) { return i + (i >> 4); }
constexpr int CF_SW = RS_TILE + RS_TILE / 16;

// ------------------------------------------------------ pair offsets --
// Exclusive int64 scans over users / queries (pair_off[u] = sum_{v<u} L_v^2,
// the recall's candidate offsets): one workgroup of 1024 threads walks tiles
// of 8,192 values -- coalesced loads into LDS, one thread-contiguous chunk of
// 8 per thread, a wave shuffle scan + 16 wave totals, coalesced stores -- and
// carries the running total.  No workspace (the C ABI of these two entry
// points has none, and the library allocates nothing), in place when the
// values alias out (every tile is loaded before it is written); out[n] = total.
// Round 1's version read one 245-value chunk per thread, chunk-strided
// (0.52 ms at 250k users).
struct ScanPairs {  // L_u^2 from the CSR offsets
    const int64_t* offsets;
    __device__ int64_t operator()(int64_t u) const {
        const int64_t L = offsets[u + 1] - offsets[u];
        return L * L;
    }
};
struct ScanVals {
    const int64_t* v;
    __device__ int64_t operator()(int64_t u) const { return v[u]; }
};

constexpr int SCAN_PT = 8, SCAN_TILE = 1024 * SCAN_PT;

template <typename F>
__global__ __launch_bounds__(1024) void scan_exclusive_kernel(F f, int64_t n, int64_t* out) {  // out may alias f's values
    __shared__ int64_t sv[SCAN_TILE + SCAN_TILE / 16];
    __shared__ int64_t wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int64_t carry = 0;
    // the next tile's values load while this one is scanned (round 6: one
    // load round trip per tile was most of the time; tiles never overlap, so
    // an aliased out is still read before it is written)
    int64_t v[SCAN_PT];
#pragma unroll
    for (int j = 0; j < SCAN_PT; ++j) {
        const int64_t e = j * 1024 + tid;
        v[j] = e < n ? f(e) : 0;
    }
    for (int64_t t0 = 0; t0 < n; t0 += SCAN_TILE) {
#pragma unroll
        for (int j = 0; j < SCAN_PT; ++j) sv[cf_pad(j * 1024 + tid)] = v[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SCAN_PT; ++j) {
            const int64_t e = t0 + SCAN_TILE + j * 1024 + tid;
            v[j] = e < n ? f(e) : 0;
        }
        int64_t c[SCAN_PT], sum = 0;
#pragma unroll
        for (int r = 0; r < SCAN_PT; ++r) {
            c[r] = sv[cf_pad(tid * SCAN_PT + r)];
            sum += c[r];
        }
        int64_t x = sum;  // inclusive over the wave
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        int64_t wbase = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const int64_t t = wsum[w];
            wbase += w < wv ? t : 0;
            total += t;
        }
        int64_t run = carry + wbase + x - sum;
#pragma unroll
        for (int r = 0; r < SCAN_PT; ++r) {
            sv[cf_pad(tid * SCAN_PT + r)] = run;
            run += c[r];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SCAN_PT; ++j) {
            const int64_t e = t0 + j * 1024 + tid;
            if (e < n) out[e] = sv[cf_pad(j * 1024 + tid)];
        }
        carry += total;
        __syncthreads();  // sv / wsum are rewritten by the next tile
    }
    if (tid == 0) out[n] = carry;
}

// ------------------------------------------------------------- 1. pairs --
struct CfParams {
    double loc_alpha, loc_alpha_rev, loc_beta, time_alpha, created_alpha;
    int64_t dt_zero;  // |dt| >= dt_zero -> pow(time_alpha, dt) is +0 (cf_dt_zero)
    double ln_time, ln_created;  // cf_ln of the two alphas
};

// Smallest |dt| from which time_alpha^|dt| lies below 2^-1100 for every dt
// at or past it: any faithfully rounded pow returns +0 there, so the
// kernels skip the pow (and exp(+0) = 1 exactly) -- bit-identical to
// evaluating it.  Click timestamps are milliseconds (0.7^dt underflows from
// dt ~ 2,100 ms on), so this is nearly every pair.  No shortcut unless
// 0 < time_alpha < 1.
// The two time-decay factors are exp(alpha^x) (weights.py time_decay_weight).
// Round 6 evaluates alpha^x as exp(x ln alpha) with ln alpha formed once on
// the host: the device pow re-derives log(alpha) in double-double on every
// call, most of its cost, in the kernel that spends its time on these
// factors.  The exponent carries an absolute error <= |y| 2^-52 (y = x ln
// alpha), so alpha^x is off by a relative |y| 2^-52 and exp(alpha^x) by
// e^y |y| 2^-52 <= 2^-52 / e relative: below half an ulp of the factor (the
// ItemCF bar is rtol 1e-12; device and host libm already differ by an ulp).
// ln is NaN (-> the device pow) unless alpha is positive and finite.
static inline double cf_ln(double alpha) {
    return alpha > 0.0 && std::isfinite(alpha) ? std::log(alpha) : NAN;
}
__device__ __forceinline__ double cf_apow(double alpha, double ln_alpha, double x) {
    return ln_alpha == ln_alpha ? exp(x * ln_alpha) : pow(alpha, x);
}

static inline int64_t cf_dt_zero(double time_alpha) {
    if (!(time_alpha > 0.0 && time_alpha < 1.0)) return INT64_MAX;
    const double l2 = -std::log2(time_alpha);  // > 0
    const double d = std::ceil(1100.0 / l2) + 1.0;
    return d < 9.0e18 ? (int64_t)d : INT64_MAX;
}

// item_cnt[i] += the occurrences of i in the users' clicks (item_cf.py:43,
// cnt[i] += 1 per occurrence).  Round 5 counted with one global atomic per
// click from the pairs kernel: a popular item's counter took tens of
// thousands of same-address atomics in a row, 1.65 of that kernel's 1.89 ms.
// Here a workgroup folds 4,096 clicks into an LDS hash table (open
// addressing, load <= 1/2) and adds each distinct item's count once: a hot
// item's counter sees one atomic per chunk.
constexpr int CF_CNT_CHUNK = 4096;
constexpr int CF_CNT_SLOTS = 8192;
constexpr int CF_CNT_THREADS = 512;

__global__ __launch_bounds__(CF_CNT_THREADS) void cf_item_count_kernel(const int64_t* __restrict__ offsets,
                                                                     int64_t n_users,
                                                                     const int32_t* __restrict__ items,
                                                                     unsigned long long* __restrict__ cnt) {
    __shared__ int32_t hk[CF_CNT_SLOTS];
    __shared__ uint32_t hc[CF_CNT_SLOTS];
    const int64_t c0 = offsets[0], c1 = offsets[n_users];
    for (int64_t a = c0 + (int64_t)blockIdx.x * CF_CNT_CHUNK; a < c1; a += (int64_t)gridDim.x * CF_CNT_CHUNK) {
        for (int t = threadIdx.x; t < CF_CNT_SLOTS; t += CF_CNT_THREADS) {
            hk[t] = -1;
            hc[t] = 0;
        }
        __syncthreads();
        const int64_t e1 = a + CF_CNT_CHUNK < c1 ? a + CF_CNT_CHUNK : c1;
        for (int64_t e = a + threadIdx.x; e < e1; e += CF_CNT_THREADS) {
            const int32_t it = items[e];  // >= 0
            uint32_t t = ((uint32_t)it * 2654435761u) >> 19;  // 13-bit multiplicative hash
            for (;;) {
                const int32_t prev = atomicCAS(&hk[t], -1, it);
                if (prev == -1 || prev == it) {
                    atomicAdd(&hc[t], 1u);
                    break;
                }
                t = (t + 1) & (CF_CNT_SLOTS - 1);
            }
        }
        __syncthreads();
        for (int t = threadIdx.x; t < CF_CNT_SLOTS; t += CF_CNT_THREADS)
            if (hc[t]) atomicAdd(&cnt[hk[t]], (unsigned long long)hc[t]);
        __syncthreads();
    }
}

// cf_pairs_flat_kernel: every ordered position pair's key, global slot and
// weight, flat over the global pair index (round 6; round 5's one wave per
// user left the kernel waiting on its heaviest users -- a user with L
// clicks has L^2 pairs (a capped 250-click history: 62,500, one wave's
// ~980 serial steps of fp64 pow / exp while the average user needs 1.3).
// Here a wave takes chunks of CF_CHUNK consecutive pair slots (slot order =
// the reference's (user, loc1, loc2) order, pair_off = the exclusive scan
// of L^2) and every lane finds its pair's user in a window of 64 pair ends
// that follows the chunk.  Same keys and slots as round 5; the weights differ only by
// cf_apow's sub-ulp rounding.
constexpr int CF_CHUNK = 64 * 8;

__global__ __launch_bounds__(256) void cf_pairs_flat_kernel(
    const int64_t* __restrict__ offsets, int64_t n_users, const int32_t* __restrict__ items,
    const int64_t* __restrict__ ts, const double* __restrict__ created,
    const int64_t* __restrict__ pair_off, int64_t slot_base, CfParams prm, int bj, uint64_t sentinel,
    uint64_t* __restrict__ keys, int32_t* __restrict__ vals, double* __restrict__ w) {
    const int lane = threadIdx.x & 63;
    __shared__ double lwt[64];
    if (threadIdx.x < 64) lwt[threadIdx.x] = pow(prm.loc_beta, (double)threadIdx.x);
    __syncthreads();
    const int64_t total = pair_off[n_users];
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t c0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * CF_CHUNK; c0 < total; c0 += nw * CF_CHUNK) {
        // the chunk's first user, the largest u with pair_off[u] <= c0 (it has
        // pairs: pair_off[u + 1] > c0): a 64-ary search by the whole wave
        int64_t lo = 0, hi = n_users;  // pair_off[lo] <= c0 < pair_off[hi]
        while (hi - lo > 1) {
            const int64_t step = (hi - lo + 63) >> 6;
            const int64_t q = lo + step * lane;
            const uint64_t le = __ballot(q < hi && pair_off[q] <= c0);  // a prefix of the lanes
            const int64_t nlo = lo + step * (63 - __builtin_clzll(le));
            hi = nlo + step < hi ? nlo + step : hi;
            lo = nlo;
        }
        // a window of 64 users' pair ends, one per lane; each lane finds its
        // pair's user by a 6-step search over the window (shuffles), the
        // window moving on to the last lane's user after every 64 pairs
        int64_t ub = lo;
        int64_t wend = ub + lane < n_users ? pair_off[ub + lane + 1] : INT64_MAX;
        int64_t cu = -1, b = 0, L = 1, base = 0;
        double pen = 0.0;
        for (int it = 0; it < CF_CHUNK / 64; ++it) {
            if (c0 + it * 64 >= total) break;  // wave-uniform
            const int64_t p = c0 + it * 64 + lane;
            const bool live = p < total;
            int64_t u = -1;
            for (;;) {  // converged: the shuffles below need every lane
                int k = 0;
#pragma unroll
                for (int st = 32; st >= 1; st >>= 1)
                    if (__shfl(wend, k + st - 1, WAVE) <= p) k += st;
                if (u < 0 && k < 64) u = ub + k;
                if (!__any(live && u < 0)) break;  // users with no pairs pushed a lane past the window
                ub += 64;
                wend = ub + lane < n_users ? pair_off[ub + lane + 1] : INT64_MAX;
            }
            const int64_t un = __shfl(u, 63, WAVE);
            if (un >= 0 && un != ub) {
                ub = un;
                wend = ub + lane < n_users ? pair_off[ub + lane + 1] : INT64_MAX;
            }
            if (!live) break;
            if (u != cu) {
                cu = u;
                b = offsets[u];
                L = offsets[u + 1] - b;
                base = pair_off[u];
                // user_penalty = 1 / log_penalty(len) = 1 / log(L + 1) (item_cf.py:69-71)
                pen = 1.0 / log((double)(L + 1));
            }
            const int64_t sl = p - base;
            const bool small = L * L < (1ll << 31);  // 32-bit pair -> (l1, l2) division
            const int64_t l1 = small ? (int64_t)((uint32_t)sl / (uint32_t)L) : sl / L, l2 = sl - l1 * L;
            const int32_t i = items[b + l1], j = items[b + l2];
            uint64_t key = sentinel;
            double wt = 0.0;
            if (i != j) {
                const double la = l2 > l1 ? prm.loc_alpha : prm.loc_alpha_rev;
                const int64_t dl = (l2 > l1 ? l2 - l1 : l1 - l2) - 1;
                const double loc_w = la * (dl < 64 ? lwt[dl] : pow(prm.loc_beta, (double)dl));
                const int64_t ti = ts[b + l1], tj = ts[b + l2];
                const int64_t dt = ti > tj ? ti - tj : tj - ti;
                const double click_w = dt >= prm.dt_zero ? 1.0 : exp(cf_apow(prm.time_alpha, prm.ln_time, (double)dt));
                const double created_w = exp(cf_apow(prm.created_alpha, prm.ln_created, fabs(created[i] - created[j])));
                wt = loc_w * click_w * created_w * pen;
                key = ((uint64_t)(uint32_t)i << bj) | (uint32_t)j;
            }
            keys[p] = key;
            vals[p] = (int32_t)(slot_base + p);  // the pair's global slot
            w[p] = wt;
        }
    }
}

// ------------------------------------------------------- 2. radix sort --
// Stable LSD radix sort of (u64 key, i32 value), 8 bits per pass.
// counts is digit-major [256][nblk] so each digit's row scans contiguously.
__global__ __launch_bounds__(RS_THREADS) void rs_upsweep(const uint64_t* __restrict__ keys, int64_t n,
                                                        int shift, int nblk,
                                                        uint32_t* __restrict__ counts,
                                                        const int64_t* __restrict__ n_dev = nullptr) {
    if (n_dev) n = *n_dev;  // the count on the device (rc_query_kernel's overflow), nblk its bound
    if ((int64_t)blockIdx.x * RS_TILE >= n && n_dev) {  // past the end: an empty tile
        counts[(size_t)threadIdx.x * nblk + blockIdx.x] = 0;
        return;
    }
    __shared__ uint32_t hist[256];
    const int tid = threadIdx.x;
    hist[tid] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int r = 0; r < RS_ITEMS; ++r) {
        const int64_t e = t0 + r * RS_THREADS + tid;
        if (e < n) atomicAdd(&hist[(keys[e] >> shift) & 255], 1u);
    }
    __syncthreads();
    counts[(size_t)tid * nblk + blockIdx.x] = hist[tid];
}

// One workgroup per digit: exclusive scan of its row in place + row total.
__global__ __launch_bounds__(256) void rs_scan_rows(uint32_t* __restrict__ counts, int nblk,
                                                   uint32_t* __restrict__ totals) {
    __shared__ uint32_t part[256];
    const int tid = threadIdx.x;
    uint32_t* row = counts + (size_t)blockIdx.x * nblk;
    const int chunk = (nblk + 255) / 256;
    const int a = tid * chunk, e = a + chunk < nblk ? a + chunk : nblk;
    uint32_t s = 0;
    for (int k = a; k < e; ++k) s += row[k];
    part[tid] = s;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
        const uint32_t v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint32_t run = part[tid] - s;
    for (int k = a; k < e; ++k) {
        const uint32_t c = row[k];
        row[k] = run;
        run += c;
    }
    if (tid == 255) totals[blockIdx.x] = part[255];
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Scatter pass.  Round 6: the tile is ranked into LDS first (digit-major,
// stable: round-major input order within a digit) and then written out in
// that order, so consecutive threads store consecutive addresses of a digit's
// run (~16 keys per digit per tile) -- round 5 stored each 256-key round
// straight from the ranking, one partial line per lane.  The tile's own digit
// counts are the differences of the block-scanned counts row.  LDS: 52 KB
// (three workgroups per CU).
__global__ __launch_bounds__(RS_THREADS) void rs_downsweep(
    const uint64_t* __restrict__ kin, const int32_t* __restrict__ vin, uint64_t* __restrict__ kout,
    int32_t* __restrict__ vout, int64_t n, int shift, int nblk, const uint32_t* __restrict__ counts,
    const uint32_t* __restrict__ totals, const int64_t* __restrict__ n_dev = nullptr) {
    if (n_dev) n = *n_dev;
    if ((int64_t)blockIdx.x * RS_TILE >= n) return;  // an empty tile writes nothing
    __shared__ uint64_t sk[RS_TILE];
    __shared__ int32_t sv[RS_TILE];
    __shared__ uint32_t base[256];    // global start of digit d minus its tile-local start
    __shared__ uint16_t run[256];     // tile-local write position of digit d
    __shared__ uint16_t wc[4][256];
    const int tid = threadIdx.x, wv = tid >> 6;
    {
        // exclusive scans over the digits: the global starts (totals) and the
        // tile-local starts (this tile's counts), both in one pass
        const uint32_t t = totals[tid];
        const uint32_t cb = counts[(size_t)tid * nblk + blockIdx.x];
        const uint32_t cn = (blockIdx.x + 1 < (unsigned)nblk ? counts[(size_t)tid * nblk + blockIdx.x + 1] : t) - cb;
        uint32_t* sg = reinterpret_cast<uint32_t*>(sv);  // scan scratch (sv is filled later)
        uint32_t* sl = sg + 256;
        sg[tid] = t;
        sl[tid] = cn;
        __syncthreads();
        for (int d = 1; d < 256; d <<= 1) {
            const uint32_t vg = tid >= d ? sg[tid - d] : 0, vl = tid >= d ? sl[tid - d] : 0;
            __syncthreads();
            sg[tid] += vg;
            sl[tid] += vl;
            __syncthreads();
        }
        const uint32_t lstart = sl[tid] - cn;
        base[tid] = (sg[tid] - t) + cb - lstart;  // mod 2^32: base + local position = global position
        run[tid] = (uint16_t)lstart;
    }
    const int64_t t0 = (int64_t)blockIdx.x * RS_TILE;
    // the tile's 16 keys / values per thread, all in flight at once
    uint64_t kr[RS_ITEMS];
    int32_t vr[RS_ITEMS];
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const int64_t e = t0 + r * RS_THREADS + tid;
        kr[r] = e < n ? kin[e] : 0;
        vr[r] = e < n ? vin[e] : 0;
    }
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) wc[k][tid] = 0;
        const bool ok = t0 + r * RS_THREADS + tid < n;
        const uint64_t key = kr[r];
        const int32_t val = vr[r];
        const uint32_t d = (uint32_t)(key >> shift) & 255u;
        uint64_t m = __ballot(ok);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const bool on = (d >> bit) & 1u;
            const uint64_t bb = __ballot(on);
            m &= on ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
        __syncthreads();
        if (ok && rank == 0) wc[wv][d] = (uint16_t)__popcll(m);
        __syncthreads();
        {
            const uint32_t c0 = wc[0][tid], c1 = wc[1][tid], c2 = wc[2][tid], c3 = wc[3][tid];
            const uint32_t r0 = run[tid];
            wc[0][tid] = (uint16_t)r0;
            wc[1][tid] = (uint16_t)(r0 + c0);
            wc[2][tid] = (uint16_t)(r0 + c0 + c1);
            wc[3][tid] = (uint16_t)(r0 + c0 + c1 + c2);
            run[tid] = (uint16_t)(r0 + c0 + c1 + c2 + c3);
        }
        __syncthreads();
        if (ok) {
            const uint32_t lp = wc[wv][d] + rank;
            sk[lp] = key;
            sv[lp] = val;
        }
    }
    __syncthreads();
    const int nloc = n - t0 < RS_TILE ? (int)(n - t0) : RS_TILE;
    for (int i = tid; i < nloc; i += RS_THREADS) {
        const uint64_t key = sk[i];
        const uint32_t gp = base[(uint32_t)(key >> shift) & 255u] + (uint32_t)i;
        kout[gp] = key;
        vout[gp] = sv[i];
    }
}

// -------------------------------------------------------------- 3. emit --
__device__ __forceinline__ bool cf_head(const uint64_t* keys, int64_t e, uint64_t sentinel) {
    const uint64_t k = keys[e];
    return k != sentinel && (e == 0 || keys[e - 1] != k);
}

// Per-key sums in sorted order as a deterministic segmented reduction (a
// popular pair's run can be thousands of keys long, far too long for one
// lane): every key change starts a segment, and fp64 sums are formed per
// thread chunk (sequential), then combined across the threads of a tile and
// across tiles by segmented scans with the fixed combine
//   (f1, v1) . (f2, v2) = (f1 | f2, f2 ? v2 : v1 + v2).
// The association differs from the reference's strictly sequential
// S[i][j] += w only in rounding order (values agree to rtol 1e-12, the ItemCF
// bar), and is the same on every run.
struct SegSum {
    double v;
    int f;
};
__device__ __forceinline__ SegSum seg_combine(SegSum a, SegSum b) {
    return SegSum{b.f ? b.v : a.v + b.v, a.f | b.f};
}

// The per-thread chunks below (thread t owns keys [16t, 16t + 16) of the
// tile: the fixed association of the segmented sums) are read from LDS.  The
// tile is staged by coalesced loads first -- chunk-strided global reads (a
// 128-B stride across the lanes) re-fetched each line once per element:
//   fl[i]  = run-break (key differs from the previous one, or e = 0) | sentinel << 1
//            for keys t0 + i, i in [0, RS_TILE] (one past the tile: the
//            last-of-run test of the tile's final key);
//   sw[.]  = the weights, padded by one slot per 16 (conflict-free chunk reads).
// Keys themselves are only read at run heads / ends (once per distinct key).
constexpr int CF_FL = RS_TILE + 16;

__device__ __forceinline__ void cf_stage_flags(const uint64_t* __restrict__ keys, int64_t n, int64_t t0,
                                               uint64_t sentinel, uint8_t* fl) {
    for (int i = threadIdx.x; i <= RS_TILE; i += RS_THREADS) {
        const int64_t e = t0 + i;
        uint8_t f = 0;
        if (e < n) {
            const uint64_t k = keys[e];
            f = (uint8_t)(((e == 0 || keys[e - 1] != k) ? 1 : 0) | (k == sentinel ? 2 : 0));
        }
        fl[i] = f;
    }
}

// this thread's 16 flags (one 16-B LDS read) + the next chunk's first
__device__ __forceinline__ void cf_chunk_flags(const uint8_t* fl, int l0, uint8_t (&f)[RS_ITEMS + 1]) {
    const uint4 v = *reinterpret_cast<const uint4*>(fl + l0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) f[r] = (uint8_t)(w[r >> 2] >> (8 * (r & 3)));
    f[RS_ITEMS] = fl[l0 + RS_ITEMS];
}

// 1. per tile: emitted-head count, the tile's segmented aggregate, and the
//    gathered weights w[vals[e]] in sorted order (ws)
__global__ __launch_bounds__(RS_THREADS) void cf_tile_reduce(
    const uint64_t* __restrict__ keys, const int32_t* __restrict__ vals, const double* __restrict__ w,
    int64_t n, uint64_t sentinel, uint32_t* __restrict__ blkcnt, double* __restrict__ tail,
    int32_t* __restrict__ brk, double* __restrict__ ws, const int64_t* __restrict__ n_dev = nullptr) {
    if (n_dev) n = *n_dev;
    if ((int64_t)blockIdx.x * RS_TILE >= n) {  // an empty tile: no heads, no sum, no break
        if (threadIdx.x == 0) {
            tail[blockIdx.x] = 0.0;
            brk[blockIdx.x] = 0;
            blkcnt[blockIdx.x] = 0;
        }
        return;
    }
    __shared__ __attribute__((aligned(16))) uint8_t fl[CF_FL];
    __shared__ double sw[CF_SW];
    __shared__ double tv[RS_THREADS];
    __shared__ int tf[RS_THREADS];
    __shared__ uint32_t c;
    const int tid = threadIdx.x;
    if (tid == 0) c = 0;
    const int64_t t0 = (int64_t)blockIdx.x * RS_TILE;
    cf_stage_flags(keys, n, t0, sentinel, fl);
#pragma unroll 4
    for (int i = tid; i < RS_TILE; i += RS_THREADS) {
        const int64_t e = t0 + i;
        if (e < n) {
            const double x = w[vals[e]];
            ws[e] = x;
            sw[cf_pad(i)] = x;
        }
    }
    __syncthreads();
    const int l0 = tid * RS_ITEMS;
    const int64_t a = t0 + l0;
    uint8_t f[RS_ITEMS + 1];
    cf_chunk_flags(fl, l0, f);
    SegSum agg{0.0, 0};
    uint32_t my = 0;
    for (int r = 0; r < RS_ITEMS; ++r) {
        if (a + r >= n) break;
        const bool b = f[r] & 1;
        if (f[r] == 1) ++my;  // a run head that is not the sentinel
        agg = seg_combine(agg, SegSum{sw[cf_pad(l0 + r)], b ? 1 : 0});
    }
    tv[tid] = agg.v;
    tf[tid] = agg.f;
    __syncthreads();
    atomicAdd(&c, my);
    __syncthreads();
    if (tid == 0) {
        SegSum t{0.0, 0};
        for (int i = 0; i < RS_THREADS; ++i) t = seg_combine(t, SegSum{tv[i], tf[i]});
        tail[blockIdx.x] = t.v;
        brk[blockIdx.x] = t.f;
        blkcnt[blockIdx.x] = c;
    }
}

// 2. carry into every tile: segmented exclusive scan of the tile aggregates
__global__ __launch_bounds__(1024) void cf_carry_scan(const double* __restrict__ tail,
                                                    const int32_t* __restrict__ brk, int nblk,
                                                    double* __restrict__ carry) {
    __shared__ double pv[1024];
    __shared__ int pf[1024];
    const int tid = threadIdx.x;
    const int chunk = (nblk + 1023) / 1024;
    const int a = tid * chunk, e = a + chunk < nblk ? a + chunk : nblk;
    SegSum s{0.0, 0};
    for (int k = a; k < e; ++k) s = seg_combine(s, SegSum{tail[k], brk[k]});
    pv[tid] = s.v;
    pf[tid] = s.f;
    __syncthreads();
    for (int dd = 1; dd < 1024; dd <<= 1) {  // inclusive Hillis-Steele, fixed order
        SegSum o{0.0, 0};
        const bool has = tid >= dd;
        if (has) o = SegSum{pv[tid - dd], pf[tid - dd]};
        __syncthreads();
        if (has) {
            const SegSum m = seg_combine(o, SegSum{pv[tid], pf[tid]});
            pv[tid] = m.v;
            pf[tid] = m.f;
        }
        __syncthreads();
    }
    SegSum run = tid > 0 ? SegSum{pv[tid - 1], pf[tid - 1]} : SegSum{0.0, 0};
    for (int k = a; k < e; ++k) {
        carry[k] = run.v;
        run = seg_combine(run, SegSum{tail[k], brk[k]});
    }
}

__global__ __launch_bounds__(1024) void cf_head_scan(const uint32_t* __restrict__ blkcnt, int nblk,
                                                   uint32_t* __restrict__ blkoff, int64_t* __restrict__ out_n) {
    __shared__ uint32_t part[1024];
    const int tid = threadIdx.x;
    const int chunk = (nblk + 1023) / 1024;
    const int a = tid * chunk, e = a + chunk < nblk ? a + chunk : nblk;
    uint32_t s = 0;
    for (int k = a; k < e; ++k) s += blkcnt[k];
    part[tid] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const uint32_t v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint32_t run = part[tid] - s;
    for (int k = a; k < e; ++k) {
        blkoff[k] = run;
        run += blkcnt[k];
    }
    if (tid == 1023) *out_n = part[1023];
}

// 3. one entry per distinct key: (i, j), the run's sum (normalised by
//    sqrt(cnt_i cnt_j) when cnt is given, item_cf.py:81-84) and the first slot
//    (the dict insertion order the reference's stable sorts break ties by).
//    Round 6: the tile's heads are compacted in LDS (their tile positions and
//    sums) and written by consecutive threads to consecutive entries -- round
//    5 stored them from the per-thread chunk walk, every lane to its own line
//    of each of the four outputs.  A run that ends in a later tile gets its sum
//    from that tile (the only global scalar store left, one per tile at most).
__global__ __launch_bounds__(RS_THREADS) void cf_emit(
    const uint64_t* __restrict__ keys, const int32_t* __restrict__ vals, const double* __restrict__ ws,
    int64_t n, uint64_t sentinel, const uint32_t* __restrict__ blkoff, const double* __restrict__ carry,
    const unsigned long long* __restrict__ cnt, const int32_t* __restrict__ slots, int bj,
    int32_t* __restrict__ out_i, int32_t* __restrict__ out_j, double* __restrict__ out_v,
    int64_t* __restrict__ out_first, const int64_t* __restrict__ n_dev = nullptr) {
    if (n_dev) n = *n_dev;
    if ((int64_t)blockIdx.x * RS_TILE >= n) return;
    __shared__ __attribute__((aligned(16))) uint8_t fl[CF_FL];
    __shared__ double sw[CF_SW];  // the sorted weights, then the heads' sums
    __shared__ uint16_t hpos[RS_TILE];
    __shared__ double pv[RS_THREADS];
    __shared__ int pf[RS_THREADS];
    __shared__ uint32_t ph[RS_THREADS];
    const int tid = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * RS_TILE;
    const int nloc = n - t0 < RS_TILE ? (int)(n - t0) : RS_TILE;
    cf_stage_flags(keys, n, t0, sentinel, fl);
#pragma unroll 4
    for (int i = tid; i < nloc; i += RS_THREADS) sw[cf_pad(i)] = ws[t0 + i];
    __syncthreads();
    const int l0 = tid * RS_ITEMS;
    uint8_t f[RS_ITEMS + 1];
    cf_chunk_flags(fl, l0, f);
    double x[RS_ITEMS];
    SegSum agg{0.0, 0};
    uint32_t my = 0;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        x[r] = l0 + r < nloc ? sw[cf_pad(l0 + r)] : 0.0;
        if (l0 + r < nloc) {
            if (f[r] == 1) ++my;
            agg = seg_combine(agg, SegSum{x[r], (f[r] & 1) ? 1 : 0});
        }
    }
    pv[tid] = agg.v;
    pf[tid] = agg.f;
    ph[tid] = my;
    __syncthreads();
    for (int dd = 1; dd < RS_THREADS; dd <<= 1) {  // inclusive scans, fixed order
        SegSum o{0.0, 0};
        uint32_t oh = 0;
        const bool has = tid >= dd;
        if (has) {
            o = SegSum{pv[tid - dd], pf[tid - dd]};
            oh = ph[tid - dd];
        }
        __syncthreads();
        if (has) {
            const SegSum m = seg_combine(o, SegSum{pv[tid], pf[tid]});
            pv[tid] = m.v;
            pf[tid] = m.f;
            ph[tid] += oh;
        }
        __syncthreads();
    }
    SegSum run{carry[blockIdx.x], 0};
    if (tid > 0) run = seg_combine(run, SegSum{pv[tid - 1], pf[tid - 1]});
    const uint32_t g0 = blkoff[blockIdx.x];
    uint32_t lidx = ph[tid] - my;  // the tile's heads before this thread's chunk
    const uint64_t jmask = (1ull << bj) - 1;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        if (l0 + r >= nloc) break;
        const bool b = f[r] & 1;
        run = seg_combine(run, SegSum{x[r], b ? 1 : 0});
        if (f[r] & 2) continue;  // sentinel
        if (b) hpos[lidx++] = (uint16_t)(l0 + r);
        const int64_t e = t0 + l0 + r;
        if (e + 1 == n || (f[r + 1] & 1)) {  // last of the run: its sum
            double v = run.v;
            if (cnt) {
                const uint64_t k = keys[e];
                const int32_t i = (int32_t)(k >> bj), j = (int32_t)(k & jmask);
                v = v / sqrt((double)(cnt[i] * cnt[j]));
            }
            if (lidx > 0) sw[lidx - 1] = v;  // sw's weights are all in registers by now
            else out_v[(int64_t)g0 - 1] = v;  // the run began in an earlier tile
        }
    }
    __syncthreads();
    const uint32_t nh = ph[RS_THREADS - 1];
    // the last head's sum is set here unless its run (the run of the tile's
    // last key, not the sentinel) continues into the next tile
    const bool tail_open = t0 + nloc < n && !(fl[nloc] & 1) && !(fl[nloc - 1] & 2);
    for (uint32_t h = tid; h < nh; h += RS_THREADS) {
        const int64_t e = t0 + hpos[h];
        const uint64_t k = keys[e];
        const int64_t g = (int64_t)g0 + h;
        out_i[g] = (int32_t)(k >> bj);
        out_j[g] = (int32_t)(k & jmask);
        out_first[g] = slots ? slots[vals[e]] : vals[e];
        if (!(tail_open && h + 1 == nh)) out_v[g] = sw[h];
    }
}

// -------------------------------------------------------------- top-n --
// One wave per row: running top-64 by (score desc, first asc), 64-entry
// chunks bitonic-sorted and merged.
struct CfEnt {
    double s;
    int64_t f;
    int32_t c;
};

__device__ __forceinline__ bool cf_better(double as, int64_t af, double bs, int64_t bf) {
    return as > bs || (as == bs && af < bf);
}

// compare-exchange with lane ^ J through lane_xor (DPP / ds_swizzle /
// permlane swaps; round 6: __shfl_xor's ds_bpermute made these sorts most of
// the top-n and recall kernels' LDS instructions)
template <int J>
__device__ __forceinline__ void cf_cmpx(CfEnt& x, bool keep_better) {
    const double ys = lane_xor_f64<J>(x.s);
    const uint64_t fb = (uint64_t)x.f;
    const int64_t yf =
        (int64_t)(((uint64_t)lane_xor<J>((uint32_t)(fb >> 32)) << 32) | (uint64_t)lane_xor<J>((uint32_t)fb));
    const int32_t yc = (int32_t)lane_xor<J>((uint32_t)x.c);
    const bool xb = cf_better(x.s, x.f, ys, yf);
    if (keep_better != xb) {
        x.s = ys;
        x.f = yf;
        x.c = yc;
    }
}

__device__ __forceinline__ void cf_sort64(CfEnt& x) {
    const int lane = threadIdx.x & 63;
    static_for<6>([&](auto klc) {
        constexpr int k = 2 << decltype(klc)::value;
        static_for<decltype(klc)::value + 1>([&](auto jc) {
            constexpr int j = (k >> 1) >> decltype(jc)::value;
            const bool lower = (lane & j) == 0;
            const bool up = (lane & k) == 0;
            cf_cmpx<j>(x, lower == up);
        });
    });
}

// the bitonic clean of a 64-entry bitonic sequence, best first
__device__ __forceinline__ void cf_clean64(CfEnt& x) {
    const int lane = threadIdx.x & 63;
    static_for<6>([&](auto jc) {
        constexpr int j = 32 >> decltype(jc)::value;
        cf_cmpx<j>(x, (lane & j) == 0);
    });
}

// True when no lane of the (unsorted) chunk x beats the current n-th best
// entry (n <= 64): such a chunk cannot change the top n, and is skipped
// without its sort (round 6; in a long row almost every chunk after the
// first few).  (score, first) is a strict total order, so the kept top n is
// the same.
__device__ __forceinline__ bool cf_prunable(const CfEnt& cur, const CfEnt& x, int n) {
    const double ts = __shfl(cur.s, n - 1, WAVE);
    const int64_t tf = __shfl(cur.f, n - 1, WAVE);
    return !__any(cf_better(x.s, x.f, ts, tf));
}

__global__ __launch_bounds__(256) void cf_topn_kernel(const int64_t* __restrict__ row_off, int64_t n_rows,
                                                    const int32_t* __restrict__ cols,
                                                    const double* __restrict__ vals,
                                                    const int64_t* __restrict__ first, int topn,
                                                    int32_t* __restrict__ out_cols,
                                                    double* __restrict__ out_vals,
                                                    int32_t* __restrict__ out_cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n_rows; row += nw) {
        const int64_t a = row_off[row], n = row_off[row + 1] - a;
        if (n > CF_HEAVY) {  // a popular item's long row: cf_topn_heavy_kernel, a workgroup per row
            if (lane == 0) out_cnt[row] = -1;
            continue;
        }
        CfEnt cur{-INFINITY, INT64_MAX, -1};
        for (int64_t c0 = 0; c0 < n; c0 += 64) {
            CfEnt x{-INFINITY, INT64_MAX, -1};
            if (c0 + lane < n) {
                x.s = vals[a + c0 + lane];
                x.f = first[a + c0 + lane];
                x.c = cols[a + c0 + lane];
            }
            if (c0 > 0 && cf_prunable(cur, x, topn)) continue;
            cf_sort64(x);
            if (c0 == 0) {
                cur = x;
            } else {
                // top 64 of two sorted lists: cur[l] vs x[63 - l] -> bitonic, then clean
                const double ys = __shfl(x.s, 63 - lane, WAVE);
                const int64_t yf = __shfl(x.f, 63 - lane, WAVE);
                const int32_t yc = __shfl(x.c, 63 - lane, WAVE);
                if (cf_better(ys, yf, cur.s, cur.f)) {
                    cur.s = ys;
                    cur.f = yf;
                    cur.c = yc;
                }
                cf_clean64(cur);
            }
        }
        const int64_t m = n < topn ? n : topn;
        if (lane < topn) {
            const bool ok = lane < m;
            out_cols[row * topn + lane] = ok ? cur.c : -1;
            out_vals[row * topn + lane] = ok ? cur.s : 0.0;
        }
        if (lane == 0) out_cnt[row] = (int32_t)m;
    }
}

// ------------------------------------------------------------- recall --
// ItemCFRecaller.recall (itemcf_recaller.py:56-129) for a batch of query
// users.  The reference accumulates item_rank[j] += w over (loc, x) -- the
// history position and the rank in item i's top-n list -- and breaks score
// ties by dict insertion order.  Every candidate (q, loc, x) gets a sequence
// number c = cand_off[q] + (position in that walk):
//   rc_count / rc_scan   C_q = sum_loc nbr_cnt[items[loc]], exclusive offsets;
//   rc_cand              one wave per query: key (q << bj | j) (sentinel for
//                        j in the history), c and the contribution
//                        exp(alpha^|ct_i - ct_j|) * beta^(L - loc) * content * w_ij;
//   rc_query             (topk <= 64, C_q <= RC_CAP; round 6) one wave per
//                        query: a register sort by (j, walk position), per-j
//                        sums in walk order, top-k and the hot fill
//                        (rc_finish_query);
//   the radix path       (the larger queries, listed by rc_query and
//                        compacted; every query when topk > 64) the stable
//                        (key, c) radix sort + ordered segment sums
//                        of the similarity pass, cf_emit (q, j, score, first
//                        c) per distinct key; rc_topk: one wave per query, the
//                        hot-item fill while fewer than topk entries
//                        (:116-122), then the top-k by (score desc, insertion
//                        order asc), as sorted(...)[:topk].
__global__ __launch_bounds__(256) void rc_count_kernel(const int64_t* __restrict__ q_slot, int64_t nq,
                                                       const int64_t* __restrict__ offsets,
                                                       const int32_t* __restrict__ items,
                                                       const int32_t* __restrict__ nbr_cnt,
                                                       int64_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); q < nq; q += nw) {
        const int64_t sl = q_slot[q];
        int64_t c = 0;
        if (sl >= 0)
            for (int64_t l = offsets[sl] + lane; l < offsets[sl + 1]; l += 64) c += nbr_cnt[items[l]];
#pragma unroll
        for (int k = 32; k > 0; k >>= 1) c += __shfl_xor(c, k, WAVE);
        if (lane == 0) cnt[q] = c;
    }
}


struct RcParams {
    double loc_beta, created_alpha, ln_created;
    int topn, ke, bj;
};

__device__ __forceinline__ bool rc_find(const int32_t* __restrict__ cols, const double* __restrict__ vals,
                                        int n, int32_t key, double& v) {
    for (int x = 0; x < n; ++x)
        if (cols[x] == key) {
            v = vals[x];
            return true;
        }
    return false;
}

// One query's candidates in the reference's walk order (loc, x), handed to
// sink(f, inh, j, v) for every flat candidate f < C_q (inh: j is in the
// history -> no item_rank entry).  History positions in chunks of 64, one
// per lane; the (loc, neighbour) candidates of a chunk's positions are
// flattened over the wave -- lane f takes flat candidate f0 + f, its position
// found by a binary search of the lane-scanned neighbour counts (a row has <=
// topn neighbours, so one position per pass would leave most lanes idle).
// The in-history test is shuffles over the history held one per lane (chunk
// by chunk past 64 clicks) -- round 5 walked histories longer than 64 by
// dependent loads, one position per pass, and its few 200-click users set
// the kernel's length.
template <class Sink>
__device__ __forceinline__ void rc_gen_query(int64_t b, int64_t L, const int32_t* __restrict__ items,
                                             const int32_t* __restrict__ nbr_cols,
                                             const double* __restrict__ nbr_vals,
                                             const int32_t* __restrict__ nbr_cnt, const double* __restrict__ created,
                                             const int32_t* __restrict__ emb_cols,
                                             const double* __restrict__ emb_vals,
                                             const int32_t* __restrict__ emb_cnt, const RcParams& prm, Sink&& sink) {
    const int lane = threadIdx.x & 63;
    int64_t c = 0;
    const int32_t h0 = lane < L ? items[b + lane] : -1;  // the first 64 clicks
    for (int64_t p0 = 0; p0 < L; p0 += 64) {
        const int32_t hl = p0 == 0 ? h0 : (p0 + lane < L ? items[b + p0 + lane] : -1);
        const int nl = p0 + lane < L ? nbr_cnt[hl] : 0;
        int inc = nl;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        const int total = __shfl(inc, 63, 64);
        // position_weight(len(hist) - loc) (:92-95), lane loc
        const double lwl = p0 + lane < L ? pow(prm.loc_beta, (double)(L - p0 - lane)) : 0.0;
        for (int f0 = 0; f0 < total; f0 += 64) {  // uniform: the shuffles run converged
            const int f = f0 + lane;
            int loc = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1)
                if (__shfl(inc, loc + step - 1, 64) <= f) loc += step;
            const int32_t i = __shfl(hl, loc, 64);
            const int x = f - (__shfl(inc, loc, 64) - __shfl(nl, loc, 64));
            const double lw = __shfl(lwl, loc, 64);
            const bool ok = f < total;
            const int32_t j = ok ? nbr_cols[(int64_t)i * prm.topn + x] : -2;
            bool inh = false;
            for (int l = 0; l < (int)(L < 64 ? L : 64); ++l) inh |= __shfl(h0, l, 64) == j;
            for (int64_t hc = 64; hc < L; hc += 64) {
                const int32_t hv = hc + lane < L ? items[b + hc + lane] : -1;
                const int nh = (int)(L - hc < 64 ? L - hc : 64);
                for (int l = 0; l < nh; ++l) inh |= __shfl(hv, l, 64) == j;
            }
            if (!ok) continue;
            const double wij = nbr_vals[(int64_t)i * prm.topn + x];
            double v = 0.0;
            if (!inh) {
                // time_decay_weight(created_i, created_j) (:86-90)
                const double cw = exp(cf_apow(prm.created_alpha, prm.ln_created, fabs(created[i] - created[j])));
                double content = 1.0;  // (:98-103)
                if (prm.ke > 0) {
                    double e;
                    if (rc_find(emb_cols + (int64_t)i * prm.ke, emb_vals + (int64_t)i * prm.ke, emb_cnt[i], j, e))
                        content += e;
                    if (rc_find(emb_cols + (int64_t)j * prm.ke, emb_vals + (int64_t)j * prm.ke, emb_cnt[j], i, e))
                        content += e;
                }
                v = cw * lw * content * wij;
            }
            sink(c + f, inh, j, v);
        }
        c += total;
    }
}

// Every query's candidates to global memory at cand_off[q]: key (q << bj |
// j) or the sentinel, the global slot, the contribution.
__global__ __launch_bounds__(256) void rc_cand_kernel(
    const int64_t* __restrict__ q_slot, int64_t nq, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ items, const int32_t* __restrict__ nbr_cols,
    const double* __restrict__ nbr_vals, const int32_t* __restrict__ nbr_cnt,
    const double* __restrict__ created, const int32_t* __restrict__ emb_cols,
    const double* __restrict__ emb_vals, const int32_t* __restrict__ emb_cnt, RcParams prm,
    const int64_t* __restrict__ cand_off, uint64_t sentinel, uint64_t* __restrict__ keys,
    int32_t* __restrict__ vals, double* __restrict__ contrib) {
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); q < nq; q += nw) {
        const int64_t sl = q_slot[q];
        if (sl < 0) continue;
        const int64_t b = offsets[sl], L = offsets[sl + 1] - b;
        const int64_t c = cand_off[q];
        rc_gen_query(b, L, items, nbr_cols, nbr_vals, nbr_cnt, created, emb_cols, emb_vals, emb_cnt, prm,
                     [&](int64_t f, bool inh, int32_t j, double v) {
                         keys[c + f] = inh ? sentinel : (((uint64_t)q << prm.bj) | (uint32_t)j);
                         vals[c + f] = (int32_t)(c + f);
                         contrib[c + f] = v;
                     });
    }
}

// lower bound of q in the emitted (q, j) run (sorted by q), searched by the
// whole wave 64 probes at a time: ~4 dependent rounds over millions of
// entries where round 5's per-lane bisection made ~23 (the query's two
// bounds were most of rc_topk's time).  Probes below q form a lane prefix.
__device__ __forceinline__ int64_t rc_lower(const int32_t* __restrict__ oq, int64_t n, int64_t q) {
    const int lane = threadIdx.x & 63;
    int64_t lo = 0, hi = n;  // oq[< lo] < q <= oq[>= hi]
    while (lo < hi) {
        const int64_t step = (hi - lo + 63) >> 6;
        const int64_t p = lo + step * lane;
        const int c = __popcll(__ballot(p < hi && (int64_t)oq[p] < q));
        if (c == 0) break;  // oq[lo] >= q
        const int64_t nhi = lo + step * c;
        lo += step * (c - 1) + 1;
        hi = nhi < hi ? nhi : hi;
    }
    return lo;
}

// The end of one query's recall (itemcf_recaller.py:116-129): the top-k
// (k <= 64) of its distinct candidates by (score desc, first slot asc) --
// chunk(c0) gives each lane its entry of positions [c0, c0 + 64) of a source
// of nsrc positions (or c = -1: none there) -- then the hot-item fill while
// fewer than topk (:116-122; in_cands(h): h is one of the candidates, only
// asked when there are some), then the output row.
template <class Chunk, class InCands>
__device__ __forceinline__ void rc_finish_query(int64_t q, int64_t nsrc, Chunk&& chunk, InCands&& in_cands,
                                                int64_t b, int64_t L, const int32_t* __restrict__ items,
                                                const int32_t* __restrict__ hot, int n_hot, int topk,
                                                int32_t* __restrict__ out_items, double* __restrict__ out_scores,
                                                int32_t* __restrict__ out_src, int32_t* __restrict__ out_cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t HOT_FIRST = (int64_t)1 << 62;  // after every candidate (insertion order)
    CfEnt cur{-INFINITY, INT64_MAX, -1};
    bool started = false;
    auto merge = [&](CfEnt x) {
        cf_sort64(x);
        if (!started) {
            cur = x;
            started = true;
            return;
        }
        const double ys = __shfl(x.s, 63 - lane, WAVE);
        const int64_t yf = __shfl(x.f, 63 - lane, WAVE);
        const int32_t yc = __shfl(x.c, 63 - lane, WAVE);
        if (cf_better(ys, yf, cur.s, cur.f)) {
            cur.s = ys;
            cur.f = yf;
            cur.c = yc;
        }
        cf_clean64(cur);
    };
    int64_t n = 0;  // distinct candidates
    for (int64_t c0 = 0; c0 < nsrc; c0 += 64) {
        const CfEnt x = chunk(c0);
        n += __popcll(__ballot(x.c >= 0));
        if (started && cf_prunable(cur, x, topk)) continue;
        merge(x);
    }
    int64_t total = n;
    if (n < topk) {
        // fill with popular items not yet ranked and not in the history,
        // scored -x - 100, until topk entries (:116-122)
        int need = (int)(topk - n);
        CfEnt hx{-INFINITY, INT64_MAX, -1};
        int got = 0;
        for (int x0 = 0; x0 < n_hot && need > 0; x0 += 64) {
            const int x = x0 + lane;
            const int32_t h = x < n_hot ? hot[x] : -1;
            bool ok = x < n_hot;
            // not in the history: its clicks 64 at a time, one per lane, each
            // compared by a uniform-index read (round 5: every lane walked the
            // history by dependent loads)
            for (int64_t hc = 0; hc < L; hc += 64) {
                const int32_t hv = hc + lane < L ? items[b + hc + lane] : -1;
                const int nh = (int)(L - hc < 64 ? L - hc : 64);
                for (int l = 0; l < nh; ++l) {
                    const int32_t hl = __shfl(hv, l, WAVE);  // every lane active: a shuffle under
                    ok = ok && hl != h;                      // a short-circuit reads stale lanes
                }
            }
            if (ok && n > 0) ok = !in_cands(h);
            const uint64_t bal = __builtin_amdgcn_ballot_w64(ok);
            const int take = __builtin_popcountll(bal) < need ? __builtin_popcountll(bal) : need;
            // the first `take' accepted entries, in hot order, into hx lanes
            // got ..: lane got + t takes the t-th set bit of bal (the smallest
            // p with t + 1 set bits in [0, p], by bisection)
            const int t = lane - got;
            int src = 0;
#pragma unroll
            for (int st = 32; st >= 1; st >>= 1)
                if (__builtin_popcountll(bal & ((2ull << (src + st - 1)) - 1ull)) < t + 1) src += st;
            const int32_t hv = __shfl(h, src, WAVE);
            if (t >= 0 && t < take) {
                hx.s = (double)(-(x0 + src) - 100);
                hx.f = HOT_FIRST + x0 + src;
                hx.c = hv;
            }
            got += take;
            need -= take;
        }
        total += got;
        if (got > 0) merge(hx);
    }
    const int64_t m = total < topk ? total : topk;
    if (lane < topk) {
        const bool ok = lane < m;
        out_items[q * topk + lane] = ok ? cur.c : -1;
        out_scores[q * topk + lane] = ok ? cur.s : 0.0;
        out_src[q * topk + lane] = ok ? (cur.f >= HOT_FIRST ? 1 : 0) : -1;
    }
    if (lane == 0) out_cnt[q] = (int32_t)m;
}

// cold start: [(hot[i], -i) for i < topk] (:68-70)
__device__ __forceinline__ void rc_cold(int64_t q, const int32_t* __restrict__ hot, int n_hot, int topk,
                                        int32_t* __restrict__ out_items, double* __restrict__ out_scores,
                                        int32_t* __restrict__ out_src, int32_t* __restrict__ out_cnt) {
    const int lane = threadIdx.x & 63;
    const int m = n_hot < topk ? n_hot : topk;
    if (lane < topk) {
        out_items[q * topk + lane] = lane < m ? hot[lane] : -1;
        out_scores[q * topk + lane] = lane < m ? -(double)lane : 0.0;
        out_src[q * topk + lane] = lane < m ? 2 : -1;
    }
    if (lane == 0) out_cnt[q] = m;
}

// rc_finish_query for at most 64 distinct candidates, lane i < nd holding
// entry x: the hot fill goes to lanes [nd, nd + got) (it only runs when nd <
// topk <= 64), then one 64-wide sort gives the output row.
template <class InCands>
__device__ __forceinline__ void rc_finish_small(int64_t q, CfEnt x, int nd, InCands&& in_cands, int64_t b,
                                                int64_t L, const int32_t* __restrict__ items,
                                                const int32_t* __restrict__ hot, int n_hot, int topk,
                                                int32_t* __restrict__ out_items, double* __restrict__ out_scores,
                                                int32_t* __restrict__ out_src, int32_t* __restrict__ out_cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t HOT_FIRST = (int64_t)1 << 62;
    int total = nd;
    if (nd < topk) {
        int need = topk - nd, got = 0;
        for (int x0 = 0; x0 < n_hot && need > 0; x0 += 64) {
            const int xi = x0 + lane;
            const int32_t h = xi < n_hot ? hot[xi] : -1;
            bool ok = xi < n_hot;
            for (int64_t hc = 0; hc < L; hc += 64) {
                const int32_t hv = hc + lane < L ? items[b + hc + lane] : -1;
                const int nh = (int)(L - hc < 64 ? L - hc : 64);
                for (int l = 0; l < nh; ++l) {
                    const int32_t hl = __shfl(hv, l, WAVE);  // every lane active: a shuffle under
                    ok = ok && hl != h;                      // a short-circuit reads stale lanes
                }
            }
            if (ok && nd > 0) ok = !in_cands(h);
            const uint64_t bal = __builtin_amdgcn_ballot_w64(ok);
            const int take = __builtin_popcountll(bal) < need ? __builtin_popcountll(bal) : need;
            const int t = lane - nd - got;
            int src = 0;
#pragma unroll
            for (int st = 32; st >= 1; st >>= 1)
                if (__builtin_popcountll(bal & ((2ull << (src + st - 1)) - 1ull)) < t + 1) src += st;
            const int32_t hv = __shfl(h, src, WAVE);
            if (t >= 0 && t < take) x = CfEnt{(double)(-(x0 + src) - 100), HOT_FIRST + x0 + src, hv};
            got += take;
            need -= take;
        }
        total += got;
    }
    cf_sort64(x);
    const int m = total < topk ? total : topk;
    if (lane < topk) {
        const bool ok = lane < m;
        out_items[q * topk + lane] = ok ? x.c : -1;
        out_scores[q * topk + lane] = ok ? x.s : 0.0;
        out_src[q * topk + lane] = ok ? (x.f >= HOT_FIRST ? 1 : 0) : -1;
    }
    if (lane == 0) out_cnt[q] = m;
}

// The radix path's top-k: one wave per query over its emitted (q, j) run
// (every query, or the *qcount listed ones).
__global__ __launch_bounds__(256) void rc_topk_kernel(
    const int64_t* __restrict__ q_slot, int64_t nq, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ items, const int32_t* __restrict__ hot, int n_hot,
    const int32_t* __restrict__ eq, const int32_t* __restrict__ ej, const double* __restrict__ ev,
    const int64_t* __restrict__ ef, const int64_t* __restrict__ n_emit, int topk,
    int32_t* __restrict__ out_items, double* __restrict__ out_scores, int32_t* __restrict__ out_src,
    int32_t* __restrict__ out_cnt, const int2* __restrict__ qlist = nullptr,
    const int32_t* __restrict__ qcount = nullptr) {
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int64_t ne = *n_emit;
    const int64_t nl = qlist ? (int64_t)*qcount : nq;
    for (int64_t iq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); iq < nl; iq += nw) {
        const int64_t q = qlist ? (int64_t)qlist[iq].x : iq;
        const int64_t sl = q_slot[q];
        if (sl < 0) {
            rc_cold(q, hot, n_hot, topk, out_items, out_scores, out_src, out_cnt);
            continue;
        }
        const int64_t a = rc_lower(eq, ne, q), e = rc_lower(eq, ne, q + 1);
        const int64_t b = offsets[sl], L = offsets[sl + 1] - b;
        rc_finish_query(
            q, e - a,
            [&](int64_t c0) {
                const int64_t i = a + c0 + (threadIdx.x & 63);
                return i < e ? CfEnt{ev[i], ef[i], ej[i]} : CfEnt{-INFINITY, INT64_MAX, -1};
            },
            [&](int32_t h) {  // binary search in the query's candidate js (sorted)
                int64_t lo = a, hi = e;
                while (lo < hi) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (ej[mid] < h) lo = mid + 1;
                    else hi = mid;
                }
                return lo < e && ej[lo] == h;
            },
            b, L, items, hot, n_hot, topk, out_items, out_scores, out_src, out_cnt);
    }
}

// lane ^ stride's key (stride < 64, a constant once the sort below is
// unrolled: lane_xor's DPP / swizzle / permlane forms)
__device__ __forceinline__ uint64_t lane_xor_u64(uint64_t v, int stride) {
    auto x = [&](auto jc) {
        constexpr int J = decltype(jc)::value;
        return ((uint64_t)lane_xor<J>((uint32_t)(v >> 32)) << 32) | (uint64_t)lane_xor<J>((uint32_t)v);
    };
    switch (stride) {
        case 1: return x(std::integral_constant<int, 1>{});
        case 2: return x(std::integral_constant<int, 2>{});
        case 4: return x(std::integral_constant<int, 4>{});
        case 8: return x(std::integral_constant<int, 8>{});
        case 16: return x(std::integral_constant<int, 16>{});
        default: return x(std::integral_constant<int, 32>{});
    }
}

// ascending bitonic sort of 64 E keys, key e * 64 + lane in k[e]
template <int E>
__device__ __forceinline__ void wave_sort_u64(uint64_t (&k)[E]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int size = 2; size <= 64 * E; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {
                const int es = stride >> 6;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if (e & es) continue;
                    const bool up = ((e * 64 + lane) & size) == 0;
                    const uint64_t x = k[e], y = k[e | es];
                    if ((x > y) == up) {
                        k[e] = y;
                        k[e | es] = x;
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const uint64_t y = lane_xor_u64(k[e], stride);
                    const bool up = ((e * 64 + lane) & size) == 0;
                    const bool lower = (lane & stride) == 0;
                    k[e] = (lower == up) ? (k[e] < y ? k[e] : y) : (k[e] > y ? k[e] : y);
                }
            }
        }
    }
}

template <int E>
__device__ __forceinline__ void rc_sort_lds(uint64_t* kw, int c) {
    const int lane = threadIdx.x & 63;
    uint64_t k[E];
#pragma unroll
    for (int e = 0; e < E; ++e) k[e] = e * 64 + lane < c ? kw[e * 64 + lane] : ~0ull;
    wave_sort_u64<E>(k);
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (e * 64 + lane < c) kw[e * 64 + lane] = k[e];
}

// The recall of a query with at most RC_CAP candidates in one wave (round 6;
// topk <= 64), from rc_cand's keys and contributions: the keys as (j << 32 |
// f), f the walk position (in-history: j = 0xFFFFFFFF, sorted last), a
// register bitonic sort of them (j, then walk order), the contributions in
// LDS by f, then per distinct j the sum of its contributions in walk order --
// exactly the reference's item_rank[j] += w sequence -- and the first walk
// position, fed to rc_finish_query.  Queries with more candidates are listed
// (q, compacted offset) for the radix path.  Round 5 sent every query through
// the global radix sort (five 8-bit passes over all candidates, tile sums,
// emit, rc_topk).  rc_cand stays a kernel of its own: with the gathers and
// fp64 exp of the candidate walk inlined here the wave needed 150 VGPRs (3 per
// SIMD).  Measured at 250k users: the single-kernel form 1.92 ms and a 4.47 ms
// recall; split, rc_cand 0.85 + this kernel 1.53 ms and a 4.06 ms recall (the
// same step let empty radix tiles exit early); this kernel is 0.97 ms since
// its sorts use DPP exchanges and small queries finish with one 64-wide sort.
constexpr int RC_CAP = 512;

__global__ __launch_bounds__(256) void rc_query_kernel(
    const int64_t* __restrict__ q_slot, int64_t nq, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ items, const int64_t* __restrict__ cand_off, const uint64_t* __restrict__ keys,
    const double* __restrict__ contrib, uint64_t sentinel, int bj, const int32_t* __restrict__ hot, int n_hot,
    int topk, int32_t* __restrict__ out_items, double* __restrict__ out_scores, int32_t* __restrict__ out_src,
    int32_t* __restrict__ out_cnt, int2* __restrict__ hlist, int32_t* __restrict__ hcnt,
    unsigned long long* __restrict__ htot) {
    __shared__ uint64_t sk[4][RC_CAP];
    __shared__ double rv[4][RC_CAP];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t* kw = sk[wave];
    double* vw = rv[wave];
    const uint64_t jmask = (1ull << bj) - 1;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t q = (int64_t)blockIdx.x * 4 + wave; q < nq; q += nw) {
        const int64_t sl = q_slot[q];
        if (sl < 0) {
            rc_cold(q, hot, n_hot, topk, out_items, out_scores, out_src, out_cnt);
            continue;
        }
        const int64_t c0 = cand_off[q], cq = cand_off[q + 1] - c0;
        if (cq > RC_CAP) {
            if (lane == 0) {
                const int i = atomicAdd(hcnt, 1);
                hlist[i] = make_int2((int)q, (int)atomicAdd(htot, (unsigned long long)cq));
            }
            continue;
        }
        const int c = (int)cq;
        const int64_t b = offsets[sl], L = offsets[sl + 1] - b;
        wave_sync_lds();  // the previous query's reads of kw / vw are done
        // (1) keys (j << 32 | f) sorted in registers; (2) per distinct j, its
        // sum in walk order by the run's first lane (registers); (3) the
        // distinct entries compacted in j order into the front of kw / vw
        // (key, sum) -- every read of (1) / (2) is done first.  Returns nd.
        auto distinct = [&](auto e_c) -> int {
            constexpr int E = decltype(e_c)::value;
            uint64_t k[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int i = e * 64 + lane;
                k[e] = ~0ull;
                if (i < c) {
                    const uint64_t kk = keys[c0 + i];
                    k[e] = ((kk == sentinel ? 0xFFFFFFFFull : (kk & jmask)) << 32) | (uint32_t)i;
                    vw[i] = contrib[c0 + i];
                }
            }
            wave_sort_u64<E>(k);
#pragma unroll
            for (int e = 0; e < E; ++e)
                if (e * 64 + lane < c) kw[e * 64 + lane] = k[e];
            wave_sync_lds();
            bool hd[E];
            double hs[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int i = e * 64 + lane;
                const uint32_t j = (uint32_t)(k[e] >> 32);
                hd[e] = i < c && j != 0xFFFFFFFFu && (i == 0 || (uint32_t)(kw[i - 1] >> 32) != j);
                hs[e] = 0.0;
                if (hd[e]) {
                    double sum = 0.0;  // item_rank[j] += w, walk order (:118-119)
                    for (int t = i; t < c; ++t) {
                        const uint64_t kt = kw[t];
                        if ((uint32_t)(kt >> 32) != j) break;
                        sum += vw[(uint32_t)kt];
                    }
                    hs[e] = sum;
                }
            }
            wave_sync_lds();
            int nd = 0;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint64_t bal = __ballot(hd[e]);
                if (hd[e]) {
                    const int pos = nd + __popcll(bal & ((1ull << lane) - 1ull));
                    kw[pos] = k[e];
                    vw[pos] = hs[e];
                }
                nd += __popcll(bal);
            }
            return nd;
        };
        int nd;
        if (c <= 64) nd = distinct(std::integral_constant<int, 1>{});
        else if (c <= 128) nd = distinct(std::integral_constant<int, 2>{});
        else if (c <= 256) nd = distinct(std::integral_constant<int, 4>{});
        else nd = distinct(std::integral_constant<int, 8>{});
        wave_sync_lds();
        auto in_cands = [&](int32_t h) {  // h among the distinct js: bisection
            const uint64_t kh = (uint64_t)(uint32_t)h << 32;
            int lo = 0, hi = nd;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (kw[mid] < kh) lo = mid + 1;
                else hi = mid;
            }
            return lo < nd && (uint32_t)(kw[lo] >> 32) == (uint32_t)h;
        };
        auto ent = [&](int i) {
            return i < nd ? CfEnt{vw[i], c0 + (int64_t)(uint32_t)kw[i], (int32_t)(kw[i] >> 32)}
                          : CfEnt{-INFINITY, INT64_MAX, -1};
        };
        if (nd <= 64) {
            // one sort: the distinct entries in lanes [0, nd), the hot fill
            // (only when nd < topk <= 64) behind them
            rc_finish_small(q, ent(lane), nd, in_cands, b, L, items, hot, n_hot, topk, out_items, out_scores,
                            out_src, out_cnt);
        } else {
            rc_finish_query(
                q, nd, [&](int64_t p0) { return ent((int)p0 + lane); }, in_cands, b, L, items, hot, n_hot, topk,
                out_items, out_scores, out_src, out_cnt);
        }
    }
}

// The listed queries' keys and slots to the front of (kout, vout), query by
// query (the contributions stay where rc_cand wrote them: the slots index
// them).  One wave per listed query.
__global__ __launch_bounds__(256) void rc_compact_kernel(const int64_t* __restrict__ cand_off,
                                                         const uint64_t* __restrict__ kin,
                                                         const int32_t* __restrict__ vin,
                                                         const int2* __restrict__ hlist,
                                                         const int32_t* __restrict__ hcnt,
                                                         uint64_t* __restrict__ kout, int32_t* __restrict__ vout) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4, nl = *hcnt;
    for (int64_t iq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); iq < nl; iq += nw) {
        const int2 h = hlist[iq];
        const int64_t c0 = cand_off[h.x], cq = cand_off[h.x + 1] - c0;
        for (int64_t i = lane; i < cq; i += 64) {
            kout[h.y + i] = kin[c0 + i];
            vout[h.y + i] = vin[c0 + i];
        }
    }
}

// Rows longer than CF_HEAVY (flagged out_cnt = -1 by cf_topn_kernel): 16 waves
// run the same running top-64 over interleaved 64-entry chunks, then wave 0
// merges the 16 lists.  (score, first) is a total order, so the result does
// not depend on the partition.
__global__ __launch_bounds__(1024) void cf_topn_heavy_kernel(const int64_t* __restrict__ row_off, int64_t n_rows,
                                                           const int32_t* __restrict__ cols,
                                                           const double* __restrict__ vals,
                                                           const int64_t* __restrict__ first, int topn,
                                                           int32_t* __restrict__ out_cols,
                                                           double* __restrict__ out_vals,
                                                           int32_t* __restrict__ out_cnt) {
    __shared__ double ls[16][64];
    __shared__ int64_t lf[16][64];
    __shared__ int32_t lc[16][64];
    __shared__ int64_t hrow[1024];
    __shared__ int nh;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // the flagged rows of a 1,024-row window, found by one coalesced read
    // (round 6: each workgroup tested its rows one dependent load at a time,
    // ~560 round trips per workgroup before any heavy row)
    for (int64_t base = (int64_t)blockIdx.x * 1024; base < n_rows; base += (int64_t)gridDim.x * 1024) {
    if (threadIdx.x == 0) nh = 0;
    __syncthreads();
    {
        const int64_t r = base + threadIdx.x;
        if (r < n_rows && out_cnt[r] == -1) hrow[atomicAdd(&nh, 1)] = r;
    }
    __syncthreads();
    const int nhv = nh;
    for (int ih = 0; ih < nhv; ++ih) {
        const int64_t row = hrow[ih];
        const int64_t a = row_off[row], n = row_off[row + 1] - a;
        CfEnt cur{-INFINITY, INT64_MAX, -1};
        auto merge_in = [&](CfEnt x) {  // x sorted desc; keep the top 64 of cur + x
            const double ys = __shfl(x.s, 63 - lane, WAVE);
            const int64_t yf = __shfl(x.f, 63 - lane, WAVE);
            const int32_t yc = __shfl(x.c, 63 - lane, WAVE);
            if (cf_better(ys, yf, cur.s, cur.f)) {
                cur.s = ys;
                cur.f = yf;
                cur.c = yc;
            }
            cf_clean64(cur);
        };
        bool started = false;
        // the wave's chunks wv, wv + 16, ... in that order, CF_HB of them
        // loaded at once (round 6: one chunk's loads per round trip, and most
        // chunks are pruned without a sort, so the loads were the time)
        constexpr int CF_HB = 4;
        for (int64_t c0 = (int64_t)wv * 64; c0 < n; c0 += CF_HB * 16 * 64) {
            CfEnt xs[CF_HB];
#pragma unroll
            for (int t = 0; t < CF_HB; ++t) {
                const int64_t e = c0 + (int64_t)t * 16 * 64 + lane;
                xs[t] = CfEnt{-INFINITY, INT64_MAX, -1};
                if (e < n) {
                    xs[t].s = vals[a + e];
                    xs[t].f = first[a + e];
                    xs[t].c = cols[a + e];
                }
            }
#pragma unroll
            for (int t = 0; t < CF_HB; ++t) {
                if (c0 + (int64_t)t * 16 * 64 >= n) break;  // wave-uniform
                CfEnt x = xs[t];
                if (started && cf_prunable(cur, x, topn)) continue;
                cf_sort64(x);
                if (!started) cur = x;
                else merge_in(x);
                started = true;
            }
        }
        ls[wv][lane] = cur.s;
        lf[wv][lane] = cur.f;
        lc[wv][lane] = cur.c;
        __syncthreads();
        if (wv == 0) {
            for (int w = 1; w < 16; ++w) merge_in(CfEnt{ls[w][lane], lf[w][lane], lc[w][lane]});
            const int64_t m = n < topn ? n : topn;
            if (lane < topn) {
                const bool ok = lane < m;
                out_cols[row * topn + lane] = ok ? cur.c : -1;
                out_vals[row * topn + lane] = ok ? cur.s : 0.0;
            }
            if (lane == 0) out_cnt[row] = (int32_t)m;
        }
        __syncthreads();
    }
    __syncthreads();  // nh is reset for the next window
    }
}

// ----------------------------------------------------- wide top-k (k > 64) --
// The reference has no limit on itemcf_sim_item_topk / the recall topk
// (itemcf_recaller.py:41-54, :125) or on rank_and_recommend's topk.  Above
// the 64-lane register paths: one wave per row keeps a running top-K
// (K = next_pow2(k)) best-first in LDS; each chunk of up to K new entries
// lands behind it and the 2K are re-sorted by an LDS bitonic sort on
// (score desc, first asc) -- a total order, so the result does not depend on
// the chunking.
__device__ inline void cf_lds_sort(CfEnt* x, int n) {
    const int lane = threadIdx.x & (WAVE - 1);
    wave_sync_lds();
    for (int sz = 2; sz <= n; sz <<= 1) {
        for (int st = sz >> 1; st > 0; st >>= 1) {
            for (int i = lane; i < n / 2; i += WAVE) {
                const int lo = 2 * st * (i / st) + (i % st), hi = lo + st;
                const bool up = (lo & sz) == 0;
                const CfEnt a = x[lo], b = x[hi];
                const bool b_first = cf_better(b.s, b.f, a.s, a.f);
                if (up ? b_first : !b_first && (a.s != b.s || a.f != b.f)) {
                    x[lo] = b;
                    x[hi] = a;
                }
            }
            wave_sync_lds();
        }
    }
}

template <class Get>
__device__ inline void cf_wave_topk(CfEnt* buf, int K, int64_t n, Get get) {
    const int lane = threadIdx.x & (WAVE - 1);
    for (int i = lane; i < 2 * K; i += WAVE) buf[i] = CfEnt{-INFINITY, INT64_MAX, -1};
    for (int64_t c0 = 0; c0 < n; c0 += K) {
        wave_sync_lds();
        for (int i = lane; i < K; i += WAVE) buf[K + i] = c0 + i < n ? get(c0 + i) : CfEnt{-INFINITY, INT64_MAX, -1};
        cf_lds_sort(buf, 2 * K);
    }
    wave_sync_lds();
}

__global__ __launch_bounds__(64) void cf_topn_wide_kernel(const int64_t* __restrict__ row_off, int64_t n_rows,
                                                        const int32_t* __restrict__ cols,
                                                        const double* __restrict__ vals,
                                                        const int64_t* __restrict__ first, int topn, int K,
                                                        int32_t* __restrict__ out_cols, double* __restrict__ out_vals,
                                                        int32_t* __restrict__ out_cnt) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    CfEnt* buf = reinterpret_cast<CfEnt*>(dyn);
    const int lane = threadIdx.x;
    for (int64_t row = blockIdx.x; row < n_rows; row += gridDim.x) {
        const int64_t a = row_off[row], n = row_off[row + 1] - a;
        cf_wave_topk(buf, K, n, [&](int64_t i) { return CfEnt{vals[a + i], first[a + i], cols[a + i]}; });
        const int64_t m = n < topn ? n : topn;
        for (int i = lane; i < topn; i += WAVE) {
            const bool ok = i < m;
            out_cols[row * topn + i] = ok ? buf[i].c : -1;
            out_vals[row * topn + i] = ok ? buf[i].s : 0.0;
        }
        if (lane == 0) out_cnt[row] = (int32_t)m;
        wave_sync_lds();
    }
}

// rc_topk_kernel for topk > 64 (same outputs): candidates by the wave top-K,
// then the hot fill (:116-122) appended in hot order -- every fill score
// -x - 100 is below every candidate's (products of positive weights) and
// the fill scores decrease with x, so no re-sort is needed.
__global__ __launch_bounds__(64) void rc_topk_wide_kernel(
    const int64_t* __restrict__ q_slot, int64_t nq, const int64_t* __restrict__ offsets,
    const int32_t* __restrict__ items, const int32_t* __restrict__ hot, int n_hot,
    const int32_t* __restrict__ eq, const int32_t* __restrict__ ej, const double* __restrict__ ev,
    const int64_t* __restrict__ ef, const int64_t* __restrict__ n_emit, int topk, int K,
    int32_t* __restrict__ out_items, double* __restrict__ out_scores, int32_t* __restrict__ out_src,
    int32_t* __restrict__ out_cnt) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    CfEnt* buf = reinterpret_cast<CfEnt*>(dyn);
    const int lane = threadIdx.x;
    const int64_t ne = *n_emit;
    for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const int64_t sl = q_slot[q];
        int32_t* oi = out_items + q * topk;
        double* os = out_scores + q * topk;
        int32_t* osrc = out_src + q * topk;
        if (sl < 0) {  // cold start: [(hot[i], -i) for i < topk] (:68-70)
            const int m = n_hot < topk ? n_hot : topk;
            for (int i = lane; i < topk; i += WAVE) {
                oi[i] = i < m ? hot[i] : -1;
                os[i] = i < m ? -(double)i : 0.0;
                osrc[i] = i < m ? 2 : -1;
            }
            if (lane == 0) out_cnt[q] = m;
            continue;
        }
        const int64_t a = rc_lower(eq, ne, q), e = rc_lower(eq, ne, q + 1), n = e - a;
        cf_wave_topk(buf, K, n, [&](int64_t i) { return CfEnt{ev[a + i], ef[a + i], ej[a + i]}; });
        const int mc = (int)(n < topk ? n : topk);
        for (int i = lane; i < mc; i += WAVE) {
            oi[i] = buf[i].c;
            os[i] = buf[i].s;
            osrc[i] = 0;
        }
        int got = 0;
        if (mc < topk) {
            const int64_t b = offsets[sl], L = offsets[sl + 1] - b;
            int need = topk - mc;
            for (int x0 = 0; x0 < n_hot && need > 0; x0 += WAVE) {
                const int x = x0 + lane;
                bool ok = false;
                int32_t hv = -1;
                if (x < n_hot) {
                    hv = hot[x];
                    ok = true;
                    for (int64_t l = 0; l < L && ok; ++l) ok = items[b + l] != hv;
                    if (ok && n > 0) {  // binary search in the query's candidate js (sorted)
                        int64_t lo = a, hi = e;
                        while (lo < hi) {
                            const int64_t mid = (lo + hi) >> 1;
                            if (ej[mid] < hv) lo = mid + 1;
                            else hi = mid;
                        }
                        ok = !(lo < e && ej[lo] == hv);
                    }
                }
                const unsigned long long bal = __ballot(ok);
                const int rank = __popcll(bal & ((1ull << lane) - 1ull));
                if (ok && rank < need) {
                    oi[mc + got + rank] = hv;
                    os[mc + got + rank] = (double)(-x - 100);
                    osrc[mc + got + rank] = 1;
                }
                const int take = __popcll(bal) < need ? __popcll(bal) : need;
                got += take;
                need -= take;
            }
        }
        for (int i = mc + got + lane; i < topk; i += WAVE) {
            oi[i] = -1;
            os[i] = 0.0;
            osrc[i] = -1;
        }
        if (lane == 0) out_cnt[q] = mc + got;
        wave_sync_lds();
    }
}

// CSR row offsets of the (i, j)-sorted similarity entries: off[r] = first
// entry with i >= r (binary search per row; no atomics)
__global__ __launch_bounds__(256) void cf_row_offsets_kernel(const int32_t* __restrict__ ei, int64_t n,
                                                           int64_t n_rows, int64_t* __restrict__ off) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r <= n_rows; r += (int64_t)gridDim.x * 256) {
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)ei[mid] < r) lo = mid + 1;
            else hi = mid;
        }
        off[r] = lo;
    }
}

__global__ void cf_iota_copy_kernel(const uint64_t* __restrict__ kin, int64_t n, uint64_t* __restrict__ kout,
                                    int32_t* __restrict__ v) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        kout[e] = kin[e];
        v[e] = (int32_t)e;
    }
}

// ---------------------------------------------------------- workspace --
struct CfWs {
    uint64_t *ka, *kb;
    int32_t *va, *vb;
    double* w;
    uint32_t *counts, *totals, *blkcnt, *blkoff;
    double *tail, *carry;
    int32_t* brk;
    size_t bytes;
};

static inline size_t cf_al(size_t x) { return (x + 255) & ~(size_t)255; }

static CfWs cf_ws_layout(void* base, int64_t P) {
    CfWs w;
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    size_t o = 0;
    const size_t n = (size_t)(P > 0 ? P : 1);
    const size_t nblk = (n + RS_TILE - 1) / RS_TILE;
    auto take = [&](size_t b) { uint8_t* r = p + o; o += cf_al(b); return r; };
    w.ka = (uint64_t*)take(n * 8);
    w.kb = (uint64_t*)take(n * 8);
    w.va = (int32_t*)take(n * 4);
    w.vb = (int32_t*)take(n * 4);
    w.w = (double*)take(n * 8);
    w.counts = (uint32_t*)take(256 * nblk * 4);
    w.totals = (uint32_t*)take(256 * 4);
    w.blkcnt = (uint32_t*)take(nblk * 4);
    w.blkoff = (uint32_t*)take(nblk * 4);
    w.tail = (double*)take(nblk * 8);
    w.carry = (double*)take(nblk * 8);
    w.brk = (int32_t*)take(nblk * 4);
    w.bytes = o;
    return w;
}

struct RcWs {
    CfWs sort;
    int32_t *eq, *ej;
    double* ev;
    int64_t *ef, *n_emit;
    int2* hlist;
    int32_t* hcnt;
    unsigned long long* htot;
    size_t bytes;
};

static RcWs rc_ws_layout(void* base, int64_t n_cand) {
    RcWs w;
    w.sort = cf_ws_layout(base, n_cand);
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    size_t o = w.sort.bytes;
    const size_t n = (size_t)(n_cand > 0 ? n_cand : 1);
    auto take = [&](size_t b) { uint8_t* r = p + o; o += cf_al(b); return r; };
    w.eq = (int32_t*)take(n * 4);
    w.ej = (int32_t*)take(n * 4);
    w.ev = (double*)take(n * 8);
    w.ef = (int64_t*)take(n * 8);
    w.n_emit = (int64_t*)take(8);
    w.hlist = (int2*)take((n / RC_CAP + 1) * sizeof(int2));  // at most n / (RC_CAP + 1) overflow queries
    w.hcnt = (int32_t*)take(16);                              // + the overflow candidate total at +8
    w.htot = reinterpret_cast<unsigned long long*>(reinterpret_cast<uint8_t*>(w.hcnt) + 8);
    w.bytes = o;
    return w;
}

static int bits_for(int64_t n) {  // smallest b with 2^b > n
    int b = 1;
    while ((int64_t(1) << b) <= n) ++b;
    return b;
}

static inline int cf_wide_k(int k) {
    int p = 64;
    while (p < k) p <<= 1;
    return p;
}

}  // namespace nrk

using namespace nrk;

extern "C" {

int nrk_itemcf_pair_offsets(const int64_t* offsets, int64_t n_users, int64_t* pair_off,
                            nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(offsets && pair_off, "null pointer");
    NRK_REQUIRE(n_users >= 0, "n_users < 0");
    scan_exclusive_kernel<ScanPairs><<<1, 1024, 0, as_stream(stream)>>>(ScanPairs{offsets}, n_users, pair_off);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_itemcf_workspace_bytes(int64_t n_pairs, int32_t n_items) {
    (void)n_items;
    if (n_pairs < 0) return 0;
    return cf_ws_layout(nullptr, n_pairs).bytes;
}

int nrk_itemcf_sim(const int64_t* offsets, int64_t n_users, const int32_t* items, const int64_t* ts,
                   const double* created, int32_t n_items, const int64_t* pair_off, int64_t n_pairs,
                   double loc_alpha, double loc_alpha_rev, double loc_beta, double time_alpha,
                   double created_alpha, int32_t* out_i, int32_t* out_j, double* out_v,
                   int64_t* out_first, int64_t* out_n, int64_t* out_cnt, void* workspace,
                   size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_users >= 0 && n_pairs >= 0, "negative size");
    NRK_REQUIRE(n_items >= 1, "n_items must be >= 1");
    NRK_REQUIRE(n_pairs < (int64_t(1) << 31) - RS_TILE, "n_pairs must be < 2^31 (int32 slots)");
    NRK_REQUIRE(offsets && items && ts && created && pair_off && out_i && out_j && out_v &&
                    out_first && out_n && out_cnt && workspace,
                "null pointer");
    const CfWs w = cf_ws_layout(workspace, n_pairs);
    NRK_REQUIRE(workspace_bytes >= w.bytes, "workspace too small");
    hipStream_t s = as_stream(stream);
    const int bj = bits_for(n_items);  // 2^bj > n_items - 1 + 1: i = 2^bj - 1 is never an item
    const int nbits = 2 * bj;
    const uint64_t sentinel = (nbits >= 64) ? ~0ull : ((1ull << nbits) - 1);
    (void)hipMemsetAsync(out_cnt, 0, sizeof(int64_t) * (size_t)n_items, s);
    const CfParams prm{loc_alpha, loc_alpha_rev, loc_beta, time_alpha, created_alpha, cf_dt_zero(time_alpha),
                       cf_ln(time_alpha), cf_ln(created_alpha)};
    const int64_t pgrid = (n_pairs + 4 * CF_CHUNK - 1) / (4 * CF_CHUNK);
    if (n_users > 0 && n_pairs > 0)
        cf_pairs_flat_kernel<<<(int)(pgrid < 8192 ? pgrid : 8192), 256, 0, s>>>(
            offsets, n_users, items, ts, created, pair_off, 0, prm, bj, sentinel, w.ka, w.va, w.w);
    if (n_users > 0)
        cf_item_count_kernel<<<1024, CF_CNT_THREADS, 0, s>>>(offsets, n_users, items,
                                                             reinterpret_cast<unsigned long long*>(out_cnt));
    const int64_t n = n_pairs;
    const int nblk = (int)((n + RS_TILE - 1) / RS_TILE);
    uint64_t* kin = w.ka;
    uint64_t* kout = w.kb;
    int32_t* vin = w.va;
    int32_t* vout = w.vb;
    if (n > 0) {
        for (int shift = 0; shift < nbits; shift += 8) {
            rs_upsweep<<<nblk, RS_THREADS, 0, s>>>(kin, n, shift, nblk, w.counts);
            rs_scan_rows<<<256, 256, 0, s>>>(w.counts, nblk, w.totals);
            rs_downsweep<<<nblk, RS_THREADS, 0, s>>>(kin, vin, kout, vout, n, shift, nblk, w.counts,
                                                     w.totals);
            uint64_t* tk = kin; kin = kout; kout = tk;
            int32_t* tv = vin; vin = vout; vout = tv;
        }
        double* wsorted = reinterpret_cast<double*>(kout);  // the free ping-pong key buffer
        cf_tile_reduce<<<nblk, RS_THREADS, 0, s>>>(kin, vin, w.w, n, sentinel, w.blkcnt, w.tail, w.brk, wsorted);
        cf_head_scan<<<1, 1024, 0, s>>>(w.blkcnt, nblk, w.blkoff, out_n);
        cf_carry_scan<<<1, 1024, 0, s>>>(w.tail, w.brk, nblk, w.carry);
        cf_emit<<<nblk, RS_THREADS, 0, s>>>(kin, vin, wsorted, n, sentinel, w.blkoff, w.carry,
                                             reinterpret_cast<const unsigned long long*>(out_cnt), nullptr,
                                             bj, out_i, out_j, out_v, out_first);
    } else {
        (void)hipMemsetAsync(out_n, 0, sizeof(int64_t), s);
    }
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_itemcf_topn(const int64_t* row_off, int64_t n_rows, const int32_t* cols, const double* vals,
                    const int64_t* first, int topn, int32_t* out_cols, double* out_vals,
                    int32_t* out_cnt, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(topn >= 1, "topn must be >= 1");
    if (topn > CF_WIDE_MAX) NRK_UNSUPPORTED("topn must be <= 2048");
    NRK_REQUIRE(n_rows >= 0, "n_rows < 0");
    if (n_rows == 0) return NRK_OK;
    // cols / vals / first may be null when the CSR has no entries (empty torch tensors)
    NRK_REQUIRE(row_off && out_cols && out_vals && out_cnt, "null pointer");
    if (topn > 64) {
        const int K = cf_wide_k(topn);
        const size_t lds = (size_t)2 * K * sizeof(CfEnt);
        (void)hipFuncSetAttribute((const void*)cf_topn_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        cf_topn_wide_kernel<<<(int)(n_rows < 65536 ? n_rows : 65536), 64, lds, as_stream(stream)>>>(
            row_off, n_rows, cols, vals, first, topn, K, out_cols, out_vals, out_cnt);
        NRK_CHECK_LAUNCH();
        return NRK_OK;
    }
    const int64_t g = (n_rows + 3) / 4;
    cf_topn_kernel<<<(int)(g < 65536 ? g : 65536), 256, 0, as_stream(stream)>>>(
        row_off, n_rows, cols, vals, first, topn, out_cols, out_vals, out_cnt);
    const int64_t gw = (n_rows + 1023) / 1024;
    cf_topn_heavy_kernel<<<(int)(gw < 512 ? gw : 512), 1024, 0, as_stream(stream)>>>(
        row_off, n_rows, cols, vals, first, topn, out_cols, out_vals, out_cnt);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_itemcf_recall_offsets(const int64_t* q_slot, int64_t n_query, const int64_t* offsets,
                              const int32_t* items, const int32_t* nbr_cnt, int64_t* cand_off,
                              nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_query >= 0, "n_query < 0");
    NRK_REQUIRE(cand_off, "null pointer");
    hipStream_t s = as_stream(stream);
    if (n_query > 0) {
        NRK_REQUIRE(q_slot && offsets && items && nbr_cnt, "null pointer");
        const int64_t g = (n_query + 3) / 4;
        rc_count_kernel<<<(int)(g < 65536 ? g : 65536), 256, 0, s>>>(q_slot, n_query, offsets, items, nbr_cnt,
                                                                     cand_off);
    }
    scan_exclusive_kernel<ScanVals><<<1, 1024, 0, s>>>(ScanVals{cand_off}, n_query, cand_off);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_itemcf_recall_workspace_bytes(int64_t n_cand) {
    if (n_cand < 0) return 0;
    return rc_ws_layout(nullptr, n_cand).bytes;
}

int nrk_itemcf_recall(const int64_t* q_slot, int64_t n_query, const int64_t* offsets, const int32_t* items,
                      const int32_t* nbr_cols, const double* nbr_vals, const int32_t* nbr_cnt, int topn,
                      const double* created, int32_t n_items, const int32_t* hot, int n_hot,
                      const int32_t* emb_cols, const double* emb_vals, const int32_t* emb_cnt, int ke,
                      double loc_beta, double created_alpha, const int64_t* cand_off, int64_t n_cand,
                      int topk, int32_t* out_items, double* out_scores, int32_t* out_src,
                      int32_t* out_cnt, void* workspace, size_t workspace_bytes, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_query >= 0 && n_cand >= 0 && n_hot >= 0, "negative size");
    NRK_REQUIRE(topk >= 1, "topk must be >= 1");
    if (topk > CF_WIDE_MAX) NRK_UNSUPPORTED("topk must be <= 2048");
    NRK_REQUIRE(topn >= 1 && n_items >= 1 && ke >= 0, "bad sizes");
    NRK_REQUIRE(n_cand < (int64_t(1) << 31) - RS_TILE, "n_cand must be < 2^31");
    if (n_query == 0) return NRK_OK;
    NRK_REQUIRE(q_slot && offsets && items && nbr_cols && nbr_vals && nbr_cnt && created && cand_off &&
                    out_items && out_scores && out_src && out_cnt && workspace,
                "null pointer");
    NRK_REQUIRE(n_hot == 0 || hot, "hot is null");
    NRK_REQUIRE(ke == 0 || (emb_cols && emb_vals && emb_cnt), "emb arrays null");
    const RcWs w = rc_ws_layout(workspace, n_cand);
    NRK_REQUIRE(workspace_bytes >= w.bytes, "workspace too small");
    hipStream_t s = as_stream(stream);
    const int bj = bits_for(n_items);
    const int bq = bits_for(n_query);
    const int nbits = bj + bq;
    if (nbits > 64) NRK_UNSUPPORTED("n_query * n_items too large for 64-bit keys");
    const uint64_t sentinel = (nbits >= 64) ? ~0ull : ((1ull << nbits) - 1);
    const int64_t g = (n_query + 3) / 4;
    const int gq = (int)(g < 65536 ? g : 65536);
    const int64_t n = n_cand;
    const int nblk = (int)((n + RS_TILE - 1) / RS_TILE);
    const RcParams prm{loc_beta, created_alpha, cf_ln(created_alpha), topn, ke, bj};
    // topk <= 64: every query with <= RC_CAP candidates is finished by
    // rc_query_kernel from rc_cand's output; the radix path then runs over
    // the listed larger queries only, compacted to the front of the sort
    // buffers (device-side count: its launches exit at once when there are
    // none).  topk > 64: every query takes the radix path.
    const bool fused = topk <= 64;
    const int64_t* n_dev = nullptr;
    int gl = gq;
    if (n > 0) {
        rc_cand_kernel<<<gq, 256, 0, s>>>(q_slot, n_query, offsets, items, nbr_cols, nbr_vals, nbr_cnt, created,
                                          emb_cols, emb_vals, emb_cnt, prm, cand_off, sentinel, w.sort.ka,
                                          w.sort.va, w.sort.w);
        uint64_t* kin = w.sort.ka;
        uint64_t* kout = w.sort.kb;
        int32_t* vin = w.sort.va;
        int32_t* vout = w.sort.vb;
        if (fused) {
            (void)hipMemsetAsync(w.hcnt, 0, 16, s);
            static const int qgrid = [] {
                int dev = 0, cu = 256, per = 0;
                if (hipGetDevice(&dev) == hipSuccess)
                    (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)rc_query_kernel, 256, 0) !=
                        hipSuccess ||
                    per <= 0)
                    per = 4;
                return per * (cu > 0 ? cu : 256);
            }();
            rc_query_kernel<<<(int)(g < qgrid ? g : qgrid), 256, 0, s>>>(
                q_slot, n_query, offsets, items, cand_off, w.sort.ka, w.sort.w, sentinel, bj, hot, n_hot, topk,
                out_items, out_scores, out_src, out_cnt, w.hlist, w.hcnt, w.htot);
            const int64_t gh = (n / (RC_CAP + 1) + 4) / 4;
            gl = (int)(gh < 65536 ? gh : 65536);
            rc_compact_kernel<<<gl, 256, 0, s>>>(cand_off, kin, vin, w.hlist, w.hcnt, kout, vout);
            uint64_t* tk = kin; kin = kout; kout = tk;
            int32_t* tv = vin; vin = vout; vout = tv;
            n_dev = reinterpret_cast<const int64_t*>(w.htot);
        }
        for (int shift = 0; shift < nbits; shift += 8) {
            rs_upsweep<<<nblk, RS_THREADS, 0, s>>>(kin, n, shift, nblk, w.sort.counts, n_dev);
            rs_scan_rows<<<256, 256, 0, s>>>(w.sort.counts, nblk, w.sort.totals);
            rs_downsweep<<<nblk, RS_THREADS, 0, s>>>(kin, vin, kout, vout, n, shift, nblk, w.sort.counts,
                                                     w.sort.totals, n_dev);
            uint64_t* tk = kin; kin = kout; kout = tk;
            int32_t* tv = vin; vin = vout; vout = tv;
        }
        double* wsorted = reinterpret_cast<double*>(kout);
        cf_tile_reduce<<<nblk, RS_THREADS, 0, s>>>(kin, vin, w.sort.w, n, sentinel, w.sort.blkcnt, w.sort.tail,
                                                   w.sort.brk, wsorted, n_dev);
        cf_head_scan<<<1, 1024, 0, s>>>(w.sort.blkcnt, nblk, w.sort.blkoff, w.n_emit);
        cf_carry_scan<<<1, 1024, 0, s>>>(w.sort.tail, w.sort.brk, nblk, w.sort.carry);
        cf_emit<<<nblk, RS_THREADS, 0, s>>>(kin, vin, wsorted, n, sentinel, w.sort.blkoff, w.sort.carry, nullptr,
                                             nullptr, bj, w.eq, w.ej, w.ev, w.ef, n_dev);
    } else {
        (void)hipMemsetAsync(w.n_emit, 0, sizeof(int64_t), s);
        if (fused) (void)hipMemsetAsync(w.hcnt, 0, 16, s);
    }
    if (fused) {
        // n == 0: no listed queries, every query is a cold start or has no
        // candidates -> all of them through the list-free form
        if (n > 0)
            rc_topk_kernel<<<gl, 256, 0, s>>>(q_slot, n_query, offsets, items, hot, n_hot, w.eq, w.ej, w.ev, w.ef,
                                              w.n_emit, topk, out_items, out_scores, out_src, out_cnt, w.hlist,
                                              w.hcnt);
        else
            rc_topk_kernel<<<gq, 256, 0, s>>>(q_slot, n_query, offsets, items, hot, n_hot, w.eq, w.ej, w.ev, w.ef,
                                              w.n_emit, topk, out_items, out_scores, out_src, out_cnt);
    } else {
        const int K = cf_wide_k(topk);
        const size_t lds = (size_t)2 * K * sizeof(CfEnt);
        (void)hipFuncSetAttribute((const void*)rc_topk_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        rc_topk_wide_kernel<<<(int)(n_query < 65536 ? n_query : 65536), 64, lds, s>>>(
            q_slot, n_query, offsets, items, hot, n_hot, w.eq, w.ej, w.ev, w.ef, w.n_emit, topk, K, out_items,
            out_scores, out_src, out_cnt);
    }
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_itemcf_row_offsets(const int32_t* ei, int64_t n, int64_t n_rows, int64_t* row_off, nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n >= 0 && n_rows >= 0, "negative size");
    NRK_REQUIRE(row_off && (n == 0 || ei), "null pointer");
    const int64_t g = (n_rows + 1 + 255) / 256;
    cf_row_offsets_kernel<<<(int)(g < 65536 ? g : 65536), 256, 0, as_stream(stream)>>>(ei, n, n_rows, row_off);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

int nrk_itemcf_pairs(const int64_t* offsets, int64_t n_users, const int32_t* items, const int64_t* ts,
                     const double* created, int32_t n_items, const int64_t* pair_off, int64_t slot_base,
                     double loc_alpha, double loc_alpha_rev, double loc_beta, double time_alpha,
                     double created_alpha, uint64_t* keys, int32_t* slots, double* w, int64_t* item_cnt,
                     nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n_users >= 0 && slot_base >= 0 && n_items >= 1, "bad sizes");
    if (n_users == 0) return NRK_OK;
    NRK_REQUIRE(offsets && items && ts && created && pair_off && keys && slots && w && item_cnt, "null pointer");
    const int bj = bits_for(n_items);
    const int nbits = 2 * bj;
    const uint64_t sentinel = (nbits >= 64) ? ~0ull : ((1ull << nbits) - 1);
    const CfParams prm{loc_alpha, loc_alpha_rev, loc_beta, time_alpha, created_alpha, cf_dt_zero(time_alpha),
                       cf_ln(time_alpha), cf_ln(created_alpha)};
    // (the pair count lives on the device, pair_off[n_users]: a fixed
    // persistent grid walks it)
    cf_pairs_flat_kernel<<<2048, 256, 0, as_stream(stream)>>>(
        offsets, n_users, items, ts, created, pair_off, slot_base, prm, bj, sentinel, keys, slots, w);
    cf_item_count_kernel<<<1024, CF_CNT_THREADS, 0, as_stream(stream)>>>(
        offsets, n_users, items, reinterpret_cast<unsigned long long*>(item_cnt));
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

size_t nrk_itemcf_reduce_workspace_bytes(int64_t n) {
    if (n < 0) return 0;
    return cf_ws_layout(nullptr, n).bytes;
}

int nrk_itemcf_reduce(const uint64_t* keys, const int32_t* slots, const double* w, int64_t n, int32_t n_items,
                      const int64_t* item_cnt, int32_t* out_i, int32_t* out_j, double* out_v,
                      int64_t* out_first, int64_t* out_n, void* workspace, size_t workspace_bytes,
                      nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n >= 0 && n_items >= 1, "bad sizes");
    NRK_REQUIRE(n < (int64_t(1) << 31) - RS_TILE, "n must be < 2^31");
    NRK_REQUIRE(out_n && workspace, "null pointer");
    hipStream_t s = as_stream(stream);
    if (n == 0) {
        (void)hipMemsetAsync(out_n, 0, sizeof(int64_t), s);
        NRK_CHECK_LAUNCH();
        return NRK_OK;
    }
    NRK_REQUIRE(keys && slots && w && item_cnt && out_i && out_j && out_v && out_first, "null pointer");
    const CfWs ws = cf_ws_layout(workspace, n);
    NRK_REQUIRE(workspace_bytes >= ws.bytes, "workspace too small");
    const int bj = bits_for(n_items);
    const int nbits = 2 * bj;
    const uint64_t sentinel = (nbits >= 64) ? ~0ull : ((1ull << nbits) - 1);
    const int nblk = (int)((n + RS_TILE - 1) / RS_TILE);
    const int64_t g = (n + 255) / 256;
    cf_iota_copy_kernel<<<(int)(g < 65536 ? g : 65536), 256, 0, s>>>(keys, n, ws.ka, ws.va);
    uint64_t* kin = ws.ka;
    uint64_t* kout = ws.kb;
    int32_t* vin = ws.va;
    int32_t* vout = ws.vb;
    for (int shift = 0; shift < nbits; shift += 8) {
        rs_upsweep<<<nblk, RS_THREADS, 0, s>>>(kin, n, shift, nblk, ws.counts);
        rs_scan_rows<<<256, 256, 0, s>>>(ws.counts, nblk, ws.totals);
        rs_downsweep<<<nblk, RS_THREADS, 0, s>>>(kin, vin, kout, vout, n, shift, nblk, ws.counts, ws.totals);
        uint64_t* tk = kin; kin = kout; kout = tk;
        int32_t* tv = vin; vin = vout; vout = tv;
    }
    double* wsorted = reinterpret_cast<double*>(kout);
    cf_tile_reduce<<<nblk, RS_THREADS, 0, s>>>(kin, vin, w, n, sentinel, ws.blkcnt, ws.tail, ws.brk, wsorted);
    cf_head_scan<<<1, 1024, 0, s>>>(ws.blkcnt, nblk, ws.blkoff, out_n);
    cf_carry_scan<<<1, 1024, 0, s>>>(ws.tail, ws.brk, nblk, ws.carry);
    cf_emit<<<nblk, RS_THREADS, 0, s>>>(kin, vin, wsorted, n, sentinel, ws.blkoff, ws.carry,
                                         reinterpret_cast<const unsigned long long*>(item_cnt), slots, bj,
                                         out_i, out_j, out_v, out_first);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
