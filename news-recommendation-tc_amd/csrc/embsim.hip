// embsim.hip -- row L2 normalisation for the embedding-similarity search.
//
// EmbeddingSimilarity.calculate (src/similarity/embedding.py:35-41) builds
// the Faiss index from  item_emb_np / np.linalg.norm(item_emb_np, axis=1)
// in float32.  The self-search that follows (:46-50) is nrk_ip_topk over the
// same rows, so the normalised rows must be bit-identical to numpy's or
// near-tied neighbours could swap.  numpy computes the norm as
//   sqrt(add.reduce(x * x, axis=1))
// and float32 add.reduce over a contiguous axis is numpy's pairwise sum
// (numpy/_core/src/umath/loops_utils.h.src, @TYPE@_pairwise_sum): below 8
// elements a plain loop; up to 128 elements 8 strided accumulators combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail added in order; above
// 128 a split at n/2 rounded down to a multiple of 8, recursively.  Every
// product and sum below is a separately rounded op: the square passes through
// an empty asm so the backend cannot fuse it into the running sum (hipcc's
// fast contraction does so even across __fmul_rn / __fadd_rn); sqrt and
// division are the correctly rounded ones.
//
// One wave per 64 rows: the [64 x dim] tile is staged through LDS with
// coalesced loads, each lane reduces its own row (row stride dim | 1 words,
// so the 64 lanes hit 64 different banks), and the normalised tile is
// written back coalesced.
#include "nrk_common.h"

namespace nrk {

__device__ __forceinline__ float sq_rn(float x) {
    float p = __fmul_rn(x, x);
    asm volatile("" : "+v"(p));  // materialise the rounded product
    return p;
}

// numpy pairwise sum of squares, n <= 128 (the unrolled block)
__device__ float pw_leaf(const float* a, int n) {
    if (n < 8) {
        float r = 0.0f;
        for (int i = 0; i < n; ++i) r = __fadd_rn(r, sq_rn(a[i]));
        return r;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = sq_rn(a[j]);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], sq_rn(a[i + j]));
    }
    float res = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                          __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
    for (; i < n; ++i) res = __fadd_rn(res, sq_rn(a[i]));
    return res;
}

// two split levels cover n <= 256 (256 -> 128 + 128; 255 -> 120 + 135 -> 64 + 71)
template <int L>
__device__ float pw_sum(const float* a, int n) {
    if (L == 0 || n <= 128) return pw_leaf(a, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return __fadd_rn(pw_sum<(L > 0 ? L - 1 : 0)>(a, n2), pw_sum<(L > 0 ? L - 1 : 0)>(a + n2, n - n2));
}

__global__ __launch_bounds__(64) void row_normalize_kernel(const float* __restrict__ x, int64_t n,
                                                           int dim, float* __restrict__ out,
                                                           float* __restrict__ norms) {
    extern __shared__ float tile[];  // [64][dim | 1]
    const int st = dim | 1;
    const int lane = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * 64;
    const int rows = (int)(n - r0 < 64 ? n - r0 : 64);
    const int64_t tot = (int64_t)rows * dim;
    for (int64_t e = lane; e < tot; e += 64) {
        const int r = (int)(e / dim), d = (int)(e % dim);
        tile[r * st + d] = x[r0 * dim + e];
    }
    __syncthreads();
    float nr = 0.0f;
    if (lane < rows) {
        nr = sqrtf(pw_sum<2>(tile + lane * st, dim));
        if (norms) norms[r0 + lane] = nr;
    }
    __syncthreads();
    // every lane needs the norms of the rows it writes: stash them in LDS
    __shared__ float nrm[64];
    nrm[lane] = nr;
    __syncthreads();
    for (int64_t e = lane; e < tot; e += 64) {
        const int r = (int)(e / dim), d = (int)(e % dim);
        out[r0 * dim + e] = tile[r * st + d] / nrm[r];
    }
}

}  // namespace nrk

using namespace nrk;

extern "C" {

int nrk_row_normalize(const float* x, int64_t n, int dim, float* out, float* norms,
                      nrk_stream_t stream) {
    clear_error();
    NRK_REQUIRE(n >= 0, "negative row count");
    NRK_REQUIRE(dim >= 1 && dim <= 256, "dim must be in [1, 256]");
    if (n == 0) return NRK_OK;
    NRK_REQUIRE(x && out, "null pointer");
    const size_t lds = sizeof(float) * 64 * (size_t)(dim | 1);
    (void)hipFuncSetAttribute((const void*)row_normalize_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    row_normalize_kernel<<<(unsigned)((n + 63) / 64), 64, lds, as_stream(stream)>>>(x, n, dim, out,
                                                                                 norms);
    NRK_CHECK_LAUNCH();
    return NRK_OK;
}

}  // extern "C"
