// Counter calibration micro-kernels (dev tool, tools/pmc_busy.sh).
//
// mfma_loop: every wave issues back-to-back v_mfma_f32_32x32x16_f16 on four
//   independent accumulators, nothing else in the loop -> the matrix pipe of
//   every SIMD is busy all the time (the busy share should read 1.0).
// valu_loop: every wave issues independent v_fma_f32 (8 chains, inline asm so
//   the compiler cannot pack them), 8 waves per SIMD -> the VALU issue of
//   every SIMD is saturated.
// tools/pmc_busy.py divides the raw counter formulas of the real kernels by
// what these two read, so "1.0" means "as busy as a pure loop can make it".
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters) {
    half8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)(0.001f * (threadIdx.x & 7) + 0.01f * i);
        b[i] = (_Float16)(0.002f * (threadIdx.x & 3) - 0.01f * i);
    }
    float16v c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void valu_loop(float* out, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
          x7 = x0 + 7;
    const float m = 0.999f, c = 1e-3f;
    for (int it = 0; it < iters; ++it) {
        asm volatile(
            "v_fma_f32 %0, %0, %8, %9\n\t"
            "v_fma_f32 %1, %1, %8, %9\n\t"
            "v_fma_f32 %2, %2, %8, %9\n\t"
            "v_fma_f32 %3, %3, %8, %9\n\t"
            "v_fma_f32 %4, %4, %8, %9\n\t"
            "v_fma_f32 %5, %5, %8, %9\n\t"
            "v_fma_f32 %6, %6, %8, %9\n\t"
            "v_fma_f32 %7, %7, %8, %9"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(m), "v"(c));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main() {
    // 1024 blocks x 4 waves = 4 waves per SIMD (mfma), 2048 x 4 = 8 (valu)
    const int mfma_blocks = 1024, valu_blocks = 2048, mfma_iters = 20000, valu_iters = 100000;
    float* out;
    CK(hipMalloc(&out, sizeof(float) * valu_blocks * 256));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        CK(hipEventRecord(a));
        mfma_loop<<<mfma_blocks, 256>>>(out, mfma_iters);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        const double nm = 4.0 * mfma_iters * mfma_blocks * 4;
        printf("mfma_loop: %.3f ms, %.0f MFMA 32x32x16 -> %.1f TFLOP/s, %.2f GHz if 32 cyc/MFMA/SIMD\n", ms, nm,
               nm * 32768.0 / (ms * 1e-3) / 1e12, nm / 1024.0 * 32.0 / (ms * 1e-3) / 1e9);
        CK(hipEventRecord(a));
        valu_loop<<<valu_blocks, 256>>>(out, valu_iters);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        const double nv = 8.0 * valu_iters * valu_blocks * 4;
        printf("valu_loop: %.3f ms, %.0f wave-level v_fma_f32 -> %.2f per SIMD-ns\n", ms, nv,
               nv / 1024.0 / (ms * 1e6));
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(out));
    return 0;
}
