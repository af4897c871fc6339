// enc_common.h -- shared definitions of the DeeperImpact encoder kernels (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace di {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T>
__device__ __forceinline__ T from_f32(float x);
template <>
__device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <>
__device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// erf for f32 without branches: x clamped to [-4, 4] (erf is +-1 in f32 beyond),
// x * P(x^2) / Q(x^2) rational minimax (the coefficients of Eigen's
// generic_fast_erf_float); a few ulp, vs ~117 instructions for ocml erff.
__device__ __forceinline__ float fast_erf(float x) {
    x = fminf(fmaxf(x, -4.0f), 4.0f);
    const float x2 = x * x;
    float p = -2.72614225801306e-10f;
    p = fmaf(x2, p, 2.77068142495902e-08f);
    p = fmaf(x2, p, -2.10102402082508e-06f);
    p = fmaf(x2, p, -5.69250639462346e-05f);
    p = fmaf(x2, p, -7.34990630326855e-04f);
    p = fmaf(x2, p, -2.95459980854025e-03f);
    p = fmaf(x2, p, -1.60960333262415e-02f);
    p *= x;
    float q = -1.45660718464996e-05f;
    q = fmaf(x2, q, -2.13374055278905e-04f);
    q = fmaf(x2, q, -1.68282697438203e-03f);
    q = fmaf(x2, q, -7.37332916720468e-03f);
    q = fmaf(x2, q, -1.42647390514189e-02f);
    return __fdividef(p, q);
}

// GELU with erf, as torch.nn.functional.gelu (approximate='none')
__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + fast_erf(x * 0.70710678118654752440f));
}

// GEMM epilogues
enum GemmEpi : int {
    EPI_BIAS = 0,        // out(T) = acc + bias
    EPI_BIAS_GELU = 1,   // out(T) = gelu(acc + bias)
    EPI_BIAS_RESID = 2,  // out(f32) = acc + bias + resid(T)      (pre-LayerNorm)
    EPI_QKV = 3,         // Q,K -> qk[M][2H] (T);  V -> vt[H][ldv] transposed (T)
};

struct GemmArgs {
    const void *A;      // [M][K]
    const void *B;      // [N][K]   (nn.Linear weight layout: out x in)
    const float *bias;  // [N]
    const void *resid;  // [M][N] (EPI_BIAS_RESID)
    void *out;          // see GemmEpi
    void *out2;         // EPI_QKV: V^T buffer
    int M, N, K;
    int ld_out;         // row stride of out (elements)
    int ld_v;           // EPI_QKV: row stride of V^T (tokens, padded)
    int hidden;         // EPI_QKV: H (Q | K | V split points)
    const int32_t *vcol;  // EPI_QKV: V^T column of every token row (doc-aligned layout)
    int64_t a_rows;       // rows of A that may be read (>= M; slack lets 256-row tiles
                          // read past M without clamping)
};

}  // namespace di
