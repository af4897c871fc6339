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

// GELU with erf, as torch.nn.functional.gelu (approximate='none')
__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
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
};

}  // namespace di
