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

typedef float f32x2 __attribute__((ext_vector_type(2)));

// erf for f32 without branches: x clamped to [-4, 4] (erf is +-1 in f32 beyond),
// x * P(x^2) / Q(x^2) rational minimax (the coefficients of Eigen's
// generic_fast_erf_float); a few ulp, vs ~117 instructions for ocml erff.
// Written on pairs so the epilogues run it as packed f32 math (v_pk_fma_f32).
__device__ __forceinline__ f32x2 fast_erf2(f32x2 x) {
    x = __builtin_elementwise_min(__builtin_elementwise_max(x, f32x2{-4.0f, -4.0f}),
                                  f32x2{4.0f, 4.0f});
    const f32x2 x2 = x * x;
#define DI_C2(c) f32x2{c, c}
    f32x2 p = DI_C2(-2.72614225801306e-10f);
    p = __builtin_elementwise_fma(x2, p, DI_C2(2.77068142495902e-08f));
    p = __builtin_elementwise_fma(x2, p, DI_C2(-2.10102402082508e-06f));
    p = __builtin_elementwise_fma(x2, p, DI_C2(-5.69250639462346e-05f));
    p = __builtin_elementwise_fma(x2, p, DI_C2(-7.34990630326855e-04f));
    p = __builtin_elementwise_fma(x2, p, DI_C2(-2.95459980854025e-03f));
    p = __builtin_elementwise_fma(x2, p, DI_C2(-1.60960333262415e-02f));
    p = p * x;
    f32x2 q = DI_C2(-1.45660718464996e-05f);
    q = __builtin_elementwise_fma(x2, q, DI_C2(-2.13374055278905e-04f));
    q = __builtin_elementwise_fma(x2, q, DI_C2(-1.68282697438203e-03f));
    q = __builtin_elementwise_fma(x2, q, DI_C2(-7.37332916720468e-03f));
    q = __builtin_elementwise_fma(x2, q, DI_C2(-1.42647390514189e-02f));
#undef DI_C2
    return p * f32x2{__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
}

// GELU with erf, as torch.nn.functional.gelu (approximate='none'):
// 0.5 x (1 + erf(x / sqrt 2)) = h + h * erf(...), h = x / 2
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
    const f32x2 e = fast_erf2(x * f32x2{0.70710678118654752440f, 0.70710678118654752440f});
    const f32x2 h = x * f32x2{0.5f, 0.5f};
    return __builtin_elementwise_fma(h, e, h);
}
__device__ __forceinline__ float gelu_erf(float x) { return gelu_erf2(f32x2{x, x}).x; }

// gelu_erf2 on 8 values at once, the four pair chains advanced in lockstep: each
// Horner step of one pair depends on the previous step, so one chain at a time runs
// at the dependent-issue latency; four independent chains fill those gaps.
__device__ __forceinline__ void gelu_erf8(float (&v)[8]) {
#define DI_C2(c) f32x2{c, c}
    f32x2 x[4], x2[4], p[4], q[4], h[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2 xi = f32x2{v[2 * i], v[2 * i + 1]};
        h[i] = xi * DI_C2(0.5f);
        x[i] = __builtin_elementwise_min(
            __builtin_elementwise_max(xi * DI_C2(0.70710678118654752440f), DI_C2(-4.0f)),
            DI_C2(4.0f));
        x2[i] = x[i] * x[i];
        p[i] = DI_C2(-2.72614225801306e-10f);
        q[i] = DI_C2(-1.45660718464996e-05f);
    }
    constexpr float PC[6] = {2.77068142495902e-08f, -2.10102402082508e-06f,
                             -5.69250639462346e-05f, -7.34990630326855e-04f,
                             -2.95459980854025e-03f, -1.60960333262415e-02f};
    constexpr float QC[4] = {-2.13374055278905e-04f, -1.68282697438203e-03f,
                             -7.37332916720468e-03f, -1.42647390514189e-02f};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            p[i] = __builtin_elementwise_fma(x2[i], p[i], DI_C2(PC[k]));
            if (k < 4) q[i] = __builtin_elementwise_fma(x2[i], q[i], DI_C2(QC[k]));
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2 e = p[i] * x[i] * f32x2{__builtin_amdgcn_rcpf(q[i].x), __builtin_amdgcn_rcpf(q[i].y)};
        const f32x2 y = __builtin_elementwise_fma(h[i], e, h[i]);
        v[2 * i] = y.x;
        v[2 * i + 1] = y.y;
    }
#undef DI_C2
}

// GELU for bf16 outputs: x * sigmoid(x P(x^2)) with P a cubic fitted to
// logit(Phi(x)) / x (the tanh form's quadratic refined), as x / (1 + 2^(x P'(x^2))),
// P' = -P log2(e).  |error| <= 1.1e-4 absolute and <= 6.6e-4 relative to max(|gelu|,
// 1e-3) -- a third of a bf16 output's rounding step -- in 7 packed ops and 4
// transcendentals per pair (gelu_erf8: 16 packed, 4 max/min, 2 transcendentals).
// Large |x|: 2^(+inf) -> rcp 0 -> -0 (x < 0), 2^(-inf) = 0 -> x (x > 0), as gelu.
// Only the bf16 epilogues use it; the fp32-faithful (split) outputs keep gelu_erf8.
__device__ __forceinline__ void gelu_bf16_8(float (&v)[8]) {
#define DI_C2(c) f32x2{c, c}
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2 x = f32x2{v[2 * i], v[2 * i + 1]};
        const f32x2 x2 = x * x;
        f32x2 p = __builtin_elementwise_fma(x2, DI_C2(-5.821808827022323e-06f),
                                            DI_C2(0.001257223659195006f));
        p = __builtin_elementwise_fma(x2, p, DI_C2(-0.10838031768798828f));
        p = __builtin_elementwise_fma(x2, p, DI_C2(-2.29897403717041f));
        const f32x2 z = x * p;
        const f32x2 d = f32x2{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} +
                        DI_C2(1.0f);
        const f32x2 y = x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
        v[2 * i] = y.x;
        v[2 * i + 1] = y.y;
    }
#undef DI_C2
}

__device__ __forceinline__ float gelu_bf16(float x) {
    float v[8] = {x, x, x, x, x, x, x, x};
    gelu_bf16_8(v);
    return v[0];
}

// GEMM epilogues
enum GemmEpi : int {
    EPI_BIAS = 0,        // out(T) = acc + bias
    EPI_BIAS_GELU = 1,   // out(T) = gelu(acc + bias)
    EPI_BIAS_RESID = 2,  // out(T) = acc + bias + resid(T), one rounding (pre-LayerNorm)
    EPI_QKV = 3,         // Q,K -> qk[M][2H] (T);  V -> vt[H][ldv] transposed (T)
    // (4: a fused-LayerNorm epilogue, removed -- measured slower than GEMM + LayerNorm)
    // LayerNorm folding (bf16, 256-col tiles): the GEMM that consumes LN(x) takes the
    // un-normalised x and weights W' = W diag(gamma) and corrects per row / column:
    //   LN(x) W^T + b = r (x W'^T) - r mu s + c,  s = W' 1,  c = b + W beta
    EPI_FOLD = 5,           // out(T) = r acc - r mu s + c           (row params: row_ln)
    EPI_FOLD_GELU = 6,      // out(T) = gelu(r acc - r mu s + c)
    EPI_RESID_STATS = 7,    // out(T) = acc + bias + LNin(resid), plus per-row partial
                            // (sum, sum of squares, head dot) of the rounded out over
                            // this tile's 256 columns -> stats_out[n0/256][row]
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
    int tune_gm;          // 256-tile kernel: M tiles per group in the tile order (0 = default)
    int ablate;           // profiling only (tools/gemm_check): 1 = skip the epilogue
    float ln_eps;
    // LayerNorm folding: row statistics as float4 partials (sum, sumsq, dot, 0) per
    // 256-column tile: stats[t * stats_ld + row], t < n_part
    const float2 *row_ln;     // EPI_FOLD*: (rstd, -rstd mean) of A's rows; EPI_RESID_STATS:
                              // of resid's rows (null: plain residual)
    float4 *stats_out;        // EPI_RESID_STATS
    int stats_ld, n_part, ln_h;
    const float *col_s, *col_c;          // EPI_FOLD*
    const float *res_gamma, *res_beta;   // EPI_RESID_STATS: LN params of resid
    const float *head_wg;                // EPI_RESID_STATS: w * gamma for the dot partial
    // split-bf16 (bf16x3, the fp32-faithful mode): A and B rows are split rows (see
    // split_col: every 32 columns as 32 hi then 32 lo bf16, row stride 2K), so that one
    // 64-wide K tile holds the hi and lo halves of 32 k and each (A, B) fragment pair
    // gives three MFMAs, acc += A_hi B_hi + A_lo B_hi + A_hi B_lo, in f32.  Outputs:
    // EPI_BIAS / EPI_BIAS_GELU split rows (ld_out = 2N), EPI_BIAS_RESID f32 rows (resid
    // split).  (The fp32-faithful QKV projection is EPI_BIAS into split rows [M][6H].)
    int split;
};

// v = hi + lo with hi = bf16(v), lo = bf16(v - hi): 16 significant bits, relative
// error <= 2^-17 (the split-bf16 storage of the fp32-faithful mode)
// Split rows: logical column c of a row of width W sits at split_col(c) (hi) and
// split_col(c) + 32 (lo) of a 2W-wide bf16 row -- 32-column chunks of hi then lo.
__host__ __device__ __forceinline__ int64_t split_col(int64_t c) { return (c >> 5) * 64 + (c & 31); }
__device__ __forceinline__ bf16 split_hi(float v) { return (bf16)v; }
__device__ __forceinline__ bf16 split_lo(float v) { return (bf16)(v - (float)(bf16)v); }


}  // namespace di
