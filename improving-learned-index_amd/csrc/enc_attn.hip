// enc_attn.hip -- variable-length multi-head self-attention (head dim 64), gfx950.
//
// softmax(Q K^T / sqrt(64) + key-padding mask) V of the reference encoder
// (transformers XLMRobertaModel/BertModel self-attention, called at reference
// src/deep_impact/models/xlmr_original.py:70-75).  Documents are packed without
// padding (cu_seqlens), which equals the reference's padded computation at every
// real token: its padded keys carry a finfo.min mask and contribute exact zeros.
//
// One wave owns 16 queries of one (doc, head); a 256-thread block owns 64.
// "Swapped" products keep every operand in registers, no LDS:
//   S^T[key][q] = K Q^T          (A = K rows, B = Q rows: both 16-byte loads)
//   O^T[d][q]   = V^T P^T        (B = P^T is the S^T accumulator itself; the
//                                 MFMA k index is permuted consistently on A)
// V^T comes pre-transposed ([H][tokens]) from the QKV GEMM epilogue.
// Online softmax in f32 (exp2 with log2(e)/8 folded into the scores).
#include <hip/hip_runtime.h>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int ATT_D = 64;

template <typename T>
struct AttnOps;

// bf16: S^T tile (16 keys x 16 q) = 2 MFMA 16x16x32 over d; PV per 32 keys.
template <>
struct AttnOps<bf16> {
    static constexpr int KC = 32;  // MFMA k extent
    static constexpr int EPC = 8;  // elements per lane per k chunk
};
template <>
struct AttnOps<float> {
    static constexpr int KC = 16;  // 4 MFMA 16x16x4 per 16-byte chunk
    static constexpr int EPC = 4;
};

__device__ __forceinline__ void mma_chunk(const uint4 &a, const uint4 &b, f32x4 &acc, bf16) {
    bf16x8 av, bv;
    __builtin_memcpy(&av, &a, 16);
    __builtin_memcpy(&bv, &b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma_chunk(const uint4 &a, const uint4 &b, f32x4 &acc, float) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc,
                                               0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc,
                                               0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc,
                                               0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc,
                                               0, 0, 0);
}

// qk: [M][2H] (Q | K), vt: [H][ld_v] (V^T), ctx: [M][H]
template <typename T>
__global__ void __launch_bounds__(256)
attention_kernel(const T *__restrict__ qk, const T *__restrict__ vt,
                 const int32_t *__restrict__ cu_seqlens, int H, int ld_v, T *__restrict__ ctx) {
    constexpr int KC = AttnOps<T>::KC, EPC = AttnOps<T>::EPC;
    constexpr int NCH = ATT_D / KC;  // k chunks over the head dim
    const int doc = blockIdx.y, h = blockIdx.z;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int tok0 = cu_seqlens[doc], n = cu_seqlens[doc + 1] - tok0;
    const int q_base = blockIdx.x * 64 + wave * 16;
    if (q_base >= n) return;
    const int ldqk = 2 * H;
    const int qrow = tok0 + min(q_base + c, n - 1);

    // B operand: Q^T, lane (g, c): Q[q_base + c][chunk*KC + EPC*g + j]
    uint4 qf[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
        qf[ch] = *reinterpret_cast<const uint4 *>(qk + (int64_t)qrow * ldqk + h * ATT_D +
                                                   ch * KC + EPC * g);

    const float sc = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    float m = -INFINITY, lsum = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    const T *kbase = qk + H + h * ATT_D;
    const T *vbase = vt + (int64_t)(h * ATT_D) * ld_v + tok0;

    for (int key0 = 0; key0 < n; key0 += 32) {
        // ---- S^T for keys key0 .. key0+31 (two 16-key tiles) ----
        f32x4 s[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int krow = tok0 + min(key0 + 16 * t + c, n - 1);
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                uint4 kf = *reinterpret_cast<const uint4 *>(kbase + (int64_t)krow * ldqk +
                                                             ch * KC + EPC * g);
                mma_chunk(kf, qf[ch], s[t], T{});
            }
        }
        // lane holds S^T[key0 + 16t + 4g + r][q_base + c]
        float cmax = -INFINITY;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = key0 + 16 * t + 4 * g + r;
                float v = (key < n) ? s[t][r] * sc : -INFINITY;
                s[t][r] = v;
                cmax = fmaxf(cmax, v);
            }
        cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
        cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
        const float m_new = fmaxf(m, cmax);
        const float alpha = exp2f(m - m_new);  // 0 on the first chunk (m = -inf)
        m = m_new;
        lsum *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float p = exp2f(s[t][r] - m);
                s[t][r] = p;
                lsum += p;
            }
        // ---- O^T += V^T P^T ----
        if constexpr (sizeof(T) == 2) {
            // k permutation: slot (g, j<4) = key0 + 4g + j, (g, j>=4) = key0 + 16 + 4g + j-4
            bf16x8 pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pb[r] = (bf16)s[0][r];
                pb[4 + r] = (bf16)s[1][r];
            }
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                // V^T rows start at arbitrary token offsets: element loads (no
                // alignment assumption); the 32 keys of a chunk are one cache line pair
                const T *vrow = vbase + (int64_t)(dt * 16 + c) * ld_v + key0 + 4 * g;
                bf16x8 va;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    va[r] = vrow[r];
                    va[4 + r] = vrow[16 + r];
                }
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[dt], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const T *vrow = vbase + (int64_t)(dt * 16 + c) * ld_v + key0 + 16 * t + 4 * g;
                    float4 va = make_float4(vrow[0], vrow[1], vrow[2], vrow[3]);
                    o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(va.x, s[t][0], o[dt], 0, 0, 0);
                    o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(va.y, s[t][1], o[dt], 0, 0, 0);
                    o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(va.z, s[t][2], o[dt], 0, 0, 0);
                    o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(va.w, s[t][3], o[dt], 0, 0, 0);
                }
        }
    }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    const float inv = 1.0f / lsum;
    const int q = q_base + c;
    if (q < n) {
        T *out = ctx + (int64_t)(tok0 + q) * H + h * ATT_D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int r = 0; r < 4; ++r) out[dt * 16 + 4 * g + r] = from_f32<T>(o[dt][r] * inv);
    }
}

template <typename T>
void launch_attention(const T *qk, const T *vt, const int32_t *cu_seqlens, int n_docs,
                      int max_len, int H, int ld_v, T *ctx, hipStream_t s) {
    DI_REQUIRE(H % ATT_D == 0, DI_EINVAL, "hidden %d is not a multiple of the head dim 64", H);
    if (n_docs == 0 || max_len == 0) return;
    dim3 grid((max_len + 63) / 64, n_docs, H / ATT_D);
    hipLaunchKernelGGL(attention_kernel<T>, grid, dim3(256), 0, s, qk, vt, cu_seqlens, H, ld_v,
                       ctx);
    check_launch("attention");
}

template void launch_attention<bf16>(const bf16 *, const bf16 *, const int32_t *, int, int, int,
                                     int, bf16 *, hipStream_t);
template void launch_attention<float>(const float *, const float *, const int32_t *, int, int,
                                      int, int, float *, hipStream_t);

}  // namespace di
