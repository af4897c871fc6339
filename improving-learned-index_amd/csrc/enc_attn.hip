// enc_attn.hip -- variable-length multi-head self-attention (head dim 64), gfx950.
//
// softmax(Q K^T / sqrt(64) + key-padding mask) V of the reference encoder
// (transformers XLMRobertaModel/BertModel self-attention, called at reference
// src/deep_impact/models/xlmr_original.py:70-75).  Documents are packed without
// padding (cu_seqlens), which equals the reference's padded computation at every
// real token: its padded keys carry a finfo.min mask and contribute exact zeros.
//
// One wave owns QT*16 queries of one (doc, head).  "Swapped" products keep every
// operand in registers, no LDS:
//   S^T[key][q] = K Q^T          (A = K rows, B = Q rows: 16-byte loads)
//   O^T[d][q]   = V^T P^T        (B = P^T is the S^T accumulator itself; the
//                                 MFMA k index is permuted consistently on A)
// V^T comes pre-transposed from the QKV GEMM epilogue, laid out [H][ld_v] with
// every document starting at a 4-aligned column vbase(d) = 4*(d + cu[d]/4), so
// 4 consecutive keys are one 8-byte (bf16) / 16-byte (f32) load.
// Online softmax in f32 (exp2 with log2(e)/8 folded into the scores).
#include <hip/hip_runtime.h>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int ATT_D = 64;
constexpr int QT = 4;  // query tiles of 16 per wave

__device__ __forceinline__ int vt_base(int doc, int tok0) { return 4 * (doc + (tok0 >> 2)); }

template <typename T>
struct AttnOps;
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

// qk: [M][2H] (Q | K), vt: [H][ld_v] (V^T, doc-aligned columns), ctx: [M][H]
template <typename T>
__global__ void __launch_bounds__(64)
attention_kernel(const T *__restrict__ qk, const T *__restrict__ vt,
                 const int32_t *__restrict__ cu_seqlens, int H, int ld_v, int n_qb, int n_heads,
                 int n_pairs, T *__restrict__ ctx) {
    constexpr int KC = AttnOps<T>::KC, EPC = AttnOps<T>::EPC;
    constexpr int NCH = ATT_D / KC;  // k chunks over the head dim
    // 1-D grid, XCD-grouped (speed only): the QB query blocks of one (doc, head)
    // are ids j*8 + x for j in one run of QB -- all on XCD x under round-robin
    // dispatch -- so they share K / V^T through that XCD's L2.
    const int id = blockIdx.x, x = id & 7, j = id >> 3;
    const int pair = (j / n_qb) * 8 + x;  // (doc, head) pair index
    const int qb = j % n_qb;
    if (pair >= n_pairs) return;
    const int doc = pair / n_heads, h = pair % n_heads;
    const int lane = threadIdx.x;
    const int g = lane >> 4, c = lane & 15;
    const int tok0 = cu_seqlens[doc], n = cu_seqlens[doc + 1] - tok0;
    const int q_base = qb * (16 * QT);
    if (q_base >= n) return;
    const int ldqk = 2 * H;

    // B operands: Q^T tiles, lane (g, c): Q[q_base + 16 qt + c][chunk*KC + EPC*g + j]
    uint4 qf[QT][NCH];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int qrow = tok0 + min(q_base + 16 * qt + c, n - 1);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
            qf[qt][ch] = *reinterpret_cast<const uint4 *>(qk + (int64_t)qrow * ldqk + h * ATT_D +
                                                          ch * KC + EPC * g);
    }
    const float sc = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    float m[QT], lsum[QT];
    f32x4 o[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        m[qt] = -INFINITY;
        lsum[qt] = 0.f;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const T *kbase = qk + H + h * ATT_D;
    const T *vbase = vt + (int64_t)(h * ATT_D) * ld_v + vt_base(doc, tok0);

    for (int key0 = 0; key0 < n; key0 += 32) {
        // ---- K fragments of 32 keys (two 16-key tiles), V^T fragments ----
        uint4 kf[2][NCH];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int krow = tok0 + min(key0 + 16 * t + c, n - 1);
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch)
                kf[t][ch] = *reinterpret_cast<const uint4 *>(kbase + (int64_t)krow * ldqk +
                                                             ch * KC + EPC * g);
        }
        // V^T: lane (g, c) of d-tile dt needs d = 16 dt + c, keys key0+4g..+3 and
        // key0+16+4g..+3 (the P^T k permutation)
        uint4 vf[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const T *vrow = vbase + (int64_t)(dt * 16 + c) * ld_v + key0 + 4 * g;
            if constexpr (sizeof(T) == 2) {
                uint2 lo = *reinterpret_cast<const uint2 *>(vrow);
                uint2 hi = *reinterpret_cast<const uint2 *>(vrow + 16);
                vf[dt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
            } else {
                vf[dt] = *reinterpret_cast<const uint4 *>(vrow);  // keys 4g..4g+3 (tile 0)
            }
        }
        uint4 vf1[4];  // f32: tile 1 keys
        if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
                vf1[dt] = *reinterpret_cast<const uint4 *>(
                    vbase + (int64_t)(dt * 16 + c) * ld_v + key0 + 16 + 4 * g);
        }
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            f32x4 s[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ch = 0; ch < NCH; ++ch) mma_chunk(kf[t][ch], qf[qt][ch], s[t], T{});
            }
            // lane holds S^T[key0 + 16t + 4g + r][q_base + 16 qt + c]
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
            const float m_new = fmaxf(m[qt], cmax);
            const float alpha = exp2f(m[qt] - m_new);  // 0 on the first chunk
            m[qt] = m_new;
            lsum[qt] *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float p = exp2f(s[t][r] - m_new);
                    s[t][r] = p;
                    lsum[qt] += p;
                }
            if constexpr (sizeof(T) == 2) {
                bf16x8 pb;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    pb[r] = (bf16)s[0][r];
                    pb[4 + r] = (bf16)s[1][r];
                }
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    bf16x8 va;
                    __builtin_memcpy(&va, &vf[dt], 16);
                    o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[qt][dt], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const uint4 &a0 = vf[dt];
                    const uint4 &a1 = vf1[dt];
                    f32x4 acc = o[qt][dt];
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a0.x), s[0][0], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a0.y), s[0][1], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a0.z), s[0][2], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a0.w), s[0][3], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a1.x), s[1][0], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a1.y), s[1][1], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a1.z), s[1][2], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a1.w), s[1][3], acc, 0, 0, 0);
                    o[qt][dt] = acc;
                }
            }
        }
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        float l = lsum[qt];
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        const float inv = 1.0f / l;
        const int q = q_base + 16 * qt + c;
        if (q < n) {
            T *out = ctx + (int64_t)(tok0 + q) * H + h * ATT_D + 4 * g;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                if constexpr (sizeof(T) == 2) {
                    bf16x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[qt][dt][r] * inv);
                    *reinterpret_cast<bf16x4 *>(out + dt * 16) = v;
                } else {
                    *reinterpret_cast<float4 *>(out + dt * 16) =
                        make_float4(o[qt][dt][0] * inv, o[qt][dt][1] * inv, o[qt][dt][2] * inv,
                                    o[qt][dt][3] * inv);
                }
            }
        }
    }
}

// column of token `row` in the doc-aligned V^T layout
__global__ void vt_cols_kernel(const int32_t *__restrict__ cu, int n_docs, int M,
                               int32_t *__restrict__ vcol) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= M) return;
    int lo = 0, hi = n_docs;
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (cu[mid] <= row) lo = mid;
        else hi = mid;
    }
    vcol[row] = vt_base(lo, cu[lo]) + (row - cu[lo]);
}

void launch_vt_cols(const int32_t *cu, int n_docs, int M, int32_t *vcol, hipStream_t s) {
    if (M == 0) return;
    hipLaunchKernelGGL(vt_cols_kernel, dim3((M + 255) / 256), dim3(256), 0, s, cu, n_docs, M,
                       vcol);
    check_launch("vt_cols");
}

int vt_ld(int64_t M, int n_docs) {
    // 4*(n_docs + M/4) + 32 keys of read-ahead, rounded to 64 columns
    int64_t need = 4 * ((int64_t)n_docs + M / 4) + 64 + 32;
    return (int)((need + 63) / 64 * 64);
}

template <typename T>
void launch_attention(const T *qk, const T *vt, const int32_t *cu_seqlens, int n_docs,
                      int max_len, int H, int ld_v, T *ctx, hipStream_t s) {
    DI_REQUIRE(H % ATT_D == 0, DI_EINVAL, "hidden %d is not a multiple of the head dim 64", H);
    if (n_docs == 0 || max_len == 0) return;
    const int n_qb = (max_len + 16 * QT - 1) / (16 * QT), n_heads = H / ATT_D;
    const int n_pairs = n_docs * n_heads;
    const int64_t blocks = (int64_t)((n_pairs + 7) / 8) * 8 * n_qb;
    DI_REQUIRE(blocks < (1ll << 31), DI_ERANGE, "attention grid too large");
    hipLaunchKernelGGL(attention_kernel<T>, dim3((unsigned)blocks), dim3(64), 0, s, qk, vt,
                       cu_seqlens, H, ld_v, n_qb, n_heads, n_pairs, ctx);
    check_launch("attention");
}

template void launch_attention<bf16>(const bf16 *, const bf16 *, const int32_t *, int, int, int,
                                     int, bf16 *, hipStream_t);
template void launch_attention<float>(const float *, const float *, const int32_t *, int, int,
                                      int, int, float *, hipStream_t);

}  // namespace di
