// enc_misc.hip -- memory-bound encoder kernels (gfx950): embeddings + LayerNorm,
// LayerNorm (+ the impact head), first-token term gather with the 3-decimal
// rounding, and the 8-bit quantizer.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int LN_MAX_PER_LANE = 16;  // H <= 1024

__device__ __forceinline__ float wave_sum_f(float x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// LayerNorm of one row held as v[i] = x[lane + 64 i] (two-pass, biased variance,
// eps inside the sqrt -- torch.nn.functional.layer_norm).
template <int PL>
__device__ __forceinline__ void ln_row(float (&v)[PL], int H, const float *gamma,
                                       const float *beta, float eps) {
    const int lane = threadIdx.x & 63;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PL; ++i)
        if (lane + 64 * i < H) s += v[i];
    const float mean = wave_sum_f(s) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PL; ++i)
        if (lane + 64 * i < H) {
            float d = v[i] - mean;
            q += d * d;
        }
    const float rstd = 1.0f / sqrtf(wave_sum_f(q) / (float)H + eps);
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const int c = lane + 64 * i;
        if (c < H) v[i] = (v[i] - mean) * rstd * gamma[c] + beta[c];
    }
}

__device__ __forceinline__ int find_doc(const int32_t *cu, int n_docs, int row) {
    int lo = 0, hi = n_docs;  // cu[lo] <= row < cu[hi]
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (cu[mid] <= row) lo = mid;
        else hi = mid;
    }
    return lo;
}

// x0 = LN(word[id] + pos[p] + type[0]);  p = i (BERT) or pad + 1 + i (RoBERTa:
// create_position_ids_from_input_ids on an unpadded row).  One wave per token.
template <typename T, int PL>
__global__ void __launch_bounds__(256)
embed_ln_kernel(const int32_t *__restrict__ ids, const int32_t *__restrict__ cu, int n_docs,
                int M, int H, const T *__restrict__ word, const T *__restrict__ pos,
                const T *__restrict__ type0, const float *__restrict__ gamma,
                const float *__restrict__ beta, float eps, int pos_offset, int vocab,
                int max_pos, T *__restrict__ out, int32_t *__restrict__ err) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int lane = threadIdx.x & 63;
    const int d = find_doc(cu, n_docs, row);
    const int p = row - cu[d] + pos_offset;
    int id = ids[row];
    if (id < 0 || id >= vocab || p >= max_pos) {
        if (lane == 0) atomicOr(err, 1);
        id = min(max(id, 0), vocab - 1);
    }
    const int pp = min(p, max_pos - 1);
    const T *wr = word + (int64_t)id * H;
    const T *pr = pos + (int64_t)pp * H;
    float v[PL];
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const int c = lane + 64 * i;
        v[i] = (c < H) ? to_f32(wr[c]) + to_f32(pr[c]) + to_f32(type0[c]) : 0.f;
    }
    ln_row<PL>(v, H, gamma, beta, eps);
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const int c = lane + 64 * i;
        if (c < H) out[(int64_t)row * H + c] = from_f32<T>(v[i]);
    }
}

// Impact head of the reference (xlmr_original.py:34-38, :77-85) on the f32 LN
// output row: impact = act(x . w + b), act = Softplus(beta 1, threshold 20) or ReLU.
__device__ __forceinline__ void head_out(float s, float head_b, int act, float *impact, int row) {
    s = wave_sum_f(s) + head_b;
    if ((threadIdx.x & 63) == 0) {
        float y;
        if (act == 0)  // nn.Softplus(beta=1, threshold=20)
            y = (s > 20.0f) ? s : log1pf(expf(s));
        else
            y = s > 0.f ? s : 0.f;
        impact[row] = y;
    }
}

// x = LN(pre) (pre = GEMM output + bias + residual, T), one wave per row; with
// head_w also the impact head.  Generic layout: lane holds x[lane + 64 i].
template <typename T, int PL>
__global__ void __launch_bounds__(256)
ln_kernel(const T *__restrict__ pre, int M, int H, const float *__restrict__ gamma,
          const float *__restrict__ beta, float eps, T *__restrict__ out,
          const float *__restrict__ head_w, float head_b, int act, float *__restrict__ impact) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int lane = threadIdx.x & 63;
    float v[PL];
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const int c = lane + 64 * i;
        v[i] = (c < H) ? to_f32(pre[(int64_t)row * H + c]) : 0.f;
    }
    ln_row<PL>(v, H, gamma, beta, eps);
    if (out) {
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            const int c = lane + 64 * i;
            if (c < H) out[(int64_t)row * H + c] = from_f32<T>(v[i]);
        }
    }
    if (head_w) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            const int c = lane + 64 * i;
            if (c < H) s += v[i] * head_w[c];
        }
        head_out(s, head_b, act, impact, row);
    }
}

// Vector form for H = 256 NC: lane holds x[256 c + 4 lane + j], j < 4 -- one
// 8-byte (bf16) / 16-byte (f32) access per chunk instead of four scalar ones.
template <typename T>
__device__ __forceinline__ void ld4(const T *p, float (&f)[4]);
template <>
__device__ __forceinline__ void ld4<bf16>(const bf16 *p, float (&f)[4]) {
    const bf16x4 v = *reinterpret_cast<const bf16x4 *>(p);
    f[0] = (float)v[0]; f[1] = (float)v[1]; f[2] = (float)v[2]; f[3] = (float)v[3];
}
template <>
__device__ __forceinline__ void ld4<float>(const float *p, float (&f)[4]) {
    const float4 v = *reinterpret_cast<const float4 *>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
}
__device__ __forceinline__ void st4(bf16 *p, const float (&f)[4]) {
    *reinterpret_cast<bf16x4 *>(p) = bf16x4{(bf16)f[0], (bf16)f[1], (bf16)f[2], (bf16)f[3]};
}
__device__ __forceinline__ void st4(float *p, const float (&f)[4]) {
    *reinterpret_cast<float4 *>(p) = make_float4(f[0], f[1], f[2], f[3]);
}
// split-bf16 row store (fp32-faithful mode): 4 columns col.. of one 32-column chunk
// of the split row at p (enc_common.h split_col)
__device__ __forceinline__ void st4_split(bf16 *p, int col, const float (&f)[4]) {
    bf16x4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) hi[j] = split_hi(f[j]), lo[j] = split_lo(f[j]);
    *reinterpret_cast<bf16x4 *>(p + split_col(col)) = hi;
    *reinterpret_cast<bf16x4 *>(p + split_col(col) + 32) = lo;
}
// row store of the LayerNorm kernels: OUT = T (plain rows) or split rows of 2H bf16
template <typename T, bool SPLIT>
struct LnOut {
    typedef typename std::conditional<SPLIT, bf16, T>::type type;
};
template <bool SPLIT, typename O>
__device__ __forceinline__ void st4_row(O *out, int64_t row, int H, int col, const float (&f)[4]) {
    if constexpr (SPLIT)
        st4_split(out + row * 2 * H, col, f);
    else
        st4(out + row * H + col, f);
}

template <typename T, int NC, bool SPLIT = false>
__global__ void __launch_bounds__(256)
ln_vec_kernel(const T *__restrict__ pre, int M, const float *__restrict__ gamma,
              const float *__restrict__ beta, float eps,
              typename LnOut<T, SPLIT>::type *__restrict__ out,
              const float *__restrict__ head_w, float head_b, int act, float *__restrict__ impact) {
    constexpr int H = 256 * NC;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int lane = threadIdx.x & 63;
    float v[NC][4];
#pragma unroll
    for (int c = 0; c < NC; ++c) ld4<T>(pre + (int64_t)row * H + 256 * c + 4 * lane, v[c]);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += (v[c][0] + v[c][1]) + (v[c][2] + v[c][3]);
    const float mean = wave_sum_f(s) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float d = v[c][j] - mean;
            q += d * d;
        }
    const float rstd = 1.0f / sqrtf(wave_sum_f(q) / (float)H + eps);
    float hs = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        float gm[4], bt[4];
        ld4<float>(gamma + 256 * c + 4 * lane, gm);
        ld4<float>(beta + 256 * c + 4 * lane, bt);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[c][j] = (v[c][j] - mean) * rstd * gm[j] + bt[j];
        if (out) st4_row<SPLIT>(out, row, H, 256 * c + 4 * lane, v[c]);
        if (head_w) {
            float w[4];
            ld4<float>(head_w + 256 * c + 4 * lane, w);
#pragma unroll
            for (int j = 0; j < 4; ++j) hs += v[c][j] * w[j];
        }
    }
    if (head_w) head_out(hs, head_b, act, impact, row);
}

// embed_ln for H = 256 NC (XLM-R / BERT base and large): one workgroup per document,
// so the position is the row's offset in the document (no per-token search over the
// document offsets), 4 waves x 2 rows in flight, lane holds 4 consecutive columns of
// each 256-column chunk (8-byte loads, the ln_vec_kernel layout and arithmetic).
template <typename T, int NC, bool SPLIT = false>
__global__ void __launch_bounds__(256)
embed_ln_vec_kernel(const int32_t *__restrict__ ids, const int32_t *__restrict__ cu,
                    const T *__restrict__ word, const T *__restrict__ pos,
                    const T *__restrict__ type0, const float *__restrict__ gamma,
                    const float *__restrict__ beta, float eps, int pos_offset, int vocab,
                    int max_pos, typename LnOut<T, SPLIT>::type *__restrict__ out,
                    int32_t *__restrict__ err) {
    constexpr int H = 256 * NC, RB = 2;
    const int d = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r0 = cu[d], n = cu[d + 1] - r0;
    float gm[NC][4], bt[NC][4], ty[NC][4];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        ld4<float>(gamma + 256 * c + 4 * lane, gm[c]);
        ld4<float>(beta + 256 * c + 4 * lane, bt[c]);
        ld4<T>(type0 + 256 * c + 4 * lane, ty[c]);
    }
    for (int i0 = wave * RB; i0 < n; i0 += 4 * RB) {
        float v[RB][NC][4];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int i = min(i0 + r, n - 1);  // clamped: loads stay unconditional
            const int p = i + pos_offset;
            int id = ids[r0 + i];
            if (id < 0 || id >= vocab || p >= max_pos) {
                if (lane == 0) atomicOr(err, 1);
                id = min(max(id, 0), vocab - 1);
            }
            const T *wr = word + (int64_t)id * H + 4 * lane;
            const T *pr = pos + (int64_t)min(p, max_pos - 1) * H + 4 * lane;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                float w4[4], p4[4];
                ld4<T>(wr + 256 * c, w4);
                ld4<T>(pr + 256 * c, p4);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[r][c][j] = w4[j] + p4[j] + ty[c][j];
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            if (i0 + r >= n) break;
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) s += (v[r][c][0] + v[r][c][1]) + (v[r][c][2] + v[r][c][3]);
            const float mean = wave_sum_f(s) / (float)H;
            float q = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float dd = v[r][c][j] - mean;
                    q += dd * dd;
                }
            const float rstd = 1.0f / sqrtf(wave_sum_f(q) / (float)H + eps);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[r][c][j] = (v[r][c][j] - mean) * rstd * gm[c][j] + bt[c][j];
                st4_row<SPLIT>(out, (int64_t)(r0 + i0 + r), H, 256 * c + 4 * lane, v[r][c]);
            }
        }
    }
}

// LayerNorm folding: per-row (rstd, -rstd * mean) from the row-statistics partials
// of the producing GEMM (biased variance as torch layer_norm; fixed summation order).
__global__ void row_ln_kernel(const float4 *__restrict__ st, int ld, int n_part, int M, int H,
                              float eps, float2 *__restrict__ out) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    float s = 0.f, q = 0.f;
    for (int t = 0; t < n_part; ++t) {
        const float4 v = st[(int64_t)t * ld + m];
        s += v.x;
        q += v.y;
    }
    const float mean = s / (float)H;
    const float rstd = 1.0f / sqrtf(fmaxf(q / (float)H - mean * mean, 0.f) + eps);
    out[m] = make_float2(rstd, -rstd * mean);
}

void launch_row_ln(const float4 *st, int ld, int n_part, int M, int H, float eps, float2 *out,
                   hipStream_t s) {
    if (M == 0) return;
    hipLaunchKernelGGL(row_ln_kernel, dim3((M + 255) / 256), dim3(256), 0, s, st, ld, n_part, M,
                       H, eps, out);
    check_launch("row_ln");
}

// Impact head when the last LayerNorm is folded (encoder LN folding): from the
// row statistics of the last FFN output (sum, sumsq, dot with w * gamma),
//   LN(x) . w + b = r (x . (w gamma) - mu sw) + cw,  sw = sum(w gamma), cw = b + w . beta
__global__ void head_from_stats_kernel(const float4 *__restrict__ st, int ld, int n_part, int M,
                                       int H, float eps, float sw, float cw, int act,
                                       float *__restrict__ impact) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    float s = 0.f, q = 0.f, d = 0.f;
    for (int t = 0; t < n_part; ++t) {
        const float4 v = st[(int64_t)t * ld + m];
        s += v.x;
        q += v.y;
        d += v.z;
    }
    const float mean = s / (float)H;
    const float rstd = 1.0f / sqrtf(fmaxf(q / (float)H - mean * mean, 0.f) + eps);
    const float x = rstd * (d - mean * sw) + cw;
    impact[m] = act == 0 ? ((x > 20.0f) ? x : log1pf(expf(x))) : (x > 0.f ? x : 0.f);
}

void launch_head_from_stats(const float4 *st, int ld, int n_part, int M, int H, float eps,
                            float sw, float cw, int act, float *impact, hipStream_t s) {
    if (M == 0) return;
    hipLaunchKernelGGL(head_from_stats_kernel, dim3((M + 255) / 256), dim3(256), 0, s, st, ld,
                       n_part, M, H, eps, sw, cw, act, impact);
    check_launch("head_from_stats");
}

// numpy's round(np.float32, 3) (reference indexer.py:132): fl32(rint(fl32(x*1000))/1000)
__device__ __forceinline__ float round3(float x) {
    float t = __fmul_rn(x, 1000.0f);
    return __fdiv_rn(rintf(t), 1000.0f);
}

// compute_term_impacts (xlmr_original.py:205-225): impact of the first token of
// every unique term.  term_tok is relative to the doc's first token.
__global__ void gather_terms_kernel(const float *__restrict__ impact,
                                    const int32_t *__restrict__ cu_seq,
                                    const int32_t *__restrict__ cu_terms, int n_docs,
                                    const int32_t *__restrict__ term_tok, int n_terms, int do_round,
                                    float *__restrict__ out, int32_t *__restrict__ err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_terms) return;
    const int d = find_doc(cu_terms, n_docs, i);
    const int tok = term_tok[i];
    const int len = cu_seq[d + 1] - cu_seq[d];
    float v = 0.f;
    if (tok < 0 || tok >= len) {
        atomicOr(err, 2);
    } else {
        // pruned: the last layer computed only the terms' rows, row i = term i
        v = impact[do_round & 2 ? i : cu_seq[d] + tok];
    }
    out[i] = (do_round & 1) ? round3(v) : v;
}

// The encoder's pruned last layer: the layer-input rows (and their LayerNorm row
// parameters) of the terms' first tokens, packed in term order.  One workgroup per
// document, one wave per row, 8-byte copies.
__global__ void __launch_bounds__(256)
gather_term_rows_kernel(const bf16 *__restrict__ X, const float2 *__restrict__ rl,
                        const int32_t *__restrict__ cu_seq, const int32_t *__restrict__ cu_terms,
                        const int32_t *__restrict__ term_tok, int H, bf16 *__restrict__ Xg,
                        float2 *__restrict__ rlg) {
    const int d = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t0 = cu_seq[d], n = cu_seq[d + 1] - t0;
    for (int j = cu_terms[d] + wave; j < cu_terms[d + 1]; j += 4) {
        const int row = t0 + min(max(term_tok[j], 0), max(n - 1, 0));  // (checked by the gather)
        const uint2 *src = reinterpret_cast<const uint2 *>(X + (int64_t)row * H);
        uint2 *dst = reinterpret_cast<uint2 *>(Xg + (int64_t)j * H);
        for (int c = lane; c < H / 4; c += 64) dst[c] = src[c];
        if (rl && lane == 0) rlg[j] = rl[row];
    }
}

// The inverse for the pruned last layer's queries: packed row j (term j) -> row t0 +
// term_tok[j] (same clamp) of a [tokens][ld] matrix, its first W elements (a repeated
// token receives the same row twice: the same bytes).
__global__ void __launch_bounds__(256)
scatter_term_rows_kernel(const bf16 *__restrict__ Xg, const int32_t *__restrict__ cu_seq,
                         const int32_t *__restrict__ cu_terms, const int32_t *__restrict__ term_tok,
                         int W, int64_t ld, bf16 *__restrict__ X) {
    const int d = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t0 = cu_seq[d], n = cu_seq[d + 1] - t0;
    for (int j = cu_terms[d] + wave; j < cu_terms[d + 1]; j += 4) {
        const int row = t0 + min(max(term_tok[j], 0), max(n - 1, 0));
        const uint2 *src = reinterpret_cast<const uint2 *>(Xg + (int64_t)j * W);
        uint2 *dst = reinterpret_cast<uint2 *>(X + (int64_t)row * ld);
        for (int c = lane; c < W / 4; c += 64) dst[c] = src[c];
    }
}

void launch_scatter_term_rows(const bf16 *Xg, const int32_t *cu_seq, const int32_t *cu_terms,
                              const int32_t *term_tok, int n_docs, int W, int64_t ld, bf16 *X,
                              hipStream_t s) {
    if (n_docs == 0) return;
    DI_REQUIRE(W % 4 == 0 && ld % 4 == 0, DI_EINVAL, "scatter_term_rows: 8-byte rows");
    hipLaunchKernelGGL(scatter_term_rows_kernel, dim3(n_docs), dim3(256), 0, s, Xg, cu_seq,
                       cu_terms, term_tok, W, ld, X);
    check_launch("scatter_term_rows");
}

void launch_gather_term_rows(const bf16 *X, const float2 *rl, const int32_t *cu_seq,
                             const int32_t *cu_terms, const int32_t *term_tok, int n_docs, int H,
                             bf16 *Xg, float2 *rlg, hipStream_t s) {
    if (n_docs == 0) return;
    hipLaunchKernelGGL(gather_term_rows_kernel, dim3(n_docs), dim3(256), 0, s, X, rl, cu_seq,
                       cu_terms, term_tok, H, Xg, rlg);
    check_launch("gather_term_rows");
}

template <typename T>
void launch_embed_ln(const int32_t *ids, const int32_t *cu, int n_docs, int M, int H,
                     const T *word, const T *pos, const T *type0, const float *gamma,
                     const float *beta, float eps, int pos_offset, int vocab, int max_pos, T *out,
                     int32_t *err, hipStream_t s) {
    if (M == 0) return;
    if (H == 768 || H == 1024) {  // one workgroup per document
        if (H == 768)
            hipLaunchKernelGGL((embed_ln_vec_kernel<T, 3>), dim3(n_docs), dim3(256), 0, s, ids, cu,
                               word, pos, type0, gamma, beta, eps, pos_offset, vocab, max_pos,
                               out, err);
        else
            hipLaunchKernelGGL((embed_ln_vec_kernel<T, 4>), dim3(n_docs), dim3(256), 0, s, ids, cu,
                               word, pos, type0, gamma, beta, eps, pos_offset, vocab, max_pos,
                               out, err);
        check_launch("embed_ln");
        return;
    }
    dim3 grid((M + 3) / 4);
    if (H <= 256)
        hipLaunchKernelGGL((embed_ln_kernel<T, 4>), grid, dim3(256), 0, s, ids, cu, n_docs, M, H,
                           word, pos, type0, gamma, beta, eps, pos_offset, vocab, max_pos, out,
                           err);
    else if (H <= 768)
        hipLaunchKernelGGL((embed_ln_kernel<T, 12>), grid, dim3(256), 0, s, ids, cu, n_docs, M,
                           H, word, pos, type0, gamma, beta, eps, pos_offset, vocab, max_pos, out,
                           err);
    else
        hipLaunchKernelGGL((embed_ln_kernel<T, LN_MAX_PER_LANE>), grid, dim3(256), 0, s, ids, cu,
                           n_docs, M, H, word, pos, type0, gamma, beta, eps, pos_offset, vocab,
                           max_pos, out, err);
    check_launch("embed_ln");
}

template <typename T>
void launch_ln(const T *pre, int M, int H, const float *gamma, const float *beta, float eps,
               T *out, const float *head_w, float head_b, int act, float *impact, hipStream_t s) {
    if (M == 0) return;
    dim3 grid((M + 3) / 4);
    if (H == 768)
        hipLaunchKernelGGL((ln_vec_kernel<T, 3>), grid, dim3(256), 0, s, pre, M, gamma, beta, eps,
                           out, head_w, head_b, act, impact);
    else if (H == 1024)
        hipLaunchKernelGGL((ln_vec_kernel<T, 4>), grid, dim3(256), 0, s, pre, M, gamma, beta, eps,
                           out, head_w, head_b, act, impact);
    else if (H <= 256)
        hipLaunchKernelGGL((ln_kernel<T, 4>), grid, dim3(256), 0, s, pre, M, H, gamma, beta, eps,
                           out, head_w, head_b, act, impact);
    else if (H <= 768)
        hipLaunchKernelGGL((ln_kernel<T, 12>), grid, dim3(256), 0, s, pre, M, H, gamma, beta,
                           eps, out, head_w, head_b, act, impact);
    else
        hipLaunchKernelGGL((ln_kernel<T, LN_MAX_PER_LANE>), grid, dim3(256), 0, s, pre, M, H,
                           gamma, beta, eps, out, head_w, head_b, act, impact);
    check_launch("ln");
}

// fp32-faithful (split-bf16) mode: f32 tables / pre-LN rows in, split rows out
void launch_embed_ln_split(const int32_t *ids, const int32_t *cu, int n_docs, int M, int H,
                           const float *word, const float *pos, const float *type0,
                           const float *gamma, const float *beta, float eps, int pos_offset,
                           int vocab, int max_pos, bf16 *out, int32_t *err, hipStream_t s) {
    if (M == 0) return;
    DI_REQUIRE(H == 768 || H == 1024, DI_EINVAL, "split mode: hidden %d (768 / 1024)", H);
    if (H == 768)
        hipLaunchKernelGGL((embed_ln_vec_kernel<float, 3, true>), dim3(n_docs), dim3(256), 0, s,
                           ids, cu, word, pos, type0, gamma, beta, eps, pos_offset, vocab, max_pos,
                           out, err);
    else
        hipLaunchKernelGGL((embed_ln_vec_kernel<float, 4, true>), dim3(n_docs), dim3(256), 0, s,
                           ids, cu, word, pos, type0, gamma, beta, eps, pos_offset, vocab, max_pos,
                           out, err);
    check_launch("embed_ln_split");
}

void launch_ln_split(const float *pre, int M, int H, const float *gamma, const float *beta,
                     float eps, bf16 *out, const float *head_w, float head_b, int act,
                     float *impact, hipStream_t s) {
    if (M == 0) return;
    DI_REQUIRE(H == 768 || H == 1024, DI_EINVAL, "split mode: hidden %d (768 / 1024)", H);
    dim3 grid((M + 3) / 4);
    if (H == 768)
        hipLaunchKernelGGL((ln_vec_kernel<float, 3, true>), grid, dim3(256), 0, s, pre, M, gamma,
                           beta, eps, out, head_w, head_b, act, impact);
    else
        hipLaunchKernelGGL((ln_vec_kernel<float, 4, true>), grid, dim3(256), 0, s, pre, M, gamma,
                           beta, eps, out, head_w, head_b, act, impact);
    check_launch("ln_split");
}

void launch_gather_terms(const float *impact, const int32_t *cu_seq, const int32_t *cu_terms,
                         int n_docs, const int32_t *term_tok, int n_terms, int do_round,
                         float *out, int32_t *err, hipStream_t s) {
    if (n_terms == 0) return;
    hipLaunchKernelGGL(gather_terms_kernel, dim3((n_terms + 255) / 256), dim3(256), 0, s, impact,
                       cu_seq, cu_terms, n_docs, term_tok, n_terms, do_round, out, err);
    check_launch("gather_terms");
}

template void launch_embed_ln<bf16>(const int32_t *, const int32_t *, int, int, int, const bf16 *,
                                    const bf16 *, const bf16 *, const float *, const float *,
                                    float, int, int, int, bf16 *, int32_t *, hipStream_t);
template void launch_embed_ln<float>(const int32_t *, const int32_t *, int, int, int,
                                     const float *, const float *, const float *, const float *,
                                     const float *, float, int, int, int, float *, int32_t *,
                                     hipStream_t);
template void launch_ln<bf16>(const bf16 *, int, int, const float *, const float *, float, bf16 *,
                              const float *, float, int, float *, hipStream_t);
template void launch_ln<float>(const float *, int, int, const float *, const float *, float,
                               float *, const float *, float, int, float *, hipStream_t);

// ---------------------------------------------------------------------------
// A10 quantizer (reference src/deep_impact/indexing/quantize.py:13-47):
//   max_val = max(0, values) (fp64), scale = (2^bits - 1) / max_val (fp64),
//   q = int(v * scale) (truncation, fp64 product).
// ---------------------------------------------------------------------------
__global__ void max_f32_kernel(const float *__restrict__ v, int64_t n,
                               unsigned int *__restrict__ out_bits) {
    float m = 0.f;  // find_max_value starts at 0
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, v[i]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
    // non-negative floats order like their bit patterns (-0.0 and NaN -> 0)
    if ((threadIdx.x & 63) == 0) atomicMax(out_bits, m > 0.f ? __float_as_uint(m) : 0u);
}

__global__ void quantize_kernel(const float *__restrict__ v, int64_t n,
                                const unsigned int *__restrict__ max_bits, double max_given,
                                int bits, int32_t *__restrict__ out) {
    const double m = max_given > 0.0 ? max_given : (double)__uint_as_float(*max_bits);
    const double scale = (double)((1 << bits) - 1) / m;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double p = __dmul_rn((double)v[i], scale);
        p = fmin(fmax(p, -2147483648.0), 2147483647.0);
        out[i] = (int32_t)p;  // C conversion truncates toward zero, as Python int()
    }
}

}  // namespace di

namespace di {
// f64 inputs (values parsed from impact-TSV text, quantize_file)
__global__ void max_f64_kernel(const double *__restrict__ v, int64_t n,
                               unsigned long long *__restrict__ out_bits) {
    double m = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        m = fmax(m, v[i]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = fmax(m, __shfl_xor(m, d, 64));
    if ((threadIdx.x & 63) == 0)
        atomicMax(out_bits, m > 0.0 ? (unsigned long long)__double_as_longlong(m) : 0ull);
}

__global__ void quantize_f64_kernel(const double *__restrict__ v, int64_t n,
                                    const unsigned long long *__restrict__ max_bits,
                                    double max_given, int bits, int32_t *__restrict__ out) {
    const double m = max_given > 0.0 ? max_given : __longlong_as_double((long long)*max_bits);
    const double scale = (double)((1 << bits) - 1) / m;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double p = __dmul_rn(v[i], scale);
        p = fmin(fmax(p, -2147483648.0), 2147483647.0);
        out[i] = (int32_t)p;
    }
}

void launch_quantize_f64(const double *v, int64_t n, double max_given, int bits, int32_t *out,
                         unsigned long long *max_bits, hipStream_t s) {
    DI_HIP(hipMemsetAsync(max_bits, 0, sizeof(unsigned long long), s));
    if (n == 0) return;
    int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
    if (!(max_given > 0.0)) {
        hipLaunchKernelGGL(max_f64_kernel, dim3(blocks), dim3(256), 0, s, v, n, max_bits);
        check_launch("max_f64");
    }
    hipLaunchKernelGGL(quantize_f64_kernel, dim3(blocks), dim3(256), 0, s, v, n, max_bits,
                       max_given, bits, out);
    check_launch("quantize_f64");
}

void launch_quantize(const float *v, int64_t n, double max_given, int bits, int32_t *out,
                     unsigned int *max_bits, hipStream_t s) {
    DI_HIP(hipMemsetAsync(max_bits, 0, sizeof(unsigned int), s));
    if (n == 0) return;
    int blocks = (int)std::min<int64_t>(2048, (n + 255) / 256);
    if (!(max_given > 0.0)) {
        hipLaunchKernelGGL(max_f32_kernel, dim3(blocks), dim3(256), 0, s, v, n, max_bits);
        check_launch("max_f32");
    }
    hipLaunchKernelGGL(quantize_kernel, dim3(blocks), dim3(256), 0, s, v, n, max_bits,
                       max_given, bits, out);
    check_launch("quantize");
}
}  // namespace di

extern "C" int di_quantize(const float *impacts, int64_t n, double max_val, int32_t bits,
                           int32_t *out, double *max_used, int device, void *hip_stream,
                           uint32_t flags) {
    using namespace di;
    return guard([&] {
        DI_REQUIRE(impacts && out && n >= 0 && bits >= 1 && bits <= 16, DI_EINVAL,
                   "bad argument");
        int prev = 0;
        DI_HIP(hipGetDevice(&prev));
        DI_HIP(hipSetDevice(device));
        hipStream_t s = (hipStream_t)hip_stream;
        const bool dev = flags & DI_F_DEVICE_PTRS;
        DevBuf bin, bout, bmax;
        bmax.reserve(16);
        const float *d_in = (const float *)stage_in(impacts, (size_t)n * 4, dev, bin, s);
        int32_t *d_out = out;
        if (!dev) {
            bout.reserve((size_t)std::max<int64_t>(n, 1) * 4);
            d_out = bout.as<int32_t>();
        }
        launch_quantize(d_in, n, max_val, bits, d_out, bmax.as<unsigned int>(), s);
        unsigned int mb = 0;
        DI_HIP(hipMemcpyAsync(&mb, bmax.p, 4, hipMemcpyDeviceToHost, s));
        if (!dev && n)
            DI_HIP(hipMemcpyAsync(out, d_out, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        DI_HIP(hipStreamSynchronize(s));
        float mf;
        std::memcpy(&mf, &mb, 4);
        if (max_used) *max_used = max_val > 0.0 ? max_val : (double)mf;
        DI_REQUIRE(max_val > 0.0 || n == 0 || mf > 0.f, DI_EINVAL,
                   "max impact is 0: the reference divides by zero (quantize.py:37)");
        (void)hipSetDevice(prev);
    });
}
