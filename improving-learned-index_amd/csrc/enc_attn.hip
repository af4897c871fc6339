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
// every document starting at a 32-aligned column vt_base(d) = 32*(d + cu[d]/32), so
// 4 consecutive keys are one 8-byte (bf16) / 16-byte (f32) load.
// Online softmax in f32 (exp2 with log2(e)/8 folded into the scores).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int ATT_D = 64;
constexpr int QT = 4;  // query tiles of 16 per wave

// doc d's first V^T column: 32-aligned (one split chunk; 16 B loads for bf16 / f32),
// at most 31 gap columns per document
__host__ __device__ __forceinline__ int vt_base(int doc, int tok0) { return 32 * (doc + (tok0 >> 5)); }

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
                 int n_pairs, T *__restrict__ ctx, bf16 *__restrict__ ctx_split) {
    // ctx_split (f32 kernel, fp32-faithful mode): the output as split-bf16 rows
    // [hi(H) | lo(H)] for the next split GEMM, instead of ctx
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
        if (q < n && ctx_split) {
            bf16 *out = ctx_split + (int64_t)(tok0 + q) * 2 * H;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                bf16x4 hv, lv;
#pragma unroll
                for (int r = 0; r < 4; ++r) hv[r] = split_hi(o[qt][dt][r] * inv), lv[r] = split_lo(o[qt][dt][r] * inv);
                const int64_t sc0 = split_col(h * ATT_D + dt * 16 + 4 * g);
                *reinterpret_cast<bf16x4 *>(out + sc0) = hv;
                *reinterpret_cast<bf16x4 *>(out + sc0 + 32) = lv;
            }
        } else if (q < n) {
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

// fp32-faithful attention (precision bf16x3): every product as split bf16 (x = x_hi +
// x_lo, three 16x16x32 bf16 MFMAs per f32 product: hi*hi + lo*hi + hi*lo, f32
// accumulate, ~2^-17 relative per product) instead of f32 MFMA (1/16 of the bf16
// rate): S^T = K Q^T from split K and Q, O^T = V^T P^T from split V and the split
// probabilities; softmax and the row sums in f32.  Q | K | V arrive as split rows
// [M][6H] from the QKV GEMM (split_col over the 3H logical columns): no V^T scatter.
//
// One persistent 512-thread workgroup per CU walks the (doc, head) pairs; the 8 waves
// own 48 queries each (three 16-query tiles, QTN; documents past 384 tokens take a
// second pass), and the keys stream
// through LDS in 32-key chunks, double-buffered: chunk i+1 is copied by LDS-DMA
// (global_load_lds, every wave one 1 KiB piece of K and one of V) while chunk i is
// computed, so every K / V byte is read from memory once per pass for the workgroup.
//   K and V images (8 KiB each): key row r = the head's 256 B [ch0 hi | ch0 lo | ch1 hi
//   | ch1 lo] (16-byte slots), slot j stored at j ^ ax_swz(r).
//   S^T fragment row c of tile t = key 8 (c >> 2) + 4 t + (c & 3), so lane group g holds
//   the consecutive keys 8 g..8 g + 7 of P^T (as attention_v3_kernel); the O^T A
//   operand (V^T) is read from the V rows with ds_read_b64_tr_b16.
// Fragment reads are inline-asm ds_reads with their lgkmcnt wait in the same statement
// (the compiler would otherwise drain the in-flight prefetch with vmcnt(0) before an
// LDS read it cannot tell apart from the DMA's destination).
constexpr int AX_WAVES = 8, AX_QT = 2;
// Image swizzle: slot j of key row r at j ^ ax_swz(r), ax_swz(r) = r0 r1 r3 in bits 1-3.
// A ds_read_b128 lane group (16 lanes: rows c&3 + 8 (c>>2) + 4 t, slot bit 0 = g) and a
// ds_read_b64_tr_b16 lane group (32 lanes: rows q + 8 g + 4 h2, slot bit 0 = p>>1)
// then reach 16 distinct slots (every 256-byte row starts at bank 0): conflict-free
// (r & 15 conflicts 2-way on both).  Row bit 5 (the 32-key sub-chunk) is not used, so
// the sub-chunk stays an immediate offset.
__device__ __forceinline__ int ax_swz(int r) { return ((r & 3) << 1) | (r & 8); }
// LDS: [K image, buffer 0 | K, buffer 1 | V, buffer 0 | V, buffer 1], one image = AX_KC
// key rows of 256 B; every fragment read's (buffer, sub-chunk) offset is an immediate.
// (Measured: 128-key chunks -- half the barriers -- and raised MFMA issue priority
// were both slower, r03 ab_attn.)
constexpr int AX_KC = 64, AX_IMG = AX_KC * 256, AX_LDS = 4 * AX_IMG;
// Q through LDS: every wave copies the next unit's query fragments by LDS-DMA into a
// region of its own ([qt][ch][hi, lo] x 1 KiB, lane l's 16 B at l * 16) with the chunk
// staging, and reads them into registers once at the unit's start -- no second set of
// Q registers live across the chunk loop (and none of the moves its conditional load
// cost at every chunk)
constexpr int AX_QTB = 4096;  // Q region bytes per query tile
constexpr int ax_lds(int nw, int qtn, int kc = AX_KC) { return 4 * kc * 256 + nw * qtn * AX_QTB; }

// BAL: wave w owns the 16-query tiles w and w + 8 of a pass (instead of 2w, 2w + 1), so
// the tiles of a short pass spread over the four SIMDs (wave w runs on SIMD w % 4), and
// a tile with no query is skipped.  LAZY: the softmax's reference max moves only when a
// score exceeds it by 8 / sc (p <= 2^8): one max per lane and one ballot in the common
// case instead of the cross-lane max; the scale folds into the exponent's fma.  PIPE
// (with both, two query tiles): tile 1's S^T products interleaved with tile 0's
// exponentials, tile 0's O^T products with tile 1's (sched_group_barrier), so the
// softmax issues in the MFMAs' shadow.
// NW: waves per workgroup.  8: one workgroup per CU, 256-query passes.  4: two
// workgroups per CU (64 KiB of LDS and <= 256 VGPRs each), 128-query passes -- a SIMD
// idle at one workgroup's short last pass runs the other workgroup's wave.
// QTN: query tiles per wave and pass (2: 256-query passes; 3: 384, every document of up to
// 384 tokens in one pass -- a wave's third tile runs the generic loop, the pair PIPE).
// KC: keys per staged chunk (64; 32 halves the K / V buffers: the 4-wave form of the pruned
// last layer, two workgroups per CU).
template <bool BAL, bool LAZY, bool PIPE = false, int NW = AX_WAVES, int QTN = AX_QT,
          int KC = AX_KC>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2)))
attention_x3_kernel(const bf16 *__restrict__ qkv, const int32_t *__restrict__ cu_seqlens, int H,
                    int n_heads, int n_pairs, bf16 *__restrict__ ctx_split,
                    const int32_t *__restrict__ qsel, const int32_t *__restrict__ cu_qsel,
                    int abl) {
    // abl (developer timing ablations, wrong results): 1 no softmax arithmetic, 2 no S^T
    // products, 4 no O^T products, 16 no second pass (documents past 256 queries)
    // qsel (optional, the pruned last layer): only the query rows qsel[cu_qsel[d] ..)
    // (doc-local token indices) of document d are computed, into ctx rows cu_qsel[d] + i;
    // keys and values are every token of the document either way.
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef __attribute__((address_space(3))) void lds_void;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c = lane & 15;
    const int64_t ld = 6 * (int64_t)H;  // split row: 3H logical columns
    const uint32_t lds_base =
        (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char *)lds);
    const float sc = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    constexpr int PASS_Q = NW * QTN * 16;           // queries per pass (256, 384 or 128)
    static_assert(QTN == 2 || QTN == 3, "two or three query tiles per wave");
    constexpr int IMG = KC * 256, KVL = 4 * IMG;  // one K or V image; the four of them

    // Work units: (pair, pass), pairs blockIdx.x, + gridDim.x, ... (persistent); the
    // next unit's Q and first K / V chunk load while the current unit's last chunk
    // computes.
    struct Unit {
        int pair, pass, tok0, n, h, q0, nq;  // q0: ctx row of query 0; nq: queries
    };
    auto make_unit = [&](int pr, int pass, Unit &u) {
        const int doc = pr / n_heads;
        u.pair = pr;
        u.pass = pass;
        u.h = pr % n_heads;
        u.tok0 = cu_seqlens[doc];
        u.n = cu_seqlens[doc + 1] - u.tok0;
        u.q0 = qsel ? cu_qsel[doc] : u.tok0;
        u.nq = qsel ? cu_qsel[doc + 1] - u.q0 : u.n;
    };
    // the unit after `u` with at least one token and one query, or false
    auto next_unit = [&](const Unit &u, Unit &nu) {
        if ((u.pass + 1) * PASS_Q < u.nq && !(abl & 16)) {
            nu = u;
            nu.pass = u.pass + 1;
            return true;
        }
        for (int pr = u.pair + (int)gridDim.x; pr < n_pairs; pr += (int)gridDim.x) {
            make_unit(pr, 0, nu);
            if (nu.n > 0 && nu.nq > 0) return true;
        }
        return false;
    };
    // chunk ci of unit u -> stage buffer b: key rows RPW wave..+RPW-1 of K and of V
    // (RPW / 4 pieces of 1 KiB each), 16 B per lane, source slots permuted by the
    // swizzle (piece pc: key rows RPW wave + 4 pc + lane >> 4)
    constexpr int RPW = KC / NW;  // key rows per wave and image (8 or 16)
    const int sr = RPW * wave + (lane >> 4);
    auto stage = [&](const Unit &u, int ci, int b) {
        const bf16 *kg = qkv + split_col(H + u.h * ATT_D);      // + key row * ld: 256 B
        const bf16 *vg = qkv + split_col(2 * H + u.h * ATT_D);
#pragma unroll
        for (int pc = 0; pc < RPW / 4; ++pc) {
            const int rl = sr + 4 * pc;
            const int row = u.tok0 + min(ci * KC + rl, u.n - 1);
            const int j = (lane & 15) ^ ax_swz(rl);
            const int dst = b * IMG + (RPW * wave + 4 * pc) * 256;
            __builtin_amdgcn_global_load_lds((const void *)(kg + row * ld + j * 8),
                                             (lds_void *)(lds + dst), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *)(vg + row * ld + j * 8),
                                             (lds_void *)(lds + 2 * IMG + dst), 16, 0, 0);
        }
    };
    // first query (within its pass) of this wave's tile qt
    auto qtile = [&](int qt) { return BAL ? 16 * (wave + NW * qt) : wave * (QTN * 16) + 16 * qt; };
    // unit u's query fragments of this wave -> its Q region (LDS-DMA, 8 x 1 KiB)
    auto dma_q = [&](const Unit &u) {
        const bf16 *qbase = qkv + split_col(u.h * ATT_D) + 8 * g;
#pragma unroll
        for (int qt = 0; qt < QTN; ++qt) {
            const int qi = min(u.pass * PASS_Q + qtile(qt) + c, u.nq - 1);
            const int qloc = qsel ? min(max(qsel[u.q0 + qi], 0), u.n - 1) : qi;
            const int qrow = u.tok0 + qloc;
#pragma unroll
            for (int ch = 0; ch < 2; ++ch) {
                const bf16 *src = qbase + qrow * ld + ch * 64;
                const int dst = KVL + wave * (QTN * AX_QTB) + (qt * 2 + ch) * 2048;
                __builtin_amdgcn_global_load_lds((const void *)src, (lds_void *)(lds + dst), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void *)(src + 32),
                                                 (lds_void *)(lds + dst + 1024), 16, 0, 0);
            }
        }
    };
    // fragment addresses (buffer 0; buffer 1 is the immediate offset IMG).  Row bit 2
    // (the K tile t, the V half h2) is not in the swizzle, so those halves are the
    // immediate offset 4 * 256 = 1024 of one address register: 12 VGPRs instead of 24.
    constexpr int AX_HALF = 1024;
    uint32_t ka[2][2];  // [ch][hi, lo]: key row 8 (c >> 2) + (c & 3) (+ 4 t: + AX_HALF)
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
            const int r = 8 * (c >> 2) + (c & 3), j = ch * 8 + pt * 4 + g;
            ka[ch][pt] = lds_base + r * 256 + ((j ^ ax_swz(r)) << 4);
        }
    // [dt][hi, lo]: ds_read_b64_tr_b16 roles -- lane 4 q + p of a 16-lane group addresses
    // key row 8 g + 4 h2 + q (h2: + AX_HALF), columns 16 dt + 4 p..+3 (one 8-byte half
    // slot); lane i then holds column d = 16 dt + i for keys 8 g + 4 h2 + 0..3
    uint32_t va[4][2];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
            const int q = c >> 2, pp = c & 3;
            const int r = 8 * g + q;
            const int j = (dt >> 1) * 8 + pt * 4 + 2 * (dt & 1) + (pp >> 1);
            va[dt][pt] = lds_base + 2 * IMG + r * 256 + ((j ^ ax_swz(r)) << 4) + 8 * (pp & 1);
        }

    Unit cu;
    {
        int pr = blockIdx.x;
        for (; pr < n_pairs; pr += (int)gridDim.x) {
            make_unit(pr, 0, cu);
            if (cu.n > 0 && cu.nq > 0) break;
        }
        if (pr >= n_pairs) return;
    }
    bf16x8 qh[QTN][2], ql[QTN][2];
    const uint32_t qa = lds_base + KVL + wave * (QTN * AX_QTB) + lane * 16;
    // this wave's Q region -> qh / ql (landed: the caller waited vmcnt(0))
    auto read_q = [&]() {
        uint4 q4[8];
        asm volatile(
            "ds_read_b128 %0, %8 offset:0"
            "\n\tds_read_b128 %1, %8 offset:1024"
            "\n\tds_read_b128 %2, %8 offset:2048"
            "\n\tds_read_b128 %3, %8 offset:3072"
            "\n\tds_read_b128 %4, %8 offset:4096"
            "\n\tds_read_b128 %5, %8 offset:5120"
            "\n\tds_read_b128 %6, %8 offset:6144"
            "\n\tds_read_b128 %7, %8 offset:7168"
            "\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(q4[0]), "=&v"(q4[1]), "=&v"(q4[2]), "=&v"(q4[3]), "=&v"(q4[4]),
              "=&v"(q4[5]), "=&v"(q4[6]), "=&v"(q4[7])
            : "v"(qa)
            : "memory");
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
            for (int ch = 0; ch < 2; ++ch) {
                __builtin_memcpy(&qh[qt][ch], &q4[(qt * 2 + ch) * 2], 16);
                __builtin_memcpy(&ql[qt][ch], &q4[(qt * 2 + ch) * 2 + 1], 16);
            }
        if constexpr (QTN == 3) {
            uint4 q5[4];
            asm volatile(
                "ds_read_b128 %0, %4 offset:8192"
                "\n\tds_read_b128 %1, %4 offset:9216"
                "\n\tds_read_b128 %2, %4 offset:10240"
                "\n\tds_read_b128 %3, %4 offset:11264"
                "\n\ts_waitcnt lgkmcnt(0)"
                : "=&v"(q5[0]), "=&v"(q5[1]), "=&v"(q5[2]), "=&v"(q5[3])
                : "v"(qa)
                : "memory");
#pragma unroll
            for (int ch = 0; ch < 2; ++ch) {
                __builtin_memcpy(&qh[2][ch], &q5[ch * 2], 16);
                __builtin_memcpy(&ql[2][ch], &q5[ch * 2 + 1], 16);
            }
        }
    };
    stage(cu, 0, 0);
    dma_q(cu);
    int b = 0;  // stage buffer of the next chunk to compute
    for (;;) {
        const int n = cu.n, h = cu.h, q0 = cu.q0, nq = cu.nq;
        const int q_pass = cu.pass * PASS_Q;
        const bool has_q = q_pass + qtile(0) < nq;
        const bool two = BAL ? q_pass + qtile(1) < nq : has_q;  // (uniform) tile 1 has queries
        const bool three = QTN == 3 && (BAL ? q_pass + qtile(2) < nq : has_q);
        const int n_chunks = (n + KC - 1) / KC;
        Unit nu;
        const bool more = next_unit(cu, nu);
        float m[QTN], lsum[QTN], lim[QTN], mneg[QTN];
        f32x4 o[QTN][4];
#pragma unroll
        for (int qt = 0; qt < QTN; ++qt) {
            m[qt] = -INFINITY;
            lim[qt] = -INFINITY;
            mneg[qt] = 0.f;
            lsum[qt] = 0.f;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // The chunk loop for a unit whose wave has NQT (1 or 2) query tiles -- one loop per
        // count, not a choice per chunk: with the choice inside, the two bodies left the
        // O accumulators in different registers and the loop's back edge moved them
        // (16 v_mov_b64 + 12 v_mov per chunk in the ISA)
        // (and the unit's whole 64-key chunks in a loop of their own, the partial last chunk
        // after it: a sub-chunk loop that may stop after its first sub-chunk also left them
        // in different registers, moved at the top and the bottom of every chunk)
        // (and a wave with no query in the unit runs the staging alone: a body that may
        // skip its products also moved the accumulators)
        auto stage_next = [&](const int ci) {
            if (ci + 1 < n_chunks) {
                stage(cu, ci + 1, b ^ 1);
            } else if (more) {  // the next unit's first chunk and Q
                stage(nu, 0, b ^ 1);
                dma_q(nu);
            }
        };
        // chunk ci > 0 (chunk 0's wait is the unit's start, below)
        auto stage_step = [&](const int ci) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of chunk ci
            __syncthreads();  // every piece landed; buffer b ^ 1 no longer read
            stage_next(ci);
        };
        // unit start: chunk 0 and this wave's Q landed; Q into registers before the next
        // unit's Q copy can be issued (stage_next(0) issues it for a one-chunk unit)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        read_q();
        stage_next(0);
        auto chunk_loop = [&](auto nqt_outer) {
        auto one_chunk = [&](const int ci, auto whole_c) {
            constexpr bool WHOLE = decltype(whole_c)::value;
            if (ci > 0) stage_step(ci);
            // the chunk's sub-chunks for the wave's NQT non-empty query tiles
            auto chunk = [&](auto nqt_c) {
            constexpr int NQT = decltype(nqt_c)::value;
#pragma unroll
            for (int u = 0; u < KC / 32; ++u) {  // 32-key sub-chunks
            const int key0 = ci * KC + 32 * u;
            if (!WHOLE && key0 >= n) break;
            uint4 kf[2][2][2];
            uint2 vt2[4][2][2];
            // K fragments: one asm statement for the 8 reads and their wait (outputs
            // exist only after it); V^T fragments: likewise, one statement with its wait,
            // issued before the softmax.  The stage buffer and the sub-chunk are the
            // immediate offset.
#define AX_READ_K(OFF)                                                                             \
    asm volatile(                                                                                  \
        "ds_read_b128 %0, %8 offset:%12"                                                           \
        "\n\tds_read_b128 %1, %9 offset:%12"                                                       \
        "\n\tds_read_b128 %2, %10 offset:%12"                                                      \
        "\n\tds_read_b128 %3, %11 offset:%12"                                                      \
        "\n\tds_read_b128 %4, %8 offset:%13"                                                       \
        "\n\tds_read_b128 %5, %9 offset:%13"                                                       \
        "\n\tds_read_b128 %6, %10 offset:%13"                                                      \
        "\n\tds_read_b128 %7, %11 offset:%13"                                                      \
        "\n\ts_waitcnt lgkmcnt(0)"                                                                 \
        : "=&v"(kf[0][0][0]), "=&v"(kf[0][0][1]), "=&v"(kf[0][1][0]), "=&v"(kf[0][1][1]),          \
          "=&v"(kf[1][0][0]), "=&v"(kf[1][0][1]), "=&v"(kf[1][1][0]), "=&v"(kf[1][1][1])           \
        : "v"(ka[0][0]), "v"(ka[0][1]), "v"(ka[1][0]), "v"(ka[1][1]),                              \
          "i"(OFF), "i"((OFF) + AX_HALF)                                                           \
        : "memory")
#define AX_READ_VW(OFF)                                                                            \
    asm volatile(                                                                                  \
        "ds_read_b64_tr_b16 %0, %16 offset:%24"                                                    \
        "\n\tds_read_b64_tr_b16 %1, %16 offset:%25"                                                \
        "\n\tds_read_b64_tr_b16 %2, %17 offset:%24"                                                \
        "\n\tds_read_b64_tr_b16 %3, %17 offset:%25"                                                \
        "\n\tds_read_b64_tr_b16 %4, %18 offset:%24"                                                \
        "\n\tds_read_b64_tr_b16 %5, %18 offset:%25"                                                \
        "\n\tds_read_b64_tr_b16 %6, %19 offset:%24"                                                \
        "\n\tds_read_b64_tr_b16 %7, %19 offset:%25"                                                \
        "\n\tds_read_b64_tr_b16 %8, %20 offset:%24"                                                \
        "\n\tds_read_b64_tr_b16 %9, %20 offset:%25"                                                \
        "\n\tds_read_b64_tr_b16 %10, %21 offset:%24"                                               \
        "\n\tds_read_b64_tr_b16 %11, %21 offset:%25"                                               \
        "\n\tds_read_b64_tr_b16 %12, %22 offset:%24"                                               \
        "\n\tds_read_b64_tr_b16 %13, %22 offset:%25"                                               \
        "\n\tds_read_b64_tr_b16 %14, %23 offset:%24"                                               \
        "\n\tds_read_b64_tr_b16 %15, %23 offset:%25"                                               \
        "\n\ts_waitcnt lgkmcnt(0)"                                                                 \
        : "=&v"(vt2[0][0][0]), "=&v"(vt2[0][0][1]), "=&v"(vt2[0][1][0]), "=&v"(vt2[0][1][1]),      \
          "=&v"(vt2[1][0][0]), "=&v"(vt2[1][0][1]), "=&v"(vt2[1][1][0]), "=&v"(vt2[1][1][1]),      \
          "=&v"(vt2[2][0][0]), "=&v"(vt2[2][0][1]), "=&v"(vt2[2][1][0]), "=&v"(vt2[2][1][1]),      \
          "=&v"(vt2[3][0][0]), "=&v"(vt2[3][0][1]), "=&v"(vt2[3][1][0]), "=&v"(vt2[3][1][1])       \
        : "v"(va[0][0]), "v"(va[0][1]), "v"(va[1][0]), "v"(va[1][1]),                              \
          "v"(va[2][0]), "v"(va[2][1]), "v"(va[3][0]), "v"(va[3][1]),                              \
          "i"(OFF), "i"((OFF) + AX_HALF)                                                           \
        : "memory")
// (b, the stage buffer, is 0 or 1 at run time; u, the sub-chunk, a constant of the
// unrolled loop: one branch per site -- a switch over the offsets' value range compiled
// to a chain of compares)
static_assert((KC == 64 && IMG == 16384) || (KC == 32 && IMG == 8192), "AX_SEL's offsets");
#define AX_SEL(M)                                                                                  \
    do {                                                                                           \
        if constexpr (KC == 64) {                                                                  \
            if (b) {                                                                               \
                if (u) M(24576); else M(16384);                                                    \
            } else {                                                                               \
                if (u) M(8192); else M(0);                                                         \
            }                                                                                      \
        } else {                                                                                   \
            if (b) M(8192); else M(0);                                                             \
        }                                                                                          \
    } while (0)
            // (immediate offset: buffer b at b * IMG, sub-chunk u at u * 32 rows; u is
            // a constant of the unrolled loop, so each site keeps two cases)
            AX_SEL(AX_READ_K);
            __builtin_amdgcn_sched_barrier(0);
            bf16x8 kfr[2][2][2];  // [t][ch][hi, lo]
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int ch = 0; ch < 2; ++ch)
#pragma unroll
                    for (int pt = 0; pt < 2; ++pt) __builtin_memcpy(&kfr[t][ch][pt], &kf[t][ch][pt], 16);
            if constexpr (PIPE && NQT >= 2) {
            static_assert(BAL && LAZY, "PIPE builds on the balanced lazy form");
            const bool full = WHOLE || key0 + 32 <= n;  // (uniform) no masked key in this sub-chunk
            f32x4 s[QTN][2];
            float v[QTN][8];
            bf16x8 ph[QTN], pl[QTN];
            // S^T of tile qt (12 MFMAs; the two accumulators' chains interleaved)
            auto s_mfma = [&](int qt) {
                s[qt][0] = s[qt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ch = 0; ch < 2; ++ch)
#pragma unroll
                    for (int p = 0; p < 3; ++p)
#pragma unroll
                        for (int t = 0; t < 2; ++t)
                            s[qt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                kfr[t][ch][p == 1], p == 2 ? ql[qt][ch] : qh[qt][ch], s[qt][t],
                                0, 0, 0);
            };
            // softmax part A of tile qt: masked raw scores, the lazy max test and the rare
            // rescale (a branch: outside the interleaved regions)
            auto soft_a = [&](int qt) {
                // (a uniform branch: the common full sub-chunk takes the scores as they are,
                // without 8 compares and selects per tile)
                if (full) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[qt][e] = s[qt][e >> 2][e & 3];
                } else {
                    // (key 8 g + e of the sub-chunk is valid iff e < n - key0 - 8 g: one
                    // value per lane against constants, not 8 hoisted key offsets)
                    const int kv = n - key0 - 8 * g;
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[qt][e] = e < kv ? s[qt][e >> 2][e & 3] : -INFINITY;
                }
                // (the test by compares: the max, with its NaN-canonicalising operand
                // maxes, only on the rare path)
                bool up = false;
#pragma unroll
                for (int e = 0; e < 8; ++e) up |= v[qt][e] > lim[qt];
                if (__any(up)) {
                    float cmax = fmaxf(fmaxf(fmaxf(v[qt][0], v[qt][1]), fmaxf(v[qt][2], v[qt][3])),
                                       fmaxf(fmaxf(v[qt][4], v[qt][5]), fmaxf(v[qt][6], v[qt][7])));
                    const auto p16 = __builtin_amdgcn_permlane16_swap(
                        __float_as_uint(cmax), __float_as_uint(cmax), false, false);
                    cmax = fmaxf(__uint_as_float(p16[0]), __uint_as_float(p16[1]));
                    const auto p32 = __builtin_amdgcn_permlane32_swap(
                        __float_as_uint(cmax), __float_as_uint(cmax), false, false);
                    cmax = fmaxf(__uint_as_float(p32[0]), __uint_as_float(p32[1]));
                    const float m_new = fmaxf(m[qt], cmax);
                    if (m_new != m[qt]) {
                        const float alpha = __builtin_amdgcn_exp2f((m[qt] - m_new) * sc);
                        lsum[qt] *= alpha;
#pragma unroll
                        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
                    }
                    m[qt] = m_new;
                    lim[qt] = m_new + 8.0f / sc;
                    mneg[qt] = -m_new * sc;
                }
            };
            // softmax part B: the exponentials, row sums and split probabilities
            auto soft_b = [&](int qt) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float pr = __builtin_amdgcn_exp2f(fmaf(v[qt][e], sc, mneg[qt]));
                    lsum[qt] += pr;
                    ph[qt][e] = split_hi(pr);
                    pl[qt][e] = split_lo(pr);
                }
            };
            bf16x8 vfr[4][2];
            auto o_mfma = [&](int qt) {
#pragma unroll
                for (int p = 0; p < 3; ++p)
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt)
                        o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            vfr[dt][p == 1], p == 2 ? pl[qt] : ph[qt], o[qt][dt], 0, 0, 0);
            };
            // 1 MFMA : 4 VALU (incl. transcendental) groups over a 12-MFMA region
#define AX_INTERLEAVE()                                                                            \
    do {                                                                                           \
        _Pragma("unroll") for (int i_ = 0; i_ < 12; ++i_) {                                        \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                     \
            __builtin_amdgcn_sched_group_barrier(0x402, 4, 0);                                     \
        }                                                                                          \
    } while (0)
            s_mfma(0);
            __builtin_amdgcn_sched_barrier(0);
            AX_SEL(AX_READ_VW);  // (their wait overlaps tile 0's products)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int pt = 0; pt < 2; ++pt) {
                    const uint4 v4 = make_uint4(vt2[dt][pt][0].x, vt2[dt][pt][0].y,
                                                vt2[dt][pt][1].x, vt2[dt][pt][1].y);
                    __builtin_memcpy(&vfr[dt][pt], &v4, 16);
                }
            soft_a(0);
            __builtin_amdgcn_sched_barrier(0);
            s_mfma(1);
            soft_b(0);
            AX_INTERLEAVE();
            __builtin_amdgcn_sched_barrier(0);
            soft_a(1);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (NQT == 3) {  // tile 2's products in tile 1's and tile 2's shadows
                s_mfma(2);
                soft_b(1);
                AX_INTERLEAVE();
                __builtin_amdgcn_sched_barrier(0);
                soft_a(2);
                __builtin_amdgcn_sched_barrier(0);
                o_mfma(0);
                soft_b(2);
                AX_INTERLEAVE();
                __builtin_amdgcn_sched_barrier(0);
                o_mfma(1);
                o_mfma(2);
            } else {
                o_mfma(0);
                soft_b(1);
                AX_INTERLEAVE();
                __builtin_amdgcn_sched_barrier(0);
                o_mfma(1);
            }
#undef AX_INTERLEAVE
            } else {
            // S^T for both query tiles, each product stage over the 4 independent
            // accumulators before the next (one accumulator's 3 products are a chain)
            f32x4 s[QTN][2];
#pragma unroll
            for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
                for (int t = 0; t < 2; ++t) s[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (!(abl & 2))
#pragma unroll
            for (int ch = 0; ch < 2; ++ch)
#pragma unroll
                for (int p = 0; p < 3; ++p)
#pragma unroll
                    for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
                        for (int t = 0; t < 2; ++t)
                            s[qt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                kfr[t][ch][p == 1], p == 2 ? ql[qt][ch] : qh[qt][ch], s[qt][t], 0,
                                0, 0);
            __builtin_amdgcn_sched_barrier(0);
            // (the V^T reads with their wait in one statement: with a separate wait the
            // compiler copied V^T registers above it -- tools/asm_wait_scan.py)
            AX_SEL(AX_READ_VW);
            __builtin_amdgcn_sched_barrier(0);
            const bool full = WHOLE || key0 + 32 <= n;  // (uniform) no masked key in this sub-chunk
            bf16x8 ph[QTN], pl[QTN];
            if (abl & 1) {
#pragma unroll
                for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        ph[qt][e] = (bf16)s[qt][e >> 2][e & 3];
                        pl[qt][e] = ph[qt][e];
                    }
            } else if (LAZY) {
#pragma unroll
                for (int qt = 0; qt < NQT; ++qt) {
                    // raw scores (masked keys -inf); the reference max m is in raw units
                    float v[8];
                    const int kv = n - key0 - 8 * g;  // key 8 g + e valid iff e < kv
#pragma unroll
                    for (int e = 0; e < 8; ++e)  // (t = e >> 2, r = e & 3)
                        v[e] = (full || e < kv) ? s[qt][e >> 2][e & 3] : -INFINITY;
                    bool up = false;  // (by compares, as the PIPE form)
#pragma unroll
                    for (int e = 0; e < 8; ++e) up |= v[e] > lim[qt];
                    // (always at a unit's first sub-chunk: lim = -inf, key 0 is valid)
                    if (__any(up)) {
                        // over the 4 lane groups: permlane swaps
                        float cmax = fmaxf(fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])),
                                           fmaxf(fmaxf(v[4], v[5]), fmaxf(v[6], v[7])));
                        const auto p16 = __builtin_amdgcn_permlane16_swap(
                            __float_as_uint(cmax), __float_as_uint(cmax), false, false);
                        cmax = fmaxf(__uint_as_float(p16[0]), __uint_as_float(p16[1]));
                        const auto p32 = __builtin_amdgcn_permlane32_swap(
                            __float_as_uint(cmax), __float_as_uint(cmax), false, false);
                        cmax = fmaxf(__uint_as_float(p32[0]), __uint_as_float(p32[1]));
                        const float m_new = fmaxf(m[qt], cmax);
                        if (m_new != m[qt]) {  // (per lane; 0 at the first)
                            const float alpha = __builtin_amdgcn_exp2f((m[qt] - m_new) * sc);
                            lsum[qt] *= alpha;
#pragma unroll
                            for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
                        }
                        m[qt] = m_new;
                        lim[qt] = m_new + 8.0f / sc;
                        mneg[qt] = -m_new * sc;
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float pr = __builtin_amdgcn_exp2f(fmaf(v[e], sc, mneg[qt]));
                        lsum[qt] += pr;
                        ph[qt][e] = split_hi(pr);
                        pl[qt][e] = split_lo(pr);
                    }
                }
            } else
#pragma unroll
            for (int qt = 0; qt < NQT; ++qt) {
                // lane holds S^T[key0 + 8 g + 4 t + r][q_base + 16 qt + c]
                float cmax = -INFINITY;
                const int kv = n - key0 - 8 * g;  // key 8 g + 4 t + r valid iff 4 t + r < kv
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float v = (full || 4 * t + r < kv) ? s[qt][t][r] * sc : -INFINITY;
                        s[qt][t][r] = v;
                        cmax = fmaxf(cmax, v);
                    }
                {  // max over the 4 lane groups (lanes l, l^16, l^32, l^48): permlane swaps
                    const auto p16 = __builtin_amdgcn_permlane16_swap(
                        __float_as_uint(cmax), __float_as_uint(cmax), false, false);
                    cmax = fmaxf(__uint_as_float(p16[0]), __uint_as_float(p16[1]));
                    const auto p32 = __builtin_amdgcn_permlane32_swap(
                        __float_as_uint(cmax), __float_as_uint(cmax), false, false);
                    cmax = fmaxf(__uint_as_float(p32[0]), __uint_as_float(p32[1]));
                }
                const float m_new = fmaxf(m[qt], cmax);
                // rescale only when some running max moved (alpha == 1 exactly otherwise)
                if (__any(m_new != m[qt])) {
                    const float alpha = __builtin_amdgcn_exp2f(m[qt] - m_new);  // 0 at first
                    lsum[qt] *= alpha;
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
                }
                m[qt] = m_new;
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        // (raw v_exp_f32: no denormal-range rescale; p < 2^-126 is 0 here)
                        const float pr = __builtin_amdgcn_exp2f(s[qt][t][r] - m_new);
                        lsum[qt] += pr;
                        ph[qt][4 * t + r] = split_hi(pr);
                        pl[qt][4 * t + r] = split_lo(pr);
                    }
            }
__builtin_amdgcn_sched_barrier(0);
            bf16x8 vfr[4][2];  // [dt][hi, lo]
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int pt = 0; pt < 2; ++pt) {
                    const uint4 v4 = make_uint4(vt2[dt][pt][0].x, vt2[dt][pt][0].y,
                                                vt2[dt][pt][1].x, vt2[dt][pt][1].y);
                    __builtin_memcpy(&vfr[dt][pt], &v4, 16);
                }
            if (!(abl & 4))
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt)
                        o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            vfr[dt][p == 1], p == 2 ? pl[qt] : ph[qt], o[qt][dt], 0, 0, 0);
            }  // (PIPE)
            }
            };
            chunk(nqt_outer);
        };
        const int n_whole = n / KC;
        int ci = 0;
        for (; ci < n_whole; ++ci, b ^= 1) one_chunk(ci, std::true_type{});
        if (ci < n_chunks) {
            one_chunk(ci, std::false_type{});
            b ^= 1;
        }
        };
        if (!has_q) {
            for (int ci = 0; ci < n_chunks; ++ci, b ^= 1)
                if (ci > 0) stage_step(ci);
        } else if (three) {
            if constexpr (QTN == 3) chunk_loop(std::integral_constant<int, 3>{});
        } else if (two) {
            chunk_loop(std::integral_constant<int, 2>{});
        } else {
            chunk_loop(std::integral_constant<int, 1>{});
        }
        if (has_q) {
#pragma unroll
            for (int qt = 0; qt < QTN; ++qt) {
                float l = lsum[qt];
                l += __shfl_xor(l, 16, 64);
                l += __shfl_xor(l, 32, 64);
                const float inv = 1.0f / l;
                const int q = q_pass + qtile(qt) + c;
                if (q < nq) {
                    bf16 *out = ctx_split + (int64_t)(q0 + q) * 2 * H;
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt) {
                        bf16x4 hv, lv;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float y = o[qt][dt][r] * inv;
                            hv[r] = split_hi(y);
                            lv[r] = split_lo(y);
                        }
                        const int64_t sc0 = split_col(h * ATT_D + dt * 16 + 4 * g);
                        *reinterpret_cast<bf16x4 *>(out + sc0) = hv;
                        *reinterpret_cast<bf16x4 *>(out + sc0 + 32) = lv;
                    }
                }
            }
        }
        if (!more) break;
        cu = nu;
    }
#undef AX_READ_K
#undef AX_READ_VW
#undef AX_SEL
}

void launch_attention_x3(const bf16 *qkv, const int32_t *cu_seqlens, int n_docs, int H,
                         bf16 *ctx_split, hipStream_t s, const int32_t *qsel,
                         const int32_t *cu_qsel) {
    DI_REQUIRE(H % ATT_D == 0, DI_EINVAL, "hidden %d is not a multiple of the head dim 64", H);
    if (n_docs == 0) return;
    const int n_heads = H / ATT_D;
    const int64_t n_pairs = (int64_t)n_docs * n_heads;
    DI_REQUIRE(n_pairs < (1ll << 31), DI_ERANGE, "attention grid too large");
    // persistent: one 8-wave or two 4-wave workgroups per CU
    // balanced tiles + lazy max + interleaved softmax (r03 ab_attn: attention -8.5%,
    // then -3% per step), three query tiles per wave (384-query passes: every document of
    // up to 384 tokens in one pass; round6_o: -4.4%); DI_ATTN_X3 (developer A/B): 0 = the
    // round-2 form, 12 = no interleave, 28 = two tiles per wave
    static const int variant = [] {
        const char *e = getenv("DI_ATTN_X3");
        return e ? atoi(e) & 252 : 92;
    }();

    static const int abl = [] {
        const char *e = getenv("DI_ATTN_X3_ABLATE");
        return e ? atoi(e) : 0;
    }();
#define AX_LAUNCH(BL, LZ, PP, NW, QN, KC)                                                      \
    do {                                                                                       \
        DI_HIP(hipFuncSetAttribute((const void *)attention_x3_kernel<BL, LZ, PP, NW, QN, KC>,  \
                                   hipFuncAttributeMaxDynamicSharedMemorySize,                 \
                                   ax_lds(NW, QN, KC)));                                       \
        hipLaunchKernelGGL((attention_x3_kernel<BL, LZ, PP, NW, QN, KC>),                      \
                           dim3((int)std::min<int64_t>(                                        \
                               n_pairs, (int64_t)n_cu() * (160 * 1024 / ax_lds(NW, QN, KC)))), \
                           dim3(64 * NW), ax_lds(NW, QN, KC), s, qkv, cu_seqlens, H, n_heads,  \
                           (int)n_pairs, ctx_split, qsel, cu_qsel, abl);                       \
    } while (0)
    // The pruned last layer (qsel: the terms' rows, ~1/5 of the queries): 4-wave
    // workgroups with 32-key chunks, two per CU, so that a document's few query tiles
    // keep a workgroup's waves busy (DI_ATTN_X3_PRUNED=0: the full layers' kernel)
    static const int pruned_variant = [] {
        const char *e = getenv("DI_ATTN_X3_PRUNED");
        return e ? atoi(e) : 1;
    }();
    if (qsel && pruned_variant == 1 && variant == 92) {
        AX_LAUNCH(true, true, true, 4, 3, 32);
        check_launch("attention_x3");
        return;
    }
    // (r03 ab_attn, attention ms per step: BAL alone -3.5%, LAZY alone -5.6%, both -8.5%)
    switch (variant) {
    case 12: AX_LAUNCH(true, true, false, AX_WAVES, AX_QT, AX_KC); break;
    case 28: AX_LAUNCH(true, true, true, AX_WAVES, AX_QT, AX_KC); break;
    case 60: AX_LAUNCH(true, true, true, 4, AX_QT, AX_KC); break;  // (with the Q regions: one per CU)
    case 92: AX_LAUNCH(true, true, true, AX_WAVES, 3, AX_KC); break;  // three query tiles per wave
    case 220: AX_LAUNCH(true, true, true, 4, 3, 32); break;  // + 4 waves, 32-key chunks
    default: AX_LAUNCH(false, false, false, AX_WAVES, AX_QT, AX_KC); break;
    }
#undef AX_LAUNCH
    check_launch("attention_x3");
}

// One 32-key step of the online softmax for 16 queries (lane holds 8 raw scores of
// its query), in three parts so that attention_v3_kernel's key loop can test every
// query tile of a step with one branch and keep the common path of both tiles in one
// basic block.  Lazy rescale: the reference max m only moves when a score exceeds it
// by THR (2^8 in p) -- one compare per score and one ballot in the common case; the
// full max / rescale path runs on the first chunk and rarely after.
// p = exp2(s * sc - m * sc) by the raw v_exp_f32 (inputs <= 8; underflow to 0 is
// what softmax wants).
// lim = m + 8 / sc (kept by the caller, moved only with m)
__device__ __forceinline__ bool softmax_need(const f32x4 (&s)[2], float lim) {
    bool need = false;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) need |= s[t][r] > lim;
    return need;
}
__device__ __forceinline__ void softmax_rescale(const f32x4 (&s)[2], float &m, float &msc,
                                                f32x4 (&o)[4], f32x4 &l) {
    constexpr float sc = 0.125f * 1.4426950408889634f;
    float cmax = fmaxf(fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3])),
                       fmaxf(fmaxf(s[1][0], s[1][1]), fmaxf(s[1][2], s[1][3])));
    const auto p16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(cmax),
                                                      __float_as_uint(cmax), false, false);
    cmax = fmaxf(__uint_as_float(p16[0]), __uint_as_float(p16[1]));
    const auto p32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(cmax),
                                                      __float_as_uint(cmax), false, false);
    cmax = fmaxf(__uint_as_float(p32[0]), __uint_as_float(p32[1]));
    const float m_new = fmaxf(m, cmax);
    const float alpha = exp2f((m - m_new) * sc);  // 0 on the first chunk
    m = m_new;
    msc = m_new * sc;
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
}
__device__ __forceinline__ void softmax_p(const f32x4 (&s)[2], float msc, bf16x8 &pb) {
    constexpr float sc = 0.125f * 1.4426950408889634f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        pb[r] = (bf16)__builtin_amdgcn_exp2f(fmaf(s[0][r], sc, -msc));
        pb[4 + r] = (bf16)__builtin_amdgcn_exp2f(fmaf(s[1][r], sc, -msc));
    }
}

// ---------------------------------------------------------------------------
// Persistent, double-buffered form (bf16, max_len <= 320): the QKV projection is
// written row-major [M][3H] (Q | K | V, no V^T scatter), and one 512-thread
// workgroup per CU walks the (doc, head) pairs.  For each pair the K and V rows
// (128 B per key and head) are copied into LDS by LDS-DMA (global_load_lds,
// 16-byte XOR swizzle on the source), the NEXT pair's copy is issued before the
// current pair is computed, so the copy latency hides behind the MFMA/softmax
// work (the compute loop issues no global loads: Q fragments are loaded before
// the prefetch is issued).
//   K image: row r = 128 B, chunk q at slot q ^ (r & 7); S^T fragment row c of
//            tile t = key 8(c>>2) + 4t + (c&3) (lane group g then holds the
//            consecutive keys 8g..8g+7 of P^T).
//   V image: same row format; the O^T A operand (V^T rows) is read with
//            ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses key row
//            q of a 4-row block, columns 4p..4p+3; lane i receives column i.
// Eight waves, 32 queries (two 16-query tiles) per wave-block, blocks round robin.
// DB = true : two buffers of 320 K + 320 V rows (80 KiB each, 160 KiB: the whole
//             CU), next pair prefetched during the current one; n <= 320.
// DB = false: one buffer of 512 + 512 rows (128 KiB), no prefetch; n <= 512.
constexpr int ATT3_WAVES = 8;
template <bool DB>
struct Att3 {
    static constexpr int ROWS = DB ? 320 : 512;  // K and V image rows each
    static constexpr int BUF = 2 * ROWS * 128;
    static constexpr int LDS = DB ? 2 * BUF : BUF;
};

// K / V image swizzle: the 16-byte slot j of key row r is stored at slot
// j ^ att3_swz(r).  Bit 2 folds in row bit 3 so that the fragment reads are
// conflict-free: a ds_read_b128 lane group (16 lanes, rows 8 (c >> 2) + (c & 3) + 4 t
// of two lane groups g) and a ds_read_b64_tr_b16 lane group (32 lanes, rows
// 8 g + 4 h2 + q of two g) each see every bank once.  Bits 0-4 of a fragment row
// never depend on the 32-key chunk, so per lane every read address is a per-pair base
// plus key0 * 128 plus an immediate (see kb / vb below).
__device__ __forceinline__ int att3_swz(int r) { return (r & 7) ^ ((r >> 1) & 4); }

// f(integral_constant<K>) for K = K0, K0 + 1, .. < N until f returns true
template <int K, int N, class F>
__device__ __forceinline__ void att3_chunks(F &f) {
    if constexpr (K < N) {
        if (f(std::integral_constant<int, K>{})) return;
        att3_chunks<K + 1, N>(f);
    }
}

// The key loop is instantiated per tile count (1 or 2) and runs both tiles' S^T
// products, one shared rescale test (a branch only into the rare path) and both
// tiles' exp / O^T products as one basic block, so that one tile's softmax VALU
// overlaps the other tile's MFMAs (-2.5% attention time against a per-tile loop,
// bit-identical).
template <bool DB>
__global__ void __launch_bounds__(64 * ATT3_WAVES, 1)
attention_v3_kernel(const bf16 *__restrict__ qkv, const int32_t *__restrict__ cu_seqlens, int H,
                    int n_heads, int n_pairs, bf16 *__restrict__ ctx,
                    const int32_t *__restrict__ qsel, const int32_t *__restrict__ cu_qsel) {
    // qsel (optional): only the query rows qsel[cu_qsel[d] ..) (doc-local token
    // indices) of document d are computed, into ctx rows cu_qsel[d] + i (the encoder's
    // last layer: only the rows the term gather reads); keys are always every token.
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef __attribute__((address_space(3))) void lds_void;
    constexpr int QTB = 2;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c = lane & 15;
    const int ld = 3 * H;
    const uint32_t lds_base =
        (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char *)lds);

    // pair -> (doc, head): p / n_heads by a multiply-high (exact for p < 2^32 / n_heads)
    const uint32_t heads_magic = 0xFFFFFFFFu / (uint32_t)n_heads + 1u;
    auto doc_of = [&](int pp) { return (int)__umulhi((uint32_t)pp, heads_magic); };

    // LDS-DMA of pair p's K and V rows < round32(n) into buffer b, through a buffer
    // resource spanning the document's rows only: rows past n read zeros (their scores
    // are masked, their probabilities 0).  Slot j of row r lands at j ^ att3_swz(r); a
    // wave's pieces are all of one parity (pieces wave, wave + 8, ..; n8 is even), so
    // the swizzle is a per-lane constant: r_in ^ ((wave & 1) << 2).
    auto stage = [&](int p, int b) {
        const int doc = doc_of(p), h = p - doc * n_heads;
        const int tok0 = cu_seqlens[doc], n = cu_seqlens[doc + 1] - tok0;
        const int n8 = ((n + 31) & ~31) >> 3;  // 8-row pieces of K, and of V
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(qkv + (int64_t)tok0 * ld), (short)0, n * ld * 2, 0x00020000);
        const int r_in = lane >> 3;  // row within a piece
        const uint32_t voff = r_in * ld * 2 + (H + h * ATT_D) * 2 +
                              (((lane & 7) ^ r_in ^ ((wave & 1) << 2)) << 4);
        unsigned char *buf = lds + b * Att3<DB>::BUF;
        for (int pc = wave; pc < 2 * n8; pc += ATT3_WAVES) {
            const bool is_k = pc < n8;
            const int piece = is_k ? pc : pc - n8;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rsrc, (lds_void *)(buf + (is_k ? 0 : Att3<DB>::ROWS * 128) + piece * 1024), 16,
                voff + piece * 8 * ld * 2 + (is_k ? 0 : H * 2), 0, 0, 0);
        }
    };

    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;
    // Per-lane fragment offsets within an image (key0 = 0; see att3_swz).
    // K, S^T tile t, head-dim chunk ch: row krel + 4 t, slot 4 ch + g, stored at
    // (g ^ (c & 3)) | ((ch ^ t ^ b3) << 2)  ->  koff[ch ^ t] + 512 t.
    uint32_t koff[2];
    {
        const int krel = 8 * (c >> 2) + (c & 3), b3 = (c >> 2) & 1;
#pragma unroll
        for (int x = 0; x < 2; ++x) koff[x] = krel * 128 + ((g ^ (c & 3)) << 4) + ((x ^ b3) << 6);
    }
    // V^T by ds_read_b64_tr_b16, lane 4 q + p of a 16-lane group: row 8 g + 4 h2 + q,
    // columns 16 dt + 4 p..+3 = slot 2 dt + (p >> 1), half p & 1, stored at slot
    // u0 | ((u1 ^ dt0) << 1) | ((dt1 ^ h2 ^ g0) << 2) with u = (p >> 1) ^ q
    //   ->  voff[dt & 1][(dt >> 1) ^ h2] + 512 h2.
    uint32_t voff[2][2];
    {
        const int tq = c >> 2, tp = c & 3, u = (tp >> 1) ^ tq;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
                voff[a][bb] = (8 * g + tq) * 128 + 8 * (tp & 1) +
                              16 * ((u & 1) | (((u >> 1) ^ a) << 1) | ((bb ^ (g & 1)) << 2));
    }

    // Q of pair p comes one pair ahead (inline-asm global loads: the compiler sees no
    // pending load, so it neither waits nor drains the K/V prefetch for them), into the
    // register set not in use; the wait at the top of the pair retires it.  The two
    // sets are used in turn (the loop is unrolled by two: no register copies).
    // Query tiles (16 queries) of a document are dealt to the 8 waves in contiguous
    // runs whose lengths differ by at most one (wave w: tiles [t_first, t_first + t_cnt));
    // a wave takes its run two tiles at a time (K / V fragments shared) and an odd last
    // tile alone, so a pair costs ceil(tiles / 8) tile-steps instead of whole 32-query
    // blocks dealt round robin.
    auto tiles_of = [&](int nn, int &t_first, int &t_cnt) {
        const int n_t = (nn + 15) >> 4, base = n_t / ATT3_WAVES, extra = n_t % ATT3_WAVES;
        t_cnt = base + (wave < extra ? 1 : 0);
        t_first = wave * base + min(wave, extra);
    };
    // Q row addresses of pair pp for this wave's tile group i (tiles t_first + 2 i,
    // + 2 i + 1): [qt][ch]
    auto q_srcs = [&](int pp, int i, const bf16 *(&src)[QTB][2]) {
        const int dd = doc_of(pp), hh = pp - dd * n_heads;
        const int t0 = cu_seqlens[dd], nn = cu_seqlens[dd + 1] - t0;
        const int qs0 = qsel ? cu_qsel[dd] : 0, nq = qsel ? cu_qsel[dd + 1] - qs0 : nn;
        int t_first, t_cnt;
        tiles_of(nq, t_first, t_cnt);
        const int q_base = (t_first + 2 * i) * 16;
#pragma unroll
        for (int qt = 0; qt < QTB; ++qt) {
            const int qi = max(min(q_base + 16 * qt + c, nq - 1), 0);
            const int qloc = qsel ? (nq > 0 ? min(max(qsel[qs0 + qi], 0), max(nn - 1, 0)) : 0)
                                  : qi;
            const int qrow = t0 + qloc;
#pragma unroll
            for (int ch = 0; ch < 2; ++ch)
                src[qt][ch] = qkv + (int64_t)qrow * ld + hh * ATT_D + ch * 32 + 8 * g;
        }
    };
    // DB: tile group 0 of the next pair, one pair ahead
    auto load_q = [&](int pp, uint4 (&qd)[QTB][2]) {
        const bf16 *src[QTB][2];
        q_srcs(pp, 0, src);
#pragma unroll
        for (int qt = 0; qt < QTB; ++qt)
#pragma unroll
            for (int ch = 0; ch < 2; ++ch)
                asm volatile("global_load_dwordx4 %0, %1, off"
                             : "=v"(qd[qt][ch])
                             : "v"(src[qt][ch])
                             : "memory");
    };
    // tile group i of pair pp now, loaded together with the wait for them (one asm
    // statement: the outputs exist only after the wait, so no copy of a register
    // still being loaded can be scheduled above it).  The wait also retires any K / V
    // staging in flight (!DB: this pair's; DB, group 1: the next pair's, by then
    // mostly landed).
    auto load_q_wait = [&](int pp, int i, uint4 (&qd)[QTB][2]) {
        static_assert(QTB == 2, "load_q_wait: 4 loads");
        const bf16 *src[QTB][2];
        q_srcs(pp, i, src);
        asm volatile(
            "global_load_dwordx4 %0, %4, off\n\t"
            "global_load_dwordx4 %1, %5, off\n\t"
            "global_load_dwordx4 %2, %6, off\n\t"
            "global_load_dwordx4 %3, %7, off\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(qd[0][0]), "=&v"(qd[0][1]), "=&v"(qd[1][0]), "=&v"(qd[1][1])
            : "v"(src[0][0]), "v"(src[0][1]), "v"(src[1][0]), "v"(src[1][1])
            : "memory");
    };
    // qn: tile group 0 of pair p (DB: loaded one pair ahead, in flight); qc: the copy
    // the key loops read, made after the wait (so qn can take the next pair's loads)
    auto run_pair = [&](int p, int b, uint4 (&qc)[QTB][2], uint4 (&qn)[QTB][2])
                        __attribute__((always_inline)) {
        if (!DB) {
            stage(p, 0);
            load_q_wait(p, 0, qn);  // (also retires the staging)
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K/V and Q of this pair
#pragma unroll
        for (int qt = 0; qt < QTB; ++qt)
#pragma unroll
            for (int ch = 0; ch < 2; ++ch) {  // the loaded values exist from here on
                asm volatile("" : "+v"(qn[qt][ch].x), "+v"(qn[qt][ch].y), "+v"(qn[qt][ch].z),
                             "+v"(qn[qt][ch].w));
                qc[qt][ch] = qn[qt][ch];
            }
        __syncthreads();
        const int doc = doc_of(p), h = p - doc * n_heads;
        const int tok0 = cu_seqlens[doc], n = cu_seqlens[doc + 1] - tok0;
        const int qs0 = qsel ? cu_qsel[doc] : 0, nq = qsel ? cu_qsel[doc + 1] - qs0 : n;
        const int out0 = qsel ? qs0 : tok0;  // ctx row of query 0
        int t_first, t_cnt;
        tiles_of(nq, t_first, t_cnt);
        if (DB && p + (int)gridDim.x < n_pairs) {
            load_q(p + gridDim.x, qn);
            stage(p + gridDim.x, b ^ 1);
        }

        const uint32_t kim = lds_base + b * Att3<DB>::BUF;
        const uint32_t vim = kim + Att3<DB>::ROWS * 128;
        // Per-pair fragment bases (opaque to the compiler, so that it keeps one set
        // live instead of precomputing every buffer / chunk combination).
        uint32_t kb[2], vb[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            kb[x] = kim + koff[x];
            asm volatile("" : "+v"(kb[x]));
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
                vb[a][bb] = vim + voff[a][bb];
                asm volatile("" : "+v"(vb[a][bb]));
            }
        // Fragment reads of the 32-key chunk at key0 + SUB: key0 (a multiple of 64, one
        // address add per two chunks) in the address, SUB (compile time) and the row
        // parts in the instruction's immediate.  Inline asm: the compiler must not drain
        // the next pair's LDS-DMA with vmcnt(0) before them.  Issue and wait are
        // separate statements; the wait names every register still being written
        // ("+v"), so nothing touches one earlier (tools/asm_wait_scan.py checks the
        // assembly).
        using C0 = std::integral_constant<int, 0>;
        using C32 = std::integral_constant<int, 32>;
        auto read_k = [&](int key0, auto sub_c, bf16x8 (&kf)[2][2]) {  // [t][ch]
            constexpr int OFF = decltype(sub_c)::value * 128;
            const uint32_t k0 = kb[0] + key0 * 128, k1 = kb[1] + key0 * 128;
            asm volatile(
                "ds_read_b128 %0, %4 offset:%6\n\t"
                "ds_read_b128 %1, %5 offset:%6\n\t"
                "ds_read_b128 %2, %5 offset:%7\n\t"
                "ds_read_b128 %3, %4 offset:%7"
                : "=&v"(kf[0][0]), "=&v"(kf[0][1]), "=&v"(kf[1][0]), "=&v"(kf[1][1])
                : "v"(k0), "v"(k1), "i"(OFF), "i"(OFF + 512)
                : "memory");
        };
        auto read_v = [&](int key0, auto sub_c, uint2 (&hv)[4][2]) {  // [dt][h2]
            constexpr int OFF = decltype(sub_c)::value * 128;
            const uint32_t v00 = vb[0][0] + key0 * 128, v01 = vb[0][1] + key0 * 128,
                           v10 = vb[1][0] + key0 * 128, v11 = vb[1][1] + key0 * 128;
            asm volatile(
                "ds_read_b64_tr_b16 %0, %8 offset:%12\n\t"
                "ds_read_b64_tr_b16 %1, %9 offset:%13\n\t"
                "ds_read_b64_tr_b16 %2, %10 offset:%12\n\t"
                "ds_read_b64_tr_b16 %3, %11 offset:%13\n\t"
                "ds_read_b64_tr_b16 %4, %9 offset:%12\n\t"
                "ds_read_b64_tr_b16 %5, %8 offset:%13\n\t"
                "ds_read_b64_tr_b16 %6, %11 offset:%12\n\t"
                "ds_read_b64_tr_b16 %7, %10 offset:%13"
                : "=&v"(hv[0][0]), "=&v"(hv[0][1]), "=&v"(hv[1][0]), "=&v"(hv[1][1]),
                  "=&v"(hv[2][0]), "=&v"(hv[2][1]), "=&v"(hv[3][0]), "=&v"(hv[3][1])
                : "v"(v00), "v"(v01), "v"(v10), "v"(v11), "i"(OFF), "i"(OFF + 512)
                : "memory");
        };
        // counted waits naming the registers they retire ("+v"): LDS reads complete in
        // issue order, so lgkmcnt(N) retires all but the newest N
        auto wait_k = [&](bf16x8 (&kf)[2][2]) {  // K in flight, then the 8 V reads
            asm volatile("s_waitcnt lgkmcnt(8)"
                         : "+v"(kf[0][0]), "+v"(kf[0][1]), "+v"(kf[1][0]), "+v"(kf[1][1])
                         :
                         : "memory");
        };
        auto wait_v = [&](uint2 (&hv)[4][2], int) {  // V, then the 4 K reads
            asm volatile("s_waitcnt lgkmcnt(4)"
                         : "+v"(hv[0][0]), "+v"(hv[0][1]), "+v"(hv[1][0]), "+v"(hv[1][1]),
                           "+v"(hv[2][0]), "+v"(hv[2][1]), "+v"(hv[3][0]), "+v"(hv[3][1])
                         :
                         : "memory");
        };
        auto wait_all = [&](bf16x8 (&kf)[2][2], uint2 (&hv)[4][2]) {
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(kf[0][0]), "+v"(kf[0][1]), "+v"(kf[1][0]), "+v"(kf[1][1]),
                           "+v"(hv[0][0]), "+v"(hv[0][1]), "+v"(hv[1][0]), "+v"(hv[1][1]),
                           "+v"(hv[2][0]), "+v"(hv[2][1]), "+v"(hv[3][0]), "+v"(hv[3][1])
                         :
                         : "memory");
        };
        // merged key loop over NQ (1 or 2) query tiles starting at q_base, software
        // pipelined one chunk deep: step k issues S^T(k + 1) = K(k + 1) Q^T on the
        // matrix pipe, then computes P(k) (VALU) beside it, then O^T += V^T(k) P^T(k);
        // the LDS reads of K(k + 2) and V(k + 1) are in flight meanwhile.  Every
        // product and every f32 operation is the one of the unpipelined loop, in the
        // same order (bit-identical).
        auto key_loop = [&](auto nq_c, const uint4 (&qf)[QTB][2], int q_base)
                            __attribute__((always_inline)) {
            constexpr int NQ = decltype(nq_c)::value;
            float m[NQ], msc[NQ], lim[NQ];
            f32x4 o[NQ][4], l[NQ];
#pragma unroll
            for (int qt = 0; qt < NQ; ++qt) {
                m[qt] = -INFINITY;
                msc[qt] = -INFINITY;
                lim[qt] = -INFINITY;
                l[qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) o[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            bf16x8 qv[NQ][2];  // B operands Q^T
#pragma unroll
            for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
                for (int ch = 0; ch < 2; ++ch) __builtin_memcpy(&qv[qt][ch], &qf[qt][ch], 16);
            auto qk = [&](const bf16x8 (&kf)[2][2], f32x4 (&s)[NQ][2]) {
#pragma unroll
                for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
                    for (int t = 0; t < 2; ++t) s[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ch = 0; ch < 2; ++ch)  // independent chains adjacent
#pragma unroll
                    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
                        for (int t = 0; t < 2; ++t)
                            s[qt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][ch], qv[qt][ch], s[qt][t], 0, 0, 0);
            };
            auto rescale = [&](f32x4 (&s)[NQ][2]) {
                bool need[NQ], need_any = false;
#pragma unroll
                for (int qt = 0; qt < NQ; ++qt) {
                    need[qt] = softmax_need(s[qt], lim[qt]);
                    need_any |= need[qt];
                }
                if (__any(need_any)) {  // rare after the first chunk
#pragma unroll
                    for (int qt = 0; qt < NQ; ++qt)
                        if (__any(need[qt])) {
                            softmax_rescale(s[qt], m[qt], msc[qt], o[qt], l[qt]);
                            lim[qt] = m[qt] + 8.0f / (0.125f * 1.4426950408889634f);
                        }
                }
            };
            auto pv = [&](const f32x4 (&s)[NQ][2], const uint2 (&hv)[4][2]) {
                bf16x8 pb[NQ];
#pragma unroll
                for (int qt = 0; qt < NQ; ++qt) softmax_p(s[qt], msc[qt], pb[qt]);
                bf16x8 vf[4];
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const uint4 v4 = make_uint4(hv[dt][0].x, hv[dt][0].y, hv[dt][1].x, hv[dt][1].y);
                    __builtin_memcpy(&vf[dt], &v4, 16);
                }
#pragma unroll
                for (int qt = 0; qt < NQ; ++qt) {
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt)
                        o[qt][dt] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[dt], pb[qt], o[qt][dt], 0, 0, 0);
                    l[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[qt], l[qt], 0, 0, 0);
                }
            };
            // step at chunk key0 + SUB (not the last chunk): s = S^T(chunk) issued,
            // kn = K(chunk + 32) in flight, reloaded in place with K(chunk + 64) once the
            // S^T products have read it (MFMA A operands are read at issue; one chunk
            // past the end reads stale rows of the image, never used); sn receives
            // S^T(chunk + 32).  V(chunk) is read inside the step (its latency hides
            // behind the S^T products and the softmax).
            auto step = [&](int key0, auto sub_c, f32x4 (&s)[NQ][2], f32x4 (&sn)[NQ][2],
                            bf16x8 (&kn)[2][2]) {
                rescale(s);
                uint2 hv[4][2];
                read_v(key0, sub_c, hv);
                wait_k(kn);
                qk(kn, sn);
                read_k(key0, std::integral_constant<int, decltype(sub_c)::value + 64>{}, kn);
                wait_v(hv, 0);
                pv(s, hv);
            };
            // the last chunk: masked keys; kn (K one chunk past the end) is named by
            // the wait
            auto last = [&](int key0, auto sub_c, f32x4 (&s)[NQ][2], bf16x8 (&kn)[2][2]) {
                const int kc = key0 + decltype(sub_c)::value;
                if (kc + 32 > n) {
#pragma unroll
                    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
                        for (int t = 0; t < 2; ++t)
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (kc + 8 * g + 4 * t + r >= n) s[qt][t][r] = -INFINITY;
                }
                rescale(s);
                uint2 hv[4][2];
                read_v(key0, sub_c, hv);
                wait_all(kn, hv);
                pv(s, hv);
            };
            bf16x8 kf[2][2];
            f32x4 sa[NQ][2], sb[NQ][2];
            read_k(0, C0{}, kf);
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(kf[0][0]), "+v"(kf[0][1]), "+v"(kf[1][0]), "+v"(kf[1][1])
                         :
                         : "memory");
            qk(kf, sa);
            read_k(0, C32{}, kf);
            // two steps per iteration: S^T alternates between sa and sb without copies,
            // and the second step's addresses are the first's plus an immediate
            int key0 = 0;
            for (; key0 + 64 < n; key0 += 64) {
                step(key0, C0{}, sa, sb, kf);
                step(key0, C32{}, sb, sa, kf);
            }
            if (key0 + 32 < n) {
                step(key0, C0{}, sa, sb, kf);
                last(key0, C32{}, sb, kf);
            } else {
                last(key0, C0{}, sa, kf);
            }
#pragma unroll
            for (int qt = 0; qt < NQ; ++qt) {
                const float inv = 1.0f / l[qt][0];
                const int q = q_base + 16 * qt + c;
                if (q < nq) {
                    bf16 *out = ctx + (int64_t)(out0 + q) * H + h * ATT_D + 4 * g;
#pragma unroll
                    for (int dt = 0; dt < 4; ++dt) {
                        bf16x4 v;
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[qt][dt][r] * inv);
                        *reinterpret_cast<bf16x4 *>(out + dt * 16) = v;
                    }
                }
            }
        };
        // this wave's tiles, two at a time (documents past 8 x 32 queries, x 16 with
        // qsel, take a second group, its Q loaded here)
        for (int i = 0; 2 * i < t_cnt;) {
            if (t_cnt - 2 * i >= 2)
                key_loop(std::integral_constant<int, 2>{}, qc, (t_first + 2 * i) * 16);
            else
                key_loop(std::integral_constant<int, 1>{}, qc, (t_first + 2 * i) * 16);
            if (2 * ++i >= t_cnt) break;
            load_q_wait(p, i, qc);
        }
        // !DB: every wave is done with the buffer before the next pair restages it (DB:
        // the barrier at the top of the next pair orders buffer b's restaging, which
        // is issued after it, behind every wave's reads of this pair)
        if (!DB) __syncthreads();
    };
    uint4 qc[QTB][2], qn[QTB][2];
    int p = blockIdx.x, b = 0;
    if (DB && p < n_pairs) {
        stage(p, 0);
        load_q(p, qn);
    }
    for (; p < n_pairs; p += gridDim.x, b ^= (DB ? 1 : 0)) run_pair(p, b, qc, qn);
}

bool attention_v3_ok(int max_len, int H) { return max_len <= 512 && H % ATT_D == 0; }

void launch_attention_v3(const bf16 *qkv, const int32_t *cu_seqlens, int n_docs, int max_len,
                         int H, bf16 *ctx, hipStream_t s, const int32_t *qsel,
                         const int32_t *cu_qsel) {
    DI_REQUIRE(attention_v3_ok(max_len, H), DI_EINVAL, "attention v3: max_len %d > 512", max_len);
    if (n_docs == 0 || max_len == 0) return;
    static int n_cu = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
        return v > 0 ? v : 256;
    }();
    const int n_heads = H / ATT_D, n_pairs = n_docs * n_heads;
    // the kernel's pair -> document multiply-high is exact for pairs < 2^32 / n_heads
    DI_REQUIRE((int64_t)n_pairs * n_heads < (1ll << 32), DI_ERANGE, "attention v3: %d pairs", n_pairs);
    const int grid = std::min(n_pairs, n_cu);
    auto launch = [&](auto kern, int lds_bytes) {
        DI_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   lds_bytes));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * ATT3_WAVES), lds_bytes, s, qkv, cu_seqlens,
                           H, n_heads, n_pairs, ctx, qsel, cu_qsel);
    };
    if (max_len <= Att3<true>::ROWS)
        launch(attention_v3_kernel<true>, Att3<true>::LDS);
    else
        launch(attention_v3_kernel<false>, Att3<false>::LDS);
    check_launch("attention_v3");
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
    // 32*(n_docs + M/32) + 32 keys of read-ahead (+ slack), rounded to 64 columns
    int64_t need = 32 * ((int64_t)n_docs + M / 32) + 64 + 32;
    return (int)((need + 63) / 64 * 64);
}

template <typename T>
void launch_attention(const T *qk, const T *vt, const int32_t *cu_seqlens, int n_docs,
                      int max_len, int H, int ld_v, T *ctx, hipStream_t s, bf16 *ctx_split) {
    DI_REQUIRE(H % ATT_D == 0, DI_EINVAL, "hidden %d is not a multiple of the head dim 64", H);
    DI_REQUIRE(!ctx_split || sizeof(T) == 4, DI_EINVAL, "split output: f32 attention only");
    if (n_docs == 0 || max_len == 0) return;
    const int n_heads = H / ATT_D, n_pairs = n_docs * n_heads;
    // (bf16: the generic path of documents the persistent v3 kernel does not take)
    const int n_qb = (max_len + 16 * QT - 1) / (16 * QT);
    const int64_t blocks = (int64_t)((n_pairs + 7) / 8) * 8 * n_qb;
    DI_REQUIRE(blocks < (1ll << 31), DI_ERANGE, "attention grid too large");
    hipLaunchKernelGGL(attention_kernel<T>, dim3((unsigned)blocks), dim3(64), 0, s, qk, vt,
                       cu_seqlens, H, ld_v, n_qb, n_heads, n_pairs, ctx, ctx_split);
    check_launch("attention");
}

template void launch_attention<bf16>(const bf16 *, const bf16 *, const int32_t *, int, int, int,
                                     int, bf16 *, hipStream_t, bf16 *);
template void launch_attention<float>(const float *, const float *, const int32_t *, int, int,
                                      int, int, float *, hipStream_t, bf16 *);

}  // namespace di
