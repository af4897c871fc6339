// enc_gemm.hip -- MFMA GEMM with fused epilogues for the encoder (gfx950).
//
// C[M,N] = A[M,K] * B[N,K]^T : A = packed token activations (varlen, no padding),
// B = an nn.Linear weight (out x in) -- both operands K-contiguous, the layout the
// reference checkpoints hold (transformers Linear, called from
// src/deep_impact/models/xlmr_original.py:70-75).
//
// Tile 128x128, 4 waves (2x2, 64x64 each), K step = 128 bytes of each row
// (64 bf16 / 32 f32); LDS double buffer (2 x (16+16) KiB) filled by LDS-DMA
// (global_load_lds_dwordx4) one K step ahead, 16-byte XOR-swizzled chunks (T2,
// swizzle on the source address) read with ds_read_b128.
//   bf16: v_mfma_f32_16x16x32_bf16, f32 accumulate        (fast mode)
//   f32 : v_mfma_f32_16x16x4_f32 (exact f32 products)       (parity mode)
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "di_common.h"
#include "enc_common.h"

namespace di {

bool gemm256_ok(int epi, const GemmArgs &g);
void launch_gemm256(int epi, const GemmArgs &g, hipStream_t s);

constexpr int GB_M = 128, GB_N = 128, G_THREADS = 256;
constexpr int ROW_BYTES = 128;                 // bytes of one row per K step
constexpr int TILE_BYTES = GB_M * ROW_BYTES;   // 16 KiB

__device__ __forceinline__ int swz(int r, int c) { return r * ROW_BYTES + ((c ^ (r & 7)) << 4); }

template <typename T>
__device__ __forceinline__ void mfma_step(const uint4 &a, const uint4 &b, f32x4 &acc);

template <>
__device__ __forceinline__ void mfma_step<bf16>(const uint4 &a, const uint4 &b, f32x4 &acc) {
    bf16x8 av, bv;
    __builtin_memcpy(&av, &a, 16);
    __builtin_memcpy(&bv, &b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}

template <>
__device__ __forceinline__ void mfma_step<float>(const uint4 &a, const uint4 &b, f32x4 &acc) {
    // 4 floats per lane = 4 MFMA k-slots: k = 4*(lane>>4) + j for MFMA j
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc,
                                               0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc,
                                               0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc,
                                               0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc,
                                               0, 0, 0);
}

template <typename T, int EPI>
__global__ void __launch_bounds__(G_THREADS) gemm_nt_kernel(GemmArgs g) {
    constexpr int EPC = 16 / sizeof(T);  // elements per 16-byte chunk
    constexpr int BK = ROW_BYTES / sizeof(T);
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][2][TILE_BYTES];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // Tile order (speed only, never correctness):
    //  (1) XCD remap (T1): the dispatcher deals blocks round-robin over the 8
    //      XCDs, so block b runs on XCD b % 8; each XCD gets a contiguous range of
    //      tile ids (bijective form of cdna_hip_programming.md §5).
    //  (2) grouped order inside that range: GM M-tiles x all N-tiles, M fastest,
    //      so the ~64 blocks an XCD runs at once touch ~8 A panels and ~8 B panels
    //      (~3 MiB) -- they stay in the XCD's 4 MiB L2 instead of re-streaming
    //      the whole weight matrix for every M tile.
    const int n_tn = gridDim.x, n_tm = gridDim.y, n_tiles = n_tn * n_tm;
    int bid = blockIdx.y * gridDim.x + blockIdx.x;
    {
        const int q = n_tiles / 8, r = n_tiles % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    constexpr int GM = 8;
    const int grp = bid / (GM * n_tn), first_m = grp * GM;
    const int gsz = min(GM, n_tm - first_m);
    const int in = bid % (GM * n_tn);
    const int m0 = (first_m + in % gsz) * GB_M, n0 = (in / gsz) * GB_N;
    const T *A = static_cast<const T *>(g.A);
    const T *B = static_cast<const T *>(g.B);
    const int M = g.M, N = g.N, K = g.K;

    // Staging by LDS-DMA (global_load_lds_dwordx4): each wave moves 4 x 1 KiB of
    // A and of B per K step.  The LDS image is lane-linear (1 KiB = 8 rows of
    // 128 B), so the XOR swizzle goes on the per-lane SOURCE chunk (rule 21):
    // LDS slot p of row r holds global chunk p ^ (r & 7); swz() reads it back.
    typedef __attribute__((address_space(3))) void lds_void;
    const T *Asrc[4];
    const T *Bsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (wave * 4 + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        Asrc[i] = A + (int64_t)min(m0 + r, M - 1) * K + c * EPC;
        Bsrc[i] = B + (int64_t)min(n0 + r, N - 1) * K + c * EPC;
    }
#define STAGE(buf, k0)                                                                   \
    do {                                                                                 \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                  \
            __builtin_amdgcn_global_load_lds((const void *)(Asrc[i] + (k0)),             \
                                             (lds_void *)&lds[buf][0][(wave * 4 + i) * 1024], \
                                             16, 0, 0);                                  \
            __builtin_amdgcn_global_load_lds((const void *)(Bsrc[i] + (k0)),             \
                                             (lds_void *)&lds[buf][1][(wave * 4 + i) * 1024], \
                                             16, 0, 0);                                  \
        }                                                                                \
    } while (0)

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
    STAGE(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        if (t + 1 < nk) {
            if (cur) STAGE(0, (t + 1) * BK);
            else STAGE(1, (t + 1) * BK);
        }
        // all fragments of this K step first: one LDS round trip per step
        uint4 af[2][4], bfr[2][4];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = 4 * s + (lane >> 4);
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                int r = wm * 64 + mt * 16 + (lane & 15);
                af[s][mt] = *reinterpret_cast<const uint4 *>(&lds[cur][0][swz(r, c)]);
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                int r = wn * 64 + nt * 16 + (lane & 15);
                bfr[s][nt] = *reinterpret_cast<const uint4 *>(&lds[cur][1][swz(r, c)]);
            }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) mfma_step<T>(af[s][mt], bfr[s][nt], acc[mt][nt]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#undef STAGE

    // ---- epilogue -----------------------------------------------------------
    // V part of the QKV projection: transposed element stores into V^T
    if constexpr (EPI == EPI_QKV) {
        if (n0 >= 2 * g.hidden) {  // a 128-column tile never straddles 2H (H % 64 == 0)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const int col = n0 + wn * 64 + nt * 16 + (lane & 15);
                if (col >= N) continue;
                const float bias = g.bias[col];
                T *vt = static_cast<T *>(g.out2) + (int64_t)(col - 2 * g.hidden) * g.ld_v;
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    const int row0 = m0 + wm * 64 + mt * 16 + (lane >> 4) * 4;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (row0 + j < M)
                            vt[g.vcol[row0 + j]] = from_f32<T>(acc[mt][nt][j] + bias);
                }
            }
            return;
        }
    }
    // Everything else goes through LDS (the staging buffers are free now), 64
    // rows per pass, so that global stores are whole 16-byte chunks of rows.
    // bias / GELU are applied in registers; the residual (EPI_BIAS_RESID) is added
    // to the f32 staged value on the way out, then rounded once to T.
    using StT = typename std::conditional<EPI == EPI_BIAS_RESID, float, T>::type;
    constexpr int SE = sizeof(StT);
    constexpr int RS = GB_N * SE + 16;       // padded LDS row stride (bytes)
    constexpr int CPR = GB_N * SE / 16;      // 16-byte chunks per row
    constexpr int EPCH = 16 / SE;            // elements per chunk
    unsigned char *ot = &lds[0][0][0];
    float bias_v[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int col = n0 + wn * 64 + nt * 16 + (lane & 15);
        bias_v[nt] = (g.bias && col < N) ? g.bias[col] : 0.f;
    }
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        if (wm == pass) {
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const int lc = wn * 64 + nt * 16 + (lane & 15);
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int lr = mt * 16 + (lane >> 4) * 4 + j;  // row within the pass
                        float v = acc[mt][nt][j] + bias_v[nt];
                        if constexpr (EPI == EPI_BIAS_GELU) v = std::is_same<T, bf16>::value ? gelu_bf16(v) : gelu_erf(v);
                        *reinterpret_cast<StT *>(ot + lr * RS + lc * SE) = from_f32<StT>(v);
                    }
                }
            }
        }
        __syncthreads();
        const int row_base = m0 + pass * 64;
#pragma unroll
        for (int i = 0; i < 64 * CPR / G_THREADS; ++i) {
            const int id = tid + i * G_THREADS;
            const int lr = id / CPR, ch = id % CPR;
            const int row = row_base + lr;
            const int col0 = n0 + ch * EPCH;
            if (row >= M) continue;
            uint4 v = *reinterpret_cast<const uint4 *>(ot + lr * RS + ch * 16);
            T *op = static_cast<T *>(g.out) + (int64_t)row * g.ld_out + col0;
            if constexpr (EPI == EPI_BIAS_RESID) {
                const T *rp = static_cast<const T *>(g.resid) + (int64_t)row * N + col0;
                const float *f = reinterpret_cast<const float *>(&v);
                if (col0 + 4 <= N) {
                    if constexpr (sizeof(T) == 2) {
                        const bf16x4 rv = *reinterpret_cast<const bf16x4 *>(rp);
                        bf16x4 o;
#pragma unroll
                        for (int q = 0; q < 4; ++q) o[q] = (bf16)(f[q] + (float)rv[q]);
                        *reinterpret_cast<bf16x4 *>(op) = o;
                    } else {
                        const float4 rv = *reinterpret_cast<const float4 *>(rp);
                        *reinterpret_cast<float4 *>(op) =
                            make_float4(f[0] + rv.x, f[1] + rv.y, f[2] + rv.z, f[3] + rv.w);
                    }
                } else {  // ragged N tail
                    for (int q = 0; q < 4 && col0 + q < N; ++q)
                        op[q] = from_f32<T>(f[q] + to_f32(rp[q]));
                }
            } else if (col0 + EPCH <= N) {
                *reinterpret_cast<uint4 *>(op) = v;
            } else {  // ragged N tail: element stores
                const T *e = reinterpret_cast<const T *>(&v);
                for (int q = 0; q < EPCH && col0 + q < N; ++q) op[q] = e[q];
            }
        }
        __syncthreads();
    }
}

template <typename T>
void launch_gemm(int epi, const GemmArgs &g, hipStream_t s) {
    DI_REQUIRE(g.K % (ROW_BYTES / (int)sizeof(T)) == 0, DI_EINVAL,
               "GEMM K=%d must be a multiple of %d", g.K, ROW_BYTES / (int)sizeof(T));
    if (g.M == 0) return;
    if constexpr (std::is_same<T, bf16>::value) {
        if (gemm256_ok(epi, g)) {
            launch_gemm256(epi, g, s);
            return;
        }
    }
    dim3 grid((g.N + GB_N - 1) / GB_N, (g.M + GB_M - 1) / GB_M);
    switch (epi) {
        case EPI_BIAS:
            hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_BIAS>), grid, dim3(G_THREADS), 0, s, g);
            break;
        case EPI_BIAS_GELU:
            hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_BIAS_GELU>), grid, dim3(G_THREADS), 0, s,
                               g);
            break;
        case EPI_BIAS_RESID:
            hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_BIAS_RESID>), grid, dim3(G_THREADS), 0, s,
                               g);
            break;
        case EPI_QKV:
            hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_QKV>), grid, dim3(G_THREADS), 0, s, g);
            break;
        default:
            fail(DI_EINVAL, "bad GEMM epilogue");
    }
    check_launch("gemm_nt");
}

template void launch_gemm<bf16>(int, const GemmArgs &, hipStream_t);
template void launch_gemm<float>(int, const GemmArgs &, hipStream_t);

}  // namespace di
