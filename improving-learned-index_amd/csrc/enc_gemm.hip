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

#include "di_common.h"
#include "enc_common.h"

namespace di {

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
    // XCD-aware tile order: consecutive tile ids share an XCD's L2 when the
    // dispatcher deals blocks round-robin over the 8 XCDs (speed only).
    const int n_tn = gridDim.x, n_tiles = gridDim.x * gridDim.y;
    int bid = blockIdx.y * gridDim.x + blockIdx.x;
    {
        const int q = n_tiles / 8, r = n_tiles % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int m0 = (bid / n_tn) * GB_M, n0 = (bid % n_tn) * GB_N;
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

    // ---- epilogue: lane holds rows (lane>>4)*4 + j of column lane&15 ----------
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int col = n0 + wn * 64 + nt * 16 + (lane & 15);
        if (col >= N) continue;
        const float bias = g.bias ? g.bias[col] : 0.f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            const int row0 = m0 + wm * 64 + mt * 16 + (lane >> 4) * 4;
            if constexpr (EPI == EPI_QKV) {
                if (col >= 2 * g.hidden) {
                    T *vt = static_cast<T *>(g.out2) + (int64_t)(col - 2 * g.hidden) * g.ld_v;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (row0 + j < M)
                            vt[g.vcol[row0 + j]] = from_f32<T>(acc[mt][nt][j] + bias);
                    continue;
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = row0 + j;
                if (row >= M) break;
                float v = acc[mt][nt][j] + bias;
                if constexpr (EPI == EPI_BIAS || EPI == EPI_QKV) {
                    static_cast<T *>(g.out)[(int64_t)row * g.ld_out + col] = from_f32<T>(v);
                } else if constexpr (EPI == EPI_BIAS_GELU) {
                    static_cast<T *>(g.out)[(int64_t)row * g.ld_out + col] =
                        from_f32<T>(gelu_erf(v));
                } else {  // EPI_BIAS_RESID
                    v += to_f32(static_cast<const T *>(g.resid)[(int64_t)row * N + col]);
                    static_cast<float *>(g.out)[(int64_t)row * g.ld_out + col] = v;
                }
            }
        }
    }
}

template <typename T>
void launch_gemm(int epi, const GemmArgs &g, hipStream_t s) {
    DI_REQUIRE(g.K % (ROW_BYTES / (int)sizeof(T)) == 0, DI_EINVAL,
               "GEMM K=%d must be a multiple of %d", g.K, ROW_BYTES / (int)sizeof(T));
    if (g.M == 0) return;
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
