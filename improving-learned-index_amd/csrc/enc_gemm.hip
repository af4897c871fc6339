// enc_gemm.hip -- MFMA GEMM with fused epilogues for the encoder (gfx950).
//
// C[M,N] = A[M,K] * B[N,K]^T : A = packed token activations (varlen, no padding),
// B = an nn.Linear weight (out x in) -- both operands K-contiguous, the layout the
// reference checkpoints hold (transformers Linear, called from
// src/deep_impact/models/xlmr_original.py:70-75).
//
// Tile 128x128, 4 waves (2x2, 64x64 each), K step = 128 bytes of each row
// (64 bf16 / 32 f32); LDS double buffer (2 x (16+16) KiB), register-staged
// global loads issued one K step ahead (T14 split), 16-byte XOR-swizzled LDS
// chunks (T2) read with ds_read_b128.
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

    // staging: 4 chunks of A and 4 of B per thread per K step; thread t owns
    // chunk (row, col) = ((t + 256 i) / 8, t % 8) of each 128 x 128-byte tile
    const int scol = tid & 7;
    const int srow0 = tid >> 3;  // + 32 i
    const T *Ap[4];
    const T *Bp[4];
    int soff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = srow0 + 32 * i;
        Ap[i] = A + (int64_t)min(m0 + r, M - 1) * K + scol * EPC;
        Bp[i] = B + (int64_t)min(n0 + r, N - 1) * K + scol * EPC;
        soff[i] = swz(r, scol);
    }
    uint4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
#define GLOAD(k0)                                                        \
    do {                                                                 \
        ra0 = *reinterpret_cast<const uint4 *>(Ap[0] + (k0));            \
        ra1 = *reinterpret_cast<const uint4 *>(Ap[1] + (k0));            \
        ra2 = *reinterpret_cast<const uint4 *>(Ap[2] + (k0));            \
        ra3 = *reinterpret_cast<const uint4 *>(Ap[3] + (k0));            \
        rb0 = *reinterpret_cast<const uint4 *>(Bp[0] + (k0));            \
        rb1 = *reinterpret_cast<const uint4 *>(Bp[1] + (k0));            \
        rb2 = *reinterpret_cast<const uint4 *>(Bp[2] + (k0));            \
        rb3 = *reinterpret_cast<const uint4 *>(Bp[3] + (k0));            \
    } while (0)
#define LSTORE(buf)                                                      \
    do {                                                                 \
        *reinterpret_cast<uint4 *>(&lds[buf][0][soff[0]]) = ra0;         \
        *reinterpret_cast<uint4 *>(&lds[buf][0][soff[1]]) = ra1;         \
        *reinterpret_cast<uint4 *>(&lds[buf][0][soff[2]]) = ra2;         \
        *reinterpret_cast<uint4 *>(&lds[buf][0][soff[3]]) = ra3;         \
        *reinterpret_cast<uint4 *>(&lds[buf][1][soff[0]]) = rb0;         \
        *reinterpret_cast<uint4 *>(&lds[buf][1][soff[1]]) = rb1;         \
        *reinterpret_cast<uint4 *>(&lds[buf][1][soff[2]]) = rb2;         \
        *reinterpret_cast<uint4 *>(&lds[buf][1][soff[3]]) = rb3;         \
    } while (0)

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
    GLOAD(0);
    LSTORE(0);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        if (t + 1 < nk) GLOAD((t + 1) * BK);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = 4 * s + (lane >> 4);
            uint4 af[4], bfr[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                int r = wm * 64 + mt * 16 + (lane & 15);
                af[mt] = *reinterpret_cast<const uint4 *>(&lds[cur][0][swz(r, c)]);
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                int r = wn * 64 + nt * 16 + (lane & 15);
                bfr[nt] = *reinterpret_cast<const uint4 *>(&lds[cur][1][swz(r, c)]);
            }
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) mfma_step<T>(af[mt], bfr[nt], acc[mt][nt]);
        }
        if (t + 1 < nk) {
            if (cur) LSTORE(0);
            else LSTORE(1);
        }
        __syncthreads();
    }
#undef GLOAD
#undef LSTORE

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
                        if (row0 + j < M) vt[row0 + j] = from_f32<T>(acc[mt][nt][j] + bias);
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
