// enc_gemm2x.hip -- 256x128-tile bf16 MFMA GEMM, two workgroups per CU (gfx950).
//
// Same contract as enc_gemm256.hip (C[M,N] = A[M,K] * B[N,K]^T + fused epilogue: the
// encoder's QKV / O / FFN1 / FFN2 projections, reference xlmr_original.py:70-75) for
// N % 128 == 0, K % 64 == 0, A readable up to round_up(M, 256) rows.
//
// Experimental, opt-in (see gemm2x_enabled).
// Why: at K = 768 the 256x256 kernel spends ~35% of its time in the epilogue (bias,
// GELU, residual loads, 128 KiB of stores per tile) with the matrix cores idle, and
// with one 8-wave workgroup per CU nothing else can issue MFMAs meanwhile.  Here a
// workgroup is 4 waves (one per SIMD, 128x64 outputs each = the same 128 accumulator
// VGPRs per wave) and takes 76 KiB of LDS, so two workgroups share every CU and one's
// epilogue runs under the other's K loop.
//
// K loop: K step 32 (one v_mfma_f32_16x16x32_bf16 k extent).  A ring of three LDS
// slots (A image 256 rows + B image 128 rows, 64 B per row, 24 KiB per slot) filled by
// LDS-DMA (global_load_lds_dwordx4) two steps ahead; the fragments of step t+1 are
// read into the second register set while the 32 MFMAs of step t run (the two sets
// alternate, the loop is unrolled by two).  One barrier per step: before it every
// wave retires its fragment reads (lgkmcnt(0)) and its DMA of step t+1 (counted
// vmcnt, never 0 in steady state); after it slot t%3 is free and gets step t+3.
// Image layout: two 64-B rows per 128-B line, 16-B chunk q of line L at slot
// q ^ (L & 7) (swizzle on the DMA source address): conflict-free ds_read_b128.
// B rows are permuted inside every 32-column group exactly as in enc_gemm256.hip, so
// that in the C^T accumulator layout (weight fragment first) every lane holds 8
// consecutive output columns: 16-byte stores straight from registers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int GX_T = 256;
constexpr int GX_BM = 256, GX_BN = 128;
constexpr int GX_A = GX_BM * 64;         // A image bytes per slot (16 KiB)
constexpr int GX_B = GX_BN * 64;         // B image bytes per slot (8 KiB)
constexpr int GX_SLOT = GX_A + GX_B;     // 24 KiB
constexpr int GX_PAR = 3 * GX_SLOT;      // epilogue parameters (staged with the prologue)
constexpr int GX_PAR_ROW = 0, GX_PAR_C0 = 2048, GX_PAR_C1 = 2560, GX_PAR_C2 = 3072,
              GX_PAR_C3 = 3584;
constexpr int GX_LDS = GX_PAR + 4096 + 16;  // 76 KiB: two workgroups per CU

// per-CU workgroup arrival counters (stagger parity; never reset: only the parity
// of each launch's arrivals is used)
__device__ uint32_t g_gx_arrivals[4096];

#define GX_BAR() asm volatile("s_barrier" ::: "memory")

template <int EPI>
__global__ void __launch_bounds__(GX_T) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm2x_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    typedef __attribute__((address_space(3))) void lds_void;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;

    const int M = g.M, N = g.N, K = g.K;
    const int nk = K / 32;
    const int n_tn = N / GX_BN, n_tm = (M + GX_BM - 1) / GX_BM, n_tiles = n_tn * n_tm;
    const int GM = g.tune_gm > 0 ? g.tune_gm : 4;

    // Persistent, two workgroups per CU.  Both would start together and, with equal
    // work per tile, reach their epilogues together: the second workgroup to arrive on
    // a CU (parity of a per-CU arrival counter) starts about half a tile late, so the
    // epilogue of one runs under the other's K loop for the whole launch (speed only).
    {
        uint32_t *flag = reinterpret_cast<uint32_t *>(lds + GX_PAR + 4096);
        if (tid == 0) {
            uint32_t hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            const uint32_t key = ((xcc & 15u) << 8) | ((hw >> 8) & 0xFFu);  // XCC, SE, SH, CU
            *flag = atomicAdd(&g_gx_arrivals[key], 1u) & 1u;
        }
        __syncthreads();
        if (*flag) {
            const uint64_t d = g.stagger > 0 ? (uint64_t)g.stagger : (uint64_t)18 * K;
            const uint64_t t0 = __builtin_amdgcn_s_memtime();
            while (__builtin_amdgcn_s_memtime() - t0 < d) __builtin_amdgcn_s_sleep(8);
        }
    }
    for (int bid0 = blockIdx.x; bid0 < n_tiles; bid0 += gridDim.x) {
    // tile order: XCD remap (bijective) + grouped GM x all-N order (speed only); with
    // gridDim.x % 8 == 0 the linear id keeps the XCD of the non-persistent order
    int bid = bid0;
    {
        const int q = n_tiles / 8, r = n_tiles % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int grp = bid / (GM * n_tn), first_m = grp * GM;
    const int gsz = min(GM, n_tm - first_m);
    const int in = bid % (GM * n_tn);
    const int m0 = (first_m + in % gsz) * GX_BM;
    const int n0 = (in / gsz) * GX_BN;

    // ---- DMA sources (per lane) ------------------------------------------------
    // piece p (1 KiB = lines 8p..8p+7 of an image); lane i writes slot i&7 of line
    // 8p + (i>>3), which holds chunk q = (i&7) ^ (i>>3): image row 16p + 2(i>>3) +
    // (q>>2), k-chunk q&3.  Wave w stages A pieces w + 4j (j < 4), B pieces w + 4j (j < 2).
    const int qch = (lane & 7) ^ (lane >> 3);
    const int r_l = 2 * (lane >> 3) + (qch >> 2);
    const int c_l = (qch & 3) * 8;
    const void *A_p = g.A, *B_p = g.B;
    asm volatile("" : "+s"(A_p), "+s"(B_p));
    const bf16 *a_src = static_cast<const bf16 *>(A_p) + (int64_t)(m0 + 16 * wave + r_l) * K + c_l;
    const int64_t a_j = (int64_t)64 * K;
    auto b_row = [&](int q) {  // B image row q -> weight row (permuted in 32-col groups)
        const int qq = q & 31;
        return (q & ~31) + ((qq >> 2) & 3) * 8 + (qq >> 4) * 4 + (qq & 3);
    };
    const bf16 *b_src0 = static_cast<const bf16 *>(B_p) + (int64_t)(n0 + b_row(16 * wave + r_l)) * K + c_l;
    const bf16 *b_src1 =
        static_cast<const bf16 *>(B_p) + (int64_t)(n0 + b_row(16 * (wave + 4) + r_l)) * K + c_l;
    auto stage = [&](int kt, int slot) {
        const int ko = kt * 32;
        unsigned char *base = lds + slot * GX_SLOT + wave * 1024;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds((const void *)(a_src + j * a_j + ko),
                                             (lds_void *)(base + j * 4096), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *)(b_src0 + ko), (lds_void *)(base + GX_A),
                                         16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *)(b_src1 + ko),
                                         (lds_void *)(base + GX_A + 4096), 16, 0, 0);
    };

    // ---- fragment reads ----------------------------------------------------------
    // A fragment mt of wave wr: image row wr*128 + mt*16 + (lane&15) = line
    // wr*64 + mt*8 + ((lane&15)>>1), chunk ((lane&1)*4 + (lane>>4)) at slot chunk ^ ((lane>>1)&7);
    // B fragment nt of wave wc: image row wc*64 + nt*16 + (lane&15), same form.
    const int fchunk = ((lane & 1) * 4 + (lane >> 4)) ^ ((lane >> 1) & 7);
    const uint32_t lds_base =
        (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char *)lds);
    const uint32_t a_rd = lds_base + (wr * 64 + ((lane & 15) >> 1)) * 128 + fchunk * 16;
    const uint32_t b_rd = lds_base + GX_A + (wc * 32 + ((lane & 15) >> 1)) * 128 + fchunk * 16;
    uint4 xa[8], xb[4], ya[8], yb[4];
#define GX_LD(dst, addr, off) \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(off))
#define GX_READ(SA, SB, slot)                                                                  \
    do {                                                                                       \
        const uint32_t so = (uint32_t)(slot) * GX_SLOT;                                        \
        const uint32_t ra = a_rd + so, rb = b_rd + so;                                         \
        GX_LD(SB[0], rb, 0);                                                                   \
        GX_LD(SB[1], rb, 1024);                                                                \
        GX_LD(SB[2], rb, 2048);                                                                \
        GX_LD(SB[3], rb, 3072);                                                                \
        GX_LD(SA[0], ra, 0);                                                                   \
        GX_LD(SA[1], ra, 1024);                                                                \
        GX_LD(SA[2], ra, 2048);                                                                \
        GX_LD(SA[3], ra, 3072);                                                                \
        GX_LD(SA[4], ra, 4096);                                                                \
        GX_LD(SA[5], ra, 5120);                                                                \
        GX_LD(SA[6], ra, 6144);                                                                \
        GX_LD(SA[7], ra, 7168);                                                                \
    } while (0)

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define GX_MFMA(SA, SB)                                                                        \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        __builtin_amdgcn_s_setprio(1);                                                         \
        _Pragma("unroll") for (int mm = 0; mm < 8; ++mm)                                       \
            _Pragma("unroll") for (int nn = 0; nn < 4; ++nn) {                                 \
                bf16x8 av, bv;                                                                 \
                __builtin_memcpy(&av, &SA[mm], 16);                                            \
                __builtin_memcpy(&bv, &SB[nn], 16);                                            \
                acc[mm][nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv, av, acc[mm][nn], 0, \
                                                                      0, 0);                   \
            }                                                                                  \
        __builtin_amdgcn_s_setprio(0);                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                     \
    } while (0)

    // ---- epilogue parameters (wave 0, issued before every stage load, so the
    // prologue's counted wait retires them) -----------------------------------------
    {
        constexpr bool FOLD = EPI == EPI_FOLD || EPI == EPI_FOLD_GELU;
        constexpr bool RS = EPI == EPI_RESID_STATS;
        if (wave == 0) {
            auto par512 = [&](const void *src, int off) {  // 128 floats: 16 B x 32 lanes
                if (lane < 32)
                    __builtin_amdgcn_global_load_lds(
                        (const void *)(static_cast<const char *>(src) + lane * 16),
                        (lds_void *)(lds + GX_PAR + off), 16, 0, 0);
            };
            par512((FOLD ? g.col_c : g.bias) + n0, GX_PAR_C0);
            if (FOLD) par512(g.col_s + n0, GX_PAR_C1);
            if (RS && g.row_ln) {
                par512(g.res_gamma + n0, GX_PAR_C1);
                par512(g.res_beta + n0, GX_PAR_C2);
            }
            if (RS && g.head_wg) par512(g.head_wg + n0, GX_PAR_C3);
            if (FOLD || (RS && g.row_ln)) {
                int m0r = m0;
                asm volatile("" : "+s"(m0r));
                __builtin_amdgcn_global_load_lds(
                    (const void *)(reinterpret_cast<const char *>(g.row_ln + m0r) + lane * 16),
                    (lds_void *)(lds + GX_PAR + GX_PAR_ROW), 16, 0, 0);
                __builtin_amdgcn_global_load_lds(
                    (const void *)(reinterpret_cast<const char *>(g.row_ln + m0r + 128) + lane * 16),
                    (lds_void *)(lds + GX_PAR + GX_PAR_ROW + 1024), 16, 0, 0);
            }
        }
    }
    // ---- prologue: steps 0, 1, 2 in flight; fragments of step 0 -------------------
    stage(0, 0);
    stage(1, 1);
    stage(2, 2);  // nk >= 4
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    GX_BAR();
    GX_READ(xa, xb, 0);

    // one step: (1) wait for the DMA of step t+1 and this wave's reads of step t;
    // (2) barrier; (3) slot t%3 -> step t+3; (4) reads of step t+1; (5) MFMAs of step t
#define GX_STEP(CA, CB, NA, NB, t)                                                             \
    do {                                                                                       \
        if ((t) + 2 < nk)                                                                      \
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");                                   \
        else                                                                                   \
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                   \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                     \
        GX_BAR();                                                                              \
        if ((t) + 3 < nk) stage((t) + 3, (t) % 3);                                             \
        if ((t) + 1 < nk) GX_READ(NA, NB, ((t) + 1) % 3);                                      \
        GX_MFMA(CA, CB);                                                                       \
    } while (0)

    for (int t = 0; t < nk; t += 2) {
        GX_STEP(xa, xb, ya, yb, t);
        GX_STEP(ya, yb, xa, xb, t + 1);
    }
#undef GX_STEP
#undef GX_LD
#undef GX_READ
#undef GX_MFMA

    // ---- epilogue ------------------------------------------------------------------
    if (g.ablate & 1) {  // profiling: main loop only (accumulators kept live)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    } else {
    // C^T layout: lane l holds, for A fragment mt and weight-column half h, output row
    //   m = m0 + wr*128 + mt*16 + (l & 15)
    // and the 8 consecutive columns n = n0 + wc*64 + h*32 + (l >> 4)*8 + e, e = 0..7,
    // in acc[mt][2h][0..3], acc[mt][2h+1][0..3].
    int m0e = m0;  // opaque: keeps the per-row epilogue offsets out of the K loop
    asm volatile("" : "+s"(m0e));
    const int row_l = m0e + wr * 128 + (lane & 15);
    const int col_l = n0 + wc * 64 + (lane >> 4) * 8;
    const int prow = wr * 128 + (lane & 15);    // + mt * 16
    const int pcol = wc * 64 + (lane >> 4) * 8;  // + h * 32 + e
    auto par8 = [&](int off, int h, float (&v)[8]) {
        const float4 a = *reinterpret_cast<const float4 *>(lds + GX_PAR + off + (pcol + h * 32) * 4);
        const float4 b = *reinterpret_cast<const float4 *>(lds + GX_PAR + off + (pcol + h * 32 + 4) * 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    };
    auto prow2 = [&](int mt) {
        return *reinterpret_cast<const float2 *>(lds + GX_PAR + GX_PAR_ROW + (prow + mt * 16) * 8);
    };
    float bias_v[2][8];
    par8(GX_PAR_C0, 0, bias_v[0]);
    par8(GX_PAR_C0, 1, bias_v[1]);
    if constexpr (EPI == EPI_FOLD || EPI == EPI_FOLD_GELU) {
        // LN folded into this GEMM: y = r acc - r mu s + c  (per row r, mu; per column s, c)
        float ra[8], rb[8];
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
            const float2 p = prow2(mt);
            ra[mt] = p.x;
            rb[mt] = p.y;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float cs[8];
            par8(GX_PAR_C1, h, cs);
            const float(&cc)[8] = bias_v[h];
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
                const int row = row_l + mt * 16;
                if (row >= M) continue;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    v[e] = fmaf(ra[mt], acc[mt][2 * h + (e >> 2)][e & 3], fmaf(rb[mt], cs[e], cc[e]));
                if constexpr (EPI == EPI_FOLD_GELU) gelu_erf8(v);
                bf16x8 ov;
#pragma unroll
                for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
                *reinterpret_cast<bf16x8 *>(static_cast<bf16 *>(g.out) + (int64_t)row * g.ld_out +
                                            col_l + h * 32) = ov;
            }
        }
    } else if constexpr (EPI == EPI_RESID_STATS) {
        // out = acc + bias + LN(resid) (resid normalised on the fly from its row
        // statistics, or plain), and this tile's partial statistics of the rounded out
        const bool res_ln = g.row_ln != nullptr;
        float ra[8], rb[8], ss[8], sq[8], sd[8];
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
            ss[mt] = sq[mt] = sd[mt] = 0.f;
            ra[mt] = 1.f;
            rb[mt] = 0.f;
            if (res_ln) {
                const float2 p = prow2(mt);
                ra[mt] = p.x;
                rb[mt] = p.y;
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float gm[8], bt[8], wg[8];
            if (res_ln) {
                par8(GX_PAR_C1, h, gm);
                par8(GX_PAR_C2, h, bt);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    gm[e] = 1.f;
                    bt[e] = 0.f;
                }
            }
            if (g.head_wg) {
                par8(GX_PAR_C3, h, wg);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) wg[e] = 0.f;
            }
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
                const int row = row_l + mt * 16;
                if (row >= M) continue;
                const bf16x8 rv = *reinterpret_cast<const bf16x8 *>(
                    static_cast<const bf16 *>(g.resid) + (int64_t)row * N + col_l + h * 32);
                bf16x8 ov;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float res = fmaf(gm[e], fmaf(ra[mt], (float)rv[e], rb[mt]), bt[e]);
                    ov[e] = (bf16)(acc[mt][2 * h + (e >> 2)][e & 3] + bias_v[h][e] + res);
                    const float yb = (float)ov[e];
                    ss[mt] += yb;
                    sq[mt] = fmaf(yb, yb, sq[mt]);
                    sd[mt] = fmaf(yb, wg[e], sd[mt]);
                }
                *reinterpret_cast<bf16x8 *>(static_cast<bf16 *>(g.out) + (int64_t)row * g.ld_out +
                                            col_l + h * 32) = ov;
            }
        }
        // partials: the 4 lane groups (lanes l, l^16, l^32, l^48 share a row), then
        // the 2 wc waves through LDS (the ring is free), fixed order
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
            for (int d = 16; d <= 32; d <<= 1) {
                ss[mt] += __shfl_xor(ss[mt], d, 64);
                sq[mt] += __shfl_xor(sq[mt], d, 64);
                sd[mt] += __shfl_xor(sd[mt], d, 64);
            }
        }
        float4 *part = reinterpret_cast<float4 *>(lds);  // [2 wc][256 rows]
        if (lane < 16) {
#pragma unroll
            for (int mt = 0; mt < 8; ++mt)
                part[wc * GX_BM + wr * 128 + mt * 16 + lane] = make_float4(ss[mt], sq[mt], sd[mt], 0.f);
        }
        __syncthreads();
        if (m0e + tid < M) {  // 256 threads = the tile's 256 rows
            const float4 a = part[tid], b = part[GX_BM + tid];
            g.stats_out[(int64_t)(n0 / GX_BN) * g.stats_ld + m0e + tid] =
                make_float4(a.x + b.x, a.y + b.y, a.z + b.z, 0.f);
        }
    } else {
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
            const int row = row_l + mt * 16;
            if (row >= M) continue;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = acc[mt][2 * h + (e >> 2)][e & 3] + bias_v[h][e];
                if constexpr (EPI == EPI_BIAS_GELU) gelu_erf8(v);
                const int64_t o = (int64_t)row * g.ld_out + col_l + h * 32;
                if constexpr (EPI == EPI_BIAS_RESID) {
                    const bf16x8 rv = *reinterpret_cast<const bf16x8 *>(
                        static_cast<const bf16 *>(g.resid) + (int64_t)row * N + col_l + h * 32);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += (float)rv[e];
                }
                bf16x8 ov;
#pragma unroll
                for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
                *reinterpret_cast<bf16x8 *>(static_cast<bf16 *>(g.out) + o) = ov;
            }
        }
    }
    }  // epilogue
    // every wave is done with the LDS of this tile (parameters, partials) before the
    // next prologue overwrites it; the epilogue stores stay in flight (no vmcnt)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }  // tiles
}
#undef GX_BAR

// Opt-in (DI_GEMM2X=1): measured slower than the 256x256 8-phase kernel at every
// encoder shape (profiles/r01_gemm2x_check.log): the 256x128 tile's K loop reaches
// 775-1317 TF without its epilogue (the 256x256 one 1282-1333) and the second
// workgroup per CU did not hide the epilogue.
bool gemm2x_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("DI_GEMM2X");
        return e && e[0] == '1';
    }();
    return on;
}

bool gemm2x_ok(int epi, const GemmArgs &g) {
    const int64_t m_pad = ((int64_t)g.M + GX_BM - 1) / GX_BM * GX_BM;
    const bool epi_ok = epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_RESID ||
                        epi == EPI_FOLD || epi == EPI_FOLD_GELU || epi == EPI_RESID_STATS;
    return gemm2x_enabled() && epi_ok && g.N % GX_BN == 0 && g.K % 64 == 0 && g.K >= 128 &&
           g.a_rows >= m_pad;
}

// Columns summarised by one row-statistics partial of EPI_RESID_STATS.
int gemm_stats_cols() { return gemm2x_enabled() ? GX_BN : 256; }

void launch_gemm2x(int epi, const GemmArgs &g, hipStream_t s) {
    static_assert(2 * GX_LDS <= 160 * 1024, "two workgroups per CU");
    const int n_tiles = (g.N / GX_BN) * ((g.M + GX_BM - 1) / GX_BM);
    dim3 grid(std::min(n_tiles, 2 * n_cu()));
    switch (epi) {
#define GX_CASE(E)                                                                             \
    case E:                                                                                    \
        DI_HIP(hipFuncSetAttribute((const void *)gemm2x_kernel<E>,                             \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, GX_LDS));       \
        hipLaunchKernelGGL((gemm2x_kernel<E>), grid, dim3(GX_T), GX_LDS, s, g);                \
        break;
        GX_CASE(EPI_BIAS)
        GX_CASE(EPI_BIAS_GELU)
        GX_CASE(EPI_BIAS_RESID)
        GX_CASE(EPI_FOLD)
        GX_CASE(EPI_FOLD_GELU)
        GX_CASE(EPI_RESID_STATS)
#undef GX_CASE
        default:
            fail(DI_EINVAL, "bad GEMM epilogue");
    }
    check_launch("gemm2x");
}

}  // namespace di
