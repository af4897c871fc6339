// enc_gemm256p.hip -- persistent form of the 256x256 8-phase bf16 GEMM (gfx950).
//
// Same tile, K loop and results as enc_gemm256.hip (bit-identical: the same MFMA
// sequence per accumulator and the same epilogue arithmetic); what changes is what
// happens BETWEEN tiles.  In the one-tile-per-workgroup kernel every tile ends in
// an epilogue (parameter arithmetic, GELU, 128 KiB of stores) with the matrix
// cores idle, and the next workgroup then waits for its prologue loads.  Here one
// workgroup per CU walks a sequence of tiles, and as soon as the last K-tile
// fragments are read it issues the NEXT tile's prologue (its epilogue parameters
// into the other parameter slot and K tiles 0-1 into the two stage buffers) --
// before the current tile's epilogue.  Stores are fire-and-forget, so they drain
// while the next tile's K loop runs; the only coupling is the in-order vector
// memory counter, and the next tile's first wait counts the epilogue's memory
// operations (vmcnt(6 + S), S = memory ops of a full tile's epilogue) so that it
// retires the prologue without waiting for those stores.
//
// Tile order: the workgroups of XCD x (blockIdx % 8) walk a contiguous range of
// the grouped (GM M-tiles x all N-tiles) order, so the 32 CUs of an XCD share A
// rows in their L2 -- the same placement the one-shot kernel gets from its
// blockIdx remap.
//
// LDS: two stage buffers (128 KiB) + two 6 KiB parameter slots + 16 KiB of
// row-statistics partials (EPI_RESID_STATS) = 156 KiB, one workgroup per CU.
// Epilogue LDS accesses are inline-asm ds_read/ds_write with explicit lgkmcnt
// waits: a C++ LDS access after an LDS-DMA makes the compiler drain vmcnt, which
// would retire the in-flight prologue (and every store) at the epilogue's start.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int GP_T = 512;
constexpr int GP_TILE = 256;
constexpr int GP_BUF = 65536;
constexpr int GP_PAR = 2 * GP_BUF;  // parameter slots
constexpr int GP_SLOT = 6144;
constexpr int GP_PAR_ROW = 0, GP_PAR_C0 = 2048, GP_PAR_C1 = 3072, GP_PAR_C2 = 4096,
              GP_PAR_C3 = 5120;
constexpr int GP_PART = GP_PAR + 2 * GP_SLOT;  // [4 wc][256 rows] f32x4
constexpr int GP_LDS = GP_PART + 16384;

// memory operations a full tile's epilogue issues after the next tile's prologue
template <int EPI>
constexpr int gp_epi_ops() {
    return (EPI == EPI_BIAS_RESID || EPI == EPI_RESID_STATS) ? 24 : 16;
}

#define GP_BAR() asm volatile("s_barrier" ::: "memory")
#define GP_FENCE()                            \
    do {                                      \
        __builtin_amdgcn_sched_barrier(0);    \
        asm volatile("" ::: "memory");        \
    } while (0)

template <int EPI>
__global__ void __launch_bounds__(GP_T) gemm256p_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int M = g.M, N = g.N, K = g.K, nk = K / 64;
    constexpr bool FOLD = EPI == EPI_FOLD || EPI == EPI_FOLD_GELU;
    constexpr bool RS = EPI == EPI_RESID_STATS;
    constexpr bool RES = EPI == EPI_BIAS_RESID || RS;

    // ---- this workgroup's tiles ---------------------------------------------------
    const int n_tn = N / GP_TILE, n_tm = (M + GP_TILE - 1) / GP_TILE, n_tiles = n_tn * n_tm;
    const int G = gridDim.x;
    int first, step, count;
    if (G % 8 == 0) {
        const int x = blockIdx.x % 8, l = blockIdx.x / 8, P = G / 8;
        const int q = n_tiles / 8, r = n_tiles % 8;
        const int start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
        const int cnt = q + (x < r ? 1 : 0);
        first = start + l;
        step = P;
        count = l < cnt ? (cnt - l + P - 1) / P : 0;
    } else {
        first = blockIdx.x;
        step = G;
        count = (n_tiles - (int)blockIdx.x + G - 1) / G;
    }
    if (count <= 0) return;
    // optional first-tile delay of every other CU of an XCD (speed only), so that
    // the two halves' epilogue store bursts alternate
    if (g.stagger > 0 && ((blockIdx.x >> 3) & 1)) {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < (uint64_t)g.stagger) __builtin_amdgcn_s_sleep(8);
    }
    const int GM = g.tune_gm > 0 ? g.tune_gm : 4;
    auto tile_mn = [&](int bid, int &m0, int &n0) {
        const int grp = bid / (GM * n_tn), first_m = grp * GM;
        const int gsz = min(GM, n_tm - first_m);
        const int in = bid % (GM * n_tn);
        m0 = (first_m + in % gsz) * GP_TILE;
        n0 = (in / gsz) * GP_TILE;
    };

    // ---- staging (enc_gemm256.hip's half-tile layout) -------------------------------
    const int chunk = ((lane & 7) ^ ((lane >> 3) & 7)) * 8;
    const int qb = (wave & 3) * 8 + (lane >> 3);
    const int b_col = ((qb >> 2) & 3) * 8 + (qb >> 4) * 4 + (qb & 3);
    const int64_t a_h = (int64_t)64 * K, a_j = (int64_t)128 * K;
    const int64_t b_h = (int64_t)32 * K, b_j = (int64_t)128 * K;
    const bf16 *a_src = nullptr, *b_src = nullptr;
    auto set_src = [&](int m0, int n0) {
        const void *A_p = g.A, *B_p = g.B;
        asm volatile("" : "+s"(A_p), "+s"(B_p), "+s"(m0), "+s"(n0));
        a_src = static_cast<const bf16 *>(A_p) + (int64_t)(m0 + wave * 8 + (lane >> 3)) * K + chunk;
        b_src = static_cast<const bf16 *>(B_p) + (int64_t)(n0 + (wave >> 2) * 64 + b_col) * K + chunk;
    };
    typedef __attribute__((address_space(3))) void lds_void;
#define GP_STAGE_A(buf, h, t)                                                                  \
    do {                                                                                       \
        __builtin_amdgcn_global_load_lds((const void *)(a_src + (h) * a_h + (t) * 64),         \
                                         (lds_void *)(lds + (buf) * GP_BUF + (h) * 16384 +     \
                                                      wave * 1024),                            \
                                         16, 0, 0);                                            \
        __builtin_amdgcn_global_load_lds((const void *)(a_src + (h) * a_h + a_j + (t) * 64),   \
                                         (lds_void *)(lds + (buf) * GP_BUF + (h) * 16384 +     \
                                                      8192 + wave * 1024),                     \
                                         16, 0, 0);                                            \
    } while (0)
#define GP_STAGE_B(buf, h, t)                                                                  \
    do {                                                                                       \
        __builtin_amdgcn_global_load_lds((const void *)(b_src + (h) * b_h + (t) * 64),         \
                                         (lds_void *)(lds + (buf) * GP_BUF + 32768 +           \
                                                      (h) * 16384 + wave * 1024),              \
                                         16, 0, 0);                                            \
        __builtin_amdgcn_global_load_lds((const void *)(b_src + (h) * b_h + b_j + (t) * 64),   \
                                         (lds_void *)(lds + (buf) * GP_BUF + 32768 +           \
                                                      (h) * 16384 + 8192 + wave * 1024),       \
                                         16, 0, 0);                                            \
    } while (0)
    // epilogue parameters of tile (m0, n0) into slot `slot` (wave 0, older than the
    // stage loads, so the prologue's counted wait retires them)
    auto stage_params = [&](int slot, int m0, int n0) {
        if (wave != 0) return;
        unsigned char *dst = lds + GP_PAR + slot * GP_SLOT;
        auto par1k = [&](const void *src, int off) {
            __builtin_amdgcn_global_load_lds(
                (const void *)(static_cast<const char *>(src) + lane * 16),
                (lds_void *)(dst + off), 16, 0, 0);
        };
        par1k((FOLD ? g.col_c : g.bias) + n0, GP_PAR_C0);
        if (FOLD) par1k(g.col_s + n0, GP_PAR_C1);
        if (RS && g.row_ln) {
            par1k(g.res_gamma + n0, GP_PAR_C1);
            par1k(g.res_beta + n0, GP_PAR_C2);
        }
        if (RS && g.head_wg) par1k(g.head_wg + n0, GP_PAR_C3);
        if (FOLD || (RS && g.row_ln)) {
            par1k(g.row_ln + m0, GP_PAR_ROW);
            par1k(g.row_ln + m0 + 128, GP_PAR_ROW + 1024);
        }
    };
    // K tiles 0 and 1 whole (the one-shot kernel leaves K tile 1's B1 half to phase 1:
    // here that load would be younger than the previous tile's stores, and phase 4's
    // wait for it would wait for them too)
    auto prologue = [&]() {
        GP_STAGE_A(0, 0, 0);
        GP_STAGE_B(0, 0, 0);
        GP_STAGE_A(0, 1, 0);
        GP_STAGE_B(0, 1, 0);
        GP_STAGE_A(1, 0, 1);
        GP_STAGE_B(1, 0, 1);
        GP_STAGE_A(1, 1, 1);
        GP_STAGE_B(1, 1, 1);
    };

    // ---- fragment reads (enc_gemm256.hip) ---------------------------------------------
    const int xs = ((lane >> 4) ^ (lane & 7));
    const int c0 = xs << 4, c1 = (xs ^ 4) << 4;
    const uint32_t lds_base =
        (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char *)lds);
    const uint32_t a_rd = lds_base + (wr * 64 + (lane & 15)) * 128;
    const uint32_t b_rd = lds_base + 32768 + (wc * 32 + (lane & 15)) * 128;
    const uint32_t ra[2][2] = {{a_rd + c0, a_rd + c1}, {a_rd + GP_BUF + c0, a_rd + GP_BUF + c1}};
    const uint32_t rb[2][2] = {{b_rd + c0, b_rd + c1}, {b_rd + GP_BUF + c0, b_rd + GP_BUF + c1}};
    uint4 af[8][2], bq[4][2];
#define GP_LD(dst, addr, off) \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(off))
#define GP_READ_A(buf, mlo)                                                                    \
    do {                                                                                       \
        _Pragma("unroll") for (int mm = 0; mm < 4; ++mm) {                                     \
            GP_LD(af[(mlo) + mm][0], ra[buf][0], ((mlo) >> 2) * 16384 + mm * 2048);            \
            GP_LD(af[(mlo) + mm][1], ra[buf][1], ((mlo) >> 2) * 16384 + mm * 2048);            \
        }                                                                                      \
    } while (0)
#define GP_READ_B(buf, nlo)                                                                    \
    do {                                                                                       \
        _Pragma("unroll") for (int nn = 0; nn < 2; ++nn) {                                     \
            GP_LD(bq[(nlo) + nn][0], rb[buf][0], ((nlo) >> 1) * 16384 + nn * 2048);            \
            GP_LD(bq[(nlo) + nn][1], rb[buf][1], ((nlo) >> 1) * 16384 + nn * 2048);            \
        }                                                                                      \
    } while (0)
    f32x4 acc[8][4];
#define GP_MFMA(mlo, nlo)                                                                      \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        __builtin_amdgcn_s_setprio(1);                                                         \
        _Pragma("unroll") for (int s = 0; s < 2; ++s)                                          \
            _Pragma("unroll") for (int mm = 0; mm < 4; ++mm)                                   \
                _Pragma("unroll") for (int nn = 0; nn < 2; ++nn) {                             \
                    bf16x8 av, bv;                                                             \
                    __builtin_memcpy(&av, &af[(mlo) + mm][s], 16);                             \
                    __builtin_memcpy(&bv, &bq[(nlo) + nn][s], 16);                             \
                    acc[(mlo) + mm][(nlo) + nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(     \
                        bv, av, acc[(mlo) + mm][(nlo) + nn], 0, 0, 0);                         \
                }                                                                              \
        __builtin_amdgcn_s_setprio(0);                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                     \
    } while (0)
#define GP_SYNC_READS() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

    int bid = first;
    int m0, n0;
    tile_mn(bid, m0, n0);
    set_src(m0, n0);
    stage_params(0, m0, n0);
    prologue();
    int slot = 0;
    bool after_full = false;  // the ops between this tile's prologue and now are a
                              // full epilogue's gp_epi_ops<EPI>()
    for (int i = 0;;) {
        // K tile 0 landed: all but the 8 youngest prologue ops (+ the epilogue's)
        if (after_full) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + gp_epi_ops<EPI>()) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        GP_BAR();
        if (wr == 1) GP_BAR();  // group 1 runs one barrier behind group 0
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

        for (int t = 0; t < nk; t += 2) {
            const bool more = t + 2 < nk;
            GP_READ_B(0, 0);
            GP_READ_A(0, 0);
            if (t > 0) GP_STAGE_B(1, 1, t + 1);
            GP_SYNC_READS();
            GP_BAR();
            GP_MFMA(0, 0);
            GP_BAR();
            GP_READ_A(0, 4);
            if (more) GP_STAGE_A(0, 0, t + 2);
            GP_SYNC_READS();
            GP_BAR();
            GP_MFMA(4, 0);
            GP_BAR();
            GP_READ_B(0, 2);
            if (more) GP_STAGE_B(0, 0, t + 2);
            GP_SYNC_READS();
            GP_BAR();
            GP_MFMA(4, 2);
            GP_BAR();
            if (more) {
                GP_STAGE_A(0, 1, t + 2);
                // K tile t+1 landed (t = 0: it came with the prologue, older than the
                // previous epilogue's ops, which may stay in flight)
                if (t == 0 && after_full)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + gp_epi_ops<EPI>()) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            GP_BAR();
            GP_MFMA(0, 2);
            GP_BAR();
            GP_READ_B(1, 0);
            GP_READ_A(1, 0);
            if (more) GP_STAGE_B(0, 1, t + 2);
            GP_SYNC_READS();
            GP_BAR();
            GP_MFMA(0, 0);
            GP_BAR();
            GP_READ_A(1, 4);
            if (more) GP_STAGE_A(1, 0, t + 3);
            GP_SYNC_READS();
            GP_BAR();
            GP_MFMA(4, 0);
            GP_BAR();
            GP_READ_B(1, 2);
            if (more) GP_STAGE_B(1, 0, t + 3);
            GP_SYNC_READS();
            GP_BAR();
            GP_MFMA(4, 2);
            GP_BAR();
            if (more) {
                GP_STAGE_A(1, 1, t + 3);
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            }
            GP_BAR();
            GP_MFMA(0, 2);
            GP_BAR();
        }
        if (wr == 0) GP_BAR();  // re-aligned: every wave is past its last fragment read

        const int cm0 = m0, cn0 = n0, cslot = slot;
        const bool full = cm0 + GP_TILE <= M && g.ablate == 0;
        const bool has_next = ++i < count;
        const int row_l = cm0 + wr * 128 + (lane & 15);
        const int col_l = cn0 + wc * 64 + (lane >> 4) * 8;

        // residual rows of column half 0, issued before the prefetch so that waiting
        // for them does not wait for it (rows clamped: unconditional loads)
        uint4 rv[8];
        if constexpr (RES) {
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
                const int row = min(row_l + mt * 16, M - 1);
                rv[mt] = *reinterpret_cast<const uint4 *>(static_cast<const bf16 *>(g.resid) +
                                                          (int64_t)row * N + col_l);
            }
        }
        GP_FENCE();
        if (has_next) {
            bid += step;
            tile_mn(bid, m0, n0);
            set_src(m0, n0);
            stage_params(slot ^ 1, m0, n0);
            prologue();
            slot ^= 1;
        }
        GP_FENCE();
        after_full = full;

        if (g.ablate & 1) {  // profiling: main loop only (accumulators kept live)
#pragma unroll
            for (int a = 0; a < 8; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) asm volatile("" ::"v"(acc[a][b]));
            if (!has_next) break;
            continue;
        }

        // ---- epilogue of tile (cm0, cn0) -------------------------------------------------
        // lane geometry recomputed here from an opaque lane id (kept out of the K loop)
        int el = lane;
        asm volatile("" : "+v"(el));
        const uint32_t par = lds_base + GP_PAR + cslot * GP_SLOT;
        const uint32_t pcol = par + (wc * 64 + (el >> 4) * 8) * 4;
        const uint32_t prow = par + GP_PAR_ROW + (wr * 128 + (el & 15)) * 8;
        float ra8[8], rb8[8];
        if constexpr (FOLD || RS) {
            const bool rows = FOLD || g.row_ln != nullptr;
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
                ra8[mt] = 1.f;
                rb8[mt] = 0.f;
            }
            if (rows) {
                uint2 pr[8];
#pragma unroll
                for (int mt = 0; mt < 8; ++mt)
                    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(pr[mt]) : "v"(prow), "i"(mt * 128));
                GP_SYNC_READS();
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) asm volatile("" : "+v"(pr[mt].x), "+v"(pr[mt].y));
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    ra8[mt] = __uint_as_float(pr[mt].x);
                    rb8[mt] = __uint_as_float(pr[mt].y);
                }
            }
        }
        // 8 column parameters of half h at byte offset `off` of the slot
#define GP_PAR8(v, off, h)                                                                     \
    do {                                                                                       \
        uint4 p0_, p1_;                                                                        \
        GP_LD(p0_, pcol, (off) + (h) * 128);                                                   \
        GP_LD(p1_, pcol, (off) + (h) * 128 + 16);                                              \
        GP_SYNC_READS();                                                                       \
        asm volatile("" : "+v"(p0_.x), "+v"(p0_.y), "+v"(p0_.z), "+v"(p0_.w), "+v"(p1_.x),      \
                     "+v"(p1_.y), "+v"(p1_.z), "+v"(p1_.w)); /* results exist after the wait */ \
        as8(p0_, p1_, v);                                                                      \
    } while (0)
        auto as8 = [](const uint4 &a, const uint4 &b, float (&v)[8]) {
            v[0] = __uint_as_float(a.x); v[1] = __uint_as_float(a.y);
            v[2] = __uint_as_float(a.z); v[3] = __uint_as_float(a.w);
            v[4] = __uint_as_float(b.x); v[5] = __uint_as_float(b.y);
            v[6] = __uint_as_float(b.z); v[7] = __uint_as_float(b.w);
        };
        auto store8 = [&](int row, int h, const bf16x8 &ov) {
            if (g.ablate & 4) {
                uint4 u;
                __builtin_memcpy(&u, &ov, 16);
                asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w));
            } else {
                *reinterpret_cast<bf16x8 *>(static_cast<bf16 *>(g.out) + (int64_t)row * g.ld_out +
                                            col_l + h * 32) = ov;
            }
        };

        if constexpr (!RES) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float cc[8], cs[8];
                GP_PAR8(cc, GP_PAR_C0, h);
                if constexpr (FOLD) GP_PAR8(cs, GP_PAR_C1, h);
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    const int row = row_l + mt * 16;
                    if (row >= M) continue;
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float a = acc[mt][2 * h + (e >> 2)][e & 3];
                        if constexpr (FOLD)
                            v[e] = fmaf(ra8[mt], a, fmaf(rb8[mt], cs[e], cc[e]));
                        else
                            v[e] = a + cc[e];
                    }
                    if constexpr (EPI == EPI_FOLD_GELU || EPI == EPI_BIAS_GELU)
                        if (!(g.ablate & 2)) gelu_erf8(v);
                    bf16x8 ov;
#pragma unroll
                    for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
                    store8(row, h, ov);
                }
            }
        } else {
            // EPI_BIAS_RESID: out = acc + bias + resid (one rounding).
            // EPI_RESID_STATS: out = acc + bias + LN(resid) (normalised from its row
            // statistics, or plain), plus this tile's partial (sum, sumsq, head dot)
            // of the rounded out per row.
            float ss[8], sq[8], sd[8];
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) ss[mt] = sq[mt] = sd[mt] = 0.f;
            const bool res_ln = RS && g.row_ln != nullptr;
            const bool head = RS && g.head_wg != nullptr;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (h == 1) {
                    GP_FENCE();
#pragma unroll
                    for (int mt = 0; mt < 8; ++mt) {
                        const int row = min(row_l + mt * 16, M - 1);
                        rv[mt] = *reinterpret_cast<const uint4 *>(
                            static_cast<const bf16 *>(g.resid) + (int64_t)row * N + col_l + 32);
                    }
                }
                float bb[8], gm[8], bt[8], wg[8];
                GP_PAR8(bb, GP_PAR_C0, h);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    gm[e] = 1.f;
                    bt[e] = 0.f;
                    wg[e] = 0.f;
                }
                if constexpr (RS) {
                    if (res_ln) {
                        GP_PAR8(gm, GP_PAR_C1, h);
                        GP_PAR8(bt, GP_PAR_C2, h);
                    }
                    if (head) GP_PAR8(wg, GP_PAR_C3, h);
                }
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    const int row = row_l + mt * 16;
                    if (row >= M) continue;
                    bf16x8 rvv;
                    __builtin_memcpy(&rvv, &rv[mt], 16);
                    bf16x8 ov;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float a = acc[mt][2 * h + (e >> 2)][e & 3];
                        if constexpr (RS) {
                            const float res = fmaf(gm[e], fmaf(ra8[mt], (float)rvv[e], rb8[mt]), bt[e]);
                            ov[e] = (bf16)(a + bb[e] + res);
                            const float yb = (float)ov[e];
                            ss[mt] += yb;
                            sq[mt] = fmaf(yb, yb, sq[mt]);
                            sd[mt] = fmaf(yb, wg[e], sd[mt]);
                        } else {
                            ov[e] = (bf16)((a + bb[e]) + (float)rvv[e]);
                        }
                    }
                    store8(row, h, ov);
                }
            }
            if constexpr (RS) {
                // partials: the 4 lane groups sharing a row, then the 4 wc waves through
                // LDS in a fixed order (as enc_gemm256.hip)
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
                    for (int d = 16; d <= 32; d <<= 1) {
                        ss[mt] += __shfl_xor(ss[mt], d, 64);
                        sq[mt] += __shfl_xor(sq[mt], d, 64);
                        sd[mt] += __shfl_xor(sd[mt], d, 64);
                    }
                }
                const uint32_t part_wr = lds_base + GP_PART + (wc * GP_TILE + wr * 128 + el) * 16;
                const uint32_t part_rd = lds_base + GP_PART + (wave * 64 + el) * 16;
                if (el < 16) {
#pragma unroll
                    for (int mt = 0; mt < 8; ++mt) {
                        const f32x4 v = f32x4{ss[mt], sq[mt], sd[mt], 0.f};
                        asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(part_wr), "v"(v),
                                     "i"(mt * 256)
                                     : "memory");
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                if (tid < GP_TILE) {
                    f32x4 p[4];
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(p[w]) : "v"(part_rd), "i"(w * 4096));
                    GP_SYNC_READS();
#pragma unroll
                    for (int w = 0; w < 4; ++w) asm volatile("" : "+v"(p[w]));
                    float4 t = make_float4(p[0].x, p[0].y, p[0].z, 0.f);
#pragma unroll
                    for (int w = 1; w < 4; ++w) {
                        t.x += p[w].x;
                        t.y += p[w].y;
                        t.z += p[w].z;
                    }
                    const int r = wave * 64 + el;
                    if (cm0 + r < M && !(g.ablate & 4))
                        g.stats_out[(int64_t)(cn0 / GP_TILE) * g.stats_ld + cm0 + r] = t;
                }
            }
        }
        if (!has_next) break;
    }
#undef GP_STAGE_A
#undef GP_STAGE_B
#undef GP_LD
#undef GP_READ_A
#undef GP_READ_B
#undef GP_MFMA
#undef GP_SYNC_READS
#undef GP_PAR8
}
#undef GP_BAR
#undef GP_FENCE

static bool gemm256p_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("DI_GEMM_PERSIST");
        return e && e[0] == '1';
    }();
    return on;
}

// The persistent kernel takes the shapes of gemm256_ok for these epilogues.
bool gemm256p_ok(int epi) {
    return gemm256p_enabled() && (epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_RESID ||
                                  epi == EPI_FOLD || epi == EPI_FOLD_GELU || epi == EPI_RESID_STATS);
}

void launch_gemm256p(int epi, const GemmArgs &g, hipStream_t s) {
    static_assert(GP_LDS <= 160 * 1024, "LDS");
    const int n_tiles = (g.N / GP_TILE) * ((g.M + GP_TILE - 1) / GP_TILE);
    int grid = n_tiles < n_cu() ? n_tiles : n_cu();
    if (grid >= 8) grid &= ~7;  // whole XCDs: the XCD-contiguous tile ranges
    switch (epi) {
#define GP_CASE(E)                                                                             \
    case E:                                                                                    \
        DI_HIP(hipFuncSetAttribute((const void *)gemm256p_kernel<E>,                           \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, GP_LDS));       \
        hipLaunchKernelGGL((gemm256p_kernel<E>), dim3(grid), dim3(GP_T), GP_LDS, s, g);        \
        break;
        GP_CASE(EPI_BIAS)
        GP_CASE(EPI_BIAS_GELU)
        GP_CASE(EPI_BIAS_RESID)
        GP_CASE(EPI_FOLD)
        GP_CASE(EPI_FOLD_GELU)
        GP_CASE(EPI_RESID_STATS)
#undef GP_CASE
        default:
            fail(DI_EINVAL, "bad GEMM epilogue");
    }
    check_launch("gemm256p");
}

}  // namespace di
