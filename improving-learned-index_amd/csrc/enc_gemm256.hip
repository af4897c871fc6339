// enc_gemm256.hip -- 256x256-tile bf16 MFMA GEMM, 8-phase pipelined K loop (gfx950).
//
// Same contract as enc_gemm.hip (C[M,N] = A[M,K] * B[N,K]^T + fused epilogue; the
// encoder's QKV / O / FFN1 / FFN2 projections, reference xlmr_original.py:70-75),
// for the shapes of the encoder hot loop: N % 256 == 0, K % 128 == 0, A readable up
// to round_up(M, 256) rows (the encoder's activation buffers carry that slack).
//
// Geometry: 512 threads = 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns output rows
// wr*128..+128 and columns wc*64..+64 = 8 x 4 fragments of 16x16 (128 accumulator
// VGPRs).  K step (one "K tile") = 64; two LDS buffers of one K tile each
// (A and B images 256 rows x 128 B, 64 KiB per buffer, 128 KiB total).
//
// Each K tile is split into four "half tiles" of 128 rows x 64 k (16 KiB, two
// global_load_lds_dwordx4 per thread), chosen so that each half is read by the
// fragment loads of exactly one phase:
//   A0 = tile rows {0-63, 128-191}   read in phase 1   (A fragments mt 0..3 of both wr)
//   A1 = tile rows {64-127, 192-255} read in phase 2   (mt 4..7)
//   B0 = columns {wc*64 + 0..31}      read in phase 1   (nt 0..1)
//   B1 = columns {wc*64 + 32..63}     read in phase 3   (nt 2..3)
// Four phases per K tile, 16 MFMAs (16x16x32) each; the wave keeps the whole K
// tile's fragments in registers (A 64 + B 32 VGPRs), so phase 4 reads nothing:
//   phase: 1 A0+B0 -> C[mt0-3][nt0-1]   2 A1 -> C[mt4-7][nt0-1]
//          3 B1    -> C[mt4-7][nt2-3]   4 --  -> C[mt0-3][nt2-3]
// One half tile is prefetched per phase into the region read in the phase before
// (write-after-read one phase later is safe because every wave retires its
// fragment reads, lgkmcnt(0), before the phase's first barrier).  Per iteration of
// 8 phases (K tiles 2i in buffer 0, 2i+1 in buffer 1):
//   ph1 buf1<-B1(2i+1)  ph2 buf0<-A0(2i+2)  ph3 buf0<-B0(2i+2)  ph4 buf0<-A1(2i+2)
//   ph5 buf0<-B1(2i+2)  ph6 buf1<-A0(2i+3)  ph7 buf1<-B0(2i+3)  ph8 buf1<-A1(2i+3)
// Counted waits (never 0 in steady state): phase 4 waits vmcnt(6) -- everything
// but the last three half tiles, i.e. all of K tile 2i+1 -- which phase 5 reads
// after the barrier; phase 8 likewise retires K tile 2i+2 for the next phase 1.
// The two wave groups (wr = 0, 1) run one barrier apart (group 1 executes one extra
// barrier up front, group 0 one at the end), so on every SIMD one wave issues
// MFMAs while the other loads fragments and issues its prefetch (ping-pong).
// Raw s_barrier (inline asm, a compiler memory fence but no vmcnt(0)) keeps the
// prefetch in flight across barriers; all LDS is one dynamic array.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int G2_T = 512;
constexpr int G2_TILE = 256;
constexpr int G2_BUF = 65536;                  // one K tile: A image 32 KiB + B image 32 KiB
// Epilogue parameters of the tile, staged by LDS-DMA with the prologue (their load
// latency then hides behind the K loop): 256 row params (float2) + up to four
// 256-column float vectors (bias or c, s or gamma, beta, head w*gamma).
constexpr int G2_PAR = 2 * G2_BUF;            // byte offset of the parameter area
constexpr int G2_PAR_ROW = 0, G2_PAR_C0 = 2048, G2_PAR_C1 = 3072, G2_PAR_C2 = 4096,
              G2_PAR_C3 = 5120;
constexpr int G2_LDS = 2 * G2_BUF + 6144;

// Epilogue row store (16 B per lane).  DI_NT_STORE (experiment builds only): the
// non-temporal form, so the streamed output does not evict the operand panels.
__device__ __forceinline__ void g2_store(bf16 *p, const bf16x8 &v) {
#ifdef DI_NT_STORE
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 u;
    __builtin_memcpy(&u, &v, 16);
    __builtin_nontemporal_store(u, reinterpret_cast<u32x4 *>(p));
#else
    *reinterpret_cast<bf16x8 *>(p) = v;
#endif
}

#define G2_BAR() asm volatile("s_barrier" ::: "memory")

template <int EPI, bool SPLIT>
__global__ void __launch_bounds__(G2_T) gemm256_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    // wave-uniform in SGPRs: the LDS-DMA destination (M0) is then scalar arithmetic
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;

    // tile order: XCD remap (bijective) + grouped GM x all-N order (speed only)
    const int n_tn = gridDim.x, n_tm = gridDim.y, n_tiles = n_tn * n_tm;
    int bid = blockIdx.y * gridDim.x + blockIdx.x;
    {
        const int q = n_tiles / 8, r = n_tiles % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    }
    const int GM = g.tune_gm > 0 ? g.tune_gm : 4;
    const int grp = bid / (GM * n_tn), first_m = grp * GM;
    const int gsz = min(GM, n_tm - first_m);
    const int in = bid % (GM * n_tn);
    const int M = g.M, N = g.N, K = g.K;
    // SPLIT: K tile t covers split columns [64 t, 64 t + 64) = the hi (k-step 0) and lo
    // (k-step 1) halves of logical k [32 t, 32 t + 32)
    const int nk = SPLIT ? K / 32 : K / 64;
    const int lda = SPLIT ? 2 * K : K, ldb = lda;
#define G2_AT(t) (t)
    const int m0 = (first_m + in % gsz) * G2_TILE;
    const int n0 = (in / gsz) * G2_TILE;

    // ---- staging sources (per lane) and LDS destinations (per wave) ----------
    // LDS row i (0..127) of a half tile = instruction j (0..1), wave, lane>>3:
    //   i = j*64 + wave*8 + (lane>>3);  slot lane&7 holds global chunk
    //   (lane&7) ^ (i&7)  (XOR swizzle on the source, rule 21).
    // A half h, row i -> tile row j*128 + h*64 + (i&63)
    // B half h, row i -> tile col j*128 + (wave>>2)*64 + h*32 + (wave&3)*8 + (lane>>3)
    const int chunk = ((lane & 7) ^ ((lane >> 3) & 7)) * 8;
    // opaque per tile: stops the compiler hoisting the per-(half, instruction)
    // source addresses of every tile out of the column-tile loop (register spills)
    const void *A_p = g.A, *B_p = g.B;
    int m0s = m0;
    asm volatile("" : "+s"(A_p), "+s"(B_p), "+s"(m0s));
    const bf16 *a_src = static_cast<const bf16 *>(A_p) +
                        (int64_t)(m0s + wave * 8 + (lane >> 3)) * lda + chunk;
    // B rows are stored permuted inside each 32-column group: LDS row q = sub*16 +
    // g*4 + r holds column g*8 + sub*4 + r, so that MFMA fragment nt (rows sub*16..+15
    // of half nt>>1) gives, in the C^T layout below, every lane 8 consecutive output
    // columns across the fragment pair (2h, 2h+1).
    const int qb = (wave & 3) * 8 + (lane >> 3);  // LDS row within the 32-column group
    const int b_col = ((qb >> 2) & 3) * 8 + (qb >> 4) * 4 + (qb & 3);
    const bf16 *b_src = static_cast<const bf16 *>(B_p) +
                        (int64_t)(n0 + (wave >> 2) * 64 + b_col) * ldb + chunk;
    const int64_t a_h = (int64_t)64 * lda, a_j = (int64_t)128 * lda;
    const int64_t b_h = (int64_t)32 * ldb, b_j = (int64_t)128 * ldb;
    typedef __attribute__((address_space(3))) void lds_void;
#define G2_STAGE_A(buf, h, t)                                                                  \
    do {                                                                                       \
        __builtin_amdgcn_global_load_lds((const void *)(a_src + (h) * a_h + G2_AT(t) * 64),    \
                                         (lds_void *)(lds + (buf) * G2_BUF + (h) * 16384 +     \
                                                      wave * 1024),                            \
                                         16, 0, 0);                                            \
        __builtin_amdgcn_global_load_lds((const void *)(a_src + (h) * a_h + a_j + G2_AT(t) * 64), \
                                         (lds_void *)(lds + (buf) * G2_BUF + (h) * 16384 +     \
                                                      8192 + wave * 1024),                     \
                                         16, 0, 0);                                            \
    } while (0)
#define G2_STAGE_B(buf, h, t)                                                                  \
    do {                                                                                       \
        __builtin_amdgcn_global_load_lds((const void *)(b_src + (h) * b_h + (t) * 64),         \
                                         (lds_void *)(lds + (buf) * G2_BUF + 32768 +           \
                                                      (h) * 16384 + wave * 1024),              \
                                         16, 0, 0);                                            \
        __builtin_amdgcn_global_load_lds((const void *)(b_src + (h) * b_h + b_j + (t) * 64),   \
                                         (lds_void *)(lds + (buf) * G2_BUF + 32768 +           \
                                                      (h) * 16384 + 8192 + wave * 1024),       \
                                         16, 0, 0);                                            \
    } while (0)

    // ---- fragment reads ------------------------------------------------------
    // A fragment mt of wave wr: LDS row (mt>>2)*128 + wr*64 + (mt&3)*16 + (lane&15);
    // B fragment nt of wave wc: LDS row (nt>>1)*128 + wc*32 + (nt&1)*16 + (lane&15).
    // k-step s reads chunk 4s + (lane>>4), stored at slot chunk ^ (lane&7).
    // Fragment reads are inline-asm ds_read_b128: the compiler then cannot see an
    // LDS read behind an LDS-DMA it cannot disambiguate (one LDS object) and does
    // not drain the prefetch with vmcnt(0); the phase's own lgkmcnt(0) + barrier
    // (and sched_barrier) order them before the MFMAs.
    const int xs = ((lane >> 4) ^ (lane & 7));
    const int c0 = xs << 4, c1 = (xs ^ 4) << 4;
    const uint32_t lds_base =
        (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char *)lds);
    const uint32_t a_rd = lds_base + (wr * 64 + (lane & 15)) * 128;
    const uint32_t b_rd = lds_base + 32768 + (wc * 32 + (lane & 15)) * 128;
    // [buffer][k-step] base addresses; the fragment offsets fit the 16-bit immediate
    const uint32_t ra[2][2] = {{a_rd + c0, a_rd + c1}, {a_rd + G2_BUF + c0, a_rd + G2_BUF + c1}};
    const uint32_t rb[2][2] = {{b_rd + c0, b_rd + c1}, {b_rd + G2_BUF + c0, b_rd + G2_BUF + c1}};
    uint4 af[8][2], bq[4][2];
#define G2_LD(dst, addr, off) \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(off))
#define G2_READ_A(buf, mlo)                                                                    \
    do {                                                                                       \
        _Pragma("unroll") for (int mm = 0; mm < 4; ++mm) {                                     \
            G2_LD(af[(mlo) + mm][0], ra[buf][0], ((mlo) >> 2) * 16384 + mm * 2048);            \
            G2_LD(af[(mlo) + mm][1], ra[buf][1], ((mlo) >> 2) * 16384 + mm * 2048);            \
        }                                                                                      \
    } while (0)
#define G2_READ_B(buf, nlo)                                                                    \
    do {                                                                                       \
        _Pragma("unroll") for (int nn = 0; nn < 2; ++nn) {                                     \
            G2_LD(bq[(nlo) + nn][0], rb[buf][0], ((nlo) >> 1) * 16384 + nn * 2048);            \
            G2_LD(bq[(nlo) + nn][1], rb[buf][1], ((nlo) >> 1) * 16384 + nn * 2048);            \
        }                                                                                      \
    } while (0)

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // (k-step pairs (sa, sb): (0, 0), (1, 1) plain; SPLIT (0, 0) hi*hi, (1, 0) A_lo B_hi,
    // (0, 1) A_hi B_lo)
#define G2_MFMA(mlo, nlo)                                                                      \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        __builtin_amdgcn_s_setprio(1);                                                         \
        _Pragma("unroll") for (int p = 0; p < (SPLIT ? 3 : 2); ++p)                            \
            _Pragma("unroll") for (int mm = 0; mm < 4; ++mm)                                   \
                _Pragma("unroll") for (int nn = 0; nn < 2; ++nn) {                             \
                    const int sa = SPLIT ? (p == 1) : p, sb = SPLIT ? (p == 2) : p;            \
                    bf16x8 av, bv;                                                             \
                    __builtin_memcpy(&av, &af[(mlo) + mm][sa], 16);                            \
                    __builtin_memcpy(&bv, &bq[(nlo) + nn][sb], 16);                            \
                    acc[(mlo) + mm][(nlo) + nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(     \
                        bv, av, acc[(mlo) + mm][(nlo) + nn], 0, 0, 0);                         \
                }                                                                              \
        __builtin_amdgcn_s_setprio(0);                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                     \
    } while (0)
#define G2_SYNC_READS() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

    // ---- epilogue parameters (wave 0; older than every stage load, so the
    // prologue's counted wait retires them) -----------------------------------------
    {
        constexpr bool FOLD = EPI == EPI_FOLD || EPI == EPI_FOLD_GELU;
        constexpr bool RS = EPI == EPI_RESID_STATS;
        if (wave == 0) {
            auto par1k = [&](const void *src, int off) {  // 1 KiB: 16 B per lane
                __builtin_amdgcn_global_load_lds(
                    (const void *)(static_cast<const char *>(src) + lane * 16),
                    (lds_void *)(lds + G2_PAR + off), 16, 0, 0);
            };
            par1k((FOLD ? g.col_c : g.bias) + n0, G2_PAR_C0);
            if (FOLD) par1k(g.col_s + n0, G2_PAR_C1);
            if (RS && g.row_ln) {
                par1k(g.res_gamma + n0, G2_PAR_C1);
                par1k(g.res_beta + n0, G2_PAR_C2);
            }
            if (RS && g.head_wg) par1k(g.head_wg + n0, G2_PAR_C3);
            if (FOLD || (RS && g.row_ln)) {
                int m0r = m0;
                asm volatile("" : "+s"(m0r));
                par1k(g.row_ln + m0r, G2_PAR_ROW);
                par1k(g.row_ln + m0r + 128, G2_PAR_ROW + 1024);
            }
        }
    }
    // ---- prologue: K tile 0 whole, K tile 1 minus its B1 half --------------------
    G2_STAGE_A(0, 0, 0);
    G2_STAGE_B(0, 0, 0);
    G2_STAGE_A(0, 1, 0);
    G2_STAGE_B(0, 1, 0);
    G2_STAGE_A(1, 0, 1);
    G2_STAGE_B(1, 0, 1);
    G2_STAGE_A(1, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    G2_BAR();
    if (wr == 1) G2_BAR();  // group 1 runs one barrier behind group 0

    for (int t = 0; t < nk; t += 2) {
        const bool more = t + 2 < nk;  // K tiles t+2, t+3 exist (nk is even)
        // phase 1: buffer 0, A0 + B0
        G2_READ_B(0, 0);
        G2_READ_A(0, 0);
        G2_STAGE_B(1, 1, t + 1);
        G2_SYNC_READS();
        G2_BAR();
        G2_MFMA(0, 0);
        G2_BAR();
        // phase 2: A1
        G2_READ_A(0, 4);
        if (more) G2_STAGE_A(0, 0, t + 2);
        G2_SYNC_READS();
        G2_BAR();
        G2_MFMA(4, 0);
        G2_BAR();
        // phase 3: B1
        G2_READ_B(0, 2);
        if (more) G2_STAGE_B(0, 0, t + 2);
        G2_SYNC_READS();
        G2_BAR();
        G2_MFMA(4, 2);
        G2_BAR();
        // phase 4: registers only; retire K tile t+1 for phase 5
        if (more) {
            G2_STAGE_A(0, 1, t + 2);
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        G2_BAR();
        G2_MFMA(0, 2);
        G2_BAR();
        // phase 5: buffer 1, A0 + B0
        G2_READ_B(1, 0);
        G2_READ_A(1, 0);
        if (more) G2_STAGE_B(0, 1, t + 2);
        G2_SYNC_READS();
        G2_BAR();
        G2_MFMA(0, 0);
        G2_BAR();
        // phase 6
        G2_READ_A(1, 4);
        if (more) G2_STAGE_A(1, 0, t + 3);
        G2_SYNC_READS();
        G2_BAR();
        G2_MFMA(4, 0);
        G2_BAR();
        // phase 7
        G2_READ_B(1, 2);
        if (more) G2_STAGE_B(1, 0, t + 3);
        G2_SYNC_READS();
        G2_BAR();
        G2_MFMA(4, 2);
        G2_BAR();
        // phase 8: retire K tile t+2 for the next phase 1
        if (more) {
            G2_STAGE_A(1, 1, t + 3);
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        }
        G2_BAR();
        G2_MFMA(0, 2);
        G2_BAR();
    }
    if (wr == 0) G2_BAR();  // re-align the two groups (every barrier is matched)
#undef G2_STAGE_A
#undef G2_STAGE_B
#undef G2_AT
#undef G2_LD
#undef G2_READ_A
#undef G2_READ_B
#undef G2_MFMA
#undef G2_SYNC_READS

    // ---- epilogue ------------------------------------------------------------
    if (g.ablate & 1) {  // profiling: main loop only (accumulators kept live)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
        return;
    }
    // C^T layout (the MFMA took the weight fragment as its first operand): lane l
    // holds, for A fragment mt and weight-column half h, output row
    //   m = m0 + wr*128 + mt*16 + (l & 15)
    // and the 8 consecutive columns n = n0 + wc*64 + h*32 + (l >> 4)*8 + e, e = 0..7,
    // in acc[mt][2h][0..3], acc[mt][2h+1][0..3].  Stores go straight from registers,
    // 16 B (bf16) / 32 B (f32) per lane, no LDS round trip and no barrier.
    int m0e = m0;  // opaque: keeps the per-row epilogue offsets out of the K loop
    asm volatile("" : "+s"(m0e));
    const int row_l = m0e + wr * 128 + (lane & 15);
    const int col_l = n0 + wc * 64 + (lane >> 4) * 8;
    // tile-local indices into the staged parameters
    const int prow = wr * 128 + (lane & 15);          // + mt * 16
    const int pcol = wc * 64 + (lane >> 4) * 8;        // + h * 32 + e
    auto par8 = [&](int off, int h, float (&v)[8]) {   // 8 column params from LDS
        const float4 a = *reinterpret_cast<const float4 *>(lds + G2_PAR + off + (pcol + h * 32) * 4);
        const float4 b = *reinterpret_cast<const float4 *>(lds + G2_PAR + off + (pcol + h * 32 + 4) * 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    };
    auto prow2 = [&](int mt) {  // (rstd, -rstd mean) of row prow + 16 mt
        return *reinterpret_cast<const float2 *>(lds + G2_PAR + G2_PAR_ROW + (prow + mt * 16) * 8);
    };
    float bias_v[2][8];  // (the folded epilogues carry their bias inside col_c)
    par8(G2_PAR_C0, 0, bias_v[0]);
    par8(G2_PAR_C0, 1, bias_v[1]);
    if constexpr (EPI == EPI_QKV) {
        if (n0 >= 2 * g.hidden) {  // V columns: transposed element stores into V^T
            typedef typename std::conditional<SPLIT, float, bf16>::type VT;  // SPLIT: f32 V^T
            VT *vt = static_cast<VT *>(g.out2) + (int64_t)(col_l - 2 * g.hidden) * g.ld_v;
#pragma unroll
            for (int mt = 0; mt < 8; ++mt) {
                const int row = row_l + mt * 16;
                if (row < M) {
                    const int vc = g.vcol[row];
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            vt[(int64_t)(h * 32 + e) * g.ld_v + vc] =
                                (VT)(acc[mt][2 * h + (e >> 2)][e & 3] + bias_v[h][e]);
                }
            }
            return;
        }
    }
    if constexpr (EPI == EPI_FOLD || EPI == EPI_FOLD_GELU) {
        // LN folded into this GEMM: y = r acc - r mu s + c  (per row r, mu; per column s, c)
        float ra[8], rb[8];
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
            const float2 p = prow2(mt);
            ra[mt] = p.x;
            rb[mt] = p.y;
        }
        float cs2[2][8];
        par8(G2_PAR_C1, 0, cs2[0]);
        par8(G2_PAR_C1, 1, cs2[1]);
        // row-major order: both 64-byte halves of a row's 128-byte segment are
        // stored by consecutive instructions (FFN1 -3.5%, QKV -2% against the
        // column-half-major order; same values)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float(&cs)[8] = cs2[h];
                const float(&cc)[8] = bias_v[h];
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
                g2_store(static_cast<bf16 *>(g.out) + (int64_t)row * g.ld_out + col_l + h * 32, ov);
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
        // row-major order, as in the folded epilogues (O -4%)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
            float gm[8], bt[8], wg[8];
            if (res_ln) {
                par8(G2_PAR_C1, h, gm);
                par8(G2_PAR_C2, h, bt);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    gm[e] = 1.f;
                    bt[e] = 0.f;
                }
            }
            if (g.head_wg) {
                par8(G2_PAR_C3, h, wg);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) wg[e] = 0.f;
            }
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
                g2_store(static_cast<bf16 *>(g.out) + (int64_t)row * g.ld_out + col_l + h * 32, ov);
            }
        }
        // partials: the 4 lane groups (lanes l, l^16, l^32, l^48 share a row), then
        // the 4 wc waves through LDS (the staging buffers are free), fixed order
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
            for (int d = 16; d <= 32; d <<= 1) {
                ss[mt] += __shfl_xor(ss[mt], d, 64);
                sq[mt] += __shfl_xor(sq[mt], d, 64);
                sd[mt] += __shfl_xor(sd[mt], d, 64);
            }
        }
        float4 *part = reinterpret_cast<float4 *>(lds);  // [4 wc][256 rows]
        if (lane < 16) {
#pragma unroll
            for (int mt = 0; mt < 8; ++mt)
                part[wc * G2_TILE + wr * 128 + mt * 16 + lane] = make_float4(ss[mt], sq[mt], sd[mt], 0.f);
        }
        __syncthreads();
        if (tid < G2_TILE && m0e + tid < M) {
            float4 t = part[tid];
#pragma unroll
            for (int w = 1; w < 4; ++w) {
                const float4 u = part[w * G2_TILE + tid];
                t.x += u.x;
                t.y += u.y;
                t.z += u.z;
            }
            g.stats_out[(int64_t)(n0 / G2_TILE) * g.stats_ld + m0e + tid] = t;
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
            if (EPI == EPI_BIAS_GELU && !(g.ablate & 2)) gelu_erf8(v);  // ablate 2: no GELU (profiling)
            const int64_t o = (int64_t)row * g.ld_out + col_l + h * 32;
            if constexpr (EPI == EPI_BIAS_RESID) {
                if constexpr (SPLIT) {  // split residual rows
                    const bf16 *rp = static_cast<const bf16 *>(g.resid) + (int64_t)row * 2 * N +
                                     split_col(col_l + h * 32);
                    const bf16x8 rh = *reinterpret_cast<const bf16x8 *>(rp);
                    const bf16x8 rl = *reinterpret_cast<const bf16x8 *>(rp + 32);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += (float)rh[e] + (float)rl[e];
                } else {
                    const bf16x8 rv = *reinterpret_cast<const bf16x8 *>(
                        static_cast<const bf16 *>(g.resid) + (int64_t)row * N + col_l + h * 32);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += (float)rv[e];
                }
            }
            if constexpr (SPLIT) {
                if constexpr (EPI == EPI_QKV || EPI == EPI_BIAS_RESID) {  // f32 rows
                    float *op = static_cast<float *>(g.out) + o;
                    *reinterpret_cast<float4 *>(op) = make_float4(v[0], v[1], v[2], v[3]);
                    *reinterpret_cast<float4 *>(op + 4) = make_float4(v[4], v[5], v[6], v[7]);
                } else {  // split rows (ld_out = 2N): 8 columns of one 32-column chunk
                    bf16x8 hv, lv;
#pragma unroll
                    for (int e = 0; e < 8; ++e) hv[e] = split_hi(v[e]), lv[e] = split_lo(v[e]);
                    bf16 *op = static_cast<bf16 *>(g.out) + (int64_t)row * g.ld_out +
                               split_col(col_l + h * 32);
                    g2_store(op, hv);
                    g2_store(op + 32, lv);
                }
                continue;
            }
            bf16x8 ov;
#pragma unroll
            for (int e = 0; e < 8; ++e) ov[e] = (bf16)v[e];
            if (g.ablate & 4) {  // profiling: no stores (values kept live)
                uint4 u;
                __builtin_memcpy(&u, &ov, 16);
                asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w));
            } else {
                g2_store(static_cast<bf16 *>(g.out) + o, ov);
            }
        }
    }
    }  // generic epilogues
}
#undef G2_BAR

// Shapes the 8-phase kernel takes; everything else goes to the 128x128 kernel.
bool gemm256_ok(int epi, const GemmArgs &g) {
    const int64_t m_pad = ((int64_t)g.M + G2_TILE - 1) / G2_TILE * G2_TILE;
    if (g.split && !(epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_RESID ||
                     epi == EPI_QKV))
        return false;
    // (SPLIT: K tiles of 32 logical k, K % 64 == 0 keeps their count even)
    return g.N % G2_TILE == 0 && g.K % (g.split ? 64 : 128) == 0 && g.K >= 128 &&
           g.a_rows >= m_pad &&
           (epi != EPI_QKV || (2 * g.hidden) % G2_TILE == 0);
}

// column width of one partial-statistics slot of the residual epilogues (the
// encoder sizes its statistics buffers by it)
int gemm_stats_cols() { return G2_TILE; }

void launch_gemm256(int epi, const GemmArgs &g, hipStream_t s) {
    static_assert(G2_LDS <= 160 * 1024, "LDS");
    dim3 grid(g.N / G2_TILE, (g.M + G2_TILE - 1) / G2_TILE);
    DI_REQUIRE(gemm256_ok(epi, g), DI_EINVAL, "gemm256: unsupported shape / epilogue");
    if (g.split) {
        switch (epi) {
#define G2_SCASE(E)                                                                            \
    case E:                                                                                    \
        DI_HIP(hipFuncSetAttribute((const void *)gemm256_kernel<E, true>,                      \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS));       \
        hipLaunchKernelGGL((gemm256_kernel<E, true>), grid, dim3(G2_T), G2_LDS, s, g);         \
        break;
            G2_SCASE(EPI_BIAS)
            G2_SCASE(EPI_BIAS_GELU)
            G2_SCASE(EPI_BIAS_RESID)
            G2_SCASE(EPI_QKV)
#undef G2_SCASE
            default:
                fail(DI_EINVAL, "bad split GEMM epilogue");
        }
        check_launch("gemm256_split");
        return;
    }
    switch (epi) {
#define G2_CASE(E)                                                                             \
    case E:                                                                                    \
        DI_HIP(hipFuncSetAttribute((const void *)gemm256_kernel<E, false>,                     \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS));       \
        hipLaunchKernelGGL((gemm256_kernel<E, false>), grid, dim3(G2_T), G2_LDS, s, g);        \
        break;
        G2_CASE(EPI_BIAS)
        G2_CASE(EPI_BIAS_GELU)
        G2_CASE(EPI_BIAS_RESID)
        G2_CASE(EPI_QKV)
        G2_CASE(EPI_FOLD)
        G2_CASE(EPI_FOLD_GELU)
        G2_CASE(EPI_RESID_STATS)
#undef G2_CASE
        default:
            fail(DI_EINVAL, "bad GEMM epilogue");
    }
    check_launch("gemm256");
}

}  // namespace di
