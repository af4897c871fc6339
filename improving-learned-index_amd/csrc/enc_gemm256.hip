// enc_gemm256.hip -- 256x256-tile bf16 MFMA GEMM, 8-phase pipelined K loop, persistent
// over tiles with the next tile's prologue in flight during the epilogue (gfx950).
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
//   (i = 0: B1(1) comes with the tile's prologue instead)
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

#include <algorithm>
#include <type_traits>

#include "di_common.h"
#include "enc_common.h"

namespace di {

constexpr int G2_T = 512;
constexpr int G2_TILE = 256;
constexpr int G2_BUF = 65536;                  // one K tile: A image 32 KiB + B image 32 KiB
// Epilogue parameters of a tile, staged by LDS-DMA with the tile's prologue (their load
// latency then hides behind the K loop): 256 row params (float2) + up to four
// 256-column float vectors (bias or c, s or gamma, beta, head w*gamma).  Two slots:
// the next tile's parameters arrive while the current tile's epilogue reads its own.
constexpr int G2_PAR = 2 * G2_BUF;            // byte offset of the parameter slots
constexpr int G2_PARSZ = 6144;
constexpr int G2_PAR_ROW = 0, G2_PAR_C0 = 2048, G2_PAR_C1 = 3072, G2_PAR_C2 = 4096,
              G2_PAR_C3 = 5120;
constexpr int G2_LDS = 2 * G2_BUF + 2 * G2_PARSZ;

// Epilogue row store (16 B per lane).
__device__ __forceinline__ void g2_store(bf16 *p, const bf16x8 &v) {
    *reinterpret_cast<bf16x8 *>(p) = v;
}

// Global stores one wave issues in the store phase of a full tile (every row < M):
// the next tile's first counted wait lets exactly these stay in flight.  (V^T tiles,
// partial tiles and the profiling ablations wait as if there were none.)
// EPI_RESID_STATS stores with its row statistics, before the prefetch: none in flight.
template <int EPI, bool SPLIT>
constexpr int g2_stores() {
    return EPI == EPI_RESID_STATS ? 0 : SPLIT ? 32 : 16;
}

#define G2_BAR() asm volatile("s_barrier" ::: "memory")
#define G2_WAITV(n) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(n) : "memory")

// Persistent: one workgroup per CU walks a chunk of tiles; after a tile's K loop it
// (1) does every epilogue step that reads LDS or global memory (parameters, residual
// rows, the row statistics exchange), (2) issues the next tile's parameter and
// prologue loads into the now idle LDS buffers, (3) computes and stores the outputs
// while those loads are in flight, and (4) starts the next K loop with a counted wait
// that leaves the stores of (3) outstanding.
template <int EPI, bool SPLIT>
__global__ void __launch_bounds__(G2_T) gemm256_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    // wave-uniform in SGPRs: the LDS-DMA destination (M0) is then scalar arithmetic
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int M = g.M, N = g.N, K = g.K;
    const int n_tn = N / G2_TILE, n_tm = (M + G2_TILE - 1) / G2_TILE, n_tiles = n_tn * n_tm;

    // tile schedule: workgroup b runs on XCD b % 8 (round-robin dispatch); XCD x owns
    // the contiguous chunk x of the tile order, walked by its workgroups in lockstep,
    // so the tiles in flight on one XCD are neighbours in the grouped order (GM
    // M-tiles x all N-tiles: A panels and weight tiles shared in that XCD's L2)
    const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
    const int wx = ((int)gridDim.x - xcd + 7) / 8;  // workgroups on this XCD
    const int cq = n_tiles / 8, cr = n_tiles % 8;
    const int c_lo = xcd * cq + min(xcd, cr), c_hi = c_lo + cq + (xcd < cr ? 1 : 0);
    int tix = c_lo + slot;
    if (tix >= c_hi) return;
    const int GM = g.tune_gm > 0 ? g.tune_gm : 4;

    // SPLIT: K tile t covers split columns [64 t, 64 t + 64) = the hi (k-step 0) and lo
    // (k-step 1) halves of logical k [32 t, 32 t + 32)
    const int nk = SPLIT ? K / 32 : K / 64;
    const int lda = SPLIT ? 2 * K : K, ldb = lda;

    // ---- staging sources (per lane) and LDS destinations (per wave) ----------
    // LDS row i (0..127) of a half tile = instruction j (0..1), wave, lane>>3:
    //   i = j*64 + wave*8 + (lane>>3);  slot lane&7 holds global chunk
    //   (lane&7) ^ (i&7)  (XOR swizzle on the source, rule 21).
    // A half h, row i -> tile row j*128 + h*64 + (i&63)
    // B half h, row i -> tile col j*128 + (wave>>2)*64 + h*32 + (wave&3)*8 + (lane>>3)
    const int chunk = ((lane & 7) ^ ((lane >> 3) & 7)) * 8;
    // B rows are stored permuted inside each 32-column group: LDS row q = sub*16 +
    // g*4 + r holds column g*8 + sub*4 + r, so that MFMA fragment nt (rows sub*16..+15
    // of half nt>>1) gives, in the C^T layout below, every lane 8 consecutive output
    // columns across the fragment pair (2h, 2h+1).
    const int qb = (wave & 3) * 8 + (lane >> 3);  // LDS row within the 32-column group
    const int b_col = ((qb >> 2) & 3) * 8 + (qb >> 4) * 4 + (qb & 3);
    // Stage addresses: a wave-uniform 64-bit base (SGPRs: tile origin, half, K tile)
    // plus a per-lane 32-bit byte offset, the global_load_lds saddr form (one offset
    // VGPR per operand instead of a 64-bit pointer per (half, instruction)).
    uint32_t a_voff = (uint32_t)(((wave * 8 + (lane >> 3)) * lda + chunk) * 2);
    uint32_t b_voff = (uint32_t)((((wave >> 2) * 64 + b_col) * ldb + chunk) * 2);
    int m0 = 0, n0 = 0;
    const char *a_base = nullptr, *b_base = nullptr;
    auto setup = [&](int t) {
        const int grp = t / (GM * n_tn), first_m = grp * GM;
        const int gsz = min(GM, n_tm - first_m);
        const int in = t % (GM * n_tn);
        m0 = (first_m + in % gsz) * G2_TILE;
        n0 = (in / gsz) * G2_TILE;
        a_base = reinterpret_cast<const char *>(static_cast<const bf16 *>(g.A) + (int64_t)m0 * lda);
        b_base = reinterpret_cast<const char *>(static_cast<const bf16 *>(g.B) + (int64_t)n0 * ldb);
    };
    const int64_t a_h = (int64_t)64 * lda * 2, a_j = (int64_t)128 * lda * 2;  // bytes
    const int64_t b_h = (int64_t)32 * ldb * 2, b_j = (int64_t)128 * ldb * 2;
    typedef __attribute__((address_space(3))) void lds_void;
#define G2_STAGE_A(buf, h, t)                                                                  \
    do {                                                                                       \
        asm volatile("" : "+v"(a_voff)); /* opaque: no hoisted 64-bit lane pointers */         \
        __builtin_amdgcn_global_load_lds((const void *)(a_base + ((h) * a_h + (t) * 128) + a_voff), \
                                         (lds_void *)(lds + (buf) * G2_BUF + (h) * 16384 +     \
                                                      wave * 1024),                            \
                                         16, 0, 0);                                            \
        __builtin_amdgcn_global_load_lds(                                                      \
            (const void *)(a_base + ((h) * a_h + a_j + (t) * 128) + a_voff),                   \
            (lds_void *)(lds + (buf) * G2_BUF + (h) * 16384 + 8192 + wave * 1024), 16, 0, 0);  \
    } while (0)
#define G2_STAGE_B(buf, h, t)                                                                  \
    do {                                                                                       \
        asm volatile("" : "+v"(b_voff));                                                       \
        __builtin_amdgcn_global_load_lds((const void *)(b_base + ((h) * b_h + (t) * 128) + b_voff), \
                                         (lds_void *)(lds + (buf) * G2_BUF + 32768 +           \
                                                      (h) * 16384 + wave * 1024),              \
                                         16, 0, 0);                                            \
        __builtin_amdgcn_global_load_lds(                                                      \
            (const void *)(b_base + ((h) * b_h + b_j + (t) * 128) + b_voff),                   \
            (lds_void *)(lds + (buf) * G2_BUF + 32768 + (h) * 16384 + 8192 + wave * 1024), 16, \
            0, 0);                                                                             \
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

    // ---- epilogue parameters of a tile (wave 0, older than the tile's stage loads,
    // so its first counted wait retires them) ---------------------------------------
    constexpr bool FOLD = EPI == EPI_FOLD || EPI == EPI_FOLD_GELU;
    constexpr bool RS = EPI == EPI_RESID_STATS;
    auto stage_params = [&](int pb) {
        if (wave != 0) return;
        uint32_t l16 = lane * 16;
        asm volatile("" : "+v"(l16));  // opaque: uniform base + 32-bit offset (saddr form)
        auto par1k = [&](const void *src, int off) {  // 1 KiB: 16 B per lane
            __builtin_amdgcn_global_load_lds(
                (const void *)(static_cast<const char *>(src) + l16),
                (lds_void *)(lds + G2_PAR + pb * G2_PARSZ + off), 16, 0, 0);
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
    };
    // prologue of a tile: K tiles 0 and 1 whole (8 loads each).  Issued before the
    // previous tile's stores, so the first iteration's phase-4 wait (K tile 1) can leave
    // those stores in flight: they must land only by phase 8 (K tile 2, issued after
    // them) instead of phase 4 -- the stores are ~12-20% of a split GEMM when exposed
    // (profiles/r03_gemm_check_ablations.txt, ablate 4).
    auto prologue = [&]() {
        G2_STAGE_A(0, 0, 0);
        G2_STAGE_B(0, 0, 0);
        G2_STAGE_A(0, 1, 0);
        G2_STAGE_B(0, 1, 0);
        G2_STAGE_A(1, 0, 1);
        G2_STAGE_B(1, 0, 1);
        G2_STAGE_A(1, 1, 1);
        G2_STAGE_B(1, 1, 1);
    };
    constexpr int NST = g2_stores<EPI, SPLIT>();
    bool pend = false;  // (uniform) the previous tile's NST stores are in flight

    int pb = 0;  // parameter slot of the current tile
    setup(tix);
    stage_params(pb);
    prologue();
    G2_WAITV(8);  // K tile 0 (and the parameters); K tile 1 in flight
    for (;;) {
        G2_BAR();
        if (wr == 1) G2_BAR();  // group 1 runs one barrier behind group 0
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        for (int t = 0; t < nk; t += 2) {
            const bool more = t + 2 < nk;  // K tiles t+2, t+3 exist (nk is even)
            // phase 1: buffer 0, A0 + B0 (K tile 1's B1 half came with the prologue)
            G2_READ_B(0, 0);
            G2_READ_A(0, 0);
            if (t > 0) G2_STAGE_B(1, 1, t + 1);
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
            // phase 4: registers only; retire K tile t+1 for phase 5 (first iteration:
            // the previous tile's stores, younger than K tile 1, may stay in flight)
            if (more) {
                G2_STAGE_A(0, 1, t + 2);
                if (t == 0 && pend)
                    G2_WAITV((6 + NST));
                else
                    G2_WAITV(6);
            } else {
                G2_WAITV(0);
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
        if (wr == 0) G2_BAR();  // re-align the two groups: every LDS read has retired

        // ---- epilogue ----------------------------------------------------------
        // C^T layout (the MFMA took the weight fragment as its first operand): lane l
        // holds, for A fragment mt and weight-column half h, output row
        //   m = m0 + wr*128 + mt*16 + (l & 15)
        // and the 8 consecutive columns n = n0 + wc*64 + h*32 + (l >> 4)*8 + e, e = 0..7,
        // in acc[mt][2h][0..3], acc[mt][2h+1][0..3].  Stores go straight from registers,
        // 16 B (bf16) / 32 B (f32) per lane, no LDS round trip.
        const int nxt = tix + wx;
        // (the residual epilogues run one tile per workgroup, see launch_gemm256)
        constexpr bool PERSIST = EPI != EPI_BIAS_RESID && EPI != EPI_RESID_STATS;
        const bool has_next = PERSIST && nxt < c_hi;
        const bool full = m0 + G2_TILE <= M;
        int m0e = m0;  // opaque: keeps the per-row epilogue offsets out of the K loop
        asm volatile("" : "+s"(m0e));
        const int row_l = m0e + wr * 128 + (lane & 15);
        // global addresses: a wave-uniform base (row m0 + wr*128, column n0 + wc*64) +
        // mt * (16 rows) in SGPRs, and one 32-bit lane offset (row lane&15, column
        // (lane>>4)*8) -- no 64-bit pointer per row held across the prefetch
        const int64_t row_w = m0e + wr * 128, col_w = n0 + wc * 64;
        auto lane_off = [&](int ld, int esz) {
            return (uint32_t)(((lane & 15) * ld + (lane >> 4) * 8) * esz);
        };
        const bool vtile = EPI == EPI_QKV && n0 >= 2 * g.hidden;
        const unsigned char *par = lds + G2_PAR + pb * G2_PARSZ;
        // tile-local indices into the staged parameters
        const int prow = wr * 128 + (lane & 15);          // + mt * 16
        const int pcol = wc * 64 + (lane >> 4) * 8;        // + h * 32 + e
        auto par8 = [&](int off, int h, float (&v)[8]) {   // 8 column params from LDS
            const float4 a = *reinterpret_cast<const float4 *>(par + off + (pcol + h * 32) * 4);
            const float4 b = *reinterpret_cast<const float4 *>(par + off + (pcol + h * 32 + 4) * 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
            v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        };
        auto prow2 = [&](int mt) {  // (rstd, -rstd mean) of row prow + 16 mt
            return *reinterpret_cast<const float2 *>(par + G2_PAR_ROW + (prow + mt * 16) * 8);
        };

        // (1) reads: parameters, residual rows, V^T columns, row statistics
        float bias_v[2][8];  // (the folded epilogues carry their bias inside col_c)
        float cs2[2][8], ra[8], rb[8];
        int vc[8];
        // (full tiles: straight-line code, no per-row guards)
        auto reads = [&](auto full_c) {
            constexpr bool FULL = decltype(full_c)::value;
            par8(G2_PAR_C0, 0, bias_v[0]);
            par8(G2_PAR_C0, 1, bias_v[1]);
            if constexpr (FOLD) {
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    const float2 p = prow2(mt);
                    ra[mt] = p.x;
                    rb[mt] = p.y;
                }
                par8(G2_PAR_C1, 0, cs2[0]);
                par8(G2_PAR_C1, 1, cs2[1]);
            }
            if (vtile) {
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    const int row = row_l + mt * 16;
                    vc[mt] = (FULL || row < M) ? g.vcol[row] : -1;
                }
#pragma unroll
                for (int mt = 0; mt < 8; ++mt)  // consumed here: the load's wait stays
                    asm volatile("" : "+v"(vc[mt]));  // ahead of the prefetch
            }
            if constexpr (EPI == EPI_BIAS_RESID) {  // acc <- (acc + bias) + resid
                // (SPLIT: split residual rows, stride 2N, 32-column chunks of hi then lo).
                const int rld = SPLIT ? 2 * N : N;
                const char *rbase = static_cast<const char *>(g.resid) +
                                    (row_w * rld + (SPLIT ? 2 * col_w : col_w)) * 2;
                const uint32_t rlo = lane_off(rld, 2);
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    if (!FULL && row_l + mt * 16 >= M) continue;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const char *rp = rbase + (int64_t)mt * 16 * rld * 2 + h * (SPLIT ? 128 : 64) + rlo;
                        float r[8];
                        if constexpr (SPLIT) {
                            const bf16x8 rh = *reinterpret_cast<const bf16x8 *>(rp);
                            const bf16x8 rl = *reinterpret_cast<const bf16x8 *>(rp + 64);
#pragma unroll
                            for (int e = 0; e < 8; ++e) r[e] = (float)rh[e] + (float)rl[e];
                        } else {
                            const bf16x8 rv = *reinterpret_cast<const bf16x8 *>(rp);
#pragma unroll
                            for (int e = 0; e < 8; ++e) r[e] = (float)rv[e];
                        }
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            acc[mt][2 * h + (e >> 2)][e & 3] =
                                (acc[mt][2 * h + (e >> 2)][e & 3] + bias_v[h][e]) + r[e];
                    }
                }
            }
            if constexpr (EPI == EPI_RESID_STATS) {
                // out = acc + bias + LN(resid) (resid normalised on the fly from its row
                // statistics, or plain), and this tile's partial statistics of the
                // rounded out
                const bool res_ln = g.row_ln != nullptr;
                float ss[8], sq[8], sd[8], rr[8], rs[8];
                float gm[2][8], bt[2][8], wg[2][8];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (res_ln) {
                        par8(G2_PAR_C1, h, gm[h]);
                        par8(G2_PAR_C2, h, bt[h]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            gm[h][e] = 1.f;
                            bt[h][e] = 0.f;
                        }
                    }
                    if (g.head_wg) {
                        par8(G2_PAR_C3, h, wg[h]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) wg[h][e] = 0.f;
                    }
                }
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    ss[mt] = sq[mt] = sd[mt] = 0.f;
                    rr[mt] = 1.f;
                    rs[mt] = 0.f;
                    if (res_ln) {
                        const float2 p = prow2(mt);
                        rr[mt] = p.x;
                        rs[mt] = p.y;
                    }
                }
                // (SPLIT: resid and out are split rows, stride 2N, every 32 columns 32 hi
                // then 32 lo; the statistics are those of hi + lo, the value the
                // consumer GEMMs read)
                const int rld = SPLIT ? 2 * N : N;
                constexpr int HS = SPLIT ? 128 : 64;  // bytes per 32 columns
                const char *rbase = static_cast<const char *>(g.resid) +
                                    (row_w * rld + (SPLIT ? 2 * col_w : col_w)) * 2;
                const uint32_t rlo = lane_off(rld, 2);
                char *ob = static_cast<char *>(g.out) +
                           (row_w * g.ld_out + (SPLIT ? 2 * col_w : col_w)) * 2;
                const uint32_t olo = lane_off(g.ld_out, 2);
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    if (!FULL && row_l + mt * 16 >= M) continue;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const char *rp = rbase + (int64_t)mt * 16 * rld * 2 + h * HS + rlo;
                        float r[8];
                        if constexpr (SPLIT) {
                            const bf16x8 rh = *reinterpret_cast<const bf16x8 *>(rp);
                            const bf16x8 rl = *reinterpret_cast<const bf16x8 *>(rp + 64);
#pragma unroll
                            for (int e = 0; e < 8; ++e) r[e] = (float)rh[e] + (float)rl[e];
                        } else {
                            const bf16x8 rv = *reinterpret_cast<const bf16x8 *>(rp);
#pragma unroll
                            for (int e = 0; e < 8; ++e) r[e] = (float)rv[e];
                        }
                        bf16x8 o, ol;
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const float res = fmaf(gm[h][e], fmaf(rr[mt], r[e], rs[mt]), bt[h][e]);
                            const float y = acc[mt][2 * h + (e >> 2)][e & 3] + bias_v[h][e] + res;
                            float yb;
                            if constexpr (SPLIT) {
                                o[e] = split_hi(y);
                                ol[e] = split_lo(y);
                                yb = (float)o[e] + (float)ol[e];
                            } else {
                                o[e] = (bf16)y;
                                yb = (float)o[e];
                            }
                            ss[mt] += yb;
                            sq[mt] = fmaf(yb, yb, sq[mt]);
                            sd[mt] = fmaf(yb, wg[h][e], sd[mt]);
                        }
                        if (!(g.ablate & 4)) {
                            char *op = ob + (int64_t)mt * 16 * g.ld_out * 2 + h * HS + olo;
                            g2_store(reinterpret_cast<bf16 *>(op), o);
                            if constexpr (SPLIT) g2_store(reinterpret_cast<bf16 *>(op + 64), ol);
                        }
                    }
                }
                // partials: the 4 lane groups (lanes l, l^16, l^32, l^48 share a row),
                // then the 4 wc waves through LDS (the staging buffers are idle until
                // the prefetch below), fixed order
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
                        part[wc * G2_TILE + wr * 128 + mt * 16 + lane] =
                            make_float4(ss[mt], sq[mt], sd[mt], 0.f);
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
                __syncthreads();  // part[] read before the prefetch overwrites it
            }
        };
        if (full && PERSIST && EPI != EPI_QKV)  // (measured: no spills)
            reads(std::true_type{});
        else
            reads(std::false_type{});

        // (2) the next tile's parameters and prologue (a compiler memory barrier: no
        // load of (1) may sink below the prefetch, whose wait would then drain it)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (has_next) {
            setup(nxt);
            stage_params(pb ^ 1);
            prologue();
        }
        __builtin_amdgcn_sched_barrier(0);

        // (3) compute and store (registers and global stores only)
        auto stores = [&](auto full_c) {
            constexpr bool FULL = decltype(full_c)::value;
            if (vtile) {  // V columns: transposed element stores into V^T
                char *vb = static_cast<char *>(g.out2) + (col_w - 2 * g.hidden) * g.ld_v * (int64_t)2;
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    if (vc[mt] < 0) continue;
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            *reinterpret_cast<bf16 *>(
                                vb + (uint32_t)((((lane >> 4) * 8 + h * 32 + e) * g.ld_v + vc[mt]) * 2)) =
                                (bf16)(acc[mt][2 * h + (e >> 2)][e & 3] + bias_v[h][e]);
                }
            } else if constexpr (FOLD) {
                // LN folded into this GEMM: y = r acc - r mu s + c  (per row r, mu; per
                // column s, c); row-major order: both 64-byte halves of a row's 128-byte
                // segment are stored by consecutive instructions
                // (SPLIT: A holds split rows of the un-normalised x, the output split rows)
                constexpr int HS = SPLIT ? 128 : 64;  // bytes per 32 columns
                char *ob = static_cast<char *>(g.out) +
                           (row_w * g.ld_out + (SPLIT ? 2 * col_w : col_w)) * 2;
                const uint32_t olo = lane_off(g.ld_out, 2);
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    const int row = row_l + mt * 16;
                    if (!FULL && row >= M) continue;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        float v[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            v[e] = fmaf(ra[mt], acc[mt][2 * h + (e >> 2)][e & 3],
                                        fmaf(rb[mt], cs2[h][e], bias_v[h][e]));
                        if constexpr (EPI == EPI_FOLD_GELU) {
                            if (!(g.ablate & 2)) {
                                if (SPLIT || (g.ablate & 8)) gelu_erf8(v);  // (A/B: the erf form)
                                else gelu_bf16_8(v);
                            }
                        }
                        if (g.ablate & 4) continue;
                        char *op = ob + (int64_t)mt * 16 * g.ld_out * 2 + h * HS + olo;
                        if constexpr (SPLIT) {
                            bf16x8 hv, lv;
#pragma unroll
                            for (int e = 0; e < 8; ++e) hv[e] = split_hi(v[e]), lv[e] = split_lo(v[e]);
                            g2_store(reinterpret_cast<bf16 *>(op), hv);
                            g2_store(reinterpret_cast<bf16 *>(op + 64), lv);
                        } else {
                            bf16x8 o;
#pragma unroll
                            for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
                            g2_store(reinterpret_cast<bf16 *>(op), o);
                        }
                    }
                }
            } else if constexpr (RS) {
                // (stored with the statistics, before the prefetch)
            } else {
                // element size and column of the output rows: bf16 rows; SPLIT: f32 rows
                // (pre-LN) or split rows (ld_out = 2N: hi chunk then lo)
                constexpr bool F32 = SPLIT && EPI == EPI_BIAS_RESID;
                constexpr int ESZ = F32 ? 4 : 2;
                constexpr int HSTEP = F32 ? 128 : (SPLIT ? 128 : 64);  // bytes per 32 columns
                char *ob = static_cast<char *>(g.out) +
                           (row_w * g.ld_out + ((SPLIT && !F32) ? 2 * col_w : col_w)) * ESZ;
                const uint32_t olo = lane_off(g.ld_out, ESZ);
#pragma unroll
                for (int mt = 0; mt < 8; ++mt) {
                    const int row = row_l + mt * 16;
                    if (!FULL && row >= M) continue;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        float v[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            v[e] = EPI == EPI_BIAS_RESID ? acc[mt][2 * h + (e >> 2)][e & 3]
                                                         : acc[mt][2 * h + (e >> 2)][e & 3] +
                                                               bias_v[h][e];
                        if constexpr (EPI == EPI_BIAS_GELU) {
                            if (!(g.ablate & 2)) {
                                if (SPLIT || (g.ablate & 8)) gelu_erf8(v);
                                else gelu_bf16_8(v);
                            }
                        }
                        if (g.ablate & 4) continue;
                        char *op = ob + (int64_t)mt * 16 * g.ld_out * ESZ + h * HSTEP + olo;
                        if constexpr (F32) {
                            *reinterpret_cast<float4 *>(op) = make_float4(v[0], v[1], v[2], v[3]);
                            *reinterpret_cast<float4 *>(op + 16) = make_float4(v[4], v[5], v[6], v[7]);
                        } else if constexpr (SPLIT) {  // 8 columns of one 32-column chunk
                            bf16x8 hv, lv;
#pragma unroll
                            for (int e = 0; e < 8; ++e) hv[e] = split_hi(v[e]), lv[e] = split_lo(v[e]);
                            g2_store(reinterpret_cast<bf16 *>(op), hv);
                            g2_store(reinterpret_cast<bf16 *>(op + 64), lv);
                        } else {
                            bf16x8 o8;
#pragma unroll
                            for (int e = 0; e < 8; ++e) o8[e] = (bf16)v[e];
                            g2_store(reinterpret_cast<bf16 *>(op), o8);
                        }
                    }
                }
            }
        };
        if (full)
            stores(std::true_type{});
        else
            stores(std::false_type{});
        if (!has_next) break;
        // (4) retire the next tile's K tile 0 (the parameters are older still), leaving
        // K tile 1 and this tile's stores in flight when their count is known
        pend = full && !vtile && !(g.ablate & 4) && NST > 0;
        if (pend)
            G2_WAITV((8 + NST));
        else
            G2_WAITV(8);
        tix = nxt;
        pb ^= 1;
    }
#undef G2_STAGE_A
#undef G2_STAGE_B
#undef G2_LD
#undef G2_READ_A
#undef G2_READ_B
#undef G2_MFMA
#undef G2_SYNC_READS
}
#undef G2_BAR
#undef G2_WAITV

// Shapes the 8-phase kernel takes; everything else goes to the 128x128 kernel.
bool gemm256_ok(int epi, const GemmArgs &g) {
    const int64_t m_pad = ((int64_t)g.M + G2_TILE - 1) / G2_TILE * G2_TILE;
    if (g.split && epi == EPI_QKV) return false;
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
    DI_REQUIRE(gemm256_ok(epi, g), DI_EINVAL, "gemm256: unsupported shape / epilogue");
    const int n_tiles = g.N / G2_TILE * ((g.M + G2_TILE - 1) / G2_TILE);
    if (n_tiles == 0) return;
    // persistent (one workgroup per CU) where the epilogue reads no global memory;
    // the residual epilogues run one tile per workgroup (their residual loads would
    // otherwise queue behind the next tile's prefetch: measured O 0.31 -> 0.36 ms)
    const bool resid = epi == EPI_BIAS_RESID || epi == EPI_RESID_STATS;
    const dim3 grid(resid ? n_tiles : std::min(n_tiles, n_cu()));
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
            G2_SCASE(EPI_FOLD)
            G2_SCASE(EPI_FOLD_GELU)
            G2_SCASE(EPI_RESID_STATS)
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
