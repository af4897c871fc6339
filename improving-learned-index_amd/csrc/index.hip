// index.hip -- quantized inverted-index scorer for MI355X (gfx950).
//
// Replaces InvertedIndex.score (reference src/deep_impact/inverted_index/
// inverted_index.py:31-62) for batches of queries, bit-exact including the
// reference's tie order.
//
// Device layout ("doc-blocked, impact-ordered postings"):
//   docs of a shard are cut into nb = ceil(n_docs / 32768) equal blocks (a multiple
//   of 64 docs each, at most 32768); every term's postings are grouped by block
//   (block-major; inside a block by impact class, bank-dealt).  One posting = one
//   u32: (doc_in_block << 8) | value.  A sparse term -> block table locates the
//   (term, block) sublists (SubIndex).
//
// score_blocks: one 1024-thread workgroup per (query, block) item, persistent.  The
//   block's 32768 accumulators live in LDS (128 KiB), one word per doc
//   score(16) | (255 - j)(8) | v_j(8)  (j = the first query term touching it, v_j its
//   value there): comparing words orders docs exactly like the reference -- score
//   descending, then first-touch order (term order, then impact desc inside that
//   term's list, then doc asc).  Terms are applied in query order; a doc occurs once
//   per term and is updated by one wave (per-wave layout) or between term barriers, so
//   a plain LDS read-modify-write is race free.  Selection: a per-query threshold
//   shared across blocks, a 4096-bin score histogram (<= 16 query terms) or a
//   block-wide radix select.
// score_long: queries of more than 256 terms (64-bit words, wide keys).
// merge_topk: one workgroup per query selects the <= NB*k block candidates by the
//   64-bit key  word(32) | ~doc(32)  and writes doc/score/key.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <memory>
#include <numeric>
#include <string>
#include <type_traits>
#include <vector>

#include "di_common.h"
#include "topk_common.h"

namespace di {

constexpr int MAX_BLOCK_DOCS = 32768;  // docs per block (one workgroup's accumulators)
constexpr int SC_THREADS = 1024;
constexpr int SC_WAVES = SC_THREADS / 64;
constexpr int SC_PER_THREAD = MAX_BLOCK_DOCS / SC_THREADS;  // 32 docs per thread in a sweep
constexpr int MAX_TERMS = DI_SHORT_QUERY_TERMS;  // query terms of the compact word
// Long sublists (>= WLONG_MIN postings in a block) carry a per-wave layout (build pass
// 3): wave w scatters only the docs of its segment.  Queries of at most WTERMS terms
// run every term that way (short terms: every wave reads the sublist, applies its own
// docs); longer ones run the all-wave form, a barrier per term.
constexpr int WSEG = SC_WAVES;
constexpr int WLONG_MIN = 128;  // (1024 / 512 / 256 / 64: within 1%, profiles/r03j; 128 vs
                                // 512 in round 4: exhaustive equal, block-max segment bounds
                                // for more terms -- f = 1 skips 0.44 vs 0.30 of the segments
                                // at 8.8 M skewed docs, gpurun_out/round4_h)
constexpr int WTERMS = 64;
// Fast selection: with at most 16 query terms every score is below 255 * 16 < 4096,
// so one pass of a 4096-bin score histogram finds the k-th score; the docs tied at
// that score (a few, typically) are ordered from a compact list in LDS.
constexpr int FAST_TERMS = 16;
constexpr int HIST_BINS = 4096;
constexpr int TIE_CAP = HIST_BINS;
constexpr int QH_BINS = 4096;  // per-query candidate-score histogram (shared threshold)
// Long queries (score_long_item): 64-bit words over half blocks.
constexpr int LONG_TERMS = DI_MAX_QUERY_TERMS;
constexpr int LH_DOCS = 16384;
constexpr int LH_PER_THREAD = LH_DOCS / SC_THREADS;  // 16
constexpr int LH_HELD = DI_MAX_TOPK / SC_THREADS;    // 4
static_assert(MAX_BLOCK_DOCS <= 2 * LH_DOCS, "two halves cover a block");
static_assert(LONG_TERMS <= 4096, "12-bit first-touch index");

struct ScoreShared {
    // the block's words score(16) | (255 - j)(8) | v_j(8) (j = the first query term
    // touching the doc, v_j its value there), + 64 per-lane dummy words; a long-query
    // item uses the array as LH_DOCS 64-bit words (score_long_item)
    uint32_t acc[MAX_BLOCK_DOCS + 64];
    union {
        RadixScratch<SC_WAVES> rs;      // general radix path
        uint32_t hist[HIST_BINS + 64];  // fast path: score histogram (+ spare bins), then the tie list
    } u;
    union {
        int64_t bounds[2][MAX_TERMS];  // scatter: sublist [lo, hi) of every query term
        uint32_t h256[256];            // fast path: digit histogram over the tie list
    } v;
    uint32_t wsum[SC_WAVES];
    uint32_t emit;   // output cursor
    uint32_t n_tie;  // tie-list cursor
    uint32_t bad;
    uint32_t thr, above, ties, bin, bin_above;
    uint32_t tq;                   // the query's shared threshold as this item read it
    uint32_t lmask[WTERMS / 32];   // terms (j < WTERMS) with a per-wave layout in this block
    uint32_t pmask[WTERMS / 32];   // packed mode: short terms read from the plain postings
    unsigned long long bm_cnt[2];  // block-max statistics of the workgroup (thread 0)
    uint32_t tqe;                  // block-max: the query's running threshold (qtq) as
                                   // thread 0 read it -- one value for every wave
    uint32_t wub[WSEG];            // block-max: each wave segment's score upper bound
    uint32_t wtab[WTERMS][WSEG];   // their per-wave runs: start << 16 | end (in the sublist)
    uint32_t wstamp[SC_WAVES];     // profiling (DI_PROFILE_ABLATE bit 64): each wave's scatter loop
    uint32_t tqn;                  // EXT: a lower bound of the query's k-th score this item
                                   // found (thread 0), raised into qtq after the item
                                   // (last: the fields above keep their alignment)
};
static_assert(offsetof(ScoreShared, acc) == 0, "accumulators at LDS address 0");
static_assert(sizeof(ScoreShared().acc) >= LH_DOCS * sizeof(uint64_t), "half-block words fit");
static_assert(sizeof(RadixScratch<SC_WAVES>) >= (HIST_BINS + 64) * 4,
              "histogram (+ 64 spare bins) overlays the radix scratch");
static_assert(sizeof(ScoreShared().wtab) >= SC_THREADS * 4, "score_long_kernel's query list");

template <class KeyF, class Pred>
__device__ __forceinline__ void score_radix_pass(ScoreShared &sh, int n_local, int shift,
                                                 uint32_t need, KeyF key, Pred pred) {
    radix_clear<SC_THREADS, SC_WAVES>(sh.u.rs);
    __syncthreads();
    RunLen rl;
#pragma unroll 4
    for (int i = 0; i < SC_PER_THREAD; ++i) {
        int idx = i * SC_THREADS + threadIdx.x;
        if (idx < n_local) {
            uint32_t w = sh.acc[idx];
            uint32_t kk = key(w, idx);
            if (pred(w, idx, kk)) rl.add(sh.u.rs, (kk >> shift) & 255u);
        }
    }
    rl.flush(sh.u.rs);
    __syncthreads();
    radix_pick<SC_THREADS, SC_WAVES>(sh.u.rs, need);
}

// Sweep of the block's accumulator words: f(w, idx) for idx < round4(n_local), 4
// consecutive words per lane per ds_read_b128, 4 reads in flight before any is
// used (a read-then-use loop is LDS-latency bound).  Words past the zeroed range
// come as 0; f runs in wave-uniform control flow (it may ballot).
template <class F>
__device__ __forceinline__ void sweep_words(const uint32_t *acc, int n_local, int tid, F f) {
    const uint4 *a4 = reinterpret_cast<const uint4 *>(acc);
    const int n4 = (n_local + 3) >> 2;
    constexpr int G = 4;  // uint4 reads in flight per lane
    for (int i0 = 0; i0 < SC_PER_THREAD / 4; i0 += G) {
        if (i0 * SC_THREADS >= n4) break;  // (uniform)
        uint4 x[G];
#pragma unroll
        for (int i = 0; i < G; ++i) {
            // q4 < 8192 always lies inside the array: load unconditionally (no branch),
            // then drop what lies past the zeroed range
            const int q4 = (i0 + i) * SC_THREADS + tid;
            const uint4 y = a4[q4];
            x[i].x = q4 < n4 ? y.x : 0u;
            x[i].y = q4 < n4 ? y.y : 0u;
            x[i].z = q4 < n4 ? y.z : 0u;
            x[i].w = q4 < n4 ? y.w : 0u;
        }
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const int base = 4 * ((i0 + i) * SC_THREADS + tid);
            f(x[i].x, base);
            f(x[i].y, base + 1);
            f(x[i].z, base + 2);
            f(x[i].w, base + 3);
        }
    }
}

// Block-wide stable compaction over the accumulator words into two lists:
// cls(w, idx) -> bit 0: list A, bit 1: list B.  One counting sweep, one exclusive
// block scan of the packed per-thread counts, one writing sweep calling
// out(list, pos, w, idx) -- no atomics.  Returns the packed totals (A | B << 16;
// each list holds at most 32768).  Ends with a barrier.
template <class Cls, class Out, class St = void (*)(int)>
__device__ __forceinline__ uint32_t compact_words(ScoreShared &sh, int n_local, int tid, Cls cls,
                                                  Out out, St st = nullptr) {
    uint32_t cnt = 0;
    sweep_words(sh.acc, n_local, tid, [&](uint32_t w, int idx) {
        const uint32_t c = cls(w, idx);
        cnt += (c & 1u) + ((c & 2u) << 15);
    });
    if constexpr (!std::is_same<St, void (*)(int)>::value) st(6);
    const int lane = tid & 63, wave = tid >> 6;
    const uint32_t incl = wave_prefix_sum(cnt);
    if (lane == 63) sh.wsum[wave] = incl;
    __syncthreads();
    uint32_t base = incl - cnt, total = 0;
    for (int w2 = 0; w2 < SC_WAVES; ++w2) {
        const uint32_t x = sh.wsum[w2];
        if (w2 < wave) base += x;
        total += x;
    }
    uint32_t pa = base & 0xFFFFu, pb = base >> 16;
    if constexpr (!std::is_same<St, void (*)(int)>::value) st(7);
    sweep_words(sh.acc, n_local, tid, [&](uint32_t w, int idx) {
        const uint32_t c = cls(w, idx);
        if (c & 1u) out(0, pa++, w, idx);
        if (c & 2u) out(1, pb++, w, idx);
    });
    __syncthreads();
    return total;
}

// Wave-aggregated append: lanes with `take` get consecutive slots of *cursor (one
// LDS atomic per wave and call).  Call from wave-uniform control flow.
// MB: the leader's base by v_readlane and the lanes below by v_mbcnt -- no LDS permute
// and no lane mask held in registers (the block-max instantiation spilled a held 64-bit
// mask and reloaded it per sweep step: 74 -> 8 scratch loads, its sweep 2x faster); the
// plain scorer keeps the permute form (measured 2.06 vs 2.09 ms per 100 k-doc launch).
template <bool MB = false>
__device__ __forceinline__ bool wave_append(bool take, uint32_t *cursor, uint32_t &pos) {
    const uint64_t m = __ballot(take);
    if (m == 0) return false;
    const int lane = threadIdx.x & 63;
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(cursor, (uint32_t)__builtin_popcountll(m));
    if constexpr (MB) {
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
        pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    } else {
        base = __shfl(base, leader, 64);
        pos = base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
    }
    return take;
}

// Device posting words are ((doc_in_block << 10) | value) XOR POST_X: bits 8-9 stay 0,
// so (word ^ POST_X) >> 8 is the doc's LDS byte address.  A buffer load
// past the descriptor's range returns 0, which decodes to doc MAX_BLOCK_DOCS -- the
// dummy accumulator word after the block -- with value 0: the padding lanes of a
// round need no clamp, no select and no branch (their update lands in the dummy).
// (Per-lane dummy words for the padding, with a quad-wise threshold sweep, measured
// 4.5% slower, r03pad; the quad sweep alone neutral, r03quad.)
constexpr uint32_t POST_X = (uint32_t)MAX_BLOCK_DOCS << 10;

// One scatter round over postings p[0 .. min(avail, UU * SC_THREADS)) (lane-
// consecutive, UU per lane; p and avail wave-uniform): all loads first -- buffer loads
// bounds-checked by the hardware, a 32-bit lane offset and no per-posting address
// arithmetic -- then the LDS reads, then the writes.  A doc occurs once per term, so
// the read-modify-write needs no atomics.
//
// wide (UU a multiple of 4): 16-byte loads, lane tid taking the postings 4 tid ..
// 4 tid + 3 of each group of 4 NT -- a quarter of the load instructions (the scatter
// is bound by them).  Any posting -> lane mapping is exact (a doc occurs
// once per term), and a multi-dword buffer load is range-checked per dword, so the
// padding past avail still reads 0.
template <int UU, int NT = SC_THREADS>
__device__ __forceinline__ void scatter_load(const uint32_t *p, int64_t avail, int tid,
                                             uint32_t (&cur)[UU], bool wide = false) {
    const uint64_t pa = reinterpret_cast<uint64_t>(p);
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)pa);
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane(
        (int)(min(avail, (int64_t)UU * NT) * 4));
    void *base = reinterpret_cast<void *>(((uint64_t)hi32 << 32) | lo32);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
    if constexpr (UU % 4 == 0) {
        if (wide) {
#pragma unroll
            for (int g = 0; g < UU / 4; ++g) {
                const auto v =
                    __builtin_amdgcn_raw_buffer_load_b128(rsrc, (4 * tid + g * 4 * NT) * 4, 0, 0);
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[4 * g + k] = v[k];
            }
            return;
        }
    }
#pragma unroll
    for (int u = 0; u < UU; ++u)
        cur[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (tid + u * NT) * 4, 0, 0);
}
// The word update: touched w + (v << 16), first touch (v << 16) | first_bits | v --
// both one 24-bit multiply-add (v < 256, first_bits = (255 - j) << 8: no carries).
__device__ __forceinline__ uint32_t word_update(uint32_t w, uint32_t v, uint32_t first_bits) {
    const uint32_t t = __umul24(v, 0x10000u) + w;
    const uint32_t f = __umul24(v, 0x10001u) + first_bits;
    return w ? t : f;
}

// FILT (the all-wave form under impact pruning): postings below vmin update the lane's
// dummy word instead.
template <int UU, bool FILT = false>
__device__ __forceinline__ void scatter_apply(uint32_t *acc, const uint32_t (&cur)[UU],
                                              uint32_t first_bits, uint32_t vmin = 0) {
    // LDS byte addresses formed here and the accesses in inline asm (the compiler's own
    // form adds the array's zero base once more per posting); the reads are retired by
    // the explicit wait, the writes by the caller's term barrier / final wait.
    // (acc is the first member of the kernel's only LDS object, the dynamic segment at
    // LDS address 0: score_blocks_kernel checks that once)
    (void)acc;
    uint32_t w[UU], a[UU];
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        a[u] = (cur[u] ^ POST_X) >> 8;
        if constexpr (FILT)
            a[u] = (cur[u] & 255u) >= vmin ? a[u] : (uint32_t)(MAX_BLOCK_DOCS + lane_id()) << 2;
        asm volatile("ds_read_b32 %0, %1" : "=v"(w[u]) : "v"(a[u]) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // the compiler sees the asm reads' results as ready at once: redefine them after
    // the wait, and fence the scheduler, so that no use is hoisted above it
#pragma unroll
    for (int u = 0; u < UU; ++u) asm volatile("" : "+v"(w[u]));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const uint32_t v = cur[u] & 255u;
        asm volatile("ds_write_b32 %0, %1" ::"v"(a[u]), "v"(word_update(w[u], v, first_bits))
                     : "memory");
    }
}

// scatter_apply restricted to the docs [dlo, dlo + dn) of one wave (a short term, whose
// sublist every wave reads in full): the other postings (and the padding) update a
// per-lane dummy word past the block instead.  (Exec-masking them off instead measured
// no faster, r03sc.)
template <int UU>
__device__ __forceinline__ void scatter_apply_own(const uint32_t (&cur)[UU], uint32_t first_bits,
                                                  uint32_t dlo, uint32_t dn, uint32_t dummy) {
    uint32_t w[UU], a[UU];
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const uint32_t d = (cur[u] ^ POST_X) >> 10;
        a[u] = (d - dlo < dn) ? d << 2 : dummy;
        asm volatile("ds_read_b32 %0, %1" : "=v"(w[u]) : "v"(a[u]) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < UU; ++u) asm volatile("" : "+v"(w[u]));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const uint32_t v = cur[u] & 255u;
        asm volatile("ds_write_b32 %0, %1" ::"v"(a[u]), "v"(word_update(w[u], v, first_bits))
                     : "memory");
    }
}

// ---------------------------------------------------------------------------
// Packed (block-compressed) postings -- BASELINE configs[4], di_index_set_packed.
// Every run (a short sublist, or one wave segment's run of a long sublist) is sorted
// by doc and cut into frames of up to 512 postings.  Lane L of a frame holds postings
// 8 L .. 8 L + 7 as eight W-bit fields, W = bd + bv rounded up to a multiple of 4
// (<= 24): field = delta | (value - vmin) << bd, delta = doc - the previous posting's
// doc in the frame (0 for the first), W / 4 dwords per lane, lanes back to back (a
// frame of n postings stores ceil(n / 8) lanes).
// Header (uint4): x = data offset (dwords), y = doc_base (the first doc, 16 bits) |
// count << 16 (10 bits) | bd << 26 (5 bits), z = vmin | bv << 8 (4 bits) | W << 12.
// Decoding happens in registers: the eight fields by static shifts, the lane's
// running delta sums, a DPP wave scan for the lanes before it (no LDS crossbar).
constexpr int PK_FRAME = 512, PK_PER_LANE = 8;

template <int W>
__device__ __forceinline__ void packed_fields(const uint32_t *data, uint32_t cnt, int lane,
                                              uint32_t (&f)[8]) {
    constexpr int ND = W / 4;  // dwords per lane
    static_assert(W % 4 == 0 && W >= 4 && W <= 24, "field width");
    const uint64_t pa = reinterpret_cast<uint64_t>(data);
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)pa);
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
    void *base = reinterpret_cast<void *>(((uint64_t)hi32 << 32) | lo32);
    // the frame's ceil(cnt / 8) lanes of data (lanes past them read 0)
    const int bytes = __builtin_amdgcn_readfirstlane((int)((cnt + PK_PER_LANE - 1) / PK_PER_LANE) * ND * 4);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
    const int off = lane * ND * 4;
    uint32_t d[ND + 1];
    if constexpr (ND == 1) {
        d[0] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
    } else if constexpr (ND == 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, 0);
        d[0] = v[0], d[1] = v[1];
    } else if constexpr (ND == 3) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rsrc, off, 0, 0);
        d[0] = v[0], d[1] = v[1], d[2] = v[2];
    } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
        d[0] = v[0], d[1] = v[1], d[2] = v[2], d[3] = v[3];
        if constexpr (ND == 5) {
            d[4] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 16, 0, 0);
        } else if constexpr (ND == 6) {
            const auto u = __builtin_amdgcn_raw_buffer_load_b64(rsrc, off + 16, 0, 0);
            d[4] = u[0], d[5] = u[1];
        }
    }
    d[ND] = 0;
    constexpr uint32_t mask = (1u << W) - 1u;
#pragma unroll
    for (int i = 0; i < PK_PER_LANE; ++i) {
        const int bit = i * W, k = bit >> 5, sft = bit & 31;
        if (sft + W <= 32)
            f[i] = (d[k] >> sft) & mask;
        else
            f[i] = __builtin_amdgcn_alignbit(d[k + 1], d[k], (uint32_t)sft) & mask;
    }
}

// One frame applied to the block's words (the read-modify-write of scatter_apply);
// OWN: only the docs [dlo, dlo + dn) (the wave's own segment), the rest to the lane's
// dummy word.
template <int W, bool OWN>
__device__ __forceinline__ void packed_apply_w(const uint4 h, const uint32_t *__restrict__ pdata,
                                               int lane, uint32_t first_bits, uint32_t dlo,
                                               uint32_t dn, uint32_t dummy) {
    uint32_t f[PK_PER_LANE];
    const uint32_t base = h.y & 0xFFFFu, cnt = (h.y >> 16) & 1023u, bd = (h.y >> 26) & 31u;
    packed_fields<W>(pdata + h.x, cnt, lane, f);
    const uint32_t vmin = h.z & 255u, bv = (h.z >> 8) & 15u;
    uint32_t run = 0, ds[PK_PER_LANE];
#pragma unroll
    for (int i = 0; i < PK_PER_LANE; ++i) {
        run += __builtin_amdgcn_ubfe(f[i], 0, bd);
        ds[i] = run;
    }
    const uint32_t first = base + wave_incl_scan_dpp(run) - run;  // doc before this lane's
    uint32_t w[PK_PER_LANE], a[PK_PER_LANE];
#pragma unroll
    for (int i = 0; i < PK_PER_LANE; ++i) {
        const uint32_t d = first + ds[i];
        bool ok = (uint32_t)(PK_PER_LANE * lane + i) < cnt;
        if constexpr (OWN) ok = ok && d - dlo < dn;  // (the wave's own docs only)
        a[i] = ok ? d << 2 : dummy;
        asm volatile("ds_read_b32 %0, %1" : "=v"(w[i]) : "v"(a[i]) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < PK_PER_LANE; ++i) asm volatile("" : "+v"(w[i]));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < PK_PER_LANE; ++i) {
        const uint32_t v = vmin + __builtin_amdgcn_ubfe(f[i], bd, bv);
        asm volatile("ds_write_b32 %0, %1" ::"v"(a[i]), "v"(word_update(w[i], v, first_bits))
                     : "memory");
    }
}

template <bool OWN>
__device__ __forceinline__ void packed_apply(const uint4 h, const uint32_t *__restrict__ pdata,
                                             int lane, uint32_t first_bits, uint32_t dlo,
                                             uint32_t dn, uint32_t dummy) {
    switch ((h.z >> 12) & 63u) {  // (wave-uniform)
    case 4: packed_apply_w<4, OWN>(h, pdata, lane, first_bits, dlo, dn, dummy); break;
    case 8: packed_apply_w<8, OWN>(h, pdata, lane, first_bits, dlo, dn, dummy); break;
    case 12: packed_apply_w<12, OWN>(h, pdata, lane, first_bits, dlo, dn, dummy); break;
    case 16: packed_apply_w<16, OWN>(h, pdata, lane, first_bits, dlo, dn, dummy); break;
    case 20: packed_apply_w<20, OWN>(h, pdata, lane, first_bits, dlo, dn, dummy); break;
    default: packed_apply_w<24, OWN>(h, pdata, lane, first_bits, dlo, dn, dummy); break;
    }
}

// Profiling (DI_PROFILE_ABLATE bit 64): per-phase shader cycles of workgroup 0's items
// accumulated here and printed by di_index_search.
__device__ unsigned long long g_sb_phase[12];  // [9] slowest wave's scatter loop, [10] mean

// The (term, block) sublists: sparse per term -- the entries of term t are
// [tb_start[t], tb_start[t+1]), one per block holding postings of t, in block order
// (eblk), at postings [epos[e], epos[e+1]); seg[8e + c] = end of impact class c inside
// the sublist; lid[e] = its long id (per-wave layout) or ~0.  A term present in every
// block is indexed directly; otherwise a binary search over its entries' blocks.
struct SubIndex {
    const uint32_t *tb_start;
    const uint16_t *eblk;
    const uint32_t *epos;
    const uint16_t *seg;
    const uint32_t *lid;
    const uint16_t *wmeta;
    const uint8_t *emax;  // block-max metadata: the sublist's largest value
    const uint8_t *wmax;  // long sublists: the largest value of each wave segment's run
    // packed (block-compressed) postings, di_index_set_packed (null: off): frames of
    // entry e = [pk_fs[e], pk_fs[e + 1]); a long entry's run w = frames pk_fs[e] +
    // [pk_fwt[17 lid + w], pk_fwt[17 lid + w + 1])
    const uint32_t *pk_fs;
    const uint16_t *pk_fwt;
    const uint4 *pk_fh;      // frame headers (PackedFrame)
    const uint32_t *pk_data;
};

// entry of (term t, block b), or -1 when t has no posting in b
__device__ __forceinline__ int64_t find_entry(const SubIndex &si, int nb, uint32_t t, int b) {
    const uint32_t e0 = si.tb_start[t], e1 = si.tb_start[t + 1];
    if (e1 - e0 == (uint32_t)nb) return (int64_t)e0 + b;
    uint32_t lo = e0, hi = e1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (si.eblk[mid] < (uint32_t)b) lo = mid + 1;
        else hi = mid;
    }
    return lo < e1 && si.eblk[lo] == (uint32_t)b ? (int64_t)lo : -1;
}

// [lo, hi) of entry e scored at impact-class prefix min_cls (7: the whole sublist)
__device__ __forceinline__ void entry_bounds(const SubIndex &si, int64_t e, int min_cls,
                                             int64_t &lo, int64_t &hi) {
    if (e < 0) {
        lo = hi = 0;
        return;
    }
    lo = si.epos[e];
    hi = min_cls >= 7 ? (int64_t)si.epos[e + 1] : lo + si.seg[e * 8 + min_cls];
}

// Per (item, query term) setup record, resolved for every item in bulk by
// item_setup_kernel before the scorer: the scorer's setup then reads one record per
// (term, wave segment) instead of walking the dependent chain query term -> entry ->
// per-wave runs (several global round trips per item).
struct ItemRec {
    int64_t lo, hi;        // the term's sublist [lo, hi) in this block (min_cls prefix)
    uint32_t wtab[WSEG];   // per-wave layout: run of wave w = start << 16 | end
    uint32_t flags;        // IR_LONG: per-wave layout; IR_BAD: invalid term id
    uint8_t wmx[WSEG];     // block-max bound of each wave segment (emax / wmax)
    uint32_t pad[3];
};
static_assert(sizeof(ItemRec) % 16 == 0, "records stay 16-byte aligned");
constexpr uint32_t IR_LONG = 1, IR_BAD = 2, IR_PLAIN = 4;
// packed mode: short sublists of fewer postings stay in the plain layout (a frame's
// header and lane rounding would cost more than their 4-byte words)
constexpr uint32_t PK_MIN = 32;

// Items (query q, block b) as the scorer numbers them (item = b * n_q + q); records
// only for queries of 1..WTERMS terms (the scorer's per-wave form), rec_slots per item
// (the batch's longest such query).
__global__ void __launch_bounds__(128)
item_setup_kernel(SubIndex si, int min_cls, int nb, int64_t n_terms,
                  const uint32_t *__restrict__ q_terms, const int32_t *__restrict__ cu_q, int n_q,
                  ItemRec *__restrict__ rec, const uint16_t *__restrict__ border, int rec_slots) {
    const int item = blockIdx.x, q = item % n_q, r_ = item / n_q;
    const int b = border ? (int)border[(int64_t)q * nb + r_] : r_;
    const int q0 = cu_q[q], nt = cu_q[q + 1] - q0;
    if (nt > rec_slots || nt <= 0) return;  // (rec_slots >= every per-wave query's terms)
    ItemRec *r = rec + (int64_t)item * rec_slots;
    for (int e = threadIdx.x; e < nt * WSEG; e += blockDim.x) {
        const int j = e / WSEG, w = e % WSEG;
        const uint32_t t = q_terms[q0 + j];
        if (t >= n_terms) {  // invalid id (device-pointer callers are not pre-checked)
            if (w == 0) {
                r[j].lo = r[j].hi = 0;
                r[j].flags = IR_BAD;
            }
            continue;
        }
        const int64_t en = find_entry(si, nb, t, b);
        const uint32_t id = en >= 0 ? si.lid[en] : 0xFFFFFFFFu;
        if (w == 0) {
            int64_t lo, hi;
            uint32_t fl = id != 0xFFFFFFFFu ? IR_LONG : 0u;
            if (si.pk_fs && en >= 0 && (id != 0xFFFFFFFFu || si.epos[en + 1] - si.epos[en] >= PK_MIN)) {
                // packed: frame ranges (exact scoring only, min_cls 7)
                lo = si.pk_fs[en];
                hi = si.pk_fs[en + 1];
            } else {
                entry_bounds(si, en, min_cls, lo, hi);
                if (si.pk_fs) fl |= IR_PLAIN;
            }
            r[j].lo = lo;
            r[j].hi = hi;
            r[j].flags = fl;
        }
        r[j].wmx[w] = en < 0 ? 0 : id != 0xFFFFFFFFu ? si.wmax[(int64_t)id * WSEG + w] : si.emax[en];
        if (id != 0xFFFFFFFFu) {
            if (si.pk_fs) {
                const uint16_t *m = si.pk_fwt + (int64_t)id * (WSEG + 1);
                r[j].wtab[w] = ((uint32_t)m[w] << 16) | m[w + 1];
            } else {
                const uint16_t *m = si.wmeta + (int64_t)id * (WSEG * 8);
                const uint32_t s0 = w ? m[(w - 1) * 8 + 7] : 0u;
                r[j].wtab[w] = (s0 << 16) | m[w * 8 + min(min_cls, 7)];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Long queries: DI_SHORT_QUERY_TERMS < known terms <= DI_MAX_QUERY_TERMS.  The packed
// score does not hold their sums (255 x 4096 > 2^16) nor the key their first-touch index
// (> 255), so an item (query, block) of such a query accumulates 64-bit words
//     score(20) | (4095 - j)(12) | v_j(8)                       (bits 39..0)
// -- ordered exactly like the short word: score, then first touch -- over half blocks
// of LH_DOCS docs (128 KiB of LDS, the accumulators of ScoreShared), and its candidates
// carry the wide merge key  word << 24 | (0xFFFFFF - doc)  (docs < 2^24).  The first
// half's candidates wait in the item's output list; the second half's selection runs
// over the union (the waiting keys held in registers, LH_HELD per thread) and rewrites
// the list, so a long item emits one list of <= k keys like a short one and the merge
// is unchanged (it decodes wide keys per query, see merge_topk_kernel).  Terms go in
// chunks of MAX_TERMS bounds, a barrier per term.  Rare (no MS MARCO query comes close),
// so simple: one posting per lane per load, a read-modify-write per posting.
__device__ __forceinline__ void score_long_item(
    ScoreShared &sh, int q, int b, const uint32_t *__restrict__ post, const SubIndex &si,
    int min_cls, int nb, int block_docs, int64_t n_terms, uint32_t n_docs, uint32_t doc_lo,
    const uint32_t *__restrict__ q_terms, const int32_t *__restrict__ cu_q, int k,
    uint64_t *__restrict__ ck, int32_t *__restrict__ cn) {
    uint64_t *acc = reinterpret_cast<uint64_t *>(sh.acc);
    int64_t *lo = sh.v.bounds[0], *hi = sh.v.bounds[1];
    const int tid = threadIdx.x;
    const int64_t block_first = (int64_t)b * block_docs;
    const int n_local = (int)min((int64_t)block_docs, (int64_t)n_docs - block_first);
    const int q0 = cu_q[q], nt = cu_q[q + 1] - q0;
    if (n_local <= 0) {
        if (tid == 0) *cn = 0;
        return;
    }
    if ((uint64_t)doc_lo + n_docs > (1ull << 24)) {  // the wide key holds 24-bit docs
        if (tid == 0) *cn = -1;
        return;
    }
    const uint32_t vmin = 1u << (7 - min(min_cls, 7));  // impact pruning: values >= vmin
    uint64_t held[LH_HELD] = {0, 0, 0, 0};
    uint32_t n_held = 0;
    for (int hb = 0; hb < n_local; hb += LH_DOCS) {
        const int hn = min(LH_DOCS, n_local - hb);
        const uint32_t gbase = doc_lo + (uint32_t)(block_first + hb);
        {
            uint4 *a4 = reinterpret_cast<uint4 *>(acc);
            for (int i = tid; i < (hn + 1) / 2; i += SC_THREADS) a4[i] = make_uint4(0, 0, 0, 0);
        }
        if (tid == 0) sh.bad = 0;
        for (int c0 = 0; c0 < nt; c0 += MAX_TERMS) {
            const int cnt = min(MAX_TERMS, nt - c0);
            __syncthreads();  // zeroing done / the previous chunk's bounds no longer read
            for (int j = tid; j < cnt; j += SC_THREADS) {
                const uint32_t t = q_terms[q0 + c0 + j];
                if (t >= n_terms) {
                    sh.bad = 1;
                    lo[j] = hi[j] = 0;
                    continue;
                }
                // the whole sublist: a long sublist is laid out per wave segment (classes
                // in order inside each), so the class prefix is not one range -- pruning
                // (min_cls < 7) filters by value in the scatter instead
                entry_bounds(si, find_entry(si, nb, t, b), 7, lo[j], hi[j]);
            }
            __syncthreads();
            if (sh.bad) {
                if (tid == 0) *cn = -1;
                return;
            }
            for (int jj = 0; jj < cnt; ++jj) {
                const uint64_t fb = (uint64_t)(4095 - (c0 + jj)) << 8;
                const int64_t L = lo[jj], H = hi[jj];
                for (int64_t p0 = L; p0 < H; p0 += 4 * SC_THREADS) {
                    uint32_t r[4];
                    scatter_load<4>(post + p0, H - p0, tid, r);  // past the end: doc 32768, v 0
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t d = ((r[u] ^ POST_X) >> 10) - (uint32_t)hb;
                        const uint64_t v = r[u] & 255u;
                        if (d < (uint32_t)hn && v >= vmin) {  // a doc occurs once per term
                            const uint64_t w = acc[d];
                            acc[d] = w ? w + (v << 20) : (v << 20) | fb | v;
                        }
                    }
                }
                __syncthreads();  // term boundary
            }
        }
        // ---- selection over this half's touched words + the held keys -------------
        auto key_of = [&](uint64_t w, int idx) {
            return (w << 24) | (uint64_t)(0xFFFFFFu - (gbase + (uint32_t)idx));
        };
        uint64_t prefix = 0, mask = 0;
        uint32_t need = (uint32_t)k;
        for (int shift = 56; shift >= 0; shift -= 8) {
            radix_clear<SC_THREADS, SC_WAVES>(sh.u.rs);
            __syncthreads();
            RunLen rl;
            for (int i = 0; i < LH_PER_THREAD; ++i) {
                const int idx = i * SC_THREADS + tid;
                const uint64_t w = idx < hn ? acc[idx] : 0ull;
                if (w) {
                    const uint64_t x = key_of(w, idx);
                    if ((x & mask) == prefix) rl.add(sh.u.rs, (uint32_t)(x >> shift) & 255u);
                }
            }
#pragma unroll
            for (int i = 0; i < LH_HELD; ++i)
                if ((uint32_t)(i * SC_THREADS + tid) < n_held && (held[i] & mask) == prefix)
                    rl.add(sh.u.rs, (uint32_t)(held[i] >> shift) & 255u);
            rl.flush(sh.u.rs);
            __syncthreads();
            radix_pick<SC_THREADS, SC_WAVES>(sh.u.rs, need);
            if (shift == 56 && sh.u.rs.total <= (uint32_t)k) {  // every key is a candidate
                prefix = 0;
                break;
            }
            prefix |= (uint64_t)sh.u.rs.bin << shift;
            mask |= (uint64_t)255 << shift;
            need -= sh.u.rs.above;
        }
        // keys are unique: the keys >= prefix are exactly min(k, total) (prefix = the
        // k-th largest key, or 0 when there are at most k)
        if (tid == 0) sh.emit = 0;
        __syncthreads();
        for (int i = 0; i < LH_PER_THREAD; ++i) {
            const int idx = i * SC_THREADS + tid;
            const uint64_t w = idx < hn ? acc[idx] : 0ull;
            const uint64_t x = w ? key_of(w, idx) : 0ull;
            uint32_t pos;
            if (wave_append(w != 0 && x >= prefix, &sh.emit, pos) && pos < (uint32_t)k) ck[pos] = x;
        }
#pragma unroll
        for (int i = 0; i < LH_HELD; ++i) {
            const bool ok = (uint32_t)(i * SC_THREADS + tid) < n_held && held[i] >= prefix;
            uint32_t pos;
            if (wave_append(ok, &sh.emit, pos) && pos < (uint32_t)k) ck[pos] = held[i];
        }
        __syncthreads();
        n_held = min(sh.emit, (uint32_t)k);
        if (hb + LH_DOCS < n_local) {  // the next half: hold this list (written above)
#pragma unroll
            for (int i = 0; i < LH_HELD; ++i) {
                const uint32_t p = (uint32_t)(i * SC_THREADS + tid);
                held[i] = p < n_held ? ck[p] : 0ull;
            }
        }
        __syncthreads();  // the list is held before the next selection rewrites it
    }
    if (tid == 0) *cn = (int32_t)n_held;
}

// One work item = (query q, doc block b): accumulate, select the block's top-k.
// EXT: the configs[4] extensions -- 0 none (the plain scorer: its code and registers
// stay exactly as without them), EXT_BM block-max skipping over the plain postings
// (bm_factor, per-query block order, the cooperative form), EXT_PK the packed postings
// (si.pk_fs; with or without block-max) -- one kernel each.
constexpr int EXT_BM = 1, EXT_PK = 2, EXT_FEW = 4;  // (EXT_FEW: the emit-above selection of
                                                   // few-block shards, its own kernel so
                                                   // the plain one keeps its code)
template <int EXT>
__device__ __forceinline__ void score_item(ScoreShared &sh, int q, int b,
                                           const uint32_t *__restrict__ post, const SubIndex &si,
                                           int min_cls, int nb,
                                           int block_docs, int64_t n_terms, uint32_t n_docs,
                                           uint32_t doc_lo, const uint32_t *__restrict__ q_terms,
                                           const int32_t *__restrict__ cu_q, int k,
                                           uint64_t *__restrict__ cand_key,
                                           int32_t *__restrict__ cand_n,
                                           uint32_t *__restrict__ qhist, int ablate,
                                           const ItemRec *__restrict__ ir,
                                           uint32_t *__restrict__ long_flag, float bm_factor,
                                           uint32_t *__restrict__ qtq, int kl, int tq_sched) {
    int64_t *lo = sh.v.bounds[0], *hi = sh.v.bounds[1];

    // opaque per item: keeps the per-thread index arithmetic of the sweeps from being
    // hoisted out of the persistent item loop (it spilled there)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t block_first = (int64_t)b * block_docs;
    const int n_local = (int)min((int64_t)block_docs, (int64_t)n_docs - block_first);
    const int q0 = cu_q[q], nt = cu_q[q + 1] - q0;
    uint64_t *ck = cand_key + ((int64_t)q * nb + b) * kl;
    int32_t *cn = cand_n + (int64_t)q * nb + b;

    if (nt > MAX_TERMS && nt <= LONG_TERMS) {  // score_long_kernel's item (it runs next)
        if (tid == 0) {
            *cn = 0;
            *long_flag = 1;
        }
        return;
    }
    if (nt > MAX_TERMS || nt < 0 || n_local <= 0) {
        if (tid == 0) *cn = (nt > MAX_TERMS || nt < 0) ? -1 : 0;
        return;
    }
    const bool fast = nt <= FAST_TERMS;
    const bool stamps = (ablate & 64) && blockIdx.x == 0 && tid == 0;
    uint64_t t_prev = stamps ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int ph) {
        if (stamps) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            atomicAdd(&g_sb_phase[ph], (unsigned long long)(t - t_prev));
            t_prev = t;
        }
    };
    if (tid == 0) {
        sh.bad = 0;
        sh.emit = 0;
        sh.n_tie = 0;
        for (int i = 0; i < WTERMS / 32; ++i) sh.lmask[i] = sh.pmask[i] = 0;
        for (int i = 0; i < WSEG; ++i) sh.wub[i] = 0;
        sh.tq = 0;
    }
    __syncthreads();

    // per-wave form (at most WTERMS terms): every term applied by each wave to its own
    // docs -- long terms over their per-wave runs, short ones read in full by every wave
    // -- so no term needs a barrier; longer queries: the all-wave form, a barrier per term
    const bool wl = nt <= WTERMS && !(ablate & 524288);  // (bit 524288: the all-wave form, A/B)
    // block-max skipping (opt-in, configs[4]): per-wave segment upper bounds (wub)
    // (XBM: the block-max / packed instantiations; EXT_FEW is the plain scorer + the
    // emit-above selection, with only the running-threshold bookkeeping of the others)
    constexpr bool XBM = EXT == EXT_BM || EXT == EXT_PK;
    const bool bm = XBM && bm_factor > 0.0f && wl && qhist != nullptr;
    // block-max: the query's running threshold as one word (qtq, raised by every item's
    // selection with a lower bound of the final k-th score), loaded with the setup's
    // loads -- the skip decision needs no histogram copy, no extra barrier
    // (thread 0 alone loads it and publishes it through LDS at the setup barrier: waves
    // that read the word themselves could see different values -- other CUs raise it --
    // and disagree on skipping, i.e. on which barriers they reach)
    // (few blocks, no qhist: the same word bounds the emit-above selection, see below)
    uint32_t tq_early = 0;
    if (qtq && threadIdx.x == 0)
        tq_early = __hip_atomic_load(&qtq[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // The query's shared threshold histogram (qhist, below) is copied by LDS-DMA into
    // the selection histogram (idle until the selection) here, so its round trip
    // overlaps the scatter and the selection reads it from LDS; the fast selection
    // path zeroes the histogram itself when it runs.
    uint32_t *qh = qhist ? qhist + (int64_t)q * QH_BINS : nullptr;
    // Threshold refresh schedule (tq_sched = first << 16 | every; plain exact scoring with
    // the running word qtq): only the items of blocks b < first and b % every == 0 copy
    // and read the histogram (and raise qtq with the Tq it gives); the others take qtq,
    // one word read with the setup loads -- no 16 KiB copy to wait for, no threshold read.
    // qtq only ever holds lower bounds of the final k-th score, so any schedule is exact.
    const int tq_every = tq_sched & 0xFFFF, tq_first = tq_sched >> 16;
    const bool qpre = qh != nullptr &&
                      (!qtq || tq_every <= 1 || b < tq_first || b % tq_every == 0);
    static_assert(QH_BINS == 4 * SC_THREADS && QH_BINS <= HIST_BINS, "qhist prefetch");
    if (qpre) {
        typedef __attribute__((address_space(3))) void lds_void;
        __builtin_amdgcn_global_load_lds((const void *)(qh + 4 * tid),
                                         (lds_void *)(sh.u.hist + wave * 256), 16, 0, 0);
    }
    // zeroing of the accumulators (and the fast path's histogram): LDS stores only,
    // placed where the setup's global loads are in flight
    auto zero = [&]() {
        uint4 *a4 = reinterpret_cast<uint4 *>(sh.acc);
        const int n4 = (n_local + 3) >> 2;
        for (int i = tid; i < n4; i += SC_THREADS) a4[i] = make_uint4(0, 0, 0, 0);
        if (fast && !qpre) reinterpret_cast<uint4 *>(sh.u.hist)[tid] = make_uint4(0, 0, 0, 0);
        // (the 64 spare bins past them are written, never read: no zeroing needed)
    };
    if (wl && ir != nullptr) {
        // the item's records (item_setup_kernel): one (term j, wave segment w) per thread
        const int e = tid;
        const bool act = e < nt * WSEG;
        const int j = act ? e / WSEG : 0, w = e % WSEG;
        uint32_t f = 0, wt = 0, ub = 0;
        int64_t rlo = 0, rhi = 0;
        if (act) {
            const ItemRec &R = ir[j];
            f = R.flags;
            wt = R.wtab[w];
            if (bm) ub = R.wmx[w];
            if (w == 0) {
                rlo = R.lo;
                rhi = R.hi;
            }
        }
        zero();
        if (act) {
            if (bm && ub) atomicAdd(&sh.wub[w], ub);
            if (w == 0) {
                lo[j] = rlo;
                hi[j] = rhi;
                if (f & IR_BAD) sh.bad = 1;
                if (f & IR_LONG) atomicOr(&sh.lmask[j >> 5], 1u << (j & 31));
                if (EXT == EXT_PK && (f & IR_PLAIN)) atomicOr(&sh.pmask[j >> 5], 1u << (j & 31));
            }
            if (f & IR_LONG) sh.wtab[j][w] = wt;
        }
    } else if (wl) {
        // nt * WSEG <= SC_THREADS: one (term j, wave segment w) per thread.  The entry
        // lookup and the loads that depend on it (bounds, long id) are issued, the
        // accumulators zeroed while they are in flight, then the per-wave runs read.
        static_assert(WTERMS * WSEG <= SC_THREADS, "one setup entry per thread");
        const int e = tid;
        const bool act = e < nt * WSEG;
        const int j = act ? e / WSEG : 0, w = e % WSEG;
        const uint32_t t = act ? q_terms[q0 + j] : 0u;
        const bool tok = act && t < n_terms;  // (device-pointer callers are not pre-checked)
        int64_t en = -1, blo = 0, bhi = 0;
        uint32_t id = 0xFFFFFFFFu, ub = 0;
        if (tok) {
            en = find_entry(si, nb, t, b);
            if (en >= 0) id = si.lid[en];
            if (w == 0) entry_bounds(si, en, min_cls, blo, bhi);
            if (bm && en >= 0)
                ub = id != 0xFFFFFFFFu ? si.wmax[(int64_t)id * WSEG + w] : si.emax[en];
        }
        zero();
        if (bm && ub) atomicAdd(&sh.wub[w], ub);
        if (act && !tok) {  // invalid term id
            if (w == 0) {
                sh.bad = 1;
                lo[j] = hi[j] = 0;
            }
        } else if (act) {
            if (w == 0) {
                lo[j] = blo;
                hi[j] = bhi;
            }
            if (id != 0xFFFFFFFFu) {
                const uint16_t *m = si.wmeta + (int64_t)id * (WSEG * 8);
                const uint32_t s0 = w ? m[(w - 1) * 8 + 7] : 0u;
                sh.wtab[j][w] = (s0 << 16) | m[w * 8 + min(min_cls, 7)];
                if (w == 0) atomicOr(&sh.lmask[j >> 5], 1u << (j & 31));
            }
        }
    } else {
        // all-wave form: whole sublists (a long one is laid out per wave segment, so its
        // class prefix is not one range); impact pruning filters by value (vmin below)
        for (int j = tid; j < nt; j += SC_THREADS) {
            const uint32_t t = q_terms[q0 + j];
            if (t >= n_terms) {
                sh.bad = 1;
                lo[j] = hi[j] = 0;
                continue;
            }
            entry_bounds(si, find_entry(si, nb, t, b), 7, lo[j], hi[j]);
        }
        zero();
    }
    if (qtq && tid == 0) sh.tqe = tq_early;
    __syncthreads();
    if (sh.bad) {
        // (the histogram copy lands before the next item touches the histogram)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) *cn = -1;
        return;
    }

    stamp(0);  // setup + zeroing
    const bool wstamps = (ablate & 64) && blockIdx.x == 0;
    const uint64_t t_w0 = wstamps ? __builtin_amdgcn_s_memtime() : 0;
    // The query's shared threshold (qhist, when given) counts the scores of every
    // candidate its finished blocks emitted (distinct docs, full scores; bin 4095 =
    // 4095 and above).  read_tq -> the largest s with >= k counted candidates scoring
    // >= s: at least k docs score >= s, so the final k-th score is >= s.  A stale
    // (smaller) count still gives a valid lower bound.  Block-wide (barriers).
    auto read_tq = [&]() -> uint32_t {
        // thread t: bins 4t..4t+3 (relaxed atomic loads: other CUs add to them; or the
        // LDS copy made at the item's start)
        uint32_t hv[4], c = 0;
        if (qpre) {
            const uint4 h = reinterpret_cast<const uint4 *>(sh.u.hist)[tid];
            hv[0] = h.x, hv[1] = h.y, hv[2] = h.z, hv[3] = h.w;
            c = h.x + h.y + h.z + h.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                c += (hv[e] = __hip_atomic_load(&qh[4 * tid + e], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));
        }
        uint32_t sfx = wave_suffix_sum(c);
        if (lane == 0) sh.wsum[wave] = sfx;
        if (tid == 0) sh.tq = 0;
        __syncthreads();
        for (int w2 = wave + 1; w2 < SC_WAVES; ++w2) sfx += sh.wsum[w2];
        // one thread holds the crossing: count(>= 4t + e) >= k > count(>= 4t + e + 1)
        if (sfx >= (uint32_t)k && sfx - c < (uint32_t)k) {
            uint32_t above = sfx - c;
            int e = 3;
            for (; e > 0; --e) {
                if (above + hv[e] >= (uint32_t)k) break;
                above += hv[e];
            }
            sh.tq = (uint32_t)(4 * tid + e);
        }
        __syncthreads();
        const uint32_t r = sh.tq;
        __syncthreads();  // (wsum / tq are reused)
        return r;
    };
    // Block-max skipping (bm, opt-in; configs[4]): a wave segment whose upper bound
    // wub = sum over the query terms of the segment's largest value in their sublists
    // stays below the query's shared threshold Tq cannot hold a top-k doc (every doc of
    // it scores <= wub < Tq <= the final k-th score): its wave skips its scatter and its
    // docs stay 0.  bm_factor 1 is exact; > 1 skips segments below factor x Tq -- an
    // approximation (the QPS-vs-recall sweep).  Every segment below: the item ends.
    bool skip_wave = false;
    uint32_t live16 = 0xFFFFu;  // bm: the wave segments that are scored (bit w)
    if (bm) {
        uint32_t tq0;
        if (qtq) {
            tq0 = sh.tqe;  // (written before the setup barrier)
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the threshold copy (read_tq)
            tq0 = read_tq();
        }
        const float thr = bm_factor * (float)tq0;
        skip_wave = tq0 > 0 && (float)sh.wub[wave] < thr && !(ablate & 131072);  // (bit 131072: no skips, A/B)
        // every segment below: lanes 0..15 of each wave check one each (no block
        // reduction: __syncthreads_and would take static LDS, and the scatter needs the
        // dynamic segment at address 0)
        static_assert(WSEG <= 64, "one lane per segment");
        const bool below = lane >= WSEG || (tq0 > 0 && (float)sh.wub[lane] < thr);
        const uint64_t below_m = __ballot(below);
        const bool all_below = below_m == ~0ull && !(ablate & 131072);
        live16 = (uint32_t)~below_m & 0xFFFFu;
        // skip statistics (di_index_timing "bm_segments" / "bm_segments_skipped"): every
        // evaluated item counts its WSEG segments, every skipped segment one -- in the
        // workgroup's LDS, added to the device counters once per workgroup at the kernel's
        // end (an atomic per item and skipping wave on one address cost tens of ms per
        // 8.8 M-doc batch)
        if (tid == 0) {
            sh.bm_cnt[0] += WSEG;
            sh.bm_cnt[1] += (unsigned long long)__builtin_popcount(~live16 & 0xFFFFu);
        }
        if (all_below) {
            // the item's threshold-histogram copy (LDS-DMA into sh.u.hist) lands before
            // the next item uses that LDS (it would overwrite the next query's copy)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (tid == 0) *cn = 0;
            return;
        }
    }
    // ---- scatter: terms in query order, barrier between terms -------------
    // A term's sublist goes in rounds of 16 postings per lane while 16 k remain, then
    // 4 per lane while more than 1 k remain, then 1: a short tail does not pay for a
    // full round of issue (loads, LDS reads and writes of masked lanes).  Each round
    // has all its loads in flight before any is applied; the 16 waves of the CU
    // overlap one another's load latency with their LDS work.
    // The last round of a term also loads the next term's first 4 k postings, before
    // the term barrier (a raw one: LDS writes retired, loads left in flight), so the
    // barrier does not expose a load round trip per term.
    // A long term (per-wave layout) is scattered by each wave over its own doc segment,
    // rounds of up to 16 postings per lane: no other wave touches those docs, so a run
    // of long terms needs no barrier between its terms, only at its ends.
    uint32_t pre[4];
    bool have_pre = false;
    auto is_long = [&](int j) { return wl && ((sh.lmask[j >> 5] >> (j & 31)) & 1u); };
    const uint32_t wseg = ((uint32_t)block_docs + WSEG - 1) / WSEG;
    // (A cooperative form -- every wave on every scored segment, barriers between terms,
    // so that a skipped segment's wave does not idle -- measured no faster at 8.8 M skewed
    // docs, 45.8 k vs 46.3 k q/s, and was removed; round-4 DESIGN §3.)
    if (EXT == 0) {
        // (the plain kernel: the per-wave / all-wave loops below)
    } else if (EXT == EXT_PK && si.pk_fs && wl) {
        // packed postings (configs[4]), the per-wave form of the plain scorer: a long
        // term's frames of the wave's own segment run; a short term read whole by every
        // wave (its frame, or its plain words when short of PK_MIN), applied to the
        // wave's own docs only -- no barrier between terms; a skipped segment's wave
        // scores nothing (skip_wave)
        const uint32_t wd = (uint32_t)(MAX_BLOCK_DOCS + lane) << 2;
        const uint32_t dlo = (uint32_t)wave * wseg;
        const uint32_t dn = wave == WSEG - 1 ? 0x7FFFFFFFu - dlo : wseg;
        for (int j = skip_wave ? nt : 0; j < nt; ++j) {
            const uint32_t first_bits = (uint32_t)(255 - j) << 8;
            if (is_long(j)) {
                const uint32_t se = sh.wtab[j][wave];
                const int64_t f1 = lo[j] + (se & 0xFFFFu);
                for (int64_t f = lo[j] + (se >> 16); f < f1; ++f)
                    packed_apply<false>(si.pk_fh[f], si.pk_data, lane, first_bits, 0u, 0x7FFFFFFFu, wd);
            } else if ((sh.pmask[j >> 5] >> (j & 31)) & 1u) {
                for (int64_t pos = lo[j], end = hi[j]; pos < end;) {
                    const int64_t rem = end - pos;
                    if (rem > 4 * 64) {
                        uint32_t r[8];
                        scatter_load<8, 64>(post + pos, rem, lane, r, true);
                        scatter_apply_own<8>(r, first_bits, dlo, dn, wd);
                        pos += 8 * 64;
                    } else if (rem > 64) {
                        uint32_t r[4];
                        scatter_load<4, 64>(post + pos, rem, lane, r, true);
                        scatter_apply_own<4>(r, first_bits, dlo, dn, wd);
                        pos = end;
                    } else {
                        uint32_t r[1];
                        scatter_load<1, 64>(post + pos, rem, lane, r);
                        scatter_apply_own<1>(r, first_bits, dlo, dn, wd);
                        pos = end;
                    }
                }
            } else {
                for (int64_t f = lo[j]; f < hi[j]; ++f)
                    packed_apply<true>(si.pk_fh[f], si.pk_data, lane, first_bits, dlo, dn, wd);
            }
        }
        skip_wave = true;  // (nothing left for the per-wave loop below)
    }
    const uint32_t wdlo = (uint32_t)wave * wseg;
    const uint32_t wdn = wave == WSEG - 1 ? 0x7FFFFFFFu - wdlo : wseg;  // last: the rest
    const uint32_t wdummy = (uint32_t)(MAX_BLOCK_DOCS + lane) << 2;
    const uint32_t vmin = 1u << (7 - min(min_cls, 7));  // all-wave form: pruning by value
    const bool x4 = !(ablate & 4096);  // rounds of 4k postings per lane by 16-byte loads (bit 4096: 4-byte, A/B)
    for (int j = (ablate & 1) || skip_wave ? nt : 0; j < nt; ++j) {  // ablate bit 0: skip (profiling)
        const uint32_t first_bits = (uint32_t)(255 - j) << 8;
        const bool lj = is_long(j);
        if (lj) {
            const uint32_t se = sh.wtab[j][wave];
            int64_t pos = lo[j] + (se >> 16);
            const int64_t end = lo[j] + (se & 0xFFFFu);
            while (pos < end) {
                const int64_t rem = end - pos;
                if (rem > 8 * 64) {
                    uint32_t r[16];
                    scatter_load<16, 64>(post + pos, rem, lane, r, x4);
                    scatter_apply<16>(sh.acc, r, first_bits);
                    pos += 16 * 64;
                } else if (rem > 4 * 64) {
                    uint32_t r[8];
                    scatter_load<8, 64>(post + pos, rem, lane, r, x4);
                    scatter_apply<8>(sh.acc, r, first_bits);
                    pos = end;
                } else if (rem > 64) {
                    uint32_t r[4];
                    scatter_load<4, 64>(post + pos, rem, lane, r, x4);
                    scatter_apply<4>(sh.acc, r, first_bits);
                    pos = end;
                } else {
                    uint32_t r[1];
                    scatter_load<1, 64>(post + pos, rem, lane, r);
                    scatter_apply<1>(sh.acc, r, first_bits);
                    pos = end;
                }
            }
            continue;
        }
        if (wl) {
            // a short term (< WLONG_MIN postings in the block): every wave reads the whole
            // sublist and applies the postings of its own doc segment -- no barrier
            for (int64_t pos = lo[j], end = hi[j]; pos < end;) {
                const int64_t rem = end - pos;
                if (rem > 8 * 64) {
                    uint32_t r[16];
                    scatter_load<16, 64>(post + pos, rem, lane, r, x4);
                    scatter_apply_own<16>(r, first_bits, wdlo, wdn, wdummy);
                    pos += 16 * 64;
                } else if (rem > 4 * 64) {
                    uint32_t r[8];
                    scatter_load<8, 64>(post + pos, rem, lane, r, x4);
                    scatter_apply_own<8>(r, first_bits, wdlo, wdn, wdummy);
                    pos = end;
                } else if (rem > 64) {
                    uint32_t r[4];
                    scatter_load<4, 64>(post + pos, rem, lane, r, x4);
                    scatter_apply_own<4>(r, first_bits, wdlo, wdn, wdummy);
                    pos = end;
                } else {
                    uint32_t r[1];
                    scatter_load<1, 64>(post + pos, rem, lane, r);
                    scatter_apply_own<1>(r, first_bits, wdlo, wdn, wdummy);
                    pos = end;
                }
            }
            continue;
        }
        int64_t pos = lo[j];
        const int64_t end = hi[j];
        if (have_pre) {
            scatter_apply<4, true>(sh.acc, pre, first_bits, vmin);
            pos = min(end, pos + (int64_t)4 * SC_THREADS);
            have_pre = false;
        }
        const bool next = j + 1 < nt && hi[j + 1] > lo[j + 1] && !is_long(j + 1);
        auto prefetch_next = [&]() {
            scatter_load<4>(post + lo[j + 1], hi[j + 1] - lo[j + 1], tid, pre, x4);
            have_pre = true;
        };
        while (pos < end) {
            const int64_t rem = end - pos;
            if (rem >= 16 * SC_THREADS) {
                uint32_t r[16];
                scatter_load<16>(post + pos, rem, tid, r, x4);
                if (rem == 16 * SC_THREADS && next) prefetch_next();
                scatter_apply<16, true>(sh.acc, r, first_bits, vmin);
                pos += 16 * SC_THREADS;
            } else if (rem > SC_THREADS) {
                uint32_t r[4];
                scatter_load<4>(post + pos, rem, tid, r, x4);
                if (rem <= 4 * SC_THREADS && next) prefetch_next();
                scatter_apply<4, true>(sh.acc, r, first_bits, vmin);
                pos += 4 * SC_THREADS;
            } else {
                uint32_t r[1];
                scatter_load<1>(post + pos, rem, tid, r);
                if (next) prefetch_next();
                scatter_apply<1, true>(sh.acc, r, first_bits, vmin);
                pos = end;
            }
        }
        // term boundary: this term's LDS writes land before any wave reads the next
        if (j + 1 < nt) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // the asm LDS writes; the threshold histogram's LDS-DMA copy.  The first half of the
    // threshold read (read_tq) goes before the barrier: thread t's own 4 bins are the
    // 16 B its own LDS-DMA wrote (no barrier needed to read them), their wave suffix
    // sums go to wsum -- the barrier the scatter needs anyway publishes them.
    if (wstamps && lane == 0) sh.wstamp[wave] = (uint32_t)(__builtin_amdgcn_s_memtime() - t_w0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    uint32_t tq_hv[4] = {0, 0, 0, 0}, tq_c = 0, tq_sfx = 0;
    if (qpre) {
        const uint4 h = reinterpret_cast<const uint4 *>(sh.u.hist)[tid];
        tq_hv[0] = h.x, tq_hv[1] = h.y, tq_hv[2] = h.z, tq_hv[3] = h.w;
        tq_c = h.x + h.y + h.z + h.w;
        tq_sfx = wave_suffix_sum(tq_c);
        if (lane == 0) sh.wsum[wave] = tq_sfx;
    }
    __syncthreads();

    stamp(1);  // scatter
    if (stamps) {
        uint32_t mx = 0, sm = 0;
        for (int w2 = 0; w2 < SC_WAVES; ++w2) {
            mx = max(mx, sh.wstamp[w2]);
            sm += sh.wstamp[w2];
        }
        atomicAdd(&g_sb_phase[9], (unsigned long long)mx);
        atomicAdd(&g_sb_phase[10], (unsigned long long)(sm / SC_WAVES));
    }
    if (ablate & 2) {  // profiling: skip the selection
        if (tid == 0) *cn = 0;
        return;
    }
    const uint64_t doc_base = (uint64_t)doc_lo + (uint64_t)block_first;
    // Candidates are staged in the unused tail of the accumulator array when they fit
    // there and copied out coalesced (a lane-scattered 8-byte store per candidate slot
    // costs a store instruction per slot and wave); else they go straight out.
    const int n4z = (n_local + 3) >> 2;
    const bool tail_fits = 2 * k <= MAX_BLOCK_DOCS - 4 * n4z;
    uint64_t *const acc_tail = reinterpret_cast<uint64_t *>(sh.acc + 4 * n4z);
    // (full blocks leave no tail: the one-sweep selections below stage in the histogram
    // area instead, free by then -- otherwise the flush re-read the keys from global
    // memory, a round trip per item at 1.1 M / 8.8 M docs)
    uint64_t *const hist_stage = reinterpret_cast<uint64_t *>(sh.u.hist);
    static_assert(sizeof(ScoreShared().u) >= (size_t)HIST_BINS * 4, "histogram stage");
    const bool hist_fits = (uint32_t)k * 8u <= (uint32_t)HIST_BINS * 4u;
    uint64_t *stage = tail_fits ? acc_tail : nullptr;  // null: straight to ck
    uint32_t cap = (uint32_t)k;  // list capacity of the current selection (emit-above: kl)
    auto cand = [&](uint32_t pos, uint32_t w, int idx) {
        const uint32_t doc = (uint32_t)(doc_base + (uint64_t)idx);
        const uint64_t key = ((uint64_t)w << 32) | (uint64_t)(0xFFFFFFFFu - doc);
        if (pos < cap) {
            if (stage)
                stage[pos] = key;
            else
                ck[pos] = key;
        }
    };
    // final candidates: copied out (staged) and counted into the query's score
    // histogram (qhist, see read_tq); called once per item, after a barrier
    auto flush = [&](uint32_t n_c) {
        // (thread order reversed: the last waves issue these stores and atomics, so the
        // next item's record loads -- issued by the first waves -- do not wait for their
        // acknowledgements behind them in the in-order vmcnt)
        for (uint32_t i = (uint32_t)(SC_THREADS - 1 - tid); i < n_c; i += SC_THREADS) {
            const uint64_t key = stage ? stage[i] : ck[i];
            if (stage) ck[i] = key;
            if (qh) atomicAdd(&qh[min((uint32_t)(key >> 48), (uint32_t)QH_BINS - 1)], 1u);
        }
    };
    auto emit_all_touched = [&]() {
        const uint32_t n = compact_words(sh, n_local, tid, [](uint32_t w, int) { return w ? 1u : 0u; },
                                         [&](int, uint32_t pos, uint32_t w, int idx) {
                                             cand(pos, w, idx);
                                         });
        flush(min(n & 0xFFFFu, (uint32_t)k));
        if (tid == 0) *cn = (int32_t)min(n & 0xFFFFu, (uint32_t)k);
    };

    // Shared per-query threshold.  qhist[q] (when given) counts the scores of every
    // candidate the query's finished blocks emitted (distinct docs, full scores; bin
    // 4095 = 4095 and above).  Tq = the largest s with >= k counted candidates scoring
    // >= s: at least k docs score >= Tq, so the final k-th score is >= Tq and a doc
    // below Tq cannot be in the query's top-k.  When at most k of this block's docs
    // reach Tq they are its only candidates (no histogram, no tie order -- the merge
    // orders them by key); else the full selection below runs.  Items run block-major
    // (all queries' block 0 first), so Tq is close to the final k-th score after the
    // first blocks and the later blocks emit few candidates.  A stale (smaller) count
    // still gives a valid lower bound.
    // Emit-above (few blocks: no qhist, a list capacity kl > k): the query's running
    // threshold T1 (qtq = the largest k-th score of its finished blocks' full selections,
    // read at the item's start) is a lower bound of its final k-th score, so only this
    // block's docs scoring >= T1 can reach the top-k.  When at most kl of them do, one
    // append sweep emits them all -- no histogram, no tie order, no compaction (the merge
    // orders by key); else the full selection below runs (and raises qtq).  Items are
    // block-major, so every block after a query's first finds the first block's k-th
    // score: at 100 k docs (4 blocks) ~k docs of each pass it, <= kl = 2 k.
    if (EXT == EXT_FEW && !qh && qtq && kl > k) {
        const uint32_t T1 = sh.tqe;  // (written before the setup barrier)
        if (T1 > 0) {
            const bool tail_kl = 2 * kl <= MAX_BLOCK_DOCS - 4 * n4z;
            if (!tail_kl && (uint32_t)kl * 8u <= (uint32_t)HIST_BINS * 4u) stage = hist_stage;
            else if (!tail_kl) stage = nullptr;
            cap = (uint32_t)kl;
            const uint32_t thr_w = T1 << 16;
            sweep_words(sh.acc, n_local, tid, [&](uint32_t w, int idx) {
                uint32_t pos;
                if (wave_append<true>(w >= thr_w, &sh.emit, pos)) cand(pos, w, idx);
            });
            __syncthreads();
            const uint32_t na = sh.emit;
            if (na <= (uint32_t)kl) {
                flush(na);
                if (tid == 0) *cn = (int32_t)na;
                return;
            }
            // (too many: the full selection, k keys; sh.emit is reset by the paths that use
            // it -- the radix ties set it, the fast path's compaction does not read it)
            // The sweep may have staged up to kl keys in the histogram area (a near-full
            // block leaves no accumulator tail); the fast path counts into those bins and
            // they were zeroed only at the setup, so zero them again here.
            if (fast && stage == hist_stage) reinterpret_cast<uint4 *>(sh.u.hist)[tid] = make_uint4(0, 0, 0, 0);
            cap = (uint32_t)k;
            stage = tail_fits ? acc_tail : nullptr;
            __syncthreads();  // every wave has read sh.emit (and the bins are zero again)
            if (tid == 0) sh.emit = 0;
        }
    }
    uint32_t Tq = 0;
    bool hist_dirty = false;  // keys staged in the histogram area by a sweep that overflowed
    if (qh) {
        if (qpre) {
            // second half of read_tq over the suffix sums published by the scatter
            // barrier: the crossing thread writes tq (0 from the item's start when the
            // histogram holds fewer than k candidates); one barrier
            for (int w2 = wave + 1; w2 < SC_WAVES; ++w2) tq_sfx += sh.wsum[w2];
            if (tq_sfx >= (uint32_t)k && tq_sfx - tq_c < (uint32_t)k) {
                uint32_t above = tq_sfx - tq_c;
                int e = 3;
                for (; e > 0; --e) {
                    if (above + tq_hv[e] >= (uint32_t)k) break;
                    above += tq_hv[e];
                }
                sh.tq = (uint32_t)(4 * tid + e);
            }
            __syncthreads();
            Tq = sh.tq;
        } else {
            Tq = sh.tqe;  // (the running word, published by the setup barrier)
        }
        if (tid == 0) sh.tqn = max(sh.tqn, Tq);
        stamp(8);  // threshold read (the part of tq-select before the sweep)
        // (wsum is written again only after a barrier of the selection below; tq only
        // at the next item's start)
        if (Tq > 0) {
            // one sweep: the docs reaching Tq (usually a few dozen) are appended by
            // wave-aggregated LDS atomics in any order (the merge orders them by key)
            // (the histogram copy is consumed: its area stages the keys of a full block)
            if (!tail_fits && hist_fits && !(ablate & 1048576)) stage = hist_stage;
            const uint32_t thr_w = Tq << 16;
            sweep_words(sh.acc, n_local, tid, [&](uint32_t w, int idx) {
                uint32_t pos;
                if (wave_append<XBM>(w >= thr_w, &sh.emit, pos)) cand(pos, w, idx);
            });
            __syncthreads();
            const uint32_t na = sh.emit;
            stamp(7);  // shared-threshold selection
            if (na <= (uint32_t)k) {
                flush(na);
                if (tid == 0) *cn = (int32_t)na;
                return;
            }
            hist_dirty = stage == hist_stage;
            stage = tail_fits ? acc_tail : nullptr;  // (the selections below use the histogram)
        }
    }

    if (EXT == EXT_BM && fast) {
        // A sparse item: at most k postings were scattered, so at most k docs are touched
        // and every touched doc is a candidate.  One append sweep (any order: the merge
        // orders by key) replaces the histogram sweep (an LDS atomic per word) and the two
        // compaction sweeps.  Every wave sums the scattered postings itself from the LDS
        // bounds (lane j: term j; a long term: its per-wave runs), so the branch is uniform
        // with no barrier.  In the EXT_BM instantiation only, which impact-pruned searches
        // use (di_index_search): in the plain kernel the same code cost the dense 100 k-doc
        // items 4% (2.148 vs 2.062 ms per launch, profiles/round4_p5_sparse_items_ab.txt);
        // here it takes 8.8 M skewed docs at min_impact 128 from 70.6 to 48.9 ms per batch.
        uint32_t np = 0;
        if (lane < nt) {
            if (is_long(lane)) {
#pragma unroll
                for (int w = 0; w < WSEG; ++w) {
                    const uint32_t se = sh.wtab[lane][w];
                    const uint32_t s0 = se >> 16, s1 = se & 0xFFFFu;
                    np += s1 > s0 ? s1 - s0 : 0u;
                }
            } else {
                np = (uint32_t)min(hi[lane] - lo[lane], (int64_t)0xFFFFFF);
            }
        }
        np = (uint32_t)__shfl(wave_prefix_sum(np), 63, 64);
        if (np <= (uint32_t)k) {
            if (!tail_fits && hist_fits && !(ablate & 1048576)) stage = hist_stage;
            sweep_words(sh.acc, n_local, tid, [&](uint32_t w, int idx) {
                uint32_t pos;
                if (wave_append<true>(w != 0, &sh.emit, pos)) cand(pos, w, idx);
            });
            __syncthreads();
            const uint32_t na = sh.emit;
            flush(na);
            if (tid == 0) *cn = (int32_t)na;
            return;
        }
    }

    uint32_t prefix = 0, mask = 0, need = (uint32_t)k;
    int shift = 24;  // next digit of the general radix path
    if (fast) {
        // ---- fast path: score histogram -> k-th score T -------------------
        uint32_t *hist = sh.u.hist;
        // branch-free: an untouched doc (w = 0) counts into a per-lane spare bin past
        // the 4096 score bins (no same-address conflicts), never read
        const uint32_t spare = HIST_BINS + (uint32_t)lane;
        if (qpre || hist_dirty) {  // the threshold copy was read (read_tq's barriers), or
            // keys were staged there: zero the bins
            reinterpret_cast<uint4 *>(hist)[tid] = make_uint4(0, 0, 0, 0);
            __syncthreads();
        }
        sweep_words(sh.acc, n_local, tid, [&](uint32_t w, int) {
            atomicAdd(&hist[w ? (w >> 16) : spare], 1u);
        });
        __syncthreads();
        // thread t owns bins 4t..4t+3; s = touched docs with score >= 4t
        const uint4 h4 = reinterpret_cast<const uint4 *>(hist)[tid];
        const uint32_t c = h4.x + h4.y + h4.z + h4.w;
        uint32_t s = wave_suffix_sum(c);
        if (lane == 0) sh.wsum[wave] = s;
        __syncthreads();
        uint32_t total = 0;
        for (int w2 = 0; w2 < SC_WAVES; ++w2) {
            const uint32_t x = sh.wsum[w2];
            total += x;
            if (w2 > wave) s += x;
        }
        __syncthreads();  // wsum is reused by the compaction
        if (total <= (uint32_t)k) {  // every touched doc is a candidate
            emit_all_touched();
            return;
        }
        if (s >= need && s - c < need) {  // exactly one thread: T is in its bins
            const uint32_t hv[4] = {h4.x, h4.y, h4.z, h4.w};
            uint32_t above = s - c;
            int e = 3;
            for (; e > 0; --e) {
                if (above + hv[e] >= need) break;
                above += hv[e];
            }
            sh.thr = (uint32_t)(4 * tid + e);
            sh.above = above;
            sh.ties = hv[e];
        }
        __syncthreads();
        stamp(2);  // histogram + threshold
        if (ablate & 4) {  // profiling: stop after the threshold
            if (tid == 0) *cn = 0;
            return;
        }
        // (this block alone has >= k docs scoring >= T: a lower bound of the query's final
        // k-th score for block-max, qtq)
        if (tid == 0) sh.tqn = max(sh.tqn, sh.thr);
        const uint32_t T = sh.thr, ties = sh.ties;  // T >= 1: every touched score is
        const uint32_t above = sh.above;             // nonzero

        need -= above;
        if (ties == need || ties <= (uint32_t)TIE_CAP) {
            // scores above T are in; the ties at T all go in, or into a list (the
            // histogram is consumed) as (low 16 bits of the word, 0xFFFF - idx):
            // unique, and larger = first-touch earlier, then doc smaller.
            // Compaction: one sweep marks each lane's candidates and ties in two
            // 32-bit masks over its 32 words (4 per ds_read_b128); a block scan of the
            // counts gives positions; the write loop visits only the marked words
            // (~1 per lane), not all 32.
            const bool all_ties = ties == need;
            const uint32_t thr_a = (all_ties ? T : T + 1) << 16;  // list A: w >= thr_a
            uint32_t *tl = sh.u.hist;
            uint32_t ma = 0, mb = 0;
            {
                const uint4 *a4 = reinterpret_cast<const uint4 *>(sh.acc);
                const int n4 = (n_local + 3) >> 2;
#pragma unroll
                for (int i = 0; i < SC_PER_THREAD / 4; ++i) {
                    const int q4 = i * SC_THREADS + tid;
                    const uint4 y = a4[q4];  // q4 < 8192: inside the array
                    const bool ok = q4 < n4;
                    const uint32_t wv[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const uint32_t w = ok ? wv[e] : 0u;
                        ma |= (uint32_t)(w >= thr_a) << (4 * i + e);
                        mb |= (uint32_t)((w >> 16) == T) << (4 * i + e);
                    }
                }
                if (all_ties) mb = 0;
            }
            const uint32_t cnt = (uint32_t)__builtin_popcount(ma) +
                                 ((uint32_t)__builtin_popcount(mb) << 16);
            const uint32_t incl = wave_prefix_sum(cnt);
            if (lane == 63) sh.wsum[wave] = incl;
            __syncthreads();
            uint32_t base = incl - cnt;
            for (int w2 = 0; w2 < wave; ++w2) base += sh.wsum[w2];
            stamp(6);
            {
                uint32_t pa = base & 0xFFFFu, pb = base >> 16;
                auto idx_of = [&](int bit) { return 4 * ((bit >> 2) * SC_THREADS + tid) + (bit & 3); };
                while (ma) {
                    const int bit = __builtin_ctz(ma);
                    ma &= ma - 1;
                    const int idx = idx_of(bit);
                    cand(pa++, sh.acc[idx], idx);
                }
                while (mb) {
                    const int bit = __builtin_ctz(mb);
                    mb &= mb - 1;
                    const int idx = idx_of(bit);
                    tl[pb++] = ((sh.acc[idx] & 0xFFFFu) << 16) | (0xFFFFu - (uint32_t)idx);
                }
            }
            __syncthreads();
            stamp(3);  // compaction
            if (ablate & 8) {  // profiling: stop after the compaction
                if (tid == 0) *cn = 0;
                return;
            }
            if (!all_ties && ties <= 64) {
                // few ties (the common case): one wave ranks them -- lane i holds tie
                // key i and counts the larger keys among all lanes (keys are unique);
                // the `need` largest go right after the `above` candidates, in rank
                // order, with no atomics and no further block barrier
                if (wave == 0) {
                    const uint32_t x = lane < (int)ties ? tl[lane] : 0u;
                    uint32_t rank = 0;
                    for (int j = 0; j < (int)ties; ++j) rank += __shfl(x, j, 64) > x;
                    if (lane < (int)ties && rank < need)
                        cand(above + rank, (T << 16) | (x >> 16), (int)(0xFFFFu - (x & 0xFFFFu)));
                }
                __syncthreads();
                stamp(4);  // tie order
                flush((uint32_t)k);
                stamp(5);  // copy-out
                if (tid == 0) *cn = k;
            } else if (!all_ties) {
                // radix select of the `need` largest tie keys (4 digits)
                uint32_t *h = sh.v.h256;
                uint32_t tp = 0, tm = 0, tneed = need;
                for (int sft = 24; sft >= 0; sft -= 8) {
                    if (tid < 256) h[tid] = 0;
                    __syncthreads();
                    for (uint32_t i = tid; i < ties; i += SC_THREADS) {
                        const uint32_t x = tl[i];
                        if ((x & tm) == tp) atomicAdd(&h[(x >> sft) & 255u], 1u);
                    }
                    __syncthreads();
                    if (wave == 0) {
                        const uint32_t c4 = h[4 * lane] + h[4 * lane + 1] + h[4 * lane + 2] +
                                            h[4 * lane + 3];
                        const uint32_t S = wave_suffix_sum(c4);
                        if (S >= tneed && S - c4 < tneed) {
                            uint32_t ab = S - c4;
                            int e = 3;
                            for (; e > 0; --e) {
                                const uint32_t he = h[4 * lane + e];
                                if (ab + he >= tneed) break;
                                ab += he;
                            }
                            sh.bin = (uint32_t)(4 * lane + e);
                            sh.bin_above = ab;
                        }
                    }
                    __syncthreads();
                    tp |= sh.bin << sft;
                    tm |= 255u << sft;
                    tneed -= sh.bin_above;
                }
                // the keys are unique: exactly `need` ties are >= tp; they follow the
                // `above` candidates
                if (tid == 0) sh.emit = above;
                __syncthreads();
                for (uint32_t i0 = 0; i0 < ties; i0 += SC_THREADS) {
                    const uint32_t i = i0 + tid;
                    const uint32_t x = i < ties ? tl[i] : 0u;
                    uint32_t pos;
                    if (wave_append<XBM>(i < ties && x >= tp, &sh.emit, pos))
                        cand(pos, (T << 16) | (x >> 16), (int)(0xFFFFu - (x & 0xFFFFu)));
                }
                __syncthreads();
                flush((uint32_t)k);
                // sh.emit == k by construction; anything else is a selection bug
                if (tid == 0) *cn = sh.emit == (uint32_t)k ? k : -2;
            } else {
                flush((uint32_t)k);
                if (tid == 0) *cn = k;
            }
            return;
        }
        // more ties than the list holds: the general path finishes from score T
        // (digits 15..8 and 7..0 of the word, then doc order)
        prefix = T << 16;
        mask = 0xFFFF0000u;
        shift = 8;
    }

    // ---- general path: block-wide radix select on the 32-bit words ----------
    auto id_key = [](uint32_t w, int) { return w; };
    if (shift == 24) {  // pass 0 also counts touched docs
        score_radix_pass(sh, n_local, 24, need, id_key,
                         [](uint32_t w, int, uint32_t) { return w != 0; });
        if (sh.u.rs.total <= (uint32_t)k) {
            __syncthreads();
            emit_all_touched();
            return;
        }
    } else {
        score_radix_pass(sh, n_local, shift, need, id_key,
                         [prefix, mask](uint32_t w, int, uint32_t) {
                             return w != 0 && (w & mask) == prefix;
                         });
    }
    for (;; shift -= 8) {
        prefix |= sh.u.rs.bin << shift;
        mask |= 255u << shift;
        need -= sh.u.rs.above;
        if (shift == 0) break;
        __syncthreads();
        score_radix_pass(sh, n_local, shift - 8, need, id_key,
                         [prefix, mask](uint32_t w, int, uint32_t) {
                             return w != 0 && (w & mask) == prefix;
                         });
    }
    const uint32_t T = prefix;
    if (tid == 0) sh.tqn = max(sh.tqn, T >> 16);
    const uint32_t ties = sh.u.rs.tot[sh.u.rs.bin];

    // doc-order cut among the ties: the `need` smallest doc indices
    // (all ties when exactly `need` of them exist)
    uint32_t dcut = 0;
    if (ties != need) {
        uint32_t dneed = need, dprefix = 0, dmask = 0;
        auto dkey = [](uint32_t, int idx) { return 0xFFFFu - (uint32_t)idx; };
        for (int sft = 8;; sft -= 8) {
            __syncthreads();
            score_radix_pass(sh, n_local, sft, dneed, dkey,
                             [T, dprefix, dmask](uint32_t w, int, uint32_t kk) {
                                 return w == T && (kk & dmask) == dprefix;
                             });
            dprefix |= sh.u.rs.bin << sft;
            dmask |= 255u << sft;
            dneed -= sh.u.rs.above;
            if (sft == 0) break;
        }
        dcut = dprefix;  // keep ties whose (0xFFFF - idx) >= dcut
    }
    __syncthreads();
    const uint32_t n = compact_words(
        sh, n_local, tid,
        [T, dcut](uint32_t w, int idx) -> uint32_t {
            return (w != 0 && (w > T || (w == T && (0xFFFFu - (uint32_t)idx) >= dcut))) ? 1u : 0u;
        },
        [&](int, uint32_t pos, uint32_t w, int idx) { cand(pos, w, idx); });
    flush((uint32_t)k);
    // exactly k by construction; anything else is a selection bug -> flag it
    if (tid == 0) *cn = (n & 0xFFFFu) == (uint32_t)k ? k : -2;
}

// Block order of each query for block-max scoring (BASELINE configs[4]): blocks by
// descending upper bound sum_j emax(t_j, b) (ties: block order), so the query's shared
// threshold -- the k-th score among the candidates of its finished blocks -- rises to
// near its final value within the first blocks and the later, weaker blocks skip more
// of their wave segments.  Any order is exact (the threshold is a lower bound of the
// final k-th score whatever blocks it has seen; the merge orders by key).  One
// workgroup per query; rank by counting (nb <= BO_MAX_BLOCKS).
constexpr int BO_MAX_BLOCKS = 1024;
__global__ void __launch_bounds__(256)
block_order_kernel(SubIndex si, int nb, int64_t n_terms, const uint32_t *__restrict__ q_terms,
                   const int32_t *__restrict__ cu_q, uint16_t *__restrict__ border) {
    __shared__ uint32_t bound[BO_MAX_BLOCKS];
    const int q = blockIdx.x;
    const int q0 = cu_q[q], nt = cu_q[q + 1] - q0;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        uint32_t u = 0;
        for (int j = 0; j < nt && j < WTERMS; ++j) {
            const uint32_t t = q_terms[q0 + j];
            if (t >= n_terms) continue;
            const int64_t e = find_entry(si, nb, t, b);
            if (e >= 0) u += si.emax[e];
        }
        bound[b] = u;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        const uint32_t u = bound[b];
        int r = 0;
        for (int x = 0; x < nb; ++x) {
            const uint32_t v = bound[x];
            r += v > u || (v == u && x < b);
        }
        border[(int64_t)q * nb + r] = (uint16_t)b;
    }
}

// Persistent: one workgroup per CU walks the (query, block) items, so the per-
// workgroup launch cost (16 waves, 154 KiB of LDS) is paid once per CU, not per item.
template <int EXT>
__global__ void __launch_bounds__(SC_THREADS)
score_blocks_kernel(const uint32_t *__restrict__ post, SubIndex si, int min_cls, int nb,
                    int block_docs, int64_t n_terms, uint32_t n_docs, uint32_t doc_lo,
                    const uint32_t *__restrict__ q_terms, const int32_t *__restrict__ cu_q, int k,
                    uint64_t *__restrict__ cand_key, int32_t *__restrict__ cand_n, int n_items,
                    int n_q, uint32_t *__restrict__ qhist, int ablate,
                    const ItemRec *__restrict__ rec, uint32_t *__restrict__ long_flag,
                    float bm_factor, unsigned long long *__restrict__ bm_stat,
                    const uint16_t *__restrict__ border, uint32_t *__restrict__ qtq,
                    int rec_slots, int kl, int tq_sched) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ScoreShared &sh = *reinterpret_cast<ScoreShared *>(smem);
    if ((uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char *)smem) != 0) {
        // scatter_apply addresses the accumulators from LDS address 0 (folded away when
        // the segment starts there, as it does): otherwise fail every item loudly
        for (int item = blockIdx.x; item < n_items; item += gridDim.x)
            if (threadIdx.x == 0) cand_n[item] = -1;
        return;
    }
    if (threadIdx.x == 0) {  // (the first item's barriers publish them)
        sh.bm_cnt[0] = sh.bm_cnt[1] = 0ull;
        sh.tqn = 0;
    }
    // items block-major: item = b * n_q + q (the shared threshold, see score_item)
    for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
        const int q = item % n_q, r_ = item / n_q;
        score_item<EXT>(sh, q, (EXT == EXT_BM || EXT == EXT_PK) && border ? (int)border[(int64_t)q * nb + r_] : r_, post, si,
                   min_cls, nb,
                   block_docs, n_terms,
                   n_docs, doc_lo, q_terms, cu_q, k, cand_key, cand_n, qhist, ablate,
                   rec ? rec + (int64_t)item * rec_slots : nullptr, long_flag, bm_factor, qtq, kl,
                   tq_sched);
        __syncthreads();  // every wave is done with the LDS of this item
        // the item's threshold into the query's running one, here rather than inside the
        // selection: qtq and the value read at the item's start need no registers across
        // the scatter (they cost the instantiation spills)
        if (threadIdx.x == 0) {
            const uint32_t t = sh.tqn;
            if (qtq && t > sh.tqe) atomicMax(&qtq[q], t);
            sh.tqn = 0;
        }
    }
    if ((EXT == EXT_BM || EXT == EXT_PK) && bm_stat && threadIdx.x == 0 && sh.bm_cnt[0]) {
        atomicAdd(&bm_stat[0], sh.bm_cnt[0]);
        atomicAdd(&bm_stat[1], sh.bm_cnt[1]);
    }
}

// The items of the long queries (score_long_item), after score_blocks_kernel on the
// same stream: it gave them no candidates and raised *long_flag (0: every workgroup
// leaves at once).  Persistent: every workgroup lists the long queries of each round of
// SC_THREADS queries in query order (a block scan: the same list in every workgroup)
// and takes its share of their (query, block) items.
__global__ void __launch_bounds__(SC_THREADS)
score_long_kernel(const uint32_t *__restrict__ post, SubIndex si, int min_cls, int nb,
                  int block_docs, int64_t n_terms, uint32_t n_docs, uint32_t doc_lo,
                  const uint32_t *__restrict__ q_terms, const int32_t *__restrict__ cu_q, int k,
                  uint64_t *__restrict__ cand_key, int32_t *__restrict__ cand_n, int n_q,
                  const uint32_t *__restrict__ long_flag, int kl) {
    if (__builtin_amdgcn_readfirstlane(*long_flag) == 0) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ScoreShared &sh = *reinterpret_cast<ScoreShared *>(smem);
    uint32_t *list = &sh.wtab[0][0];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int r0 = 0; r0 < n_q; r0 += SC_THREADS) {
        const int q = r0 + tid;
        int nt = 0;
        if (q < n_q) nt = cu_q[q + 1] - cu_q[q];
        const uint32_t is_long = nt > MAX_TERMS && nt <= LONG_TERMS ? 1u : 0u;
        const uint32_t incl = wave_prefix_sum(is_long);
        if (lane == 63) sh.wsum[wave] = incl;
        __syncthreads();
        uint32_t base = incl - is_long, n = 0;
        for (int w2 = 0; w2 < SC_WAVES; ++w2) {
            const uint32_t x = sh.wsum[w2];
            if (w2 < wave) base += x;
            n += x;
        }
        if (is_long) list[base] = (uint32_t)q;
        __syncthreads();
        const int n_items = (int)n * nb;
        for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
            const int lq = (int)list[it % n], b = it / n;
            score_long_item(sh, lq, b, post, si, min_cls, nb, block_docs, n_terms, n_docs,
                            doc_lo, q_terms, cu_q, k, cand_key + ((int64_t)lq * nb + b) * kl,
                            cand_n + (int64_t)lq * nb + b);
            __syncthreads();  // the item's LDS (and the list) stay consistent
        }
        __syncthreads();  // the list and wsum are rewritten by the next round
    }
}

// ---------------------------------------------------------------------------
// merge: per query, the top-k of n_lists candidate lists by 64-bit key
// ---------------------------------------------------------------------------
constexpr int MG_LDS_KEYS = 16384;  // fast path: every candidate fits in LDS

// Selection without a sort (fast path, > MG_SEL_MIN candidates, see the kernel):
// a 4096-bin histogram of the keys' score bits, then counting ranks.
constexpr int MG_SEL_MIN = 1024;
constexpr int MG_SEL_BINS = 4096;   // 16 KiB of LDS after the key array
constexpr int MG_SEL_KEYS = 2048;   // + 16 KiB: up to 2048 selected keys
constexpr int MG_SEL_CAP = 8192;    // key arrays up to 64 KiB (+32 KiB within the LDS max)

template <int THREADS>
struct alignas(16) MergeHead {  // 16-byte multiple: the u64 key array follows it
    RadixScratch<THREADS / 64> rs;
    int32_t off[1025];
    uint32_t cnt;
    int32_t bad;
    uint32_t thr, above;
    uint32_t wtot[THREADS / 64];
};

enum DecodeMode : int { DECODE_QUANT = 0, DECODE_SPARSE = 1, DECODE_NONE = 2 };

// keys: the LDS key array holds `cap` entries (power of two, <= MG_LDS_KEYS)
template <int THREADS>
__global__ void __launch_bounds__(THREADS)
merge_topk_kernel(const uint64_t *__restrict__ keys, const int32_t *__restrict__ counts,
                  int n_lists, int k_in, int k, int64_t list_stride, int64_t cnt_stride,
                  int64_t q_stride, int64_t cq_stride, int cap,
                  uint64_t *__restrict__ out_key, uint32_t *__restrict__ out_doc,
                  uint32_t *__restrict__ out_score, int32_t *__restrict__ out_n, int mode,
                  int select, const int32_t *__restrict__ cu_q) {
    // key i of list l of query q: keys[q*q_stride + l*list_stride + i]
    // its count:                  counts[q*cq_stride + l*cnt_stride]
    constexpr int WAVES = THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    MergeHead<THREADS> &sh = *reinterpret_cast<MergeHead<THREADS> *>(smem);
    static_assert(sizeof(MergeHead<THREADS>) % 16 == 0, "key array must stay 16-byte aligned");
    uint64_t *lk = reinterpret_cast<uint64_t *>(smem + sizeof(MergeHead<THREADS>));
    const int q = blockIdx.x, tid = threadIdx.x;
    const int32_t *cnt0 = counts + (int64_t)q * cq_stride;
    auto cnt = [&](int l) { return cnt0[(int64_t)l * cnt_stride]; };
    const uint64_t *src0 = keys + (int64_t)q * q_stride;

    if (tid == 0) sh.bad = 0;
    __syncthreads();
    int64_t total = 0;
    const bool fast_lists = n_lists <= 1024;
    if (fast_lists) {
        // list offsets by a block scan (thread t owns lists LPT t .. LPT t + LPT - 1):
        // a serial scan by one thread cost ~10 us per query at 269 lists
        constexpr int LPT = (1024 + THREADS - 1) / THREADS;
        int c[LPT];
        uint32_t run = 0;
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const int l = tid * LPT + j;
            c[j] = l < n_lists ? cnt(l) : 0;
            if (c[j] < 0) sh.bad = 1;
            c[j] = min(max(c[j], 0), k_in);
            run += (uint32_t)c[j];
        }
        const uint32_t incl = wave_prefix_sum(run);
        const int lane = tid & 63, w = tid >> 6;
        if (lane == 63) sh.wtot[w] = incl;
        __syncthreads();
        uint32_t base = incl - run;
        for (int v = 0; v < w; ++v) base += sh.wtot[v];
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const int l = tid * LPT + j;
            base += (uint32_t)c[j];
            if (l < n_lists) sh.off[l + 1] = (int32_t)base;
        }
        if (tid == 0) sh.off[0] = 0;
        __syncthreads();
        total = sh.off[n_lists];
    } else {
        int64_t part = 0;
        for (int l = tid; l < n_lists; l += THREADS) {
            int c = cnt(l);
            if (c < 0) sh.bad = 1;
            part += min(max(c, 0), k_in);
        }
        if (tid == 0) sh.cnt = 0;
        __syncthreads();
        atomicAdd(&sh.cnt, (uint32_t)part);
        __syncthreads();
        total = sh.cnt;
        __syncthreads();
    }
    if (sh.bad) {
        if (tid == 0) out_n[q] = -1;
        return;
    }
    const int take = (int)min<int64_t>(total, k);
    uint64_t *ok = out_key ? out_key + (int64_t)q * k : nullptr;
    if (fast_lists && total <= cap) {
        // flattened over the lists, 8 loads per lane in flight (clamped addresses:
        // unconditional loads), list of key i by binary search over the offsets
        constexpr int U = 8;
        const int tot = (int)total;
        for (int base = 0; base < tot; base += U * THREADS) {
            uint64_t v[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int i = min(base + j * THREADS + tid, tot - 1);
                int lo = 0, hi = n_lists - 1;  // last list with off[l] <= i
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (sh.off[mid] <= i) lo = mid;
                    else hi = mid - 1;
                }
                v[j] = src0[(int64_t)lo * list_stride + (i - sh.off[lo])];
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int i = base + j * THREADS + tid;
                if (i < tot) lk[i] = v[j];
            }
        }
        __syncthreads();
    }
    // Over the LDS capacity (many lists, e.g. the early blocks of an 8.8 M-doc query
    // emitted full lists before the shared threshold rose): two passes over the lists, a
    // wave per list -- the score histogram of every key, then only the keys in bins at or
    // above the take-th key's bin into LDS -- and the selection below on those.  Every
    // key >= the take-th largest is kept, so the result is the same.  Wide keys (score
    // bits past 4095), or more kept keys than the LDS holds: the radix select below.
    // (select bit 2: on; DI_PROFILE_MERGE=2 turns it off, A/B)
    bool over = !(fast_lists && total <= cap);
    if (over && fast_lists && (select & 2) && cap > MG_SEL_MIN && cap <= MG_SEL_CAP) {
        uint32_t *hist = reinterpret_cast<uint32_t *>(lk + cap);
        auto bin = [](uint64_t x) { return (uint32_t)(x >> 48) & (MG_SEL_BINS - 1); };
        for (int i = tid; i < MG_SEL_BINS; i += THREADS) hist[i] = 0;
        if (tid == 0) sh.cnt = 0;
        __syncthreads();
        const int lane = tid & 63, w = tid >> 6;
        constexpr int UL = 4;  // loads per lane in flight
        bool big = false;
        for (int l = w; l < n_lists; l += WAVES) {
            const int o = sh.off[l], c = sh.off[l + 1] - o;
            const uint64_t *src = src0 + (int64_t)l * list_stride;
            for (int i0 = 0; i0 < c; i0 += UL * 64) {
                uint64_t v[UL];
#pragma unroll
                for (int u = 0; u < UL; ++u) {
                    const int i = i0 + u * 64 + lane;
                    v[u] = i < c ? src[i] : 0ull;
                }
#pragma unroll
                for (int u = 0; u < UL; ++u) {
                    if (i0 + u * 64 + lane < c) {
                        big |= (v[u] >> 60) != 0;
                        atomicAdd(&hist[bin(v[u])], 1u);
                    }
                }
            }
        }
        if (!__syncthreads_or(big)) {
            // T = the bin of the take-th largest key, n_keep = the keys in bins >= T
            constexpr int BPT = MG_SEL_BINS / THREADS;
            const int top = MG_SEL_BINS - 1 - tid * BPT;
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < BPT; ++j) c += hist[top - j];
            const uint32_t incl = wave_prefix_sum(c);
            if (lane == 63) sh.wtot[w] = incl;
            __syncthreads();
            uint32_t run = incl - c;
            for (int v = 0; v < w; ++v) run += sh.wtot[v];
#pragma unroll
            for (int j = 0; j < BPT; ++j) {
                const uint32_t h = hist[top - j];
                if (run < (uint32_t)take && run + h >= (uint32_t)take) {
                    sh.thr = (uint32_t)(top - j);
                    sh.above = run + h;
                }
                run += h;
            }
            __syncthreads();
            const uint32_t T = sh.thr, n_keep = sh.above;
            if (n_keep <= (uint32_t)cap) {
                for (int l = w; l < n_lists; l += WAVES) {
                    const int o = sh.off[l], c2 = sh.off[l + 1] - o;
                    const uint64_t *src = src0 + (int64_t)l * list_stride;
                    for (int i0 = 0; i0 < c2; i0 += UL * 64) {
                        uint64_t v[UL];
#pragma unroll
                        for (int u = 0; u < UL; ++u) {
                            const int i = i0 + u * 64 + lane;
                            v[u] = i < c2 ? src[i] : 0ull;
                        }
#pragma unroll
                        for (int u = 0; u < UL; ++u) {
                            uint32_t pos;
                            const bool keep = i0 + u * 64 + lane < c2 && bin(v[u]) >= T;
                            if (wave_append(keep, &sh.cnt, pos)) lk[pos] = v[u];
                        }
                    }
                }
                __syncthreads();
                total = n_keep;
                over = false;
            }
        }
        __syncthreads();  // (the histogram area is reused by the selection)
    }
    if (over) {
        // slow path: radix select the take-th largest key straight from global
        uint64_t prefix = 0, mask = 0;
        uint32_t need = (uint32_t)take;
        for (int shift = 56; shift >= 0; shift -= 8) {
            radix_clear<THREADS, WAVES>(sh.rs);
            __syncthreads();
            RunLen rl;
            for (int l = 0; l < n_lists; ++l) {
                int c = min(cnt(l), k_in);
                const uint64_t *s = src0 + (int64_t)l * list_stride;
                for (int i = tid; i < c; i += THREADS) {
                    uint64_t x = s[i];
                    if ((x & mask) == prefix) rl.add(sh.rs, (uint32_t)(x >> shift) & 255u);
                }
            }
            rl.flush(sh.rs);
            __syncthreads();
            radix_pick<THREADS, WAVES>(sh.rs, need);
            prefix |= (uint64_t)sh.rs.bin << shift;
            mask |= (uint64_t)255 << shift;
            need -= sh.rs.above;
            __syncthreads();
        }
        // keys are unique: exactly `take` keys are >= prefix
        if (tid == 0) sh.cnt = 0;
        __syncthreads();
        for (int l = 0; l < n_lists; ++l) {
            int c = min(cnt(l), k_in);
            const uint64_t *s = src0 + (int64_t)l * list_stride;
            for (int i = tid; i < c; i += THREADS) {
                uint64_t x = s[i];
                if (x >= prefix) {
                    uint32_t pos = atomicAdd(&sh.cnt, 1u);
                    if (pos < (uint32_t)cap) lk[pos] = x;
                }
            }
        }
        __syncthreads();
        total = take;
    }
    // a long query's keys are wide (score_long_item)
    const bool wide = mode == DECODE_QUANT && cu_q && cu_q[q + 1] - cu_q[q] > MAX_TERMS;
    auto emit = [&](int i, uint64_t x) {  // output rank i
        if (ok) ok[i] = x;
        if (mode == DECODE_QUANT) {
            out_doc[(int64_t)q * k + i] =
                wide ? 0xFFFFFFu - (uint32_t)(x & 0xFFFFFFu) : 0xFFFFFFFFu - (uint32_t)x;
            out_score[(int64_t)q * k + i] = (uint32_t)(x >> (wide ? 44 : 48));
        } else if (mode == DECODE_SPARSE) {
            out_doc[(int64_t)q * k + i] = 0xFFFFFFu - (uint32_t)(x & 0xFFFFFFu);
            out_score[(int64_t)q * k + i] = (uint32_t)(x >> 32);  // f32 bits
        }
    };
    if (select && fast_lists && total > MG_SEL_MIN && cap <= MG_SEL_CAP && take < total) {
        // Selection by counting instead of a sort.  Every key below 2^60 (score <
        // 4096)?  Then bin = key bits 48..59 (the score) orders the keys up to ties
        // inside a bin: a histogram gives the bin T of the take-th largest key and
        // every bin's start rank; the keys of bins >= T are placed bin by bin, and a
        // key's rank is its bin's start + the keys of its own bin that are larger.
        bool big = false;
        for (int i = tid; i < total; i += THREADS) big |= (lk[i] >> 60) != 0;
        if (!__syncthreads_or(big)) {
            uint32_t *hist = reinterpret_cast<uint32_t *>(lk + cap);
            uint64_t *out = reinterpret_cast<uint64_t *>(hist + MG_SEL_BINS);
            auto bin = [](uint64_t x) { return (uint32_t)(x >> 48) & (MG_SEL_BINS - 1); };
            for (int i = tid; i < MG_SEL_BINS; i += THREADS) hist[i] = 0;
            __syncthreads();
            for (int i = tid; i < total; i += THREADS) atomicAdd(&hist[bin(lk[i])], 1u);
            __syncthreads();
            // thread t owns BPT consecutive bins from the top, in descending order
            constexpr int BPT = MG_SEL_BINS / THREADS;
            const int top = MG_SEL_BINS - 1 - tid * BPT;
            uint32_t hc[BPT], c = 0;
#pragma unroll
            for (int j = 0; j < BPT; ++j) c += (hc[j] = hist[top - j]);
            const uint32_t incl = wave_prefix_sum(c);
            const int lane = tid & 63, w = tid >> 6;
            if (lane == 63) sh.wtot[w] = incl;
            __syncthreads();
            uint32_t run = incl - c;
            for (int v = 0; v < w; ++v) run += sh.wtot[v];
            // counts -> start ranks (keys in higher bins); T = the take-th key's bin
#pragma unroll
            for (int j = 0; j < BPT; ++j) {
                if (run < (uint32_t)take && run + hc[j] >= (uint32_t)take) {
                    sh.thr = (uint32_t)(top - j);
                    sh.above = run + hc[j];  // keys in bins >= T
                }
                hist[top - j] = run;
                run += hc[j];
            }
            __syncthreads();
            const uint32_t T = sh.thr, n_sel = sh.above;
            if (n_sel <= (uint32_t)MG_SEL_KEYS) {
                // place (hist[b] becomes the end of bin b = the start of bin b - 1)
                for (int i = tid; i < total; i += THREADS) {
                    const uint64_t x = lk[i];
                    const uint32_t b = bin(x);
                    if (b >= T) out[atomicAdd(&hist[b], 1u)] = x;
                }
                __syncthreads();
                for (int p = tid; p < (int)n_sel; p += THREADS) {
                    const uint64_t x = out[p];
                    const uint32_t b = bin(x);
                    const uint32_t lo = b == MG_SEL_BINS - 1 ? 0u : hist[b + 1], hi = hist[b];
                    uint32_t r = lo;
                    for (uint32_t j = lo; j < hi; ++j) r += out[j] > x;
                    if (r < (uint32_t)take) emit((int)r, x);
                }
                if (tid == 0) out_n[q] = take;
                return;
            }
            __syncthreads();  // (the sort below reuses nothing of this)
        }
    }
    int n2 = 64;
    while (n2 < total) n2 <<= 1;
    for (int i = (int)total + tid; i < n2; i += THREADS) lk[i] = 0;
    __syncthreads();
    bitonic_sort_desc<THREADS>(lk, n2);
    for (int i = tid; i < take; i += THREADS) emit(i, lk[i]);
    if (tid == 0) out_n[q] = take;
}

// Merge of few short lists (n_lists <= MS_LISTS, all candidates <= MS_U per thread,
// k <= MG_SEL_KEYS; the 4-block x 1000-candidate retrieve merge): the candidates stay
// in registers (MS_U per thread), the score histogram and the selected keys are the
// only LDS -- 33 KiB instead of the general kernel's 77 KiB, so four workgroups share
// a CU instead of two.  Same selection as merge_topk_kernel's counting path; keys at or
// past score 4096 (wide keys), more than MG_SEL_KEYS selected keys or at most
// MG_SEL_MIN candidates take a radix select over the registers and a sort of the take
// winners in the same LDS.  Output identical to merge_topk_kernel (the keys are unique
// and totally ordered).
constexpr int MS_LISTS = 64;  // (MS_U: candidates per thread, 8, or 16 for the few-block
                               // emit-above lists of up to 2 k keys)

template <int THREADS>
struct alignas(16) MergeSelHead {
    union {
        RadixScratch<THREADS / 64> rs;
        uint32_t hist[MG_SEL_BINS];
    } u;
    int32_t off[MS_LISTS + 1];
    uint32_t thr, above, cnt, pad;
};

template <int THREADS, int MS_U = 8>
__global__ void __launch_bounds__(THREADS)
merge_sel_kernel(const uint64_t *__restrict__ keys, const int32_t *__restrict__ counts,
                 int n_lists, int k_in, int k, int64_t list_stride, int64_t cnt_stride,
                 int64_t q_stride, int64_t cq_stride, uint64_t *__restrict__ out_key,
                 uint32_t *__restrict__ out_doc, uint32_t *__restrict__ out_score,
                 int32_t *__restrict__ out_n, int mode, const int32_t *__restrict__ cu_q) {
    constexpr int WAVES = THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    MergeSelHead<THREADS> &sh = *reinterpret_cast<MergeSelHead<THREADS> *>(smem);
    static_assert(sizeof(MergeSelHead<THREADS>) % 16 == 0, "key array must stay 16-byte aligned");
    uint64_t *out = reinterpret_cast<uint64_t *>(smem + sizeof(MergeSelHead<THREADS>));
    const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int32_t *cnt0 = counts + (int64_t)q * cq_stride;
    const uint64_t *src0 = keys + (int64_t)q * q_stride;

    // list offsets (one wave; n_lists <= 64); a negative count marks a rejected query
    if (tid < 64) {
        int c = lane < n_lists ? cnt0[(int64_t)lane * cnt_stride] : 0;
        const bool bad = __any(c < 0);
        c = min(max(c, 0), k_in);
        const uint32_t incl = wave_prefix_sum((uint32_t)c);
        if (lane < n_lists) sh.off[lane + 1] = (int32_t)incl;
        if (lane == 0) {
            sh.off[0] = 0;
            sh.cnt = bad ? 1u : 0u;
        }
    }
    __syncthreads();
    if (sh.cnt) {
        if (tid == 0) out_n[q] = -1;
        return;
    }
    const int total = sh.off[n_lists];
    const int take = min(total, k);
    // the candidates, MS_U per thread (i = j THREADS + tid), in registers
    uint64_t v[MS_U];
#pragma unroll
    for (int j = 0; j < MS_U; ++j) {
        const int i = min(j * THREADS + tid, max(total - 1, 0));
        int lo = 0, hi = n_lists - 1;  // last list with off[l] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (sh.off[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        v[j] = total > 0 ? src0[(int64_t)lo * list_stride + (i - sh.off[lo])] : 0;
    }
    auto valid = [&](int j) { return j * THREADS + tid < total; };
    const bool wide = mode == DECODE_QUANT && cu_q && cu_q[q + 1] - cu_q[q] > MAX_TERMS;
    uint64_t *ok = out_key ? out_key + (int64_t)q * k : nullptr;
    auto emit = [&](int i, uint64_t x) {  // output rank i
        if (ok) ok[i] = x;
        if (mode == DECODE_QUANT) {
            out_doc[(int64_t)q * k + i] =
                wide ? 0xFFFFFFu - (uint32_t)(x & 0xFFFFFFu) : 0xFFFFFFFFu - (uint32_t)x;
            out_score[(int64_t)q * k + i] = (uint32_t)(x >> (wide ? 44 : 48));
        } else if (mode == DECODE_SPARSE) {
            out_doc[(int64_t)q * k + i] = 0xFFFFFFu - (uint32_t)(x & 0xFFFFFFu);
            out_score[(int64_t)q * k + i] = (uint32_t)(x >> 32);  // f32 bits
        }
    };
    bool big = false;
#pragma unroll
    for (int j = 0; j < MS_U; ++j) big |= valid(j) && (v[j] >> 60) != 0;
    const bool counting = !__syncthreads_or(big) && total > MG_SEL_MIN && take < total;
    if (counting) {
        // counting selection (merge_topk_kernel's): bin = key bits 48..59 (the score)
        uint32_t *hist = sh.u.hist;
        auto bin = [](uint64_t x) { return (uint32_t)(x >> 48) & (MG_SEL_BINS - 1); };
        for (int i = tid; i < MG_SEL_BINS; i += THREADS) hist[i] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < MS_U; ++j)
            if (valid(j)) atomicAdd(&hist[bin(v[j])], 1u);
        __syncthreads();
        constexpr int BPT = MG_SEL_BINS / THREADS;
        const int top = MG_SEL_BINS - 1 - tid * BPT;
        uint32_t hc[BPT], c = 0;
#pragma unroll
        for (int j = 0; j < BPT; ++j) c += (hc[j] = hist[top - j]);
        const uint32_t incl = wave_prefix_sum(c);
        const int w = tid >> 6;
        __syncthreads();  // (every thread read its bins; the wave totals go to off's tail)
        uint32_t *wtot = reinterpret_cast<uint32_t *>(out);  // (out is idle until placing)
        if (lane == 63) wtot[w] = incl;
        __syncthreads();
        uint32_t run = incl - c;
        for (int u = 0; u < w; ++u) run += wtot[u];
#pragma unroll
        for (int j = 0; j < BPT; ++j) {
            if (run < (uint32_t)take && run + hc[j] >= (uint32_t)take) {
                sh.thr = (uint32_t)(top - j);
                sh.above = run + hc[j];  // keys in bins >= T
            }
            hist[top - j] = run;
            run += hc[j];
        }
        __syncthreads();
        const uint32_t T = sh.thr, n_sel = sh.above;
        if (n_sel <= (uint32_t)MG_SEL_KEYS) {
#pragma unroll
            for (int j = 0; j < MS_U; ++j)
                if (valid(j) && bin(v[j]) >= T) out[atomicAdd(&hist[bin(v[j])], 1u)] = v[j];
            __syncthreads();
            for (int p = tid; p < (int)n_sel; p += THREADS) {
                const uint64_t x = out[p];
                const uint32_t b = bin(x);
                const uint32_t lo = b == MG_SEL_BINS - 1 ? 0u : hist[b + 1], hi = hist[b];
                uint32_t r = lo;
                for (uint32_t j = lo; j < hi; ++j) r += out[j] > x;
                if (r < (uint32_t)take) emit((int)r, x);
            }
            if (tid == 0) out_n[q] = take;
            return;
        }
        __syncthreads();  // (the radix select below reuses the histogram's LDS)
    }
    // radix select of the take-th largest key over the registers, then the take winners
    // (keys are unique: exactly `take` are >= the selected prefix) sorted in LDS
    uint64_t prefix = 0, mask = 0;
    uint32_t need = (uint32_t)take;
    if (take < total) {
        for (int shift = 56; shift >= 0; shift -= 8) {
            radix_clear<THREADS, WAVES>(sh.u.rs);
            __syncthreads();
            RunLen rl;
#pragma unroll
            for (int j = 0; j < MS_U; ++j)
                if (valid(j) && (v[j] & mask) == prefix)
                    rl.add(sh.u.rs, (uint32_t)(v[j] >> shift) & 255u);
            rl.flush(sh.u.rs);
            __syncthreads();
            radix_pick<THREADS, WAVES>(sh.u.rs, need);
            prefix |= (uint64_t)sh.u.rs.bin << shift;
            mask |= (uint64_t)255 << shift;
            need -= sh.u.rs.above;
            __syncthreads();
        }
    }
    if (tid == 0) sh.cnt = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MS_U; ++j)
        if (valid(j) && v[j] >= prefix) out[atomicAdd(&sh.cnt, 1u)] = v[j];
    int n2 = 64;
    while (n2 < take) n2 <<= 1;
    __syncthreads();
    for (int i = take + tid; i < n2; i += THREADS) out[i] = 0;
    __syncthreads();
    bitonic_sort_desc<THREADS>(out, n2);
    for (int i = tid; i < take; i += THREADS) emit(i, out[i]);
    if (tid == 0) out_n[q] = take;
}

}  // namespace di

// ===========================================================================
// host side
// ===========================================================================
using namespace di;

struct di_index {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int64_t n_terms = 0, n_post = 0, n_ent = 0, n_long = 0;
    uint32_t n_docs = 0, doc_lo = 0;  // shard [doc_lo, doc_lo + n_docs)
    int nb = 0, block_docs = 0;
    int min_cls = 7;                 // impact-class prefix scored (7 = every posting: exact)
    float bm_factor = 0.0f;          // block-max skipping: 0 off, 1 exact, > 1 approximate
    // postings and the sparse (term, block) entries (SubIndex)
    DevBuf post, tb_start, eblk, epos, seg, lid, wmeta, emax, wmax;
    DevBuf post_flat;      // exact scoring: the per-wave runs dealt flat (build_index)
    bool has_flat = false;
    // the posting array a search reads: flat for exact scoring, class-ordered under pruning
    const uint32_t *post_for(int mc) const {
        return has_flat && mc >= 7 ? post_flat.as<uint32_t>() : post.as<uint32_t>();
    }
    DevBuf ws_q, ws_cu, ws_ck, ws_cn, ws_doc, ws_score, ws_n, ws_key, ws_thr;
    DevBuf ws_rec;  // ItemRec per (item, term slot): item_setup_kernel -> score_blocks
    DevBuf ws_long;  // score_blocks -> score_long_kernel: the batch has long queries
    DevBuf bm_stat;  // block-max statistics: u64 {segments evaluated, segments skipped}
    DevBuf ws_border;  // block-max: each query's block order (block_order_kernel)
    DevBuf ws_tq;      // block-max: each query's running threshold (one word)
    // packed (block-compressed) postings, built by di_index_set_packed (SubIndex pk_*)
    DevBuf pk_fs, pk_fwt, pk_fh, pk_data;
    bool pk_built = false, packed = false;
    int64_t pk_frames = 0, pk_bytes = 0;
    // per-query threshold shared across blocks: -1 = auto (on from 8 blocks: at 4 blocks it
    // measured 2.31 vs 2.14 ms per 6980-query batch, at 34 / 269 blocks 16.9 vs 19.5 and
    // 130 vs 161 ms, merge 0.5 vs 7.1 and 1.4 vs 74 ms); DI_SCORE_THRESHOLD=0 / 1 forces
    int shared_thr = -1;
    bool block_order = false;  // DI_BLOCK_ORDER=1: block-max items in per-query bound order
    // threshold refresh schedule (score_item): with the shared threshold, the items of
    // blocks b < tq_first and b % tq_every == 0 read the query's histogram, the others
    // the running word qtq (DI_TQ_EVERY / DI_TQ_FIRST; tq_every 1: every item reads it,
    // as before round 6).  8 / 4 from the sweep (profiles/round6_d_tq_sweep_*.json, one
    // box): 8.8 M skewed docs 94.0 -> 102.7 k q/s (score_blocks 70.7 -> 64.0 ms per
    // 6980-query batch), 1.1 M docs 14.47 -> 14.13-14.23 ms; 4 / 0 and 8 / 0 were slower
    // at 1.1 M (their stale thresholds overflow more sweeps), 16 / 4 and 32 / 8 no faster.
    int tq_every = 8, tq_first = 4;
    int ablate = 0;  // DI_PROFILE_ABLATE: profiling only (1 no scatter, 2 no selection, 4 stop at the k-th score)
    Timer timer;

    // Few blocks (2..7, no shared qhist threshold): the emit-above selection (score_item)
    // lists up to 2 k keys per (query, block) against the running threshold qtq
    // (DI_PROFILE_ABLATE bit 2097152: off, A/B).  One predicate for search and reserve.
    bool few_blocks(int k) const {
        return nb >= 2 && nb < 8 && shared_thr != 1 && 2 * k <= 2048 && !(ablate & 2097152);
    }
    int list_cap(int k) const { return few_blocks(k) ? 2 * k : k; }

    SubIndex sub(bool with_packed = false) const {
        const bool pk = with_packed && packed && pk_built;
        return SubIndex{tb_start.as<uint32_t>(), eblk.as<uint16_t>(), epos.as<uint32_t>(),
                        seg.as<uint16_t>(), lid.as<uint32_t>(), wmeta.as<uint16_t>(),
                        emax.as<uint8_t>(), wmax.as<uint8_t>(),
                        pk ? pk_fs.as<uint32_t>() : nullptr, pk ? pk_fwt.as<uint16_t>() : nullptr,
                        pk ? pk_fh.as<uint4>() : nullptr, pk ? pk_data.as<uint32_t>() : nullptr};
    }
};

namespace {

struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        DI_HIP(hipGetDevice(&prev));
        if (prev != dev) DI_HIP(hipSetDevice(dev));
    }
    ~DeviceScope() {
        int cur;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

template <class T>
void upload(DevBuf &d, const std::vector<T> &h) {
    d.reserve(std::max<size_t>(h.size() * sizeof(T), 16));
    if (!h.empty()) DI_HIP(hipMemcpy(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
}

// The device index of postings given in the reference file order (term-major, value
// desc / doc asc): the shard's docs in nb equal blocks; per term only the blocks it has
// postings in get an entry (the sparse term -> block table: a multi-million-term
// vocabulary costs its entries, not n_terms x nb).  Every pass runs over term ranges on
// host_threads() threads (a term owns disjoint output ranges); the result does not
// depend on the thread count.
void build_index(di_index *ix, const int64_t *term_off, int64_t n_terms, const uint32_t *pdoc,
                 const uint8_t *pval, uint32_t doc_lo, uint32_t doc_hi) {
    DI_REQUIRE(n_terms >= 0, DI_EINVAL, "n_terms < 0");
    DI_REQUIRE(n_terms < (int64_t)0xFFFFFFFF, DI_ERANGE, "n_terms %lld >= 2^32",
               (long long)n_terms);
    DI_REQUIRE(term_off[0] >= 0, DI_EINVAL, "term_off[0] < 0");
    for (int64_t t = 0; t < n_terms; ++t)
        DI_REQUIRE(term_off[t + 1] >= term_off[t], DI_EINVAL, "term_off not monotone at %lld",
                   (long long)t);
    if (doc_hi == 0) {
        uint32_t mx = 0;
        bool any = false;
        for (int64_t p = term_off[0]; p < term_off[n_terms]; ++p) {
            mx = std::max(mx, pdoc[p]);
            any = true;
        }
        doc_hi = any ? mx + 1 : doc_lo;
    }
    DI_REQUIRE(doc_hi >= doc_lo, DI_EINVAL, "doc_hi < doc_lo");
    const uint32_t nd = doc_hi - doc_lo;
    const int nb = (int)((nd + MAX_BLOCK_DOCS - 1) / MAX_BLOCK_DOCS);
    DI_REQUIRE(nb <= 65535, DI_ERANGE, "%u docs in one shard: more than 65535 blocks", nd);
    // equal blocks (no small tail block costing a whole workgroup per query)
    const uint32_t bd =
        nb ? (uint32_t)std::min<uint64_t>(MAX_BLOCK_DOCS, ((nd + nb - 1) / nb + 63) / 64 * 64)
           : (uint32_t)MAX_BLOCK_DOCS;
    ix->n_terms = n_terms;
    ix->n_docs = nd;
    ix->doc_lo = doc_lo;
    ix->nb = nb;
    ix->block_docs = (int)bd;
    const uint32_t NO = 0xFFFFFFFFu;

    // pass 1: per term, kept postings and the blocks holding them
    std::vector<uint32_t> n_kept((size_t)n_terms + 1, 0), n_ent_t((size_t)n_terms + 1, 0);
    parallel_for(n_terms, [&](int64_t t0, int64_t t1, int) {
        std::vector<uint32_t> cnt((size_t)std::max(nb, 1), 0);
        std::vector<int> touched;
        for (int64_t t = t0; t < t1; ++t) {
            uint32_t kept = 0;
            touched.clear();
            for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
                if (pval[p] == 0) break;  // inverted_index.py:50-51
                const uint32_t d = pdoc[p];
                if (d < doc_lo || d >= doc_hi) continue;
                const int b = (int)((d - doc_lo) / bd);
                if (cnt[b]++ == 0) touched.push_back(b);
                ++kept;
            }
            for (int b : touched) cnt[b] = 0;
            n_kept[t] = kept;
            n_ent_t[t] = (uint32_t)touched.size();
        }
    });
    std::vector<uint32_t> tb_start((size_t)n_terms + 1, 0);
    std::vector<uint64_t> tstart((size_t)n_terms + 1, 0);
    uint64_t total = 0, n_ent = 0;
    for (int64_t t = 0; t < n_terms; ++t) {
        tstart[t] = total;
        tb_start[t] = (uint32_t)n_ent;
        total += n_kept[t];
        n_ent += n_ent_t[t];
        DI_REQUIRE(total < NO && n_ent < NO, DI_ERANGE,
                   "more than 2^32 postings / (term, block) entries in one shard");
    }
    tstart[n_terms] = total;
    tb_start[n_terms] = (uint32_t)n_ent;
    std::vector<uint32_t>().swap(n_kept);
    std::vector<uint32_t>().swap(n_ent_t);
    ix->n_post = (int64_t)total;
    ix->n_ent = (int64_t)n_ent;

    // pass 2: the entries (block, start) and the postings placed by block (stable: the
    // reference order inside each sublist)
    std::vector<uint16_t> eblk((size_t)std::max<uint64_t>(n_ent, 1));
    std::vector<uint32_t> epos((size_t)n_ent + 1);
    std::vector<uint32_t> packed((size_t)std::max<uint64_t>(total, 4));
    parallel_for(n_terms, [&](int64_t t0, int64_t t1, int) {
        std::vector<uint32_t> cur((size_t)std::max(nb, 1), 0);
        std::vector<int> touched;
        for (int64_t t = t0; t < t1; ++t) {
            touched.clear();
            for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
                if (pval[p] == 0) break;
                const uint32_t d = pdoc[p];
                if (d < doc_lo || d >= doc_hi) continue;
                const int b = (int)((d - doc_lo) / bd);
                if (cur[b]++ == 0) touched.push_back(b);
            }
            std::sort(touched.begin(), touched.end());
            uint32_t run = (uint32_t)tstart[t];
            uint32_t e = tb_start[t];
            for (int b : touched) {
                eblk[e] = (uint16_t)b;
                epos[e++] = run;
                const uint32_t c = cur[b];
                cur[b] = run;  // now the block's write cursor
                run += c;
            }
            for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
                if (pval[p] == 0) break;
                const uint32_t d = pdoc[p];
                if (d < doc_lo || d >= doc_hi) continue;
                const uint32_t r = d - doc_lo;
                packed[cur[r / bd]++] = ((r % bd) << 8) | pval[p];
            }
            for (int b : touched) cur[b] = 0;
        }
    });
    epos[n_ent] = (uint32_t)total;

    // long sublists (>= WLONG_MIN postings) get ids in entry order (DI_WLONG_MIN
    // overrides the threshold: layout A/B only, any value is exact)
    uint32_t wlong_min = WLONG_MIN;
    if (const char *e = std::getenv("DI_WLONG_MIN")) wlong_min = (uint32_t)std::max(1, std::atoi(e));
    std::vector<uint32_t> lid((size_t)std::max<uint64_t>(n_ent, 1), NO);
    uint32_t n_long = 0;
    for (uint64_t e = 0; e < n_ent; ++e)
        if (epos[e + 1] - epos[e] >= wlong_min) lid[e] = n_long++;
    ix->n_long = n_long;

    // pass 3: order inside every sublist, the impact-class offsets and the block max.
    // Postings are grouped by impact class c = 7 - floor(log2 value) (class 0 = values
    // 128..255, ..., class 7 = value 1), classes in order, so that "every posting with
    // value >= 2^(7-c)" is a prefix of the sublist: seg[8e + c] = its length
    // (di_index_set_min_impact prunes with it; class 7 = the whole sublist = exact).
    // Inside a class, postings are dealt from their 32 LDS bank buckets (doc_in_block
    // mod 32, distinct banks per aligned 32-posting block where the class allows, see
    // emit_group): the scorer's lanes read consecutive postings and update
    // acc[doc_in_block], and a 32-lane group of a ds_read_b32 / ds_write_b32 conflicts
    // on equal banks.  Any order is exact: a doc occurs once per term, and its key (first term,
    // value there) does not depend on the order inside the term.
    // Long sublists are laid out by wave segment first: wave w of the scorer owns the
    // block's docs [w S, (w + 1) S), S = ceil(bd / 16), and its postings of the sublist
    // form one run (classes in order, bank-dealt inside), so that no two waves touch one
    // doc.  wmeta[lid * 128 + 8 w + c] = end of class c of segment w (offset in the
    // sublist).  emax[e] = the sublist's largest value (block-max metadata).
    std::vector<uint16_t> seg((size_t)std::max<uint64_t>(n_ent * 8, 8), 0);
    std::vector<uint16_t> wmeta((size_t)std::max<uint32_t>(n_long, 1) * WSEG * 8, 0);
    std::vector<uint8_t> emax((size_t)std::max<uint64_t>(n_ent, 1), 0);
    std::vector<uint8_t> wmax((size_t)std::max<uint32_t>(n_long, 1) * WSEG, 0);
    auto cls_of = [](uint32_t w) { return 7 - (31 - __builtin_clz(w & 255u)); };
    auto bank_of = [](uint32_t w) { return (w >> 8) & 31u; };  // doc_in_block mod 32
    const uint32_t S = (bd + WSEG - 1) / WSEG;
    // The scorer's 16-byte loads (scatter_load wide) give a 32-lane group of one LDS
    // update the positions 4 L + k (L < 32) of an aligned 128-position block; DI_DEAL_X4=0
    // deals for the 4-byte loads' lane-consecutive groups instead (A/B).
    bool deal_x4 = true;
    if (const char *e = std::getenv("DI_DEAL_X4")) deal_x4 = std::atoi(e) != 0;
    // A second posting array for exact scoring, `flat`: the per-wave runs of long
    // sublists dealt without the impact-class order.  Class boundaries leave each 32-lane
    // set of a run with ~1.1 repeated LDS banks (a simulation of this dealing over i.i.d.
    // runs of 300-1200 postings, tools/deal_sim.py), flat runs 0.26-0.68, and the scatter's
    // reads conflict accordingly (PMC at 100 k docs: 0.45 of its LDS cycles).  Impact
    // pruning keeps the class-ordered array, whose prefixes it scores.  Same offsets in both
    // (a run is the same postings in another order); 4 B per posting more in HBM.
    // DI_DEAL_CLASSES=1: one array, class-ordered (A/B).
    bool flat_runs = true;
    if (const char *e = std::getenv("DI_DEAL_CLASSES")) flat_runs = std::atoi(e) == 0;
    std::vector<uint32_t> flat;
    if (flat_runs) flat.resize(packed.size());
    parallel_for(n_terms, [&](int64_t t0, int64_t t1, int) {
        std::vector<uint32_t> grp, tmp, bk, seg_in, cls_cnt(8), cls_pos(8), bucket_cnt(32),
            head(32), fill(32);
        // one group (any order in): classes in order (stable), each dealt round-robin
        // from its 32 LDS bank buckets into packed[o..]; cum[c] = end of class c
        // relative to the sublist start s0
        // one_class: dealt without class boundaries (the flat array's per-wave runs)
        auto emit_group = [&](const uint32_t *in, size_t n, int64_t &o, int64_t s0,
                              uint16_t *cum, uint32_t *dst, bool one_class = false) {
            auto cls_g = [&](uint32_t w) { return one_class ? 0 : cls_of(w); };
            std::fill(cls_cnt.begin(), cls_cnt.end(), 0);
            for (size_t i = 0; i < n; ++i) cls_cnt[cls_g(in[i])]++;
            uint32_t run = 0;
            for (int c = 0; c < 8; ++c) {
                cls_pos[c] = run;
                run += cls_cnt[c];
            }
            tmp.resize(n);
            for (size_t i = 0; i < n; ++i) tmp[cls_pos[cls_g(in[i])]++] = in[i];
            // The scorer's lanes take the group's postings in rounds from its start,
            // and a 32-lane group of its LDS updates is one set of 32 positions (by
            // 16-byte loads: p = 4 L + k of an aligned 128-block, one set per k; by
            // 4-byte loads: an aligned 32-block): each position takes, from its class,
            // a posting whose bank is not yet used in its set (bank cursor carried on
            // across sweeps and class boundaries), else any.
            uint32_t c0 = 0, usedq[4] = {0, 0, 0, 0};
            int cursor = 0;
            const int64_t o_start = o;
            for (int c = 0; c < 8; ++c) {
                const uint32_t c1 = c0 + cls_cnt[c];
                std::fill(bucket_cnt.begin(), bucket_cnt.end(), 0);
                for (uint32_t i = c0; i < c1; ++i) bucket_cnt[bank_of(tmp[i])]++;
                uint32_t r = 0, avail = 0;
                for (int k = 0; k < 32; ++k) {
                    head[k] = r;
                    r += bucket_cnt[k];
                    if (bucket_cnt[k]) avail |= 1u << k;
                }
                bk.resize(c1 - c0);
                fill = head;
                for (uint32_t i = c0; i < c1; ++i) bk[fill[bank_of(tmp[i])]++] = tmp[i];
                for (uint32_t i = c0; i < c1; ++i) {
                    const int64_t rp = o - o_start;
                    if ((rp & (deal_x4 ? 127 : 31)) == 0) usedq[0] = usedq[1] = usedq[2] = usedq[3] = 0;
                    uint32_t &used = usedq[deal_x4 ? (rp & 3) : 0];
                    uint32_t cand = avail & ~used;
                    if (!cand) cand = avail;  // every bank left is taken in this block
                    const uint32_t rot = cursor ? (cand >> cursor) | (cand << (32 - cursor)) : cand;
                    const int k = (__builtin_ctz(rot) + cursor) & 31;
                    dst[o++] = bk[head[k]++];
                    if (--bucket_cnt[k] == 0) avail &= ~(1u << k);
                    used |= 1u << k;
                    cursor = (k + 1) & 31;
                }
                if (cum) cum[c] = (uint16_t)(o - s0);
                c0 = c1;
            }
        };
        for (int64_t t = t0; t < t1; ++t) {
            for (uint32_t e = tb_start[t]; e < tb_start[t + 1]; ++e) {
                const int64_t s0 = epos[e], s1 = epos[e + 1];
                uint16_t *sg = &seg[(size_t)e * 8];
                grp.assign(packed.begin() + s0, packed.begin() + s1);
                uint32_t mx = 0;
                for (uint32_t x : grp) mx = std::max(mx, x & 255u);
                emax[e] = (uint8_t)mx;
                int64_t o = s0;
                const uint32_t id = lid[e];
                if (id == NO) {
                    emit_group(grp.data(), grp.size(), o, s0, sg, packed.data());
                    if (flat_runs)
                        std::copy(packed.begin() + s0, packed.begin() + o, flat.begin() + s0);
                    continue;
                }
                {  // whole-sublist class counts (seg), then the per-wave layout
                    uint32_t run = 0, cc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    for (uint32_t x : grp) cc[cls_of(x)]++;
                    for (int c = 0; c < 8; ++c) sg[c] = (uint16_t)(run += cc[c]);
                }
                for (int w = 0; w < WSEG; ++w) {
                    seg_in.clear();
                    uint32_t wm = 0;
                    for (uint32_t x : grp)
                        if (std::min<uint32_t>((x >> 8) / S, WSEG - 1) == (uint32_t)w) {
                            seg_in.push_back(x);
                            wm = std::max(wm, x & 255u);
                        }
                    wmax[(size_t)id * WSEG + w] = (uint8_t)wm;
                    const int64_t ow = o;
                    emit_group(seg_in.data(), seg_in.size(), o, s0,
                               &wmeta[(size_t)id * WSEG * 8 + w * 8], packed.data());
                    if (flat_runs) {
                        int64_t of = ow;
                        emit_group(seg_in.data(), seg_in.size(), of, s0, nullptr, flat.data(),
                                   true);
                    }
                }
            }
        }
    });
    for (auto &w : packed) w = (((w >> 8) << 10) | (w & 255u)) ^ POST_X;  // device encoding (see POST_X)
    for (auto &w : flat) w = (((w >> 8) << 10) | (w & 255u)) ^ POST_X;
    upload(ix->post, packed);
    if (flat_runs) upload(ix->post_flat, flat);
    ix->has_flat = flat_runs;
    upload(ix->tb_start, tb_start);
    upload(ix->eblk, eblk);
    upload(ix->epos, epos);
    upload(ix->seg, seg);
    upload(ix->lid, lid);
    upload(ix->wmeta, wmeta);
    upload(ix->emax, emax);
    upload(ix->wmax, wmax);
}

}  // namespace

namespace di {
// Kernels using more than 64 KiB of dynamic LDS must opt in, once per device.
void enable_big_lds() {
    static_assert(sizeof(ScoreShared) <= 160 * 1024, "ScoreShared exceeds LDS");
    DI_HIP(hipFuncSetAttribute((const void *)score_blocks_kernel<0>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ScoreShared)));
    DI_HIP(hipFuncSetAttribute((const void *)score_blocks_kernel<EXT_BM>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ScoreShared)));
    DI_HIP(hipFuncSetAttribute((const void *)score_blocks_kernel<EXT_FEW>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ScoreShared)));
    DI_HIP(hipFuncSetAttribute((const void *)score_blocks_kernel<EXT_PK>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ScoreShared)));
    DI_HIP(hipFuncSetAttribute((const void *)score_long_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ScoreShared)));
    DI_HIP(hipFuncSetAttribute((const void *)merge_topk_kernel<1024>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(MergeHead<1024>) + MG_LDS_KEYS * 8)));
    DI_HIP(hipFuncSetAttribute((const void *)merge_topk_kernel<256>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(MergeHead<256>) + MG_LDS_KEYS * 8)));
    DI_HIP(hipFuncSetAttribute((const void *)merge_topk_kernel<512>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(MergeHead<512>) + MG_LDS_KEYS * 8)));
    DI_HIP(hipFuncSetAttribute((const void *)merge_sel_kernel<512, 16>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(MergeSelHead<512>) + MG_SEL_KEYS * 8)));
    DI_HIP(hipFuncSetAttribute((const void *)merge_sel_kernel<512>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(MergeSelHead<512>) + MG_SEL_KEYS * 8)));
}

void launch_merge(const uint64_t *keys, const int32_t *counts, int n_q, int n_lists, int k_in,
                  int k, uint64_t *out_key, uint32_t *out_doc, uint32_t *out_score,
                  int32_t *out_n, int mode, hipStream_t s, bool lists_major = false,
                  const int32_t *cu_q = nullptr) {
    if (n_q == 0) return;
    int64_t ls = k_in, cs = 1, qs = (int64_t)n_lists * k_in, cqs = n_lists;
    if (lists_major) {
        ls = (int64_t)n_q * k_in;
        cs = n_q;
        qs = k_in;
        cqs = 1;
    }
    // few short lists: the register-resident merge (DI_PROFILE_MERGE=0: the general one, A/B)
    // (DI_PROFILE_MERGE=2: the radix select for candidates past the LDS capacity instead
    // of the two-pass histogram filter, A/B)
    static const bool sel_ok = [] {
        const char *e = std::getenv("DI_PROFILE_MERGE");
        return !(e && e[0] == '0');
    }();
    static const int two_pass = [] {
        const char *e = std::getenv("DI_PROFILE_MERGE");
        return (e && e[0] == '2') ? 0 : 2;
    }();
    if (sel_ok && n_lists <= MS_LISTS && (int64_t)n_lists * k_in <= (int64_t)16 * 512 &&
        k <= MG_SEL_KEYS) {
        auto kern = (int64_t)n_lists * k_in <= (int64_t)8 * 512 ? merge_sel_kernel<512, 8>
                                                                : merge_sel_kernel<512, 16>;
        hipLaunchKernelGGL(kern, dim3(n_q), dim3(512),
                           sizeof(MergeSelHead<512>) + (size_t)MG_SEL_KEYS * 8, s, keys, counts,
                           n_lists, k_in, k, ls, cs, qs, cqs, out_key, out_doc, out_score, out_n,
                           mode, cu_q);
        check_launch("merge_sel");
        return;
    }
    // LDS key capacity: all candidates when they fit, else the k survivors of the
    // slow path's radix select
    // (many lists: the score_blocks shared threshold leaves ~k + a few candidates per
    // query, so an 8192-key array -- the selection path's maximum -- usually holds them)
    // (DI_MERGE_CAP: the LDS key array past MG_LDS_KEYS candidates, A/B; default
    // MG_SEL_CAP)
    static const int64_t over_cap = [] {
        const char *e = std::getenv("DI_MERGE_CAP");
        return e ? std::max<int64_t>(64, std::atoll(e)) : (int64_t)MG_SEL_CAP;
    }();
    int64_t want = (int64_t)n_lists * k_in;
    if (n_lists > 1024 || want > MG_LDS_KEYS) want = std::max<int64_t>(k, over_cap);
    int cap = 64;
    while (cap < want) cap <<= 1;
    // workgroup size of the merge: 512 measured best for the 4-block x 1000-candidate
    // bench merge (0.68 vs 0.73 ms at 1024, 0.86 at 256); score-histogram selection
    // before the sort (a full sort of 4000 candidates took 0.80 ms, selection 0.17)
    constexpr int mt = 512;
    const int select = 1 | two_pass;
    // (the histogram follows the keys; only for cap <= MG_SEL_CAP, inside the attribute's max)
    const size_t sel_lds = cap > MG_SEL_MIN && cap <= MG_SEL_CAP ? (size_t)MG_SEL_BINS * 4 + MG_SEL_KEYS * 8 : 0;
    if (cap <= 256 || mt == 256) {
        size_t lds = sizeof(MergeHead<256>) + (size_t)cap * 8 + sel_lds;
        hipLaunchKernelGGL(merge_topk_kernel<256>, dim3(n_q), dim3(256), lds, s, keys, counts,
                           n_lists, k_in, k, ls, cs, qs, cqs, cap, out_key, out_doc, out_score,
                           out_n, mode, select, cu_q);
    } else if (mt == 512) {
        size_t lds = sizeof(MergeHead<512>) + (size_t)cap * 8 + sel_lds;
        hipLaunchKernelGGL(merge_topk_kernel<512>, dim3(n_q), dim3(512), lds, s, keys, counts,
                           n_lists, k_in, k, ls, cs, qs, cqs, cap, out_key, out_doc, out_score,
                           out_n, mode, select, cu_q);
    } else {
        size_t lds = sizeof(MergeHead<1024>) + (size_t)cap * 8 + sel_lds;
        hipLaunchKernelGGL(merge_topk_kernel<1024>, dim3(n_q), dim3(1024), lds, s, keys,
                           counts, n_lists, k_in, k, ls, cs, qs, cqs, cap, out_key, out_doc,
                           out_score, out_n, mode, select, cu_q);
    }
    check_launch("merge_topk");
}

}  // namespace di

extern "C" {

int di_index_create(const int64_t *term_off, int64_t n_terms, const uint32_t *pdoc,
                    const uint8_t *pval, uint32_t doc_lo, uint32_t doc_hi, int device,
                    di_index **out) {
    return guard([&] {
        DI_REQUIRE(out && term_off && (n_terms == 0 || (pdoc && pval)), DI_EINVAL,
                   "null argument");
        int ndev = 0;
        DI_REQUIRE(hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0, DI_ENODEV,
                   "no HIP device");
        DI_REQUIRE(device >= 0 && device < ndev, DI_EINVAL, "bad device %d", device);
        DeviceScope ds(device);
        std::unique_ptr<di_index> ix(new di_index());
        ix->device = device;
        DI_HIP(hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking));
        ix->own_stream = true;
        enable_big_lds();
        if (const char *ab = std::getenv("DI_PROFILE_ABLATE")) ix->ablate = std::atoi(ab);
        if (const char *bo = std::getenv("DI_BLOCK_ORDER")) ix->block_order = bo[0] == '1';
        if (const char *st = std::getenv("DI_SCORE_THRESHOLD"))  // (tested both ways)
            ix->shared_thr = st[0] != '0' ? 1 : 0;
        if (const char *e = std::getenv("DI_TQ_EVERY")) ix->tq_every = std::max(1, std::atoi(e));
        if (const char *e = std::getenv("DI_TQ_FIRST")) ix->tq_first = std::max(0, std::atoi(e));
        build_index(ix.get(), term_off, n_terms, pdoc, pval, doc_lo, doc_hi);
        *out = ix.release();
    });
}

int di_index_load_reference(const char *dir, uint32_t doc_lo, uint32_t doc_hi, int device,
                            di_index **out) {
    return guard([&] {
        DI_REQUIRE(dir && out, DI_EINVAL, "null argument");
        std::string d(dir);
        // .idx read whole (16 B per term); .dat mapped: a doc-id shard reads only its
        // own postings out of it, on host_threads() threads (every rank of a sharded
        // rank CLI maps the same file: one page-cache copy, no per-rank whole-file copy)
        std::ifstream fi(d + "/inverted_index.idx", std::ios::binary | std::ios::ate);
        DI_REQUIRE(fi, DI_EIO, "cannot open %s/inverted_index.idx", dir);
        const size_t isz = (size_t)fi.tellg();
        DI_REQUIRE(isz % 16 == 0, DI_EFORMAT, "inverted_index.idx size %zu not a multiple of 16",
                   isz);
        std::vector<uint64_t> idx(isz / 8);
        fi.seekg(0);
        fi.read(reinterpret_cast<char *>(idx.data()), (std::streamsize)isz);
        DI_REQUIRE(fi || isz == 0, DI_EIO, "cannot read %s/inverted_index.idx", dir);
        const int fd = ::open((d + "/inverted_index.dat").c_str(), O_RDONLY);
        DI_REQUIRE(fd >= 0, DI_EIO, "cannot open %s/inverted_index.dat", dir);
        struct stat st;
        if (::fstat(fd, &st) != 0) {
            ::close(fd);
            DI_REQUIRE(false, DI_EIO, "cannot stat %s/inverted_index.dat", dir);
        }
        const size_t dsz = (size_t)st.st_size;
        const unsigned char *dat = nullptr;
        if (dsz) {
            void *m = ::mmap(nullptr, dsz, PROT_READ, MAP_SHARED, fd, 0);
            ::close(fd);
            DI_REQUIRE(m != MAP_FAILED, DI_EIO, "cannot map %s/inverted_index.dat", dir);
            dat = static_cast<const unsigned char *>(m);
        } else {
            ::close(fd);
        }
        struct Unmap {
            const void *p;
            size_t n;
            ~Unmap() {
                if (p) ::munmap(const_cast<void *>(p), n);
            }
        } unmap{dat, dsz};
        DI_REQUIRE(dsz % 5 == 0, DI_EFORMAT, "inverted_index.dat size %zu not a multiple of 5",
                   dsz);
        const int64_t nt = (int64_t)(isz / 16);
        for (int64_t t = 0; t < nt; ++t) {
            const uint64_t s = idx[2 * t], e = idx[2 * t + 1];
            DI_REQUIRE(s % 5 == 0 && e % 5 == 0 && s <= e && e <= dsz, DI_EFORMAT,
                       "bad (start,end) for term %lld", (long long)t);
        }
        const uint64_t hi = doc_hi ? doc_hi : 0x100000000ull;
        // postings of term t: records [start/5, end/5) up to its first 0 value
        // (create.py:45-51, inverted_index.py:50-51), docs of the shard only
        auto rec_doc = [&](uint64_t r) {
            uint32_t doc;
            std::memcpy(&doc, dat + r * 5, 4);
            return doc;
        };
        std::vector<int64_t> term_off((size_t)nt + 1, 0);
        parallel_for(nt, [&](int64_t t0, int64_t t1, int) {
            for (int64_t t = t0; t < t1; ++t) {
                int64_t c = 0;
                for (uint64_t r = idx[2 * t] / 5; r < idx[2 * t + 1] / 5; ++r) {
                    if (dat[r * 5 + 4] == 0) break;
                    const uint32_t doc = rec_doc(r);
                    c += doc >= doc_lo && doc < hi;
                }
                term_off[(size_t)t + 1] = c;
            }
        });
        for (int64_t t = 0; t < nt; ++t) term_off[(size_t)t + 1] += term_off[(size_t)t];
        const int64_t np = term_off[(size_t)nt];
        std::vector<uint32_t> pdoc((size_t)std::max<int64_t>(np, 1));
        std::vector<uint8_t> pval((size_t)std::max<int64_t>(np, 1));
        parallel_for(nt, [&](int64_t t0, int64_t t1, int) {
            for (int64_t t = t0; t < t1; ++t) {
                int64_t o = term_off[(size_t)t];
                for (uint64_t r = idx[2 * t] / 5; r < idx[2 * t + 1] / 5; ++r) {
                    const uint8_t v = dat[r * 5 + 4];
                    if (v == 0) break;
                    const uint32_t doc = rec_doc(r);
                    if (doc >= doc_lo && doc < hi) {
                        pdoc[(size_t)o] = doc;
                        pval[(size_t)o++] = v;
                    }
                }
            }
        });
        int rc = di_index_create(term_off.data(), nt, pdoc.data(), pval.data(), doc_lo, doc_hi,
                                 device, out);
        if (rc != DI_OK) throw Error{rc};
    });
}

int di_index_reserve(di_index *ix, int32_t max_q, int32_t k) {
    return guard([&] {
        DI_REQUIRE(ix && max_q >= 0 && k > 0 && k <= DI_MAX_TOPK, DI_EINVAL, "bad argument");
        DeviceScope ds(ix->device);
        // (the few-block emit-above selection lists up to 2 k keys per item, see search)
        const int kl = ix->list_cap(k);
        size_t nbk = (size_t)max_q * std::max(ix->nb, 1) * kl;
        ix->ws_ck.reserve(nbk * 8);
        ix->ws_cn.reserve((size_t)max_q * std::max(ix->nb, 1) * 4);
    });
}

int di_index_search(di_index *ix, const uint32_t *q_terms, const int32_t *cu_q, int32_t n_q,
                    int32_t k, uint32_t *out_doc, uint32_t *out_score, int32_t *out_n,
                    uint64_t *out_key, uint32_t flags) {
    return guard([&] {
        DI_REQUIRE(ix && cu_q && out_doc && out_score && out_n, DI_EINVAL, "null argument");
        DI_REQUIRE(n_q >= 0, DI_EINVAL, "n_q < 0");
        DI_REQUIRE(k > 0 && k <= DI_MAX_TOPK, DI_ERANGE, "k=%d outside [1, %d]", k,
                   DI_MAX_TOPK);
        DeviceScope ds(ix->device);
        const bool dev = flags & DI_F_DEVICE_PTRS;
        const bool timing = flags & DI_F_TIMING;
        hipStream_t s = ix->stream;
        if (n_q == 0) return;
        int64_t nterms_total = 0;
        int max_nt = WTERMS;  // record slots per item (device pointers: the per-wave maximum)
        if (!dev) {
            max_nt = 1;
            for (int q = 0; q < n_q; ++q) {
                int32_t c = cu_q[q + 1] - cu_q[q];
                max_nt = std::max(max_nt, (int)c);
                DI_REQUIRE(c >= 0, DI_EINVAL, "cu_q not monotone at %d", q);
                DI_REQUIRE(c <= DI_MAX_QUERY_TERMS, DI_ERANGE,
                           "query %d has %d terms (limit %d)", q, c, DI_MAX_QUERY_TERMS);
                DI_REQUIRE(c <= DI_SHORT_QUERY_TERMS ||
                               (uint64_t)ix->doc_lo + ix->n_docs <= (1ull << 24),
                           DI_ERANGE,
                           "query %d has %d terms: queries over %d terms need shard docs < 2^24",
                           q, c, DI_SHORT_QUERY_TERMS);
            }
            nterms_total = cu_q[n_q];
            for (int64_t i = 0; i < nterms_total; ++i)
                DI_REQUIRE(q_terms[i] < (uint64_t)ix->n_terms, DI_EINVAL,
                           "term id %u out of range", q_terms[i]);
        }
        const int nb = std::max(ix->nb, 1);
        // query chunking keeps the candidate workspace bounded: 4 GiB of the 288 GB HBM
        // (DI_CAND_WS_MIB overrides, A/B).  A 1 GiB cap cut 8.8 M-doc batches into 14
        // chunks of 499 queries, whose merge launches had ~2 workgroups per CU
        // (round-4 DESIGN §4).
        // The item records (item_setup_kernel) take rec_slots per item -- the batch's
        // longest query up to WTERMS (~6 for MS MARCO queries, 64 with device-pointer
        // queries) -- and are capped at twice the candidate cap, which bounds the chunk
        // too: one setting (DI_CAND_WS_MIB) sizes both.  Peak workspace of a handle
        // ~3x the cap.
        const int rec_slots = std::min(std::max(max_nt, 1), WTERMS);
        // Few blocks: the emit-above selection (di_index::few_blocks)
        const bool few = ix->few_blocks(k);
        const int kl = ix->list_cap(k);
        const int64_t per_q = (int64_t)nb * kl * 8;
        const int64_t rec_per_q = (int64_t)nb * rec_slots * (int64_t)sizeof(ItemRec);
        int64_t ws_cap = 4ll << 30;
        if (const char *e = std::getenv("DI_CAND_WS_MIB")) ws_cap = std::max(1ll, std::atoll(e)) << 20;
        const int chunk = (int)std::max<int64_t>(
            1, std::min<int64_t>({(int64_t)n_q, ws_cap / per_q, 2 * ws_cap / rec_per_q}));
        ix->ws_ck.reserve((size_t)chunk * per_q);
        ix->ws_cn.reserve((size_t)chunk * nb * 4);
        ix->ws_thr.reserve((size_t)chunk * QH_BINS * 4);
        ix->ws_long.reserve(4);
        if (!ix->bm_stat.p) {
            ix->bm_stat.reserve(16);
            DI_HIP(hipMemsetAsync(ix->bm_stat.p, 0, 16, s));
        }
        // (DI_PROFILE_ABLATE bit 1024: no records -- the scorer walks the chain itself, A/B
        // and the fallback test)
        const size_t rec_bytes = (size_t)chunk * rec_per_q;
        const bool use_rec = !(ix->ablate & 1024);
        if (use_rec) ix->ws_rec.reserve(rec_bytes);
        const uint32_t *dq = (const uint32_t *)stage_in(
            q_terms, (size_t)nterms_total * 4, dev, ix->ws_q, s);
        const int32_t *dcu =
            (const int32_t *)stage_in(cu_q, (size_t)(n_q + 1) * 4, dev, ix->ws_cu, s);
        uint32_t *ddoc = out_doc, *dscore = out_score;
        int32_t *dn = out_n;
        uint64_t *dkey = out_key;
        if (!dev) {
            ix->ws_doc.reserve((size_t)n_q * k * 4);
            ix->ws_score.reserve((size_t)n_q * k * 4);
            ix->ws_n.reserve((size_t)n_q * 4);
            ddoc = ix->ws_doc.as<uint32_t>();
            dscore = ix->ws_score.as<uint32_t>();
            dn = ix->ws_n.as<int32_t>();
            if (out_key) {
                ix->ws_key.reserve((size_t)n_q * k * 8);
                dkey = ix->ws_key.as<uint64_t>();
            }
        }
        for (int q0 = 0; q0 < n_q; q0 += chunk) {
            const int nq = std::min(chunk, n_q - q0);
            if (ix->nb == 0) {
                DI_HIP(hipMemsetAsync(ix->ws_cn.p, 0, (size_t)nq * nb * 4, s));
            } else {
                const bool thr = nb > 1 && (ix->shared_thr < 0 ? nb >= 8 : ix->shared_thr == 1);
                if (thr) DI_HIP(hipMemsetAsync(ix->ws_thr.p, 0, (size_t)nq * QH_BINS * 4, s));
                DI_HIP(hipMemsetAsync(ix->ws_long.p, 0, 4, s));
                TimedLaunch tl(ix->timer, timing, "score_blocks", s);  // (both kernels)
                const int n_items = nq * nb;
                // packed postings (configs[4]): exact scoring from the item records only
                // (records always fit: the chunk is bounded by them; ablate bit 1024 turns
                // them off, and the packed layout with them)
                const bool pk = ix->packed && ix->pk_built && ix->min_cls >= 7 && use_rec;
                // block-max: blocks in descending order of their bound per query, opt-in
                // (DI_BLOCK_ORDER=1): it raises the running threshold sooner but gives up
                // the block-major L2 sharing of the popular sublists -- at 8.8 M docs, f = 1:
                // skewed 79.4 vs 76.7 ms per batch, i.i.d. 126.0 vs 114.2 (round-4 DESIGN §4)
                const bool order = thr && ix->bm_factor > 0.0f && nb > 1 &&
                                   nb <= BO_MAX_BLOCKS && ix->block_order;
                if (order) {
                    ix->ws_border.reserve((size_t)nq * nb * 2);
                    hipLaunchKernelGGL(block_order_kernel, dim3(nq), dim3(256), 0, s, ix->sub(),
                                       nb, ix->n_terms, dq, dcu + q0,
                                       ix->ws_border.as<uint16_t>());
                    check_launch("block_order");
                }
                const uint16_t *border = order ? ix->ws_border.as<uint16_t>() : nullptr;
                // (DI_PROFILE_ABLATE bit 32768: the histogram-copy threshold instead, A/B)
                // (DI_TQ_EVERY / DI_TQ_FIRST: the threshold refresh schedule of score_item;
                // every = 1: every item copies the histogram, as before round 6)
                const bool sched = thr && ix->tq_every > 1;
                const bool use_qtq =
                    (thr && ix->bm_factor > 0.0f && !(ix->ablate & 32768)) || few || sched;
                const int tq_sched = sched ? (ix->tq_first << 16) | ix->tq_every : 1;
                if (use_qtq) {
                    ix->ws_tq.reserve((size_t)nq * 4);
                    DI_HIP(hipMemsetAsync(ix->ws_tq.p, 0, (size_t)nq * 4, s));
                }
                if (use_rec) {
                    hipLaunchKernelGGL(item_setup_kernel, dim3(n_items), dim3(128), 0, s,
                                       ix->sub(pk), ix->min_cls, nb, ix->n_terms, dq, dcu + q0, nq,
                                       ix->ws_rec.as<ItemRec>(), border, rec_slots);
                    check_launch("item_setup");
                }
                // (DI_PROFILE_ABLATE bit 65536: the block-max instantiation with block-max
                // off, A/B of its code alone)
                // Heavily pruned searches (min_impact >= 16: min_cls <= 3) run the EXT_BM
                // instantiation too, block-max off, for its one-sweep selection of sparse
                // items (score_item).  8.8 M docs, k q/s: skewed m 16 / 32 / 64 / 128
                // 110.8 / 96.9 / 98.2 / 98.6 -> 121.4 / 124.9 / 131.2 / 133.1; i.i.d. 2.5-4%
                // slower (the instantiation's own cost, items there rarely sparse); lighter
                // pruning 1-4% slower, so it keeps the plain kernel (round-4 DESIGN §4).
                const bool ext = pk || order || (thr && ix->bm_factor > 0.0f) ||
                                 (thr && ix->min_cls <= 3) || (ix->ablate & 65536);
                hipLaunchKernelGGL(pk    ? score_blocks_kernel<EXT_PK>
                                   : ext ? score_blocks_kernel<EXT_BM>
                                   : few ? score_blocks_kernel<EXT_FEW>
                                         : score_blocks_kernel<0>,
                                   dim3(std::min(n_items, n_cu())),
                                   dim3(SC_THREADS), sizeof(ScoreShared), s,
                                   ix->post_for(ix->min_cls), ix->sub(pk),
                                   ix->min_cls, nb, ix->block_docs, ix->n_terms,
                                   ix->n_docs, ix->doc_lo, dq, dcu + q0, k,
                                   ix->ws_ck.as<uint64_t>(), ix->ws_cn.as<int32_t>(), n_items,
                                   nq, thr ? ix->ws_thr.as<uint32_t>() : nullptr, ix->ablate,
                                   use_rec ? ix->ws_rec.as<ItemRec>() : nullptr,
                                   ix->ws_long.as<uint32_t>(), thr ? ix->bm_factor : 0.0f,
                                   ix->bm_stat.as<unsigned long long>(), border,
                                   use_qtq ? ix->ws_tq.as<uint32_t>() : nullptr, rec_slots, kl,
                                   tq_sched);
                check_launch("score_blocks");
                hipLaunchKernelGGL(score_long_kernel, dim3(std::min(n_items, n_cu())),
                                   dim3(SC_THREADS), sizeof(ScoreShared), s,
                                   ix->post_for(ix->min_cls), ix->sub(),
                                   ix->min_cls, nb, ix->block_docs, ix->n_terms, ix->n_docs,
                                   ix->doc_lo, dq, dcu + q0, k, ix->ws_ck.as<uint64_t>(),
                                   ix->ws_cn.as<int32_t>(), nq, ix->ws_long.as<uint32_t>(), kl);
                check_launch("score_long");
            }
            {
                TimedLaunch tl(ix->timer, timing, "merge_topk", s);
                launch_merge(ix->ws_ck.as<uint64_t>(), ix->ws_cn.as<int32_t>(), nq, nb, kl, k,
                             dkey ? dkey + (int64_t)q0 * k : nullptr, ddoc + (int64_t)q0 * k,
                             dscore + (int64_t)q0 * k, dn + q0, DECODE_QUANT, s, false,
                             dcu + q0);
            }
        }
        if (!dev) {
            DI_HIP(hipMemcpyAsync(out_doc, ddoc, (size_t)n_q * k * 4, hipMemcpyDeviceToHost, s));
            DI_HIP(hipMemcpyAsync(out_score, dscore, (size_t)n_q * k * 4, hipMemcpyDeviceToHost,
                                  s));
            DI_HIP(hipMemcpyAsync(out_n, dn, (size_t)n_q * 4, hipMemcpyDeviceToHost, s));
            if (out_key)
                DI_HIP(hipMemcpyAsync(out_key, dkey, (size_t)n_q * k * 8, hipMemcpyDeviceToHost,
                                      s));
        }
        if (ix->ablate & 64) {
            unsigned long long ph[12];
            DI_HIP(hipStreamSynchronize(s));
            DI_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_sb_phase), sizeof ph));
            fprintf(stderr, "score_blocks phase cycles (workgroup 0, cumulative): setup %llu "
                            "scatter %llu hist %llu [count %llu] write %llu ties %llu copy %llu "
                            "tq-select %llu [tq-read %llu] scatter-loop slowest wave %llu mean wave %llu\n",
                    ph[0], ph[1], ph[2], ph[6], ph[3], ph[4], ph[5], ph[7], ph[8], ph[9], ph[10]);
        }
        if (!(flags & DI_F_ASYNC) || !dev) {
            DI_HIP(hipStreamSynchronize(s));
            ix->timer.resolve();
            if (!dev)
                for (int q = 0; q < n_q; ++q)
                    DI_REQUIRE(out_n[q] >= 0, DI_ERANGE, "query %d exceeded a kernel limit", q);
        }
    });
}

int di_index_info(const di_index *ix, int64_t *n_terms, int64_t *n_postings, uint32_t *n_docs,
                  int32_t *n_blocks) {
    return guard([&] {
        DI_REQUIRE(ix, DI_EINVAL, "null handle");
        if (n_terms) *n_terms = ix->n_terms;
        if (n_postings) *n_postings = ix->n_post;
        if (n_docs) *n_docs = ix->n_docs;
        if (n_blocks) *n_blocks = ix->nb;
    });
}

int di_index_set_min_impact(di_index *ix, int32_t min_impact) {
    return guard([&] {
        DI_REQUIRE(ix, DI_EINVAL, "null handle");
        DI_REQUIRE(min_impact >= 1 && min_impact <= 255, DI_ERANGE,
                   "min_impact=%d outside [1, 255]", min_impact);
        // postings with value >= 2^floor(log2 min_impact): the class prefix
        ix->min_cls = 7 - (31 - __builtin_clz((unsigned)min_impact));
    });
}

int di_index_set_block_max(di_index *ix, float factor) {
    return guard([&] {
        DI_REQUIRE(ix, DI_EINVAL, "null handle");
        DI_REQUIRE(factor == 0.0f || (factor >= 1.0f && factor <= 16.0f), DI_ERANGE,
                   "block-max factor %g: 0 (off) or in [1, 16]", (double)factor);
        ix->bm_factor = factor;
    });
}

// Packed (block-compressed) postings from the device layout: every run (short
// sublist, or one wave segment's run of a long one) sorted by doc, cut into frames of
// up to PK_FRAME postings, each frame bit-packed with its own widths (see
// packed_fields).  Host threads over entry ranges; three passes (frame counts, widths,
// encoding) so every entry writes its own ranges.
static void build_packed(di_index *ix) {
    const int64_t ne = ix->n_ent, np = ix->n_post, nl = ix->n_long;
    std::vector<uint32_t> post((size_t)std::max<int64_t>(np, 1)), epos((size_t)ne + 1);
    std::vector<uint32_t> lid((size_t)std::max<int64_t>(ne, 1));
    std::vector<uint16_t> wmeta((size_t)std::max<int64_t>(nl, 1) * WSEG * 8);
    if (np) DI_HIP(hipMemcpy(post.data(), ix->post.p, (size_t)np * 4, hipMemcpyDeviceToHost));
    DI_HIP(hipMemcpy(epos.data(), ix->epos.p, ((size_t)ne + 1) * 4, hipMemcpyDeviceToHost));
    if (ne) DI_HIP(hipMemcpy(lid.data(), ix->lid.p, (size_t)ne * 4, hipMemcpyDeviceToHost));
    if (nl)
        DI_HIP(hipMemcpy(wmeta.data(), ix->wmeta.p, (size_t)nl * WSEG * 8 * 2,
                         hipMemcpyDeviceToHost));
    const uint32_t NO = 0xFFFFFFFFu;
    // run r of entry e: [a, b) of the postings (w: segment of a long entry)
    auto run_of = [&](int64_t e, int w, uint32_t &a, uint32_t &b) {
        const uint32_t id = lid[(size_t)e];
        if (id == NO) {
            a = epos[(size_t)e];
            b = epos[(size_t)e + 1];
            return;
        }
        const uint16_t *m = &wmeta[(size_t)id * WSEG * 8];
        a = epos[(size_t)e] + (w ? m[(w - 1) * 8 + 7] : 0u);
        b = epos[(size_t)e] + m[w * 8 + 7];
    };
    // (a short sublist under PK_MIN postings stays plain: no run, no frame)
    auto n_runs = [&](int64_t e) {
        return lid[(size_t)e] != NO ? WSEG : epos[(size_t)e + 1] - epos[(size_t)e] >= PK_MIN ? 1 : 0;
    };
    auto frames_of = [](uint32_t n) { return (n + PK_FRAME - 1) / PK_FRAME; };
    // pass 1: frames per entry -> fs; per long entry the run starts (fwt)
    std::vector<uint32_t> fs((size_t)ne + 1, 0);
    std::vector<uint16_t> fwt((size_t)std::max<int64_t>(nl, 1) * (WSEG + 1), 0);
    parallel_for(ne, [&](int64_t e0, int64_t e1, int) {
        for (int64_t e = e0; e < e1; ++e) {
            uint32_t nf = 0;
            const uint32_t id = lid[(size_t)e];
            for (int w = 0; w < n_runs(e); ++w) {
                uint32_t a, b;
                run_of(e, w, a, b);
                if (id != NO) fwt[(size_t)id * (WSEG + 1) + w] = (uint16_t)nf;
                nf += frames_of(b - a);
            }
            if (id != NO) fwt[(size_t)id * (WSEG + 1) + WSEG] = (uint16_t)nf;
            fs[(size_t)e + 1] = nf;
        }
    });
    for (int64_t e = 0; e < ne; ++e) fs[(size_t)e + 1] += fs[(size_t)e];
    const int64_t nfr = fs[(size_t)ne];
    // one run's frames: sorted (doc, value), per frame (bd, bv, vmin, W)
    struct FrameInfo {
        uint32_t base, cnt, bd, bv, vmin, W;
    };
    auto bits = [](uint32_t x) { return x ? 32 - __builtin_clz(x) : 0; };
    auto frame_info = [&](const std::vector<std::pair<uint32_t, uint32_t>> &dv, size_t i0,
                          size_t i1) {
        FrameInfo fi{dv[i0].first, (uint32_t)(i1 - i0), 0, 0, 255, 0};
        uint32_t dmax = 0, vmax = 0;
        for (size_t i = i0; i < i1; ++i) {
            if (i > i0) dmax = std::max(dmax, dv[i].first - dv[i - 1].first);
            fi.vmin = std::min(fi.vmin, dv[i].second);
            vmax = std::max(vmax, dv[i].second);
        }
        fi.bd = (uint32_t)bits(dmax);
        fi.bv = (uint32_t)bits(vmax - fi.vmin);
        fi.W = std::max<uint32_t>(4, (fi.bd + fi.bv + 3) / 4 * 4);
        return fi;
    };
    auto sorted_run = [&](uint32_t a, uint32_t b, std::vector<std::pair<uint32_t, uint32_t>> &dv) {
        dv.resize(b - a);
        for (uint32_t p = a; p < b; ++p)
            dv[p - a] = {(post[p] ^ POST_X) >> 10, post[p] & 255u};
        std::sort(dv.begin(), dv.end());
    };
    // pass 2: data dwords per frame
    std::vector<uint32_t> fdw((size_t)std::max<int64_t>(nfr, 1) + 1, 0);
    parallel_for(ne, [&](int64_t e0, int64_t e1, int) {
        std::vector<std::pair<uint32_t, uint32_t>> dv;
        for (int64_t e = e0; e < e1; ++e) {
            uint32_t f = fs[(size_t)e];
            for (int w = 0; w < n_runs(e); ++w) {
                uint32_t a, b;
                run_of(e, w, a, b);
                sorted_run(a, b, dv);
                for (size_t i0 = 0; i0 < dv.size(); i0 += PK_FRAME, ++f) {
                    const size_t i1 = std::min(dv.size(), i0 + PK_FRAME);
                    const FrameInfo fi = frame_info(dv, i0, i1);
                    fdw[(size_t)f + 1] = (uint32_t)((fi.cnt + PK_PER_LANE - 1) / PK_PER_LANE) * (fi.W / 4);
                }
            }
        }
    });
    std::vector<uint64_t> doff((size_t)nfr + 1, 0);
    for (int64_t f = 0; f < nfr; ++f) doff[(size_t)f + 1] = doff[(size_t)f] + fdw[(size_t)f + 1];
    DI_REQUIRE(doff[(size_t)nfr] < 0xFFFFFFFFull, DI_ERANGE, "packed postings past 2^32 dwords");
    // pass 3: headers and data
    std::vector<uint4> fh((size_t)std::max<int64_t>(nfr, 1));
    std::vector<uint32_t> data((size_t)std::max<uint64_t>(doff[(size_t)nfr], 1), 0);
    parallel_for(ne, [&](int64_t e0, int64_t e1, int) {
        std::vector<std::pair<uint32_t, uint32_t>> dv;
        for (int64_t e = e0; e < e1; ++e) {
            uint32_t f = fs[(size_t)e];
            for (int w = 0; w < n_runs(e); ++w) {
                uint32_t a, b;
                run_of(e, w, a, b);
                sorted_run(a, b, dv);
                for (size_t i0 = 0; i0 < dv.size(); i0 += PK_FRAME, ++f) {
                    const size_t i1 = std::min(dv.size(), i0 + PK_FRAME);
                    const FrameInfo fi = frame_info(dv, i0, i1);
                    uint32_t *out = &data[(size_t)doff[(size_t)f]];
                    const uint32_t nd = fi.W / 4;
                    for (size_t i = i0; i < i1; ++i) {
                        const uint32_t k = (uint32_t)(i - i0);
                        const uint32_t delta = i > i0 ? dv[i].first - dv[i - 1].first : 0u;
                        const uint64_t field = (uint64_t)delta | ((uint64_t)(dv[i].second - fi.vmin) << fi.bd);
                        const uint32_t lane = k / PK_PER_LANE, slot = k % PK_PER_LANE;
                        const uint64_t bit = (uint64_t)lane * nd * 32 + (uint64_t)slot * fi.W;
                        const uint64_t sh = field << (bit & 31);
                        out[bit >> 5] |= (uint32_t)sh;
                        if ((bit & 31) + fi.W > 32) out[(bit >> 5) + 1] |= (uint32_t)(sh >> 32);
                    }
                    fh[(size_t)f] = make_uint4((uint32_t)doff[(size_t)f],
                                               fi.base | (fi.cnt << 16) | (fi.bd << 26),
                                               fi.vmin | (fi.bv << 8) | (fi.W << 12), 0u);
                }
            }
        }
    });
    upload(ix->pk_fs, fs);
    upload(ix->pk_fwt, fwt);
    upload(ix->pk_fh, fh);
    upload(ix->pk_data, data);
    ix->pk_frames = nfr;
    // bytes the packed scorer reads: headers + packed data + the plain words of the short
    // sublists it reads from the plain layout
    int64_t plain_small = 0;
    for (int64_t e = 0; e < ne; ++e)
        if (n_runs(e) == 0) plain_small += epos[(size_t)e + 1] - epos[(size_t)e];
    ix->pk_bytes = (int64_t)doff[(size_t)nfr] * 4 + nfr * (int64_t)sizeof(uint4) + 4 * plain_small;
    ix->pk_built = true;
}

int di_index_set_packed(di_index *ix, int32_t on, int64_t *packed_bytes) {
    return guard([&] {
        DI_REQUIRE(ix, DI_EINVAL, "null handle");
        DeviceScope ds(ix->device);
        if (on && !ix->pk_built) {
            DI_HIP(hipStreamSynchronize(ix->stream));
            build_packed(ix);
        }
        ix->packed = on != 0;
        if (packed_bytes) *packed_bytes = ix->pk_built ? ix->pk_bytes : 0;
    });
}

int di_index_set_stream(di_index *ix, void *stream) {
    return guard([&] {
        DI_REQUIRE(ix, DI_EINVAL, "null handle");
        DeviceScope ds(ix->device);
        if (ix->own_stream && ix->stream) DI_HIP(hipStreamDestroy(ix->stream));
        ix->own_stream = stream == nullptr;
        if (stream)
            ix->stream = (hipStream_t)stream;
        else
            DI_HIP(hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking));
    });
}

int di_index_sync(di_index *ix) {
    return guard([&] {
        DI_REQUIRE(ix, DI_EINVAL, "null handle");
        DeviceScope ds(ix->device);
        DI_HIP(hipStreamSynchronize(ix->stream));
        ix->timer.resolve();
    });
}

int di_index_timing(di_index *ix, const char *name, di_timing *out, int reset) {
    return guard([&] {
        DI_REQUIRE(ix && name && out, DI_EINVAL, "null argument");
        const std::string n(name);
        if (n == "bm_segments" || n == "bm_segments_skipped") {
            // block-max counters (launches = the count; ms = 0), accumulated on the device
            // since the last reset: reading them synchronises the index's stream
            DeviceScope ds(ix->device);
            unsigned long long st[2] = {0, 0};
            if (ix->bm_stat.p) {
                DI_HIP(hipStreamSynchronize(ix->stream));
                DI_HIP(hipMemcpy(st, ix->bm_stat.p, 16, hipMemcpyDeviceToHost));
                if (reset) DI_HIP(hipMemset(ix->bm_stat.p, 0, 16));
            }
            out->ms = 0.0;
            out->launches = (int64_t)st[n == "bm_segments" ? 0 : 1];
            return;
        }
        ix->timer.get(name, out, reset != 0);
    });
}

int di_index_destroy(di_index *ix) {
    return guard([&] {
        if (!ix) return;
        {
            DeviceScope ds(ix->device);
            if (ix->own_stream && ix->stream) (void)hipStreamDestroy(ix->stream);
        }
        delete ix;
    });
}

int di_topk_merge(const uint64_t *keys, const int32_t *counts, int32_t n_q, int32_t n_lists,
                  int32_t k, uint64_t *out_key, int32_t *out_n, int device, void *hip_stream,
                  uint32_t flags) {
    return guard([&] {
        DI_REQUIRE(keys && counts && out_key && out_n && n_q >= 0 && n_lists > 0, DI_EINVAL,
                   "bad argument");
        DI_REQUIRE(k > 0 && k <= DI_MAX_TOPK, DI_ERANGE, "k=%d outside [1, %d]", k,
                   DI_MAX_TOPK);
        DeviceScope ds(device);
        enable_big_lds();
        hipStream_t s = (hipStream_t)hip_stream;
        const bool dev = flags & DI_F_DEVICE_PTRS;
        DevBuf bk, bc, bo, bn;
        const uint64_t *dk = (const uint64_t *)stage_in(keys, (size_t)n_q * n_lists * k * 8, dev,
                                                        bk, s);
        const int32_t *dc = (const int32_t *)stage_in(counts, (size_t)n_q * n_lists * 4, dev, bc,
                                                      s);
        uint64_t *dok = out_key;
        int32_t *don = out_n;
        if (!dev) {
            bo.reserve((size_t)n_q * k * 8);
            bn.reserve((size_t)n_q * 4);
            dok = bo.as<uint64_t>();
            don = bn.as<int32_t>();
        }
        launch_merge(dk, dc, n_q, n_lists, k, k, dok, nullptr, nullptr, don, DECODE_NONE, s,
                     (flags & DI_F_LISTS_MAJOR) != 0);
        if (!dev) {
            DI_HIP(hipMemcpyAsync(out_key, dok, (size_t)n_q * k * 8, hipMemcpyDeviceToHost, s));
            DI_HIP(hipMemcpyAsync(out_n, don, (size_t)n_q * 4, hipMemcpyDeviceToHost, s));
        }
        if (!(flags & DI_F_ASYNC) || !dev) DI_HIP(hipStreamSynchronize(s));
    });
}

}  // extern "C"
