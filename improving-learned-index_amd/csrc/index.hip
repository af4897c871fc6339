// index.hip -- quantized inverted-index scorer for MI355X (gfx950).
//
// Replaces InvertedIndex.score (reference src/deep_impact/inverted_index/
// inverted_index.py:31-62) for batches of queries, bit-exact including the
// reference's tie order.
//
// Device layout ("doc-blocked, impact-ordered postings"):
//   docs of a shard are cut into blocks of BLOCK_DOCS = 32768; every term's
//   postings are grouped by block (block-major, then the reference order
//   value-desc/doc-asc).  One posting = one u32: (doc_in_block << 8) | value.
//   term_start[t] (i64) + blk_off[t*(NB+1)+b] (u32) locate the sublist (t, b).
//
// score_blocks: one 1024-thread workgroup per (query, block).  The block's
//   32768 accumulators live in LDS (128 KiB).  Terms are applied in query
//   order with a barrier between terms; inside a term every doc occurs once,
//   so plain LDS read-modify-write is race free and no atomics are needed.
//   Each LDS word is   score(16) | (255 - j)(8) | v_j(8)
//   where j is the first query term that touched the doc and v_j its value
//   there: comparing words reproduces the reference's order exactly -- score
//   descending, then first-touch order (term order, then impact desc inside
//   that term's list, then doc asc).  A block-wide radix select keeps the
//   block's top-k (ties in the last digit by doc ascending).
// merge_topk: one workgroup per query sorts the <= NB*k block candidates by
//   the 64-bit key  word(32) | ~doc(32)  and writes doc/score/key.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "di_common.h"
#include "topk_common.h"

namespace di {

constexpr int BLOCK_DOCS = 32768;
constexpr int SC_THREADS = 1024;
constexpr int SC_WAVES = SC_THREADS / 64;
constexpr int SC_PER_THREAD = BLOCK_DOCS / SC_THREADS;  // 32
constexpr int MAX_TERMS = DI_MAX_QUERY_TERMS;

struct ScoreShared {
    uint32_t acc[BLOCK_DOCS];  // 128 KiB
    RadixScratch<SC_WAVES> rs;
    int64_t lo[MAX_TERMS];
    int64_t hi[MAX_TERMS];
    uint32_t emit;  // output cursor
    uint32_t tie_need;
};

// One radix pass over the block's words (i-major: lanes read consecutive words,
// conflict-free).  KeyF: word,index -> key;  Pred: word,index,key -> bool.
template <class KeyF, class Pred>
__device__ __forceinline__ void score_radix_pass(ScoreShared &sh, int n_local, int shift,
                                                 uint32_t need, KeyF key, Pred pred) {
    radix_clear<SC_THREADS, SC_WAVES>(sh.rs);
    __syncthreads();
    RunLen rl;
#pragma unroll 4
    for (int i = 0; i < SC_PER_THREAD; ++i) {
        int idx = i * SC_THREADS + threadIdx.x;
        if (idx < n_local) {
            uint32_t w = sh.acc[idx];
            uint32_t kk = key(w, idx);
            if (pred(w, idx, kk)) rl.add(sh.rs, (kk >> shift) & 255u);
        }
    }
    rl.flush(sh.rs);
    __syncthreads();
    radix_pick<SC_THREADS, SC_WAVES>(sh.rs, need);
}

__global__ void __launch_bounds__(SC_THREADS)
score_blocks_kernel(const uint32_t *__restrict__ post, const int64_t *__restrict__ term_start,
                    const uint32_t *__restrict__ blk_off, int nb, int64_t n_terms,
                    uint32_t n_docs, uint32_t doc_lo, const uint32_t *__restrict__ q_terms,
                    const int32_t *__restrict__ cu_q, int k, uint64_t *__restrict__ cand_key,
                    int32_t *__restrict__ cand_n, int ablate) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ScoreShared &sh = *reinterpret_cast<ScoreShared *>(smem);

    const int b = blockIdx.x % nb;
    const int q = blockIdx.x / nb;
    const int tid = threadIdx.x;
    const int64_t block_first = (int64_t)b * BLOCK_DOCS;
    const int n_local = (int)min((int64_t)BLOCK_DOCS, (int64_t)n_docs - block_first);
    const int q0 = cu_q[q], nt = cu_q[q + 1] - q0;
    uint64_t *ck = cand_key + ((int64_t)q * nb + b) * k;

    if (nt > MAX_TERMS || nt < 0 || n_local <= 0) {
        if (tid == 0) cand_n[(int64_t)q * nb + b] = (nt > MAX_TERMS || nt < 0) ? -1 : 0;
        return;
    }
    if (tid == 0) sh.tie_need = 0;
    __syncthreads();

    // sublist bounds for this block, zero the accumulators
    for (int j = tid; j < nt; j += SC_THREADS) {
        uint32_t t = q_terms[q0 + j];
        if (t >= n_terms) {  // invalid id (device-pointer callers are not pre-checked)
            sh.tie_need = 1;
            sh.lo[j] = sh.hi[j] = 0;
            continue;
        }
        const uint32_t *bo = blk_off + (int64_t)t * (nb + 1) + b;
        sh.lo[j] = term_start[t] + bo[0];
        sh.hi[j] = term_start[t] + bo[1];
    }
    {
        uint4 *a4 = reinterpret_cast<uint4 *>(sh.acc);
        for (int i = tid; i < BLOCK_DOCS / 4; i += SC_THREADS) a4[i] = make_uint4(0, 0, 0, 0);
    }
    if (tid == 0) sh.emit = 0;
    __syncthreads();
    if (sh.tie_need) {
        if (tid == 0) cand_n[(int64_t)q * nb + b] = -1;
        return;
    }

    // ---- scatter: terms in query order, barrier between terms -------------
    // The postings of (term j, this block) are walked in rounds of SC_THREADS*U
    // dwords (coalesced: lane-consecutive).  The next round's loads are issued
    // before the current round is applied, also across a term boundary, so each
    // term's barrier no longer exposes a memory round trip.
    constexpr int U = 16;  // 64 B of postings in flight per lane, plus the next round
    constexpr int ROUND = SC_THREADS * U;
    auto rounds = [&](int jj) { return (int)((sh.hi[jj] - sh.lo[jj] + ROUND - 1) / ROUND); };
    auto load_round = [&](int jj, int rr, uint32_t (&r)[U]) {
        const int64_t base = sh.lo[jj] + (int64_t)rr * ROUND + tid, hi = sh.hi[jj];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t i = base + (int64_t)u * SC_THREADS;
            r[u] = (i < hi) ? post[i] : 0u;
        }
    };
    int j = (ablate & 1) ? nt : 0, rr = 0;  // ablate bit 0: skip the scatter (profiling)
    while (j < nt && rounds(j) == 0) ++j;
    uint32_t cur[U], nxt[U];
    if (j < nt) load_round(j, rr, cur);
    while (j < nt) {
        int jn = j, rn = rr + 1;
        while (jn < nt && rn >= rounds(jn)) {
            ++jn;
            rn = 0;
        }
        if (jn < nt) load_round(jn, rn, nxt);
        const uint32_t first_bits = (uint32_t)(255 - j) << 8;
        uint32_t w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = sh.acc[(cur[u] >> 8) & (BLOCK_DOCS - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = cur[u] & 255u;  // 0 only for the padding lanes
            if (v) {
                uint32_t x = w[u];
                x = x ? x + (v << 16) : ((v << 16) | first_bits | v);
                sh.acc[(cur[u] >> 8) & (BLOCK_DOCS - 1)] = x;
            }
        }
        if (jn != j) __syncthreads();  // term boundary (uniform across the block)
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        j = jn;
        rr = rn;
    }
    __syncthreads();

    if (ablate & 2) {  // profiling: skip the selection
        if (tid == 0) cand_n[(int64_t)q * nb + b] = 0;
        return;
    }
    // ---- block top-k: radix select on the 32-bit words ---------------------
    auto id_key = [](uint32_t w, int) { return w; };
    uint32_t need = (uint32_t)k, prefix = 0, mask = 0;
    // pass 0 also counts touched docs
    score_radix_pass(sh, n_local, 24, need, id_key,
                     [](uint32_t w, int, uint32_t) { return w != 0; });
    const uint32_t touched = sh.rs.total;
    const uint64_t doc_base = (uint64_t)doc_lo + (uint64_t)block_first;
    auto emit = [&](uint32_t w, int idx) {
        uint32_t pos = atomicAdd(&sh.emit, 1u);
        uint32_t doc = (uint32_t)(doc_base + (uint64_t)idx);
        if (pos < (uint32_t)k) ck[pos] = ((uint64_t)w << 32) | (uint64_t)(0xFFFFFFFFu - doc);
    };
    if (touched <= (uint32_t)k) {
        for (int i = 0; i < SC_PER_THREAD; ++i) {
            int idx = i * SC_THREADS + tid;
            if (idx < n_local && sh.acc[idx]) emit(sh.acc[idx], idx);
        }
        __syncthreads();
        if (tid == 0) cand_n[(int64_t)q * nb + b] = (int32_t)min(sh.emit, (uint32_t)k);
        return;
    }
    for (int shift = 24;; shift -= 8) {
        prefix |= sh.rs.bin << shift;
        mask |= 255u << shift;
        need -= sh.rs.above;
        if (shift == 0) break;
        __syncthreads();
        score_radix_pass(sh, n_local, shift - 8, need, id_key,
                         [prefix, mask](uint32_t w, int, uint32_t) {
                             return w != 0 && (w & mask) == prefix;
                         });
    }
    const uint32_t T = prefix;
    const uint32_t ties = sh.rs.tot[sh.rs.bin];
    // doc-order cut among the ties: the `need` smallest doc indices
    // (all ties when exactly `need` of them exist)
    uint32_t dcut = 0;
    if (ties != need) {
        uint32_t dneed = need, dprefix = 0, dmask = 0;
        auto dkey = [](uint32_t, int idx) { return 0xFFFFu - (uint32_t)idx; };
        for (int shift = 8;; shift -= 8) {
            __syncthreads();
            score_radix_pass(sh, n_local, shift, dneed, dkey,
                             [T, dprefix, dmask](uint32_t w, int, uint32_t kk) {
                                 return w == T && (kk & dmask) == dprefix;
                             });
            dprefix |= sh.rs.bin << shift;
            dmask |= 255u << shift;
            dneed -= sh.rs.above;
            if (shift == 0) break;
        }
        dcut = dprefix;  // keep ties whose (0xFFFF - idx) >= dcut
    }
    for (int i = 0; i < SC_PER_THREAD; ++i) {
        int idx = i * SC_THREADS + tid;
        if (idx >= n_local) break;
        uint32_t w = sh.acc[idx];
        if (w > T || (w == T && (0xFFFFu - (uint32_t)idx) >= dcut)) emit(w, idx);
    }
    __syncthreads();
    // sh.emit == k by construction; anything else is a selection bug -> flag it
    if (tid == 0) cand_n[(int64_t)q * nb + b] = sh.emit == (uint32_t)k ? k : -2;
}

// ---------------------------------------------------------------------------
// merge: per query, the top-k of n_lists candidate lists by 64-bit key
// ---------------------------------------------------------------------------
constexpr int MG_LDS_KEYS = 16384;  // fast path: every candidate fits in LDS

template <int THREADS>
struct alignas(16) MergeHead {  // 16-byte multiple: the u64 key array follows it
    RadixScratch<THREADS / 64> rs;
    int32_t off[1025];
    uint32_t cnt;
    int32_t bad;
    uint32_t pad[2];
};

enum DecodeMode : int { DECODE_QUANT = 0, DECODE_SPARSE = 1, DECODE_NONE = 2 };

// keys: the LDS key array holds `cap` entries (power of two, <= MG_LDS_KEYS)
template <int THREADS>
__global__ void __launch_bounds__(THREADS)
merge_topk_kernel(const uint64_t *__restrict__ keys, const int32_t *__restrict__ counts,
                  int n_lists, int k_in, int k, int64_t list_stride, int64_t cnt_stride,
                  int64_t q_stride, int64_t cq_stride, int cap,
                  uint64_t *__restrict__ out_key, uint32_t *__restrict__ out_doc,
                  uint32_t *__restrict__ out_score, int32_t *__restrict__ out_n, int mode) {
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
        for (int l = tid; l < n_lists; l += THREADS) {
            int c = cnt(l);
            if (c < 0) sh.bad = 1;
            sh.off[l + 1] = min(max(c, 0), k_in);
        }
        __syncthreads();
        if (tid == 0) {
            sh.off[0] = 0;
            for (int l = 0; l < n_lists; ++l) sh.off[l + 1] += sh.off[l];
        }
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
        for (int l = 0; l < n_lists; ++l) {
            const int o = sh.off[l], c = sh.off[l + 1] - o;
            const uint64_t *s = src0 + (int64_t)l * list_stride;
            for (int i = tid; i < c; i += THREADS) lk[o + i] = s[i];
        }
        __syncthreads();
    } else {
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
    int n2 = 64;
    while (n2 < total) n2 <<= 1;
    for (int i = (int)total + tid; i < n2; i += THREADS) lk[i] = 0;
    __syncthreads();
    bitonic_sort_desc<THREADS>(lk, n2);
    for (int i = tid; i < take; i += THREADS) {
        uint64_t x = lk[i];
        if (ok) ok[i] = x;
        if (mode == DECODE_QUANT) {
            out_doc[(int64_t)q * k + i] = 0xFFFFFFFFu - (uint32_t)x;
            out_score[(int64_t)q * k + i] = (uint32_t)(x >> 48);
        } else if (mode == DECODE_SPARSE) {
            out_doc[(int64_t)q * k + i] = 0xFFFFFFu - (uint32_t)(x & 0xFFFFFFu);
            out_score[(int64_t)q * k + i] = (uint32_t)(x >> 32);  // f32 bits
        }
    }
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
    int64_t n_terms = 0, n_post = 0;
    uint32_t n_docs = 0, doc_lo = 0;  // shard [doc_lo, doc_lo + n_docs)
    int nb = 0;
    DevBuf post, term_start, blk_off;
    DevBuf ws_q, ws_cu, ws_ck, ws_cn, ws_doc, ws_score, ws_n, ws_key;
    int ablate = 0;  // DI_PROFILE_ABLATE (profiling builds of the bench only)
    Timer timer;
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

void build_index(di_index *ix, const int64_t *term_off, int64_t n_terms, const uint32_t *pdoc,
                 const uint8_t *pval, uint32_t doc_lo, uint32_t doc_hi) {
    DI_REQUIRE(n_terms >= 0, DI_EINVAL, "n_terms < 0");
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
    const int nb = (int)((nd + BLOCK_DOCS - 1) / BLOCK_DOCS);
    ix->n_terms = n_terms;
    ix->n_docs = nd;
    ix->doc_lo = doc_lo;
    ix->nb = nb;
    const int64_t stride = nb + 1;
    std::vector<int64_t> tstart(std::max<int64_t>(n_terms, 1), 0);
    std::vector<uint32_t> boff((size_t)std::max<int64_t>(n_terms * stride, 1), 0);
    // pass 1: per (term, block) counts of kept postings
    int64_t total = 0;
    std::vector<uint32_t> cnt(stride);
    for (int64_t t = 0; t < n_terms; ++t) {
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
            if (pval[p] == 0) break;  // inverted_index.py:50-51
            uint32_t d = pdoc[p];
            if (d < doc_lo || d >= doc_hi) continue;
            cnt[(d - doc_lo) / BLOCK_DOCS]++;
        }
        tstart[t] = total;
        uint32_t run = 0;
        for (int b = 0; b < nb; ++b) {
            boff[t * stride + b] = run;
            run += cnt[b];
        }
        boff[t * stride + nb] = run;
        total += run;
    }
    ix->n_post = total;
    std::vector<uint32_t> packed((size_t)std::max<int64_t>(total, 4));
    // pass 2: place (stable: keeps value-desc/doc-asc inside each block)
    std::vector<uint32_t> cur(stride);
    for (int64_t t = 0; t < n_terms; ++t) {
        for (int b = 0; b <= nb; ++b) cur[b] = boff[t * stride + b];
        for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
            if (pval[p] == 0) break;
            uint32_t d = pdoc[p];
            if (d < doc_lo || d >= doc_hi) continue;
            uint32_t r = d - doc_lo;
            int b = (int)(r / BLOCK_DOCS);
            packed[tstart[t] + cur[b]++] = ((r % BLOCK_DOCS) << 8) | pval[p];
        }
    }
    ix->post.reserve(packed.size() * 4);
    ix->term_start.reserve(tstart.size() * 8);
    ix->blk_off.reserve(boff.size() * 4);
    DI_HIP(hipMemcpy(ix->post.p, packed.data(), packed.size() * 4, hipMemcpyHostToDevice));
    DI_HIP(hipMemcpy(ix->term_start.p, tstart.data(), tstart.size() * 8, hipMemcpyHostToDevice));
    DI_HIP(hipMemcpy(ix->blk_off.p, boff.data(), boff.size() * 4, hipMemcpyHostToDevice));
}

}  // namespace

namespace di {
// Kernels using more than 64 KiB of dynamic LDS must opt in, once per device.
void enable_big_lds() {
    static_assert(sizeof(ScoreShared) <= 160 * 1024, "ScoreShared exceeds LDS");
    DI_HIP(hipFuncSetAttribute((const void *)score_blocks_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(ScoreShared)));
    DI_HIP(hipFuncSetAttribute((const void *)merge_topk_kernel<1024>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(MergeHead<1024>) + MG_LDS_KEYS * 8)));
    DI_HIP(hipFuncSetAttribute((const void *)merge_topk_kernel<256>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(MergeHead<256>) + MG_LDS_KEYS * 8)));
}

void launch_merge(const uint64_t *keys, const int32_t *counts, int n_q, int n_lists, int k_in,
                  int k, uint64_t *out_key, uint32_t *out_doc, uint32_t *out_score,
                  int32_t *out_n, int mode, hipStream_t s, bool lists_major = false) {
    if (n_q == 0) return;
    int64_t ls = k_in, cs = 1, qs = (int64_t)n_lists * k_in, cqs = n_lists;
    if (lists_major) {
        ls = (int64_t)n_q * k_in;
        cs = n_q;
        qs = k_in;
        cqs = 1;
    }
    // LDS key capacity: all candidates when they fit, else the k survivors of the
    // slow path's radix select
    int64_t want = (int64_t)n_lists * k_in;
    if (n_lists > 1024 || want > MG_LDS_KEYS) want = k;
    int cap = 64;
    while (cap < want) cap <<= 1;
    if (cap <= 256) {
        size_t lds = sizeof(MergeHead<256>) + (size_t)cap * 8;
        hipLaunchKernelGGL(merge_topk_kernel<256>, dim3(n_q), dim3(256), lds, s, keys, counts,
                           n_lists, k_in, k, ls, cs, qs, cqs, cap, out_key, out_doc, out_score,
                           out_n, mode);
    } else {
        size_t lds = sizeof(MergeHead<1024>) + (size_t)cap * 8;
        hipLaunchKernelGGL(merge_topk_kernel<1024>, dim3(n_q), dim3(1024), lds, s, keys,
                           counts, n_lists, k_in, k, ls, cs, qs, cqs, cap, out_key, out_doc,
                           out_score, out_n, mode);
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
        build_index(ix.get(), term_off, n_terms, pdoc, pval, doc_lo, doc_hi);
        *out = ix.release();
    });
}

int di_index_load_reference(const char *dir, uint32_t doc_lo, uint32_t doc_hi, int device,
                            di_index **out) {
    return guard([&] {
        DI_REQUIRE(dir && out, DI_EINVAL, "null argument");
        std::string d(dir);
        std::ifstream fi(d + "/inverted_index.idx", std::ios::binary | std::ios::ate);
        std::ifstream fd(d + "/inverted_index.dat", std::ios::binary | std::ios::ate);
        DI_REQUIRE(fi && fd, DI_EIO, "cannot open %s/inverted_index.{idx,dat}", dir);
        size_t isz = (size_t)fi.tellg(), dsz = (size_t)fd.tellg();
        DI_REQUIRE(isz % 16 == 0, DI_EFORMAT, "inverted_index.idx size %zu not a multiple of 16",
                   isz);
        DI_REQUIRE(dsz % 5 == 0, DI_EFORMAT, "inverted_index.dat size %zu not a multiple of 5",
                   dsz);
        std::vector<uint64_t> idx(isz / 8);
        std::vector<unsigned char> dat(dsz);
        fi.seekg(0);
        fd.seekg(0);
        fi.read(reinterpret_cast<char *>(idx.data()), (std::streamsize)isz);
        fd.read(reinterpret_cast<char *>(dat.data()), (std::streamsize)dsz);
        const int64_t nt = (int64_t)(isz / 16), np = (int64_t)(dsz / 5);
        // postings of term t: records [start/5, end/5) -- create.py:45-51
        std::vector<int64_t> term_off(nt + 1, 0);
        std::vector<uint32_t> pdoc;
        std::vector<uint8_t> pval;
        pdoc.reserve(np);
        pval.reserve(np);
        for (int64_t t = 0; t < nt; ++t) {
            uint64_t s = idx[2 * t], e = idx[2 * t + 1];
            DI_REQUIRE(s % 5 == 0 && e % 5 == 0 && s <= e && e <= dsz, DI_EFORMAT,
                       "bad (start,end) for term %lld", (long long)t);
            for (uint64_t r = s / 5; r < e / 5; ++r) {
                uint32_t doc;
                std::memcpy(&doc, &dat[r * 5], 4);
                pdoc.push_back(doc);
                pval.push_back(dat[r * 5 + 4]);
            }
            term_off[t + 1] = (int64_t)pdoc.size();
        }
        int rc = di_index_create(term_off.data(), nt, pdoc.data(), pval.data(), doc_lo, doc_hi,
                                 device, out);
        if (rc != DI_OK) throw Error{rc};
    });
}

int di_index_reserve(di_index *ix, int32_t max_q, int32_t k) {
    return guard([&] {
        DI_REQUIRE(ix && max_q >= 0 && k > 0 && k <= DI_MAX_TOPK, DI_EINVAL, "bad argument");
        DeviceScope ds(ix->device);
        size_t nbk = (size_t)max_q * std::max(ix->nb, 1) * k;
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
        if (!dev) {
            for (int q = 0; q < n_q; ++q) {
                int32_t c = cu_q[q + 1] - cu_q[q];
                DI_REQUIRE(c >= 0, DI_EINVAL, "cu_q not monotone at %d", q);
                DI_REQUIRE(c <= DI_MAX_QUERY_TERMS, DI_ERANGE,
                           "query %d has %d terms (limit %d)", q, c, DI_MAX_QUERY_TERMS);
            }
            nterms_total = cu_q[n_q];
            for (int64_t i = 0; i < nterms_total; ++i)
                DI_REQUIRE(q_terms[i] < (uint64_t)ix->n_terms, DI_EINVAL,
                           "term id %u out of range", q_terms[i]);
        }
        const int nb = std::max(ix->nb, 1);
        // query chunking keeps the candidate workspace bounded (<= 1 GiB)
        const int64_t per_q = (int64_t)nb * k * 8;
        const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(n_q, (1ll << 30) / per_q));
        ix->ws_ck.reserve((size_t)chunk * per_q);
        ix->ws_cn.reserve((size_t)chunk * nb * 4);
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
                TimedLaunch tl(ix->timer, timing, "score_blocks", s);
                hipLaunchKernelGGL(score_blocks_kernel, dim3(nq * nb), dim3(SC_THREADS),
                                   sizeof(ScoreShared), s, ix->post.as<uint32_t>(),
                                   ix->term_start.as<int64_t>(), ix->blk_off.as<uint32_t>(), nb,
                                   ix->n_terms, ix->n_docs, ix->doc_lo, dq, dcu + q0, k,
                                   ix->ws_ck.as<uint64_t>(), ix->ws_cn.as<int32_t>(),
                                   ix->ablate);
                check_launch("score_blocks");
            }
            {
                TimedLaunch tl(ix->timer, timing, "merge_topk", s);
                launch_merge(ix->ws_ck.as<uint64_t>(), ix->ws_cn.as<int32_t>(), nq, nb, k, k,
                             dkey ? dkey + (int64_t)q0 * k : nullptr, ddoc + (int64_t)q0 * k,
                             dscore + (int64_t)q0 * k, dn + q0, DECODE_QUANT, s);
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
