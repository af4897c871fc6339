// sparse.hip -- the in-memory float-impact index of the NanoBEIR evaluator on
// MI355X.  Replaces SparseSearch (reference src/deep_impact/evaluation/
// nano_beir_evaluator.py:70-137): postings term -> [(doc, float32 impact)] in
// corpus order, impacts > 0 only (:96-99); per query doc_scores[doc] += impact
// over the query terms in iteration order (:113-121); top-k by score with ties
// in first-touch order (stable sorted()/heapq.nlargest, :124-133).
//
// Float32 accumulation (numpy >= 2 semantics of `0.0 + np.float32`, the
// environment the reference runs in here): terms are applied one
// after the other with a barrier in between and each doc occurs once per term, so
// every doc's sum is formed in exactly the reference's order -- bit-exact scores.
//
// Layout: docs in blocks of SP_DOCS = 16384; per term, postings grouped by block
// (doc ascending inside); SoA: u16 doc-in-block + f32 impact.
// Selection key (unique per doc): score bits(32) | 255-j(8) | 0xFFFF-local(16),
// j = first query term that touched the doc -- first-touch order is term order,
// then doc (corpus) order inside the term.  Merge key: score bits(32) |
// 255-j(8) | 0xFFFFFF-doc(24).
// Long queries (argument-style NanoBEIR queries can pass 256 unique terms): terms go
// in chunks of SP_MAX_TERMS, the accumulators carrying over, up to
// DI_MAX_SPARSE_QUERY_TERMS; the sums stay exact, and j saturates at 255, so only
// docs with EXACTLY equal scores first touched by terms 255, 256, ... are ordered by
// corpus order instead of by (term, corpus order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "di_common.h"
#include "topk_common.h"

namespace di {

constexpr int SP_DOCS = 16384;
constexpr int SP_THREADS = 1024;
constexpr int SP_WAVES = SP_THREADS / 64;
constexpr int SP_PER_THREAD = SP_DOCS / SP_THREADS;  // 16
constexpr int SP_MAX_TERMS = 256;  // term bounds per chunk (LDS)

struct SparseShared {
    float acc[SP_DOCS];          // 64 KiB
    uint8_t first[SP_DOCS];      // 16 KiB
    RadixScratch<SP_WAVES> rs;
    int64_t lo[SP_MAX_TERMS];
    int64_t hi[SP_MAX_TERMS];
    uint32_t emit;
    int32_t bad;
};

__device__ __forceinline__ uint64_t sp_key(const SparseShared &sh, int idx) {
    const float a = sh.acc[idx];
    return ((uint64_t)__float_as_uint(a) << 24) | ((uint64_t)(255u - sh.first[idx]) << 16) |
           (uint64_t)(0xFFFFu - (uint32_t)idx);
}

__global__ void __launch_bounds__(SP_THREADS)
sparse_score_kernel(const uint16_t *__restrict__ pdoc, const float *__restrict__ pimp,
                    const int64_t *__restrict__ term_start, const uint32_t *__restrict__ blk_off,
                    int nb, int64_t n_terms, uint32_t n_docs, const uint32_t *__restrict__ q_terms,
                    const int32_t *__restrict__ cu_q, int k, uint64_t *__restrict__ cand_key,
                    int32_t *__restrict__ cand_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    SparseShared &sh = *reinterpret_cast<SparseShared *>(smem);
    const int b = blockIdx.x % nb, q = blockIdx.x / nb, tid = threadIdx.x;
    const int64_t first_doc = (int64_t)b * SP_DOCS;
    const int n_local = (int)min((int64_t)SP_DOCS, (int64_t)n_docs - first_doc);
    const int q0 = cu_q[q], nt = cu_q[q + 1] - q0;
    int32_t *cn = cand_n + (int64_t)q * nb + b;
    uint64_t *ck = cand_key + ((int64_t)q * nb + b) * k;
    if (nt > DI_MAX_SPARSE_QUERY_TERMS || nt < 0 || n_local <= 0) {
        if (tid == 0) *cn = (nt > DI_MAX_SPARSE_QUERY_TERMS || nt < 0) ? -1 : 0;
        return;
    }
    if (tid == 0) {
        sh.bad = 0;
        sh.emit = 0;
    }
    for (int i = tid; i < SP_DOCS; i += SP_THREADS) sh.acc[i] = 0.f;
    // ---- accumulate: terms in query order, one barrier per term, chunks of
    // SP_MAX_TERMS term bounds ----
    for (int c0 = 0; c0 < nt; c0 += SP_MAX_TERMS) {
        const int cn_t = min(SP_MAX_TERMS, nt - c0);
        __syncthreads();  // the previous chunk's bounds are no longer read
        for (int j = tid; j < cn_t; j += SP_THREADS) {
            uint32_t t = q_terms[q0 + c0 + j];
            if (t >= n_terms) {
                sh.bad = 1;
                sh.lo[j] = sh.hi[j] = 0;
                continue;
            }
            const uint32_t *bo = blk_off + (int64_t)t * (nb + 1) + b;
            sh.lo[j] = term_start[t] + bo[0];
            sh.hi[j] = term_start[t] + bo[1];
        }
        __syncthreads();
        if (sh.bad) {
            if (tid == 0) *cn = -1;
            return;
        }
        for (int j = 0; j < cn_t; ++j) {
            const uint8_t jj = (uint8_t)min(c0 + j, 255);
            for (int64_t i = sh.lo[j] + tid; i < sh.hi[j]; i += SP_THREADS) {
                const int d = pdoc[i] & (SP_DOCS - 1);
                const float a = sh.acc[d];
                if (a == 0.f) sh.first[d] = jj;  // impacts > 0: 0 == untouched
                sh.acc[d] = a + pimp[i];
            }
            __syncthreads();
        }
    }
    // ---- block top-k over the unique 56-bit keys (untouched docs: key < 2^40) ----
    uint64_t prefix = 0, mask = 0;
    uint32_t need = (uint32_t)k;
    bool all_in = false;
    for (int shift = 48; shift >= 0; shift -= 8) {
        radix_clear<SP_THREADS, SP_WAVES>(sh.rs);
        __syncthreads();
        RunLen rl;
        for (int i = 0; i < SP_PER_THREAD; ++i) {
            const int idx = i * SP_THREADS + tid;
            if (idx < n_local && sh.acc[idx] != 0.f) {
                const uint64_t key = sp_key(sh, idx);
                if ((key & mask) == prefix) rl.add(sh.rs, (uint32_t)(key >> shift) & 255u);
            }
        }
        rl.flush(sh.rs);
        __syncthreads();
        radix_pick<SP_THREADS, SP_WAVES>(sh.rs, need);
        if (shift == 48 && sh.rs.total <= need) {  // fewer touched docs than k
            all_in = true;
            break;
        }
        prefix |= (uint64_t)sh.rs.bin << shift;
        mask |= (uint64_t)255 << shift;
        const uint32_t in_bin = sh.rs.tot[sh.rs.bin];
        need -= sh.rs.above;
        __syncthreads();
        if (in_bin == need) break;  // every key of this bin is taken: keys >= prefix
    }
    const uint64_t doc_base = (uint64_t)first_doc;
    for (int i = 0; i < SP_PER_THREAD; ++i) {
        const int idx = i * SP_THREADS + tid;
        if (idx >= n_local || sh.acc[idx] == 0.f) continue;
        const uint64_t key = sp_key(sh, idx);
        if (all_in || key >= prefix) {
            const uint32_t pos = atomicAdd(&sh.emit, 1u);
            const uint32_t doc = (uint32_t)(doc_base + (uint64_t)idx);
            if (pos < (uint32_t)k)
                ck[pos] = ((uint64_t)__float_as_uint(sh.acc[idx]) << 32) |
                          ((uint64_t)(255u - sh.first[idx]) << 24) |
                          (uint64_t)(0xFFFFFFu - doc);
        }
    }
    __syncthreads();
    if (tid == 0) *cn = (int32_t)min(sh.emit, (uint32_t)k);
}

// ---- f64 accumulation (the reference's pinned numpy 1.25: `0.0 + np.float32` is an
// np.float64, so doc_scores holds f64 sums of the f32 impacts) ----
// A 64-bit score no longer fits one 64-bit key with the tie fields, so the selection
// runs over 96-bit keys (hi = f64 bits, positive scores order as unsigned; lo =
// (255 - j) << 24 | (0xFFFFFF - doc)) with 12 radix digits.  The f64 accumulators
// take twice the LDS: a workgroup owns one half (8192 docs) of a 16384-doc block and
// skips the other half's postings.
constexpr int SP64_DOCS = SP_DOCS / 2;
constexpr int SP64_PER_THREAD = SP64_DOCS / SP_THREADS;  // 8

struct Key96 {
    uint64_t hi;
    uint32_t lo;
};
__device__ __forceinline__ bool ge96(uint64_t h, uint32_t l, uint64_t ph, uint32_t pl) {
    return h > ph || (h == ph && l >= pl);
}
__device__ __forceinline__ uint32_t digit96(uint64_t h, uint32_t l, int d) {
    return d < 8 ? (uint32_t)(h >> (56 - 8 * d)) & 255u : (l >> (24 - 8 * (d - 8))) & 255u;
}

// One radix-select round over 12 digits, shared by the block and merge kernels.
// visit(f) calls f(hi, lo) for every key of the candidate set (all threads).  Leaves
// (ph, pl) such that the k largest keys are exactly those >= (ph, pl); all_in when
// the set has at most k keys.
template <typename Visit>
__device__ __forceinline__ void select96(RadixScratch<SP_WAVES> &rs, uint32_t k, Visit visit,
                                         uint64_t &ph, uint32_t &pl, bool &all_in) {
    uint64_t mh = 0;
    uint32_t ml = 0, need = k;
    ph = 0;
    pl = 0;
    all_in = false;
    for (int d = 0; d < 12; ++d) {
        radix_clear<SP_THREADS, SP_WAVES>(rs);
        __syncthreads();
        RunLen rl;
        visit([&](uint64_t h, uint32_t l) {
            if ((h & mh) == ph && (l & ml) == pl) rl.add(rs, digit96(h, l, d));
        });
        rl.flush(rs);
        __syncthreads();
        radix_pick<SP_THREADS, SP_WAVES>(rs, need);
        if (d == 0 && rs.total <= need) {
            all_in = true;
            return;
        }
        if (d < 8) {
            ph |= (uint64_t)rs.bin << (56 - 8 * d);
            mh |= (uint64_t)255 << (56 - 8 * d);
        } else {
            pl |= rs.bin << (24 - 8 * (d - 8));
            ml |= 255u << (24 - 8 * (d - 8));
        }
        const uint32_t in_bin = rs.tot[rs.bin];
        need -= rs.above;
        __syncthreads();
        if (in_bin == need) return;  // every key of this digit is taken
    }
}

struct Sparse64Shared {
    double acc[SP64_DOCS];   // 64 KiB
    uint8_t first[SP64_DOCS];
    RadixScratch<SP_WAVES> rs;
    int64_t lo[SP_MAX_TERMS];
    int64_t hi[SP_MAX_TERMS];
    uint32_t emit;
    int32_t bad;
};

__global__ void __launch_bounds__(SP_THREADS)
sparse_score64_kernel(const uint16_t *__restrict__ pdoc, const float *__restrict__ pimp,
                      const int64_t *__restrict__ term_start, const uint32_t *__restrict__ blk_off,
                      int nb, int64_t n_terms, uint32_t n_docs,
                      const uint32_t *__restrict__ q_terms, const int32_t *__restrict__ cu_q, int k,
                      Key96 *__restrict__ cand, int32_t *__restrict__ cand_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Sparse64Shared &sh = *reinterpret_cast<Sparse64Shared *>(smem);
    const int nl = 2 * nb;
    const int l = blockIdx.x % nl, q = blockIdx.x / nl, tid = threadIdx.x;
    const int b = l >> 1, half = l & 1;
    const int64_t first_doc = (int64_t)b * SP_DOCS + half * SP64_DOCS;
    const int n_local = (int)max((int64_t)0, min((int64_t)SP64_DOCS, (int64_t)n_docs - first_doc));
    const int q0 = cu_q[q], nt = cu_q[q + 1] - q0;
    int32_t *cn = cand_n + (int64_t)q * nl + l;
    Key96 *ck = cand + ((int64_t)q * nl + l) * k;
    if (nt > DI_MAX_SPARSE_QUERY_TERMS || nt < 0 || n_local <= 0) {
        if (tid == 0) *cn = (nt > DI_MAX_SPARSE_QUERY_TERMS || nt < 0) ? -1 : 0;
        return;
    }
    if (tid == 0) {
        sh.bad = 0;
        sh.emit = 0;
    }
    for (int i = tid; i < SP64_DOCS; i += SP_THREADS) sh.acc[i] = 0.0;
    for (int c0 = 0; c0 < nt; c0 += SP_MAX_TERMS) {
        const int cn_t = min(SP_MAX_TERMS, nt - c0);
        __syncthreads();
        for (int j = tid; j < cn_t; j += SP_THREADS) {
            const uint32_t t = q_terms[q0 + c0 + j];
            if (t >= n_terms) {
                sh.bad = 1;
                sh.lo[j] = sh.hi[j] = 0;
                continue;
            }
            const uint32_t *bo = blk_off + (int64_t)t * (nb + 1) + b;
            sh.lo[j] = term_start[t] + bo[0];
            sh.hi[j] = term_start[t] + bo[1];
        }
        __syncthreads();
        if (sh.bad) {
            if (tid == 0) *cn = -1;
            return;
        }
        for (int j = 0; j < cn_t; ++j) {
            const uint8_t jj = (uint8_t)min(c0 + j, 255);
            for (int64_t i = sh.lo[j] + tid; i < sh.hi[j]; i += SP_THREADS) {
                const int dl = pdoc[i];
                if ((dl >> 13) != half) continue;
                const int d = dl & (SP64_DOCS - 1);
                const double a = sh.acc[d];
                if (a == 0.0) sh.first[d] = jj;
                sh.acc[d] = a + (double)pimp[i];  // numpy 1.25: f64 + np.float32 -> f64
            }
            __syncthreads();
        }
    }
    const uint32_t doc_base = (uint32_t)first_doc;
    auto key_of = [&](int idx, uint64_t &h, uint32_t &lo) {
        h = (uint64_t)__double_as_longlong(sh.acc[idx]);
        lo = ((255u - sh.first[idx]) << 24) | (0xFFFFFFu - (doc_base + (uint32_t)idx));
    };
    uint64_t ph;
    uint32_t pl;
    bool all_in;
    select96(sh.rs, (uint32_t)k,
             [&](auto f) {
                 for (int i = 0; i < SP64_PER_THREAD; ++i) {
                     const int idx = i * SP_THREADS + tid;
                     if (idx < n_local && sh.acc[idx] != 0.0) {
                         uint64_t h;
                         uint32_t lo;
                         key_of(idx, h, lo);
                         f(h, lo);
                     }
                 }
             },
             ph, pl, all_in);
    for (int i = 0; i < SP64_PER_THREAD; ++i) {
        const int idx = i * SP_THREADS + tid;
        if (idx >= n_local || sh.acc[idx] == 0.0) continue;
        uint64_t h;
        uint32_t lo;
        key_of(idx, h, lo);
        if (all_in || ge96(h, lo, ph, pl)) {
            const uint32_t pos = atomicAdd(&sh.emit, 1u);
            if (pos < (uint32_t)k) ck[pos] = Key96{h, lo};
        }
    }
    __syncthreads();
    if (tid == 0) *cn = (int32_t)min(sh.emit, (uint32_t)k);
}

// Per query: the k largest 96-bit keys over its 2 nb lists, sorted descending, decoded
// to (doc, f64 score).  LDS: up to DI_MAX_TOPK selected keys.
struct Merge64Shared {
    uint64_t hi[DI_MAX_TOPK];
    uint32_t lo[DI_MAX_TOPK];
    RadixScratch<SP_WAVES> rs;
    uint32_t emit;
    int32_t bad;
};

__global__ void __launch_bounds__(SP_THREADS)
sparse_merge64_kernel(const Key96 *__restrict__ cand, const int32_t *__restrict__ cand_n, int nl,
                      int k, uint32_t *__restrict__ out_doc, double *__restrict__ out_score,
                      int32_t *__restrict__ out_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Merge64Shared &sh = *reinterpret_cast<Merge64Shared *>(smem);
    const int q = blockIdx.x, tid = threadIdx.x;
    const Key96 *ck = cand + (int64_t)q * nl * k;
    const int32_t *cn = cand_n + (int64_t)q * nl;
    if (tid == 0) {
        sh.emit = 0;
        sh.bad = 0;
    }
    __syncthreads();
    for (int l = tid; l < nl; l += SP_THREADS)
        if (cn[l] < 0) sh.bad = 1;
    __syncthreads();
    if (sh.bad) {
        if (tid == 0) out_n[q] = -1;
        return;
    }
    auto visit = [&](auto f) {
        for (int l = 0; l < nl; ++l) {
            const int c = cn[l];
            for (int i = tid; i < c; i += SP_THREADS) f(ck[(int64_t)l * k + i].hi, ck[(int64_t)l * k + i].lo);
        }
    };
    uint64_t ph;
    uint32_t pl;
    bool all_in;
    select96(sh.rs, (uint32_t)k, visit, ph, pl, all_in);
    visit([&](uint64_t h, uint32_t lo) {
        if (all_in || ge96(h, lo, ph, pl)) {
            const uint32_t pos = atomicAdd(&sh.emit, 1u);
            if (pos < (uint32_t)k) {
                sh.hi[pos] = h;
                sh.lo[pos] = lo;
            }
        }
    });
    __syncthreads();
    const int n = (int)min(sh.emit, (uint32_t)k);
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = n + tid; i < np2; i += SP_THREADS) {  // padding sorts last (scores > 0)
        sh.hi[i] = 0;
        sh.lo[i] = 0;
    }
    __syncthreads();
    for (int size = 2; size <= np2; size <<= 1) {  // bitonic, descending on (hi, lo)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < (np2 >> 1); i += SP_THREADS) {
                const int a = 2 * i - (i & (stride - 1)), c = a + stride;
                const bool desc = (a & size) == 0;
                const uint64_t ha = sh.hi[a], hc = sh.hi[c];
                const uint32_t la = sh.lo[a], lc = sh.lo[c];
                const bool lt = ha < hc || (ha == hc && la < lc);
                if (lt == desc) {
                    sh.hi[a] = hc;
                    sh.lo[a] = lc;
                    sh.hi[c] = ha;
                    sh.lo[c] = la;
                }
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < n; i += SP_THREADS) {
        out_doc[(int64_t)q * k + i] = 0xFFFFFFu - (sh.lo[i] & 0xFFFFFFu);
        out_score[(int64_t)q * k + i] = __longlong_as_double((long long)sh.hi[i]);
    }
    if (tid == 0) out_n[q] = n;
}

void launch_merge(const uint64_t *keys, const int32_t *counts, int n_q, int n_lists, int k_in,
                  int k, uint64_t *out_key, uint32_t *out_doc, uint32_t *out_score,
                  int32_t *out_n, int mode, hipStream_t s, bool lists_major,
                  const int32_t *cu_q);
void enable_big_lds();

}  // namespace di

using namespace di;

struct di_sparse {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int64_t n_terms = 0, n_post = 0;
    uint32_t n_docs = 0;
    int nb = 0;
    DevBuf pdoc, pimp, term_start, blk_off;
    DevBuf ws_q, ws_cu, ws_ck, ws_cn, ws_doc, ws_score, ws_n, ws_key;
    Timer timer;
};

namespace {
struct DevScope {
    int prev = -1;
    explicit DevScope(int d) {
        DI_HIP(hipGetDevice(&prev));
        if (prev != d) DI_HIP(hipSetDevice(d));
    }
    ~DevScope() {
        int c;
        if (hipGetDevice(&c) == hipSuccess && c != prev) (void)hipSetDevice(prev);
    }
};
}  // namespace

extern "C" {

int di_sparse_create(const int64_t *term_off, int64_t n_terms, const uint32_t *pdoc,
                     const float *pimp, uint32_t n_docs, int device, di_sparse **out) {
    return guard([&] {
        DI_REQUIRE(out && term_off && n_terms >= 0, DI_EINVAL, "bad argument");
        DI_REQUIRE(n_docs <= DI_MAX_SPARSE_DOCS, DI_ERANGE, "%u docs > %u", n_docs,
                   DI_MAX_SPARSE_DOCS);
        int ndev = 0;
        DI_REQUIRE(hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0, DI_ENODEV,
                   "no HIP device");
        DevScope ds(device);
        std::unique_ptr<di_sparse> sp(new di_sparse());
        sp->device = device;
        DI_HIP(hipStreamCreateWithFlags(&sp->stream, hipStreamNonBlocking));
        sp->own_stream = true;
        enable_big_lds();
        DI_HIP(hipFuncSetAttribute((const void *)sparse_score_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)sizeof(SparseShared)));
        DI_HIP(hipFuncSetAttribute((const void *)sparse_score64_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)sizeof(Sparse64Shared)));
        DI_HIP(hipFuncSetAttribute((const void *)sparse_merge64_kernel,
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)sizeof(Merge64Shared)));
        const int nb = (int)((n_docs + SP_DOCS - 1) / SP_DOCS);
        const int64_t stride = nb + 1;
        std::vector<int64_t> tstart(std::max<int64_t>(n_terms, 1), 0);
        std::vector<uint32_t> boff((size_t)std::max<int64_t>(n_terms * stride, 1), 0);
        std::vector<uint32_t> cnt(stride);
        int64_t total = 0;
        for (int64_t t = 0; t < n_terms; ++t) {
            DI_REQUIRE(term_off[t + 1] >= term_off[t], DI_EINVAL, "term_off not monotone");
            std::fill(cnt.begin(), cnt.end(), 0);
            for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
                DI_REQUIRE(pdoc[p] < n_docs, DI_EINVAL, "doc %u >= n_docs", pdoc[p]);
                if (pimp[p] > 0.f) cnt[pdoc[p] / SP_DOCS]++;  // nano_beir_evaluator.py:98
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
        std::vector<uint16_t> hd((size_t)std::max<int64_t>(total, 1));
        std::vector<float> hi((size_t)std::max<int64_t>(total, 1));
        std::vector<uint32_t> cur(stride);
        for (int64_t t = 0; t < n_terms; ++t) {
            for (int b = 0; b <= nb; ++b) cur[b] = boff[t * stride + b];
            for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
                if (!(pimp[p] > 0.f)) continue;
                const int b = (int)(pdoc[p] / SP_DOCS);
                const int64_t o = tstart[t] + cur[b]++;
                hd[(size_t)o] = (uint16_t)(pdoc[p] % SP_DOCS);
                hi[(size_t)o] = pimp[p];
            }
        }
        sp->n_terms = n_terms;
        sp->n_post = total;
        sp->n_docs = n_docs;
        sp->nb = nb;
        sp->pdoc.reserve(hd.size() * 2);
        sp->pimp.reserve(hi.size() * 4);
        sp->term_start.reserve(tstart.size() * 8);
        sp->blk_off.reserve(boff.size() * 4);
        DI_HIP(hipMemcpy(sp->pdoc.p, hd.data(), hd.size() * 2, hipMemcpyHostToDevice));
        DI_HIP(hipMemcpy(sp->pimp.p, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
        DI_HIP(hipMemcpy(sp->term_start.p, tstart.data(), tstart.size() * 8,
                         hipMemcpyHostToDevice));
        DI_HIP(hipMemcpy(sp->blk_off.p, boff.data(), boff.size() * 4, hipMemcpyHostToDevice));
        *out = sp.release();
    });
}

int di_sparse_search(di_sparse *sp, const uint32_t *q_terms, const int32_t *cu_q, int32_t n_q,
                     int32_t k, uint32_t *out_doc, float *out_score, int32_t *out_n,
                     uint64_t *out_key, uint32_t flags) {
    return guard([&] {
        DI_REQUIRE(sp && cu_q && out_doc && out_score && out_n && n_q >= 0, DI_EINVAL,
                   "bad argument");
        DI_REQUIRE(k > 0 && k <= DI_MAX_TOPK, DI_ERANGE, "k=%d outside [1, %d]", k,
                   DI_MAX_TOPK);
        DevScope ds(sp->device);
        const bool dev = flags & DI_F_DEVICE_PTRS, timing = flags & DI_F_TIMING;
        hipStream_t s = sp->stream;
        if (n_q == 0) return;
        int64_t ntot = 0;
        if (!dev) {
            for (int q = 0; q < n_q; ++q) {
                const int32_t c = cu_q[q + 1] - cu_q[q];
                DI_REQUIRE(c >= 0 && c <= DI_MAX_SPARSE_QUERY_TERMS, DI_ERANGE,
                           "query %d has %d terms (limit %d)", q, c, DI_MAX_SPARSE_QUERY_TERMS);
            }
            ntot = cu_q[n_q];
            for (int64_t i = 0; i < ntot; ++i)
                DI_REQUIRE(q_terms[i] < (uint64_t)sp->n_terms, DI_EINVAL, "term id %u",
                           q_terms[i]);
        }
        const int nb = std::max(sp->nb, 1);
        const int64_t per_q = (int64_t)nb * k * 8;
        const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(n_q, (1ll << 30) / per_q));
        sp->ws_ck.reserve((size_t)chunk * per_q);
        sp->ws_cn.reserve((size_t)chunk * nb * 4);
        const uint32_t *dq = (const uint32_t *)stage_in(q_terms, (size_t)ntot * 4, dev,
                                                        sp->ws_q, s);
        const int32_t *dcu =
            (const int32_t *)stage_in(cu_q, (size_t)(n_q + 1) * 4, dev, sp->ws_cu, s);
        uint32_t *ddoc = out_doc, *dsc = reinterpret_cast<uint32_t *>(out_score);
        int32_t *dn = out_n;
        uint64_t *dkey = out_key;
        if (!dev) {
            sp->ws_doc.reserve((size_t)n_q * k * 4);
            sp->ws_score.reserve((size_t)n_q * k * 4);
            sp->ws_n.reserve((size_t)n_q * 4);
            ddoc = sp->ws_doc.as<uint32_t>();
            dsc = sp->ws_score.as<uint32_t>();
            dn = sp->ws_n.as<int32_t>();
            if (out_key) {
                sp->ws_key.reserve((size_t)n_q * k * 8);
                dkey = sp->ws_key.as<uint64_t>();
            }
        }
        for (int q0 = 0; q0 < n_q; q0 += chunk) {
            const int nq = std::min(chunk, n_q - q0);
            if (sp->nb == 0) {
                DI_HIP(hipMemsetAsync(sp->ws_cn.p, 0, (size_t)nq * nb * 4, s));
            } else {
                TimedLaunch tl(sp->timer, timing, "sparse_score", s);
                hipLaunchKernelGGL(sparse_score_kernel, dim3(nq * nb), dim3(SP_THREADS),
                                   sizeof(SparseShared), s, sp->pdoc.as<uint16_t>(),
                                   sp->pimp.as<float>(), sp->term_start.as<int64_t>(),
                                   sp->blk_off.as<uint32_t>(), nb, sp->n_terms, sp->n_docs, dq,
                                   dcu + q0, k, sp->ws_ck.as<uint64_t>(),
                                   sp->ws_cn.as<int32_t>());
                check_launch("sparse_score");
            }
            TimedLaunch tl(sp->timer, timing, "merge_topk", s);
            launch_merge(sp->ws_ck.as<uint64_t>(), sp->ws_cn.as<int32_t>(), nq, nb, k, k,
                         dkey ? dkey + (int64_t)q0 * k : nullptr, ddoc + (int64_t)q0 * k,
                         dsc + (int64_t)q0 * k, dn + q0, 1 /*DECODE_SPARSE*/, s, false, nullptr);
        }
        if (!dev) {
            DI_HIP(hipMemcpyAsync(out_doc, ddoc, (size_t)n_q * k * 4, hipMemcpyDeviceToHost, s));
            DI_HIP(hipMemcpyAsync(out_score, dsc, (size_t)n_q * k * 4, hipMemcpyDeviceToHost, s));
            DI_HIP(hipMemcpyAsync(out_n, dn, (size_t)n_q * 4, hipMemcpyDeviceToHost, s));
            if (out_key)
                DI_HIP(hipMemcpyAsync(out_key, dkey, (size_t)n_q * k * 8, hipMemcpyDeviceToHost,
                                      s));
        }
        if (!(flags & DI_F_ASYNC) || !dev) {
            DI_HIP(hipStreamSynchronize(s));
            sp->timer.resolve();
            if (!dev)
                for (int q = 0; q < n_q; ++q)
                    DI_REQUIRE(out_n[q] >= 0, DI_ERANGE, "query %d exceeded a kernel limit", q);
        }
    });
}

int di_sparse_search_f64(di_sparse *sp, const uint32_t *q_terms, const int32_t *cu_q,
                         int32_t n_q, int32_t k, uint32_t *out_doc, double *out_score,
                         int32_t *out_n, uint32_t flags) {
    return guard([&] {
        DI_REQUIRE(sp && cu_q && out_doc && out_score && out_n && n_q >= 0, DI_EINVAL,
                   "bad argument");
        DI_REQUIRE(k > 0 && k <= DI_MAX_TOPK, DI_ERANGE, "k=%d outside [1, %d]", k,
                   DI_MAX_TOPK);
        DevScope ds(sp->device);
        const bool dev = flags & DI_F_DEVICE_PTRS, timing = flags & DI_F_TIMING;
        hipStream_t s = sp->stream;
        if (n_q == 0) return;
        int64_t ntot = 0;
        if (!dev) {
            for (int q = 0; q < n_q; ++q) {
                const int32_t c = cu_q[q + 1] - cu_q[q];
                DI_REQUIRE(c >= 0 && c <= DI_MAX_SPARSE_QUERY_TERMS, DI_ERANGE,
                           "query %d has %d terms (limit %d)", q, c, DI_MAX_SPARSE_QUERY_TERMS);
            }
            ntot = cu_q[n_q];
            for (int64_t i = 0; i < ntot; ++i)
                DI_REQUIRE(q_terms[i] < (uint64_t)sp->n_terms, DI_EINVAL, "term id %u",
                           q_terms[i]);
        }
        const int nl = 2 * std::max(sp->nb, 1);
        const int64_t per_q = (int64_t)nl * k * (int64_t)sizeof(Key96);
        const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(n_q, (1ll << 30) / per_q));
        sp->ws_ck.reserve((size_t)chunk * per_q);
        sp->ws_cn.reserve((size_t)chunk * nl * 4);
        const uint32_t *dq = (const uint32_t *)stage_in(q_terms, (size_t)ntot * 4, dev,
                                                        sp->ws_q, s);
        const int32_t *dcu =
            (const int32_t *)stage_in(cu_q, (size_t)(n_q + 1) * 4, dev, sp->ws_cu, s);
        uint32_t *ddoc = out_doc;
        double *dsc = out_score;
        int32_t *dn = out_n;
        if (!dev) {
            sp->ws_doc.reserve((size_t)n_q * k * 4);
            sp->ws_score.reserve((size_t)n_q * k * 8);
            sp->ws_n.reserve((size_t)n_q * 4);
            ddoc = sp->ws_doc.as<uint32_t>();
            dsc = sp->ws_score.as<double>();
            dn = sp->ws_n.as<int32_t>();
        }
        for (int q0 = 0; q0 < n_q; q0 += chunk) {
            const int nq = std::min(chunk, n_q - q0);
            Key96 *ck = sp->ws_ck.as<Key96>();
            if (sp->nb == 0) {
                DI_HIP(hipMemsetAsync(sp->ws_cn.p, 0, (size_t)nq * nl * 4, s));
            } else {
                TimedLaunch tl(sp->timer, timing, "sparse_score64", s);
                hipLaunchKernelGGL(sparse_score64_kernel, dim3(nq * nl), dim3(SP_THREADS),
                                   sizeof(Sparse64Shared), s, sp->pdoc.as<uint16_t>(),
                                   sp->pimp.as<float>(), sp->term_start.as<int64_t>(),
                                   sp->blk_off.as<uint32_t>(), sp->nb, sp->n_terms, sp->n_docs,
                                   dq, dcu + q0, k, ck, sp->ws_cn.as<int32_t>());
                check_launch("sparse_score64");
            }
            TimedLaunch tl(sp->timer, timing, "sparse_merge64", s);
            hipLaunchKernelGGL(sparse_merge64_kernel, dim3(nq), dim3(SP_THREADS),
                               sizeof(Merge64Shared), s, ck, sp->ws_cn.as<int32_t>(), nl, k,
                               ddoc + (int64_t)q0 * k, dsc + (int64_t)q0 * k, dn + q0);
            check_launch("sparse_merge64");
        }
        if (!dev) {
            DI_HIP(hipMemcpyAsync(out_doc, ddoc, (size_t)n_q * k * 4, hipMemcpyDeviceToHost, s));
            DI_HIP(hipMemcpyAsync(out_score, dsc, (size_t)n_q * k * 8, hipMemcpyDeviceToHost, s));
            DI_HIP(hipMemcpyAsync(out_n, dn, (size_t)n_q * 4, hipMemcpyDeviceToHost, s));
        }
        if (!(flags & DI_F_ASYNC) || !dev) {
            DI_HIP(hipStreamSynchronize(s));
            sp->timer.resolve();
            if (!dev)
                for (int q = 0; q < n_q; ++q)
                    DI_REQUIRE(out_n[q] >= 0, DI_ERANGE, "query %d exceeded a kernel limit", q);
        }
    });
}

int di_sparse_info(const di_sparse *sp, int64_t *n_terms, int64_t *n_postings, uint32_t *n_docs,
                   int32_t *n_blocks) {
    return guard([&] {
        DI_REQUIRE(sp, DI_EINVAL, "null handle");
        if (n_terms) *n_terms = sp->n_terms;
        if (n_postings) *n_postings = sp->n_post;
        if (n_docs) *n_docs = sp->n_docs;
        if (n_blocks) *n_blocks = sp->nb;
    });
}

int di_sparse_timing(di_sparse *sp, const char *name, di_timing *out, int reset) {
    return guard([&] {
        DI_REQUIRE(sp && name && out, DI_EINVAL, "null argument");
        sp->timer.get(name, out, reset != 0);
    });
}

int di_sparse_destroy(di_sparse *sp) {
    return guard([&] {
        if (!sp) return;
        {
            DevScope ds(sp->device);
            if (sp->own_stream && sp->stream) (void)hipStreamDestroy(sp->stream);
        }
        delete sp;
    });
}

}  // extern "C"
