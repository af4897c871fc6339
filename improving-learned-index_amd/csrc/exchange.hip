// exchange.hip -- the device steps of the pruned exact top-k exchange between doc-id
// shards (parallel.exchange_topk; /root/reference/src/deep_impact/
// evaluation/ranker.py:43-48 keeps the global top-k the merge reproduces).
//
// Every rank holds, per query, its top-k u64 merge keys sorted descending (unique: they
// carry the doc).  Round 1 all-gathers a sample of every list (the keys at positions
// g-1, 2g-1, ...); T_q, the need-th largest sample of the union (need = ceil(k/g)), is a
// lower bound of the global k-th key.  Round 2 all-gathers each rank's keys >= T_q (a
// prefix of its list), padded to the largest rank's total.  The collectives are RCCL
// (torch.distributed); these kernels are the local steps around them, so that a step
// costs three collectives, one device -> host read (the padded size) and five launches
// instead of some forty small tensor operations.
//
// Keys are > 0 (a touched doc's word is >= 1 << 16), so 0 marks a missing sample.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/deepimpact.h"
#include "di_common.h"

namespace di {
namespace {

struct XDevice {
    int prev = -1;
    explicit XDevice(int dev) {
        DI_HIP(hipGetDevice(&prev));
        if (prev != dev) DI_HIP(hipSetDevice(dev));
    }
    ~XDevice() {
        int cur;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// samples[q][j] = keys[q][(j + 1) g - 1] when inside the query's valid prefix, else 0
__global__ void xchg_sample_kernel(const uint64_t *__restrict__ keys,
                                   const int32_t *__restrict__ counts, int n_q, int k, int g,
                                   int s_n, uint64_t *__restrict__ samples) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_q * s_n) return;
    const int q = (int)(i / s_n), j = (int)(i % s_n);
    const int c = min(max(counts[q], 0), k);
    const int pos = (j + 1) * g - 1;
    samples[i] = pos < c ? keys[(int64_t)q * k + pos] : 0ull;
}

// One wave per query: T_q = the need-th largest of the world * s_n gathered samples
// (0 when fewer than need are nonzero: every key passes), built bit by bit from the
// top -- the largest t with count(samples >= t) >= need, each count one ballot per
// register row of samples -- then e_q = this rank's keys >= T_q among its valid prefix.
// ec[q] = e_q, ec[n_q + q] = the scorer's count (negative: a rejected query), the two
// rows one all_gather moves.
constexpr int XR = 16;  // sample registers per lane: up to 1024 samples held
__global__ void __launch_bounds__(256) xchg_count_kernel(
    const uint64_t *__restrict__ gs, int world, int s_n, const uint64_t *__restrict__ keys,
    const int32_t *__restrict__ counts, int n_q, int k, int need, int32_t *__restrict__ ec) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (q >= n_q) return;
    const int n = world * s_n;
    // sample i = (rank r, j): gs[(r * n_q + q) * s_n + j]
    auto sample = [&](int i) -> uint64_t {
        const int r = i / s_n, j = i - r * s_n;
        return gs[((int64_t)r * n_q + q) * s_n + j];
    };
    uint64_t T = 0;
    if (n >= need) {
        if (n <= 64 * XR) {
            uint64_t s[XR];
#pragma unroll
            for (int r = 0; r < XR; ++r) {
                const int i = r * 64 + lane;
                s[r] = i < n ? sample(i) : 0ull;
            }
            for (int b = 63; b >= 0; --b) {
                const uint64_t cand = T | (1ull << b);
                uint32_t cnt = 0;
#pragma unroll
                for (int r = 0; r < XR; ++r) cnt += (uint32_t)__popcll(__ballot(s[r] >= cand));
                if (cnt >= (uint32_t)need) T = cand;
            }
        } else {  // (more samples than registers: re-read them per bit, L2-resident)
            for (int b = 63; b >= 0; --b) {
                const uint64_t cand = T | (1ull << b);
                uint32_t cnt = 0;
                for (int i0 = 0; i0 < n; i0 += 64) {
                    const int i = i0 + lane;
                    cnt += (uint32_t)__popcll(__ballot(i < n && sample(i) >= cand));
                }
                if (cnt >= (uint32_t)need) T = cand;
            }
        }
    }
    const int c = min(max(counts[q], 0), k);
    const uint64_t *kq = keys + (int64_t)q * k;
    uint32_t e = 0;
    for (int j0 = 0; j0 < c; j0 += 64) {
        const int j = j0 + lane;
        e += (uint32_t)__popcll(__ballot(j < c && kq[j] >= T));
    }
    if (lane == 0) {
        ec[q] = (int32_t)e;
        ec[n_q + q] = counts[q];
    }
}

// One workgroup per rank: exclusive scan of its e row -> offsets[r][q], totals[r].
constexpr int XS_T = 1024;
__global__ void __launch_bounds__(XS_T) xchg_offsets_kernel(const int32_t *__restrict__ gec,
                                                            int n_q, int64_t *__restrict__ off,
                                                            int64_t *__restrict__ tot) {
    __shared__ int64_t wsum[XS_T / 64];
    const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t *e = gec + (int64_t)r * 2 * n_q;  // row 0 of rank r's [2][n_q]
    const int per = (n_q + XS_T - 1) / XS_T;
    const int q0 = min(tid * per, n_q), q1 = min(q0 + per, n_q);
    int64_t s = 0;
    for (int q = q0; q < q1; ++q) s += e[q];
    // block exclusive scan of s
    int64_t incl = s;
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int64_t base = incl - s, all = 0;
    for (int w = 0; w < XS_T / 64; ++w) {
        if (w < wave) base += wsum[w];
        all += wsum[w];
    }
    int64_t *o = off + (int64_t)r * n_q;
    for (int q = q0; q < q1; ++q) {
        o[q] = base;
        base += e[q];
    }
    if (tid == 0) tot[r] = all;
}

// One wave per query: this rank's first e_q keys -> buf[off_q ..)
__global__ void __launch_bounds__(256) xchg_pack_kernel(const uint64_t *__restrict__ keys,
                                                        const int32_t *__restrict__ ec,
                                                        const int64_t *__restrict__ off, int n_q,
                                                        int k, uint64_t *__restrict__ buf) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (q >= n_q) return;
    const int e = ec[q];
    const uint64_t *src = keys + (int64_t)q * k;
    uint64_t *dst = buf + off[q];
    for (int j = lane; j < e; j += 64) dst[j] = src[j];
}

// One wave per (rank, query): rank r's e_{r,q} gathered keys -> out_keys[r][q][0 ..),
// out_n[r][q] = e_{r,q} (or the scorer's negative count: a rejected query stays flagged)
__global__ void __launch_bounds__(256) xchg_unpack_kernel(
    const uint64_t *__restrict__ g2, int64_t emax, const int32_t *__restrict__ gec,
    const int64_t *__restrict__ off, int world, int n_q, int k, uint64_t *__restrict__ out_keys,
    int32_t *__restrict__ out_n) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= (int64_t)world * n_q) return;
    const int r = (int)(i / n_q), q = (int)(i - (int64_t)r * n_q);
    const int e = gec[((int64_t)r * 2) * n_q + q];
    const int c = gec[((int64_t)r * 2 + 1) * n_q + q];
    const uint64_t *src = g2 + (int64_t)r * emax + off[i];
    uint64_t *dst = out_keys + i * k;
    for (int j = lane; j < e; j += 64) dst[j] = src[j];
    if (lane == 0) out_n[i] = c < 0 ? c : e;
}

int grid_of(int64_t n, int per) { return (int)std::max<int64_t>(1, (n + per - 1) / per); }

}  // namespace
}  // namespace di

using namespace di;

extern "C" {

int di_xchg_sample(const uint64_t *keys, const int32_t *counts, int32_t n_q, int32_t k,
                   int32_t g, uint64_t *samples, int device, void *hip_stream) {
    return guard([&] {
        DI_REQUIRE(keys && counts && samples && n_q >= 0 && k > 0 && g > 0 && g <= k,
                   DI_EINVAL, "bad argument");
        if (n_q == 0) return;
        XDevice ds(device);
        const int s_n = k / g;
        hipLaunchKernelGGL(xchg_sample_kernel, dim3(grid_of((int64_t)n_q * s_n, 256)), dim3(256),
                           0, (hipStream_t)hip_stream, keys, counts, n_q, k, g, s_n, samples);
        check_launch("xchg_sample");
    });
}

int di_xchg_count(const uint64_t *gathered_samples, int32_t world, const uint64_t *keys,
                  const int32_t *counts, int32_t n_q, int32_t k, int32_t g, int32_t *ec,
                  int device, void *hip_stream) {
    return guard([&] {
        DI_REQUIRE(gathered_samples && keys && counts && ec && world > 0 && n_q >= 0 && k > 0 &&
                       g > 0 && g <= k,
                   DI_EINVAL, "bad argument");
        if (n_q == 0) return;
        XDevice ds(device);
        const int need = (k + g - 1) / g;
        hipLaunchKernelGGL(xchg_count_kernel, dim3(grid_of(n_q, 4)), dim3(256), 0,
                           (hipStream_t)hip_stream, gathered_samples, world, k / g, keys, counts,
                           n_q, k, need, ec);
        check_launch("xchg_count");
    });
}

int di_xchg_offsets(const int32_t *gathered_ec, int32_t world, int32_t n_q, int64_t *offsets,
                    int64_t *totals, int device, void *hip_stream) {
    return guard([&] {
        DI_REQUIRE(gathered_ec && offsets && totals && world > 0 && n_q >= 0, DI_EINVAL,
                   "bad argument");
        XDevice ds(device);
        hipLaunchKernelGGL(xchg_offsets_kernel, dim3(world), dim3(XS_T), 0,
                           (hipStream_t)hip_stream, gathered_ec, n_q, offsets, totals);
        check_launch("xchg_offsets");
    });
}

int di_xchg_pack(const uint64_t *keys, const int32_t *ec, const int64_t *offsets, int32_t n_q,
                 int32_t k, uint64_t *buf, int device, void *hip_stream) {
    return guard([&] {
        DI_REQUIRE(keys && ec && offsets && buf && n_q >= 0 && k > 0, DI_EINVAL, "bad argument");
        if (n_q == 0) return;
        XDevice ds(device);
        hipLaunchKernelGGL(xchg_pack_kernel, dim3(grid_of(n_q, 4)), dim3(256), 0,
                           (hipStream_t)hip_stream, keys, ec, offsets, n_q, k, buf);
        check_launch("xchg_pack");
    });
}

int di_xchg_unpack(const uint64_t *gathered, int64_t emax, const int32_t *gathered_ec,
                   const int64_t *offsets, int32_t world, int32_t n_q, int32_t k,
                   uint64_t *out_keys, int32_t *out_n, int device, void *hip_stream) {
    return guard([&] {
        DI_REQUIRE(gathered_ec && offsets && out_keys && out_n && world > 0 && n_q >= 0 &&
                       k > 0 && emax >= 0 && (gathered || emax == 0),
                   DI_EINVAL, "bad argument");
        if (n_q == 0) return;
        XDevice ds(device);
        hipLaunchKernelGGL(xchg_unpack_kernel, dim3(grid_of((int64_t)world * n_q, 4)), dim3(256),
                           0, (hipStream_t)hip_stream, gathered, emax, gathered_ec, offsets,
                           world, n_q, k, out_keys, out_n);
        check_launch("xchg_unpack");
    });
}

}  // extern "C"
