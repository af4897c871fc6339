// topk_common.h -- device building blocks shared by the retrieval kernels:
// wave scans, block-wide radix selection over LDS-resident keys, LDS bitonic
// sort.  Wave64 (gfx950): every lane/wave constant below is 64-based.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace di {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// lane l receives sum over lanes >= l
__device__ __forceinline__ uint32_t wave_suffix_sum(uint32_t x) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_down(x, d, 64);
        if (lane_id() + d < 64) x += y;
    }
    return x;
}

// lane l receives sum over lanes <= l
__device__ __forceinline__ uint32_t wave_prefix_sum(uint32_t x) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane_id() >= d) x += y;
    }
    return x;
}

// lane l receives sum over lanes <= l, by DPP only (no LDS crossbar): a Hillis-Steele
// scan inside each 16-lane row (row_shr 1, 2, 4, 8), then row 0's total into row 1 and
// row 2's into row 3 (row_bcast:15), then rows 0-1's total into rows 2-3 (row_bcast:31).
// Lanes whose DPP source is out of the row read `old` = 0.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// Shared scratch of one radix-select pass.
template <int WAVES>
struct RadixScratch {
    uint32_t hist[WAVES][256];
    uint32_t tot[256];
    uint32_t bin;    // selected digit
    uint32_t above;  // elements with a larger digit (among the prefix)
    uint32_t total;  // elements matching the prefix
    uint32_t pad;
};

// Zero the per-wave histograms (all threads participate).
template <int THREADS, int WAVES>
__device__ __forceinline__ void radix_clear(RadixScratch<WAVES> &rs) {
    uint32_t *h = &rs.hist[0][0];
    for (int i = threadIdx.x; i < WAVES * 256; i += THREADS) h[i] = 0;
}

// Run-length aggregated histogram insert: consecutive equal digits of one lane
// become one LDS atomic (keys are often concentrated in a few digits).
struct RunLen {
    uint32_t bin = 0xFFFFFFFFu, cnt = 0;
    template <int WAVES>
    __device__ __forceinline__ void add(RadixScratch<WAVES> &rs, uint32_t b) {
        if (b == bin) {
            ++cnt;
            return;
        }
        if (cnt) atomicAdd(&rs.hist[wave_id()][bin], cnt);
        bin = b;
        cnt = 1;
    }
    template <int WAVES>
    __device__ __forceinline__ void flush(RadixScratch<WAVES> &rs) {
        if (cnt) atomicAdd(&rs.hist[wave_id()][bin], cnt);
        cnt = 0;
        bin = 0xFFFFFFFFu;
    }
};

// After the histograms are filled (and a __syncthreads()), pick the digit that
// holds the `need`-th largest element.  Ends with a __syncthreads(); the result
// is in rs.bin / rs.above / rs.total / rs.tot[].
template <int THREADS, int WAVES>
__device__ __forceinline__ void radix_pick(RadixScratch<WAVES> &rs, uint32_t need) {
    for (int b = threadIdx.x; b < 256; b += THREADS) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += rs.hist[w][b];
        rs.tot[b] = s;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        uint32_t s = rs.tot[4 * l] + rs.tot[4 * l + 1] + rs.tot[4 * l + 2] + rs.tot[4 * l + 3];
        uint32_t S = wave_suffix_sum(s);
        uint64_t ok = __ballot(S >= need);
        if (l == 0) rs.total = S;
        // highest lane whose suffix still holds `need` elements
        int L = ok ? 63 - __builtin_clzll(ok) : 0;
        if (l == L) {
            uint32_t above = S - s;
            int c = 4 * L + 3;
            for (; c > 4 * L; --c) {
                if (above + rs.tot[c] >= need) break;
                above += rs.tot[c];
            }
            rs.bin = (uint32_t)c;
            rs.above = above;
        }
    }
    __syncthreads();
}

// Bitonic sort of n (power of two) u64 keys in LDS, descending.
template <int THREADS>
__device__ __forceinline__ void bitonic_sort_desc(uint64_t *s, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < (n >> 1); i += THREADS) {
                int lo = 2 * i - (i & (stride - 1));
                int hi = lo + stride;
                bool desc = (lo & size) == 0;
                uint64_t a = s[lo], b = s[hi];
                if ((a < b) == desc) {
                    s[lo] = b;
                    s[hi] = a;
                }
            }
            __syncthreads();
        }
    }
}

}  // namespace di
