// attn_check -- developer timing/consistency check of the varlen attention kernels
// on the GPU box (bench shape: 1024 docs, lengths clip(N(200,60),8,300), 12 heads).
//   DI_ATTN=<mode> attn_check [--fixed]   modes: 0 generic, 1 LDS-staged, 2/4 register-direct
// Prints ms per launch and the max relative error vs an fp64 host reference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../improving-learned-index_amd/csrc/enc_common.h"

namespace di {
template <typename T>
void launch_attention(const T *qk, const T *vt, const int32_t *cu_seqlens, int n_docs,
                      int max_len, int H, int ld_v, T *ctx, hipStream_t s);
void launch_vt_cols(const int32_t *cu, int n_docs, int M, int32_t *vcol, hipStream_t s);
void launch_attention_v3(const bf16 *qkv, const int32_t *cu_seqlens, int n_docs, int max_len,
                         int H, bf16 *ctx, hipStream_t s, const int32_t *qsel = nullptr,
                         const int32_t *cu_qsel = nullptr);
int vt_ld(int64_t M, int n_docs);
}  // namespace di
using namespace di;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

static uint16_t f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}
static float bf2f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

__global__ void scatter_v(const __bf16 *qkv, int M, int H, const int32_t *vcol, int ld_v,
                          __bf16 *vt) {
    const int row = blockIdx.x, d = threadIdx.x;  // d < H
    for (int c = d; c < H; c += blockDim.x)
        vt[(int64_t)c * ld_v + vcol[row]] = qkv[(int64_t)row * 3 * H + 2 * H + c];
}

int main(int argc, char **argv) {
    bool fixed = false, check = true;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--fixed")) fixed = true;
        if (!strcmp(argv[i], "--nocheck")) check = false;
    }
    const int n_docs = 1024, H = 768, max_len = fixed ? 256 : 300;
    std::mt19937 rng(5);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<int32_t> cu(n_docs + 1, 0);
    for (int d = 0; d < n_docs; ++d) {
        int n = fixed ? 256 : (int)std::lround(200 + 60 * nd(rng));
        n = std::min(std::max(n, 8), 300);
        cu[d + 1] = cu[d] + n;
    }
    const int M = cu[n_docs];
    std::vector<uint16_t> hq((size_t)M * 3 * H);
    {
        std::vector<uint16_t> pool(1 << 16);
        for (auto &x : pool) x = f2bf(nd(rng) * 0.6f);
        std::uniform_int_distribution<int> ui(0, (1 << 16) - 1);
        for (size_t i = 0; i < hq.size(); ++i) hq[i] = pool[(i * 2654435761u + (i >> 16)) & 0xFFFF];
    }
    __bf16 *qkv, *qk, *vt, *ctx0, *ctx;
    int32_t *dcu, *vcol;
    const int ld_v = vt_ld(M, n_docs);
    CK(hipMalloc(&qkv, hq.size() * 2));
    CK(hipMalloc(&qk, (size_t)M * 2 * H * 2));
    CK(hipMalloc(&vt, (size_t)H * ld_v * 2));
    CK(hipMalloc(&ctx0, (size_t)M * H * 2));
    CK(hipMalloc(&ctx, (size_t)M * H * 2));
    CK(hipMalloc(&dcu, (n_docs + 1) * 4));
    CK(hipMalloc(&vcol, M * 4));
    CK(hipMemcpy(qkv, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy2D(qk, 2 * H * 2, qkv, 3 * H * 2, 2 * H * 2, M, hipMemcpyDeviceToDevice));
    CK(hipMemset(vt, 0, (size_t)H * ld_v * 2));
    CK(hipMemcpy(dcu, cu.data(), (n_docs + 1) * 4, hipMemcpyHostToDevice));
    launch_vt_cols(dcu, n_docs, M, vcol, 0);
    hipLaunchKernelGGL(scatter_v, dim3(M), dim3(256), 0, 0, qkv, M, H, vcol, ld_v, vt);
    CK(hipDeviceSynchronize());

    // the kernel variant is DI_ATTN (read once inside the library): run the tool
    // once per mode from the shell, e.g. for m in 0 1 4; do DI_ATTN=$m ./attn_check; done
    const char *self_mode = getenv("DI_ATTN") ? getenv("DI_ATTN") : "default";
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const bool v3 = !strcmp(self_mode, "3");
    auto run = [&] {
        if (v3) launch_attention_v3(qkv, dcu, n_docs, max_len, H, ctx, 0);
        else launch_attention<bf16>(qk, vt, dcu, n_docs, max_len, H, ld_v, ctx, 0);
    };
    run();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) run();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    // fp64 host reference on a few (doc, head) pairs
    std::vector<uint16_t> out((size_t)M * H);
    CK(hipMemcpy(out.data(), ctx, out.size() * 2, hipMemcpyDeviceToHost));
    double maxerr = 0;
    for (int d : {0, 1, 17, 500, 1023}) {
        if (!check) break;
        const int t0 = cu[d], n = cu[d + 1] - cu[d];
        for (int h : {0, 5, 11}) {
            for (int q = 0; q < n; q += 7) {
                std::vector<double> sc(n);
                double mx = -1e300;
                for (int k = 0; k < n; ++k) {
                    double s = 0;
                    for (int e = 0; e < 64; ++e)
                        s += (double)bf2f(hq[(size_t)(t0 + q) * 3 * H + h * 64 + e]) *
                             bf2f(hq[(size_t)(t0 + k) * 3 * H + H + h * 64 + e]);
                    sc[k] = s / 8.0;
                    mx = std::max(mx, sc[k]);
                }
                double den = 0;
                for (int k = 0; k < n; ++k) den += (sc[k] = std::exp(sc[k] - mx));
                for (int e = 0; e < 64; ++e) {
                    double o = 0;
                    for (int k = 0; k < n; ++k)
                        o += sc[k] * bf2f(hq[(size_t)(t0 + k) * 3 * H + 2 * H + h * 64 + e]);
                    o /= den;
                    const double got = bf2f(out[(size_t)(t0 + q) * H + h * 64 + e]);
                    maxerr = std::max(maxerr, std::fabs(got - o) / (std::fabs(o) + 0.02));
                }
            }
        }
    }
    double flops = 0;
    for (int d = 0; d < n_docs; ++d) flops += 4.0 * (double)(cu[d + 1] - cu[d]) * (cu[d + 1] - cu[d]) * H;
    printf("mode %s  %s  %.3f ms  %.0f TF  max_rel_err %.2e %s\n", self_mode,
           fixed ? "n=256" : "n~N(200,60)", ms, flops / ms / 1e9, maxerr, maxerr < 0.03 ? "ok" : "FAIL");
    return maxerr < 0.03 ? 0 : 1;
}
