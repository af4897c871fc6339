// gemm_check -- developer check of the encoder GEMMs on the GPU box:
//   (1) the 256x256 8-phase kernel against the 128x128 kernel, bit for bit (same
//       MFMA sequence per accumulator, same epilogue arithmetic), over ragged M,
//       every epilogue; (2) per-shape timing of both at the bench shapes.
// Build: make -C improving-learned-index_amd && make -C tools gemm_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../improving-learned-index_amd/csrc/enc_common.h"

namespace di {
template <typename T>
void launch_gemm(int epi, const GemmArgs &g, hipStream_t s);
void launch_gemm256(int epi, const GemmArgs &g, hipStream_t s);
}
using namespace di;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

static uint16_t f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

struct Case {
    int M, N, K, epi, hidden;
};

static void *dalloc(size_t b) {
    void *p;
    CK(hipMalloc(&p, b));
    CK(hipMemset(p, 0, b));
    return p;
}

int main(int argc, char **argv) {
    const bool timing_only = argc > 1 && !strcmp(argv[1], "--time");
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    const int MAXM = 206426 + 256, MAXK = 3072, MAXN = 3072;
    std::vector<uint16_t> h((size_t)MAXM * MAXK);
    for (auto &x : h) x = f2bf(nd(rng) * 0.5f);
    void *A = dalloc((size_t)MAXM * MAXK * 2);
    CK(hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    std::vector<uint16_t> hb((size_t)MAXN * MAXK);
    for (auto &x : hb) x = f2bf(nd(rng) * 0.02f);
    void *B = dalloc(hb.size() * 2);
    CK(hipMemcpy(B, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    std::vector<float> hbias(MAXN);
    for (auto &x : hbias) x = nd(rng) * 0.1f;
    float *bias = (float *)dalloc(MAXN * 4);
    CK(hipMemcpy(bias, hbias.data(), MAXN * 4, hipMemcpyHostToDevice));
    void *R = dalloc((size_t)MAXM * 768 * 2);
    CK(hipMemcpy(R, h.data(), (size_t)MAXM * 768 * 2, hipMemcpyHostToDevice));
    std::vector<int32_t> hv(MAXM);
    for (int i = 0; i < MAXM; ++i) hv[i] = i + 4 * (i / 100);  // doc-aligned-like gaps
    int32_t *vcol = (int32_t *)dalloc(MAXM * 4);
    CK(hipMemcpy(vcol, hv.data(), MAXM * 4, hipMemcpyHostToDevice));
    const size_t out_bytes = (size_t)MAXM * MAXN * 4;
    void *O1 = dalloc(out_bytes), *O2 = dalloc(out_bytes);
    const int ldv = MAXM + 4 * (MAXM / 100) + 64;
    void *V1 = dalloc((size_t)768 * ldv * 2), *V2 = dalloc((size_t)768 * ldv * 2);

    auto args = [&](const Case &c, void *out, void *out2, bool big) {
        GemmArgs g{};
        g.A = A;
        g.B = B;
        g.bias = bias;
        g.resid = R;
        g.out = out;
        g.out2 = out2;
        g.M = c.M;
        g.N = c.N;
        g.K = c.K;
        g.ld_out = c.epi == EPI_QKV ? 2 * c.hidden : c.N;
        g.ld_v = ldv;
        g.hidden = c.hidden;
        g.vcol = vcol;
        g.a_rows = big ? MAXM : c.M;  // a_rows == M forces the 128x128 kernel
        return g;
    };
    int bad = 0;
    if (!timing_only) {
        const int Ms[] = {1, 77, 256, 300, 1000, 4133, 20000};
        const Case shapes[] = {{0, 2304, 768, EPI_QKV, 768},
                               {0, 768, 768, EPI_BIAS_RESID, 768},
                               {0, 3072, 768, EPI_BIAS_GELU, 768},
                               {0, 768, 3072, EPI_BIAS_RESID, 768},
                               {0, 1024, 256, EPI_BIAS, 768}};
        for (const Case &s : shapes) {
            for (int M : Ms) {
                Case c = s;
                c.M = M;
                CK(hipMemset(O1, 0x7f, out_bytes));
                CK(hipMemset(O2, 0x7f, out_bytes));
                CK(hipMemset(V1, 0, (size_t)768 * ldv * 2));
                CK(hipMemset(V2, 0, (size_t)768 * ldv * 2));
                launch_gemm<bf16>(c.epi, args(c, O1, V1, false), 0);
                launch_gemm<bf16>(c.epi, args(c, O2, V2, true), 0);
                CK(hipDeviceSynchronize());
                const int ocols = c.epi == EPI_QKV ? 2 * c.hidden : c.N;
                const size_t esz = 2;  // every epilogue writes bf16
                const size_t nb = (size_t)M * ocols * esz;
                std::vector<unsigned char> a(nb), b(nb);
                CK(hipMemcpy(a.data(), O1, nb, hipMemcpyDeviceToHost));
                CK(hipMemcpy(b.data(), O2, nb, hipMemcpyDeviceToHost));
                size_t diff = 0;
                for (size_t i = 0; i < nb; ++i) diff += a[i] != b[i];
                size_t vdiff = 0;
                if (c.epi == EPI_QKV) {
                    const size_t vb = (size_t)768 * ldv * 2;
                    std::vector<unsigned char> va(vb), vb2(vb);
                    CK(hipMemcpy(va.data(), V1, vb, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(vb2.data(), V2, vb, hipMemcpyDeviceToHost));
                    for (size_t i = 0; i < vb; ++i) vdiff += va[i] != vb2[i];
                }
                // also an fp64 host check of one output row (row M-1), bf16/f32 tolerance
                double maxrel = 0;
                {
                    const int row = M - 1;
                    for (int col = 0; col < std::min(ocols, 64); ++col) {
                        double acc = 0;
                        for (int k = 0; k < c.K; ++k) {
                            uint32_t ua = (uint32_t)h[(size_t)row * c.K + k] << 16,
                                     ub = (uint32_t)hb[(size_t)col * c.K + k] << 16;
                            float fa, fb;
                            memcpy(&fa, &ua, 4);
                            memcpy(&fb, &ub, 4);
                            acc += (double)fa * fb;
                        }
                        acc += hbias[col];
                        if (c.epi == EPI_BIAS_GELU) acc = 0.5 * acc * (1 + erf(acc / sqrt(2.0)));
                        if (c.epi == EPI_BIAS_RESID) {
                            uint32_t ur = (uint32_t)h[(size_t)row * 768 + col] << 16;
                            float fr;
                            memcpy(&fr, &ur, 4);
                            acc += fr;
                        }
                        double got;
                        if (esz == 4) {
                            float f;
                            memcpy(&f, &b[((size_t)row * ocols + col) * 4], 4);
                            got = f;
                        } else {
                            uint32_t u = (uint32_t)(b[((size_t)row * ocols + col) * 2] |
                                                    (b[((size_t)row * ocols + col) * 2 + 1] << 8))
                                         << 16;
                            float f;
                            memcpy(&f, &u, 4);
                            got = f;
                        }
                        maxrel = std::max(maxrel, fabs(got - acc) / (fabs(acc) + 0.05));
                    }
                }
                const bool ok = diff == 0 && vdiff == 0 && maxrel < 0.02;
                bad += !ok;
                printf("%s M=%6d N=%4d K=%4d epi=%d  bytes_diff=%zu v_diff=%zu host_maxrel=%.2e\n",
                       ok ? "ok  " : "FAIL", M, c.N, c.K, c.epi, diff, vdiff, maxrel);
            }
        }
    }
    // timing at the bench shapes (M = 206426 tokens of 1024 docs)
    const Case bench[] = {{206426, 2304, 768, EPI_QKV, 768},
                          {206426, 768, 768, EPI_BIAS_RESID, 768},
                          {206426, 3072, 768, EPI_BIAS_GELU, 768},
                          {206426, 768, 3072, EPI_BIAS_RESID, 768}};
    const char *names[] = {"qkv", "o", "ffn1", "ffn2"};
    // tile-order group size and epilogue ablation sweep on the 256 kernel
    {
        hipEvent_t a0, a1;
        CK(hipEventCreate(&a0));
        CK(hipEventCreate(&a1));
        for (int i = 0; i < 4; ++i) {
            const Case &c = bench[i];
            const double flops = 2.0 * c.M * c.N * c.K;
            for (int abl : {0, 6, 8, 102, 104, 116}) {  // 1xx: full epilogue, tile group xx; 8: erf GELU
                for (int stg : {0}) {
                    const int gm = abl >= 100 ? abl - 100 : 8;
                    GemmArgs g = args(c, O1, V1, true);
                    g.tune_gm = gm;
                    g.ablate = abl >= 100 ? 0 : abl;
                    (void)stg;
                    for (int w = 0; w < 2; ++w) launch_gemm<bf16>(c.epi, g, 0);
                    CK(hipEventRecord(a0, 0));
                    for (int w = 0; w < 10; ++w) launch_gemm<bf16>(c.epi, g, 0);
                    CK(hipEventRecord(a1, 0));
                    CK(hipEventSynchronize(a1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a0, a1));
                    ms /= 10;
                    printf("sweep %-5s ablate=%d gm=%2d stagger=%5d  %.3f ms  %.0f TF\n", names[i],
                           abl, gm, stg, ms, flops / ms / 1e9);
                }
            }
        }
    }
    // split-bf16 (bf16x3) shapes: A / B as split rows (random bits; timing only).
    // ablate 6: no GELU, no stores (the K loop and the epilogue's reads)
    {
        struct SC {
            const char *name;
            int M, N, K, epi;
        };
        const SC sc[] = {{"x3_qkv", 206426, 2304, 768, EPI_BIAS},
                         {"x3_o", 206426, 768, 768, EPI_BIAS_RESID},
                         {"x3_ffn1", 206426, 3072, 768, EPI_BIAS_GELU},
                         {"x3_ffn2", 100000, 768, 3072, EPI_BIAS_RESID}};
        hipEvent_t a0, a1;
        CK(hipEventCreate(&a0));
        CK(hipEventCreate(&a1));
        for (const SC &c : sc) {
            for (int abl : {0, 2, 4, 6}) {  // 2: no GELU, 4: no stores, 6: neither
                GemmArgs g{};
                g.A = A;
                g.B = B;
                g.bias = bias;
                g.resid = O2;
                g.out = O1;
                g.M = c.M;
                g.N = c.N;
                g.K = c.K;
                g.ld_out = c.epi == EPI_BIAS_RESID ? c.N : 2 * c.N;
                g.a_rows = (c.M + 255) / 256 * 256;
                g.hidden = 768;
                g.tune_gm = abl >= 100 ? abl - 100 : (c.K == 3072 ? 4 : 8);
                g.split = 1;
                g.ablate = abl >= 100 ? 0 : abl;
                for (int w = 0; w < 2; ++w) launch_gemm256(c.epi, g, 0);
                CK(hipEventRecord(a0, 0));
                for (int w = 0; w < 10; ++w) launch_gemm256(c.epi, g, 0);
                CK(hipEventRecord(a1, 0));
                CK(hipEventSynchronize(a1));
                float ms;
                CK(hipEventElapsedTime(&ms, a0, a1));
                ms /= 10;
                const double fl = 2.0 * c.M * c.N * c.K;
                printf("split %-8s ablate=%3d  %.3f ms  %.0f TF fp32-eq  %.0f TF bf16-MFMA\n", c.name,
                       abl, ms, fl / ms / 1e9, 3 * fl / ms / 1e9);
            }
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 3; ++r) {
        for (int i = 0; i < 4; ++i) {
            const Case &c = bench[i];
            const double flops = 2.0 * c.M * c.N * c.K;
            float ms[2];
            for (int big = 0; big < 2; ++big) {
                GemmArgs g = args(c, O1, V1, big);
                for (int w = 0; w < 2; ++w) launch_gemm<bf16>(c.epi, g, 0);
                CK(hipEventRecord(e0, 0));
                const int reps = 10;
                for (int w = 0; w < reps; ++w) launch_gemm<bf16>(c.epi, g, 0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms[big], e0, e1));
                ms[big] /= reps;
            }
            printf("round %d %-5s 128x128: %.3f ms %.0f TF   256x256: %.3f ms %.0f TF   x%.2f\n", r,
                   names[i], ms[0], flops / ms[0] / 1e9, ms[1], flops / ms[1] / 1e9,
                   ms[0] / ms[1]);
        }
    }
    printf(bad ? "GEMM CHECK FAILED (%d)\n" : "GEMM CHECK OK\n", bad);
    return bad ? 1 : 0;
}
