// encoder.hip -- DeeperImpact encoder on MI355X: weight residency and the
// per-batch forward (host orchestration of the HIP kernels).
//
// Replaces, for a batch of documents, the reference's
//   DeepImpact.forward            src/deep_impact/models/xlmr_original.py:41-85
//   compute_term_impacts          src/deep_impact/models/xlmr_original.py:205-225
//   round(impact, 3)              src/deep_impact/indexing/indexer.py:132
// Documents arrive packed (cu_seqlens, no padding); every GEMM runs on real
// tokens only.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "di_common.h"
#include "enc_common.h"

namespace di {

template <typename T>
void launch_gemm(int epi, const GemmArgs &g, hipStream_t s);
template <typename T>
void launch_attention(const T *qk, const T *vt, const int32_t *cu_seqlens, int n_docs,
                      int max_len, int H, int ld_v, T *ctx, hipStream_t s,
                      bf16 *ctx_split = nullptr);
void launch_gemm256(int epi, const GemmArgs &g, hipStream_t s);
void launch_attention_x3(const bf16 *qkv, const int32_t *cu_seqlens, int n_docs, int H,
                         bf16 *ctx_split, hipStream_t s, const int32_t *qsel = nullptr,
                         const int32_t *cu_qsel = nullptr);
void launch_scatter_term_rows(const bf16 *Xg, const int32_t *cu_seq, const int32_t *cu_terms,
                              const int32_t *term_tok, int n_docs, int W, int64_t ld, bf16 *X,
                              hipStream_t s);
void launch_embed_ln_split(const int32_t *ids, const int32_t *cu, int n_docs, int M, int H,
                           const float *word, const float *pos, const float *type0,
                           const float *gamma, const float *beta, float eps, int pos_offset,
                           int vocab, int max_pos, bf16 *out, int32_t *err, hipStream_t s);
void launch_ln_split(const float *pre, int M, int H, const float *gamma, const float *beta,
                     float eps, bf16 *out, const float *head_w, float head_b, int act,
                     float *impact, hipStream_t s);
template <typename T>
void launch_embed_ln(const int32_t *ids, const int32_t *cu, int n_docs, int M, int H,
                     const T *word, const T *pos, const T *type0, const float *gamma,
                     const float *beta, float eps, int pos_offset, int vocab, int max_pos, T *out,
                     int32_t *err, hipStream_t s);
template <typename T>
void launch_ln(const T *pre, int M, int H, const float *gamma, const float *beta, float eps,
               T *out, const float *head_w, float head_b, int act, float *impact, hipStream_t s);
void launch_vt_cols(const int32_t *cu, int n_docs, int M, int32_t *vcol, hipStream_t s);
bool attention_v3_ok(int max_len, int H);
void launch_head_from_stats(const float4 *st, int ld, int n_part, int M, int H, float eps,
                            float sw, float cw, int act, float *impact, hipStream_t s);
void launch_row_ln(const float4 *st, int ld, int n_part, int M, int H, float eps, float2 *out,
                   hipStream_t s);
int gemm_stats_cols();
void launch_attention_v3(const bf16 *qkv, const int32_t *cu_seqlens, int n_docs, int max_len,
                         int H, bf16 *ctx, hipStream_t s, const int32_t *qsel = nullptr,
                         const int32_t *cu_qsel = nullptr);
void launch_gather_term_rows(const bf16 *X, const float2 *rl, const int32_t *cu_seq,
                             const int32_t *cu_terms, const int32_t *term_tok, int n_docs, int H,
                             bf16 *Xg, float2 *rlg, hipStream_t s);
int vt_ld(int64_t M, int n_docs);
void launch_gather_terms(const float *impact, const int32_t *cu_seq, const int32_t *cu_terms,
                         int n_docs, const int32_t *term_tok, int n_terms, int do_round,
                         float *out, int32_t *err, hipStream_t s);

struct Layer {
    DevBuf w_qkv, b_qkv, w_o, b_o, ln1_g, ln1_b, w_i, b_i, w_out, b_out, ln2_g, ln2_b;
    DevBuf s_qkv, c_qkv, s_i, c_i;  // LN folding: per-column s = W' 1, c = b + W beta
};

}  // namespace di

using namespace di;

struct di_encoder {
    di_encoder_cfg cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    size_t esz = 2;  // bytes per activation/weight element (bf16 or f32)
    // fp32-faithful split-bf16 mode (DI_PREC_BF16X3): esz = 4 sizes the workspace (a
    // split row of 2H bf16 = an f32 row), f32 tables, GEMM weights [N][3K] bf16
    bool split = false;
    DevBuf word, pos, type0, emb_g, emb_b, head_w;
    float head_b = 0.f;
    std::vector<std::unique_ptr<Layer>> layers;
    // workspace
    DevBuf X, qk, vt, vcol, ctx, pre, X1, Hff, impact, ids, cu, tt, cut, err;
    // LayerNorm folding (bf16): the GEMM consuming LN(x) reads x and folds LN in
    bool folded = false;
    DevBuf stats1, stats2, head_wg;  // row-statistics partials; w * gamma_last
    DevBuf rln1, rln2;               // per-row (rstd, -rstd mean) of P1 / P2
    float head_sw = 0.f, head_cw = 0.f;
    int64_t cap_tokens = 0;
    int64_t cap_rows = 0;  // allocated rows of the GEMM A operands (>= cap_tokens)
    int cap_docs = 0;
    int ld_v = 0;
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

uint16_t f32_to_bf16_bits(float f) {  // round to nearest even (NaN stays NaN)
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

float bf16_bits_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

std::string strip_prefix(const std::string &k) {
    for (const char *p : {"bert.", "roberta.", "model."})
        if (k.rfind(p, 0) == 0) return k.substr(std::strlen(p));
    return k;
}

struct HostTensor {
    const di_tensor *t;
    int64_t numel() const {
        int64_t n = 1;
        for (int i = 0; i < t->ndim; ++i) n *= t->shape[i];
        return n;
    }
    float at(int64_t i) const {
        if (t->dtype == DI_DTYPE_F32) return static_cast<const float *>(t->data)[i];
        return bf16_bits_to_f32(static_cast<const uint16_t *>(t->data)[i]);
    }
};

// LayerNorm folding of a linear layer that consumes LN(x) = (x - mu) r gamma + beta:
//   W' = W diag(gamma) (bf16),  s = W' 1 (of the rounded W'),  c = b + W beta
// so that LN(x) W^T + b = r (x W'^T) - r mu s + c  (GEMM epilogue EPI_FOLD*).
void fold_upload(DevBuf &w_dst, DevBuf &s_dst, DevBuf &c_dst,
                 const std::vector<const HostTensor *> &w_parts,
                 const std::vector<const HostTensor *> &b_parts, int K, const HostTensor *gamma,
                 const HostTensor *beta, bool split = false) {
    // split: W' as split rows (upload_split3's layout), s summed from hi + lo (the
    // weights the split GEMM multiplies by)
    int64_t rows = 0;
    for (auto *p : w_parts) rows += p->numel() / K;
    std::vector<uint16_t> w((size_t)(rows * K * (split ? 2 : 1)));
    std::vector<float> sv((size_t)rows), cv((size_t)rows);
    std::vector<float> gm((size_t)K), bt((size_t)K);
    for (int k = 0; k < K; ++k) {
        gm[(size_t)k] = gamma->at(k);
        bt[(size_t)k] = beta->at(k);
    }
    int64_t r = 0, rb = 0;
    for (auto *p : w_parts) {
        const int64_t pr = p->numel() / K;
        for (int64_t i = 0; i < pr; ++i, ++r) {
            double s = 0.0, c = 0.0;
            for (int k = 0; k < K; ++k) {
                const float wv = p->at(i * K + k);
                const float wg = wv * gm[(size_t)k];
                const uint16_t wb = f32_to_bf16_bits(wg);
                if (split) {
                    const uint16_t lo = f32_to_bf16_bits(wg - bf16_bits_to_f32(wb));
                    w[(size_t)(r * 2 * K + split_col(k))] = wb;
                    w[(size_t)(r * 2 * K + split_col(k) + 32)] = lo;
                    s += (double)bf16_bits_to_f32(wb) + (double)bf16_bits_to_f32(lo);
                } else {
                    w[(size_t)(r * K + k)] = wb;
                    s += (double)bf16_bits_to_f32(wb);
                }
                c += (double)wv * (double)bt[(size_t)k];
            }
            sv[(size_t)r] = (float)s;
            cv[(size_t)r] = (float)c;
        }
    }
    for (auto *p : b_parts)
        for (int64_t i = 0; i < p->numel(); ++i, ++rb) cv[(size_t)rb] += p->at(i);
    w_dst.reserve(w.size() * 2);
    DI_HIP(hipMemcpy(w_dst.p, w.data(), w.size() * 2, hipMemcpyHostToDevice));
    s_dst.reserve(sv.size() * 4);
    DI_HIP(hipMemcpy(s_dst.p, sv.data(), sv.size() * 4, hipMemcpyHostToDevice));
    c_dst.reserve(cv.size() * 4);
    DI_HIP(hipMemcpy(c_dst.p, cv.data(), cv.size() * 4, hipMemcpyHostToDevice));
}

void upload(DevBuf &dst, const std::vector<const HostTensor *> &parts, int64_t rows_of_first,
            bool as_f32_always, size_t esz) {
    (void)rows_of_first;
    int64_t n = 0;
    for (auto *p : parts) n += p->numel();
    const bool f32 = as_f32_always || esz == 4;
    dst.reserve((size_t)n * (f32 ? 4 : 2));
    if (f32) {
        std::vector<float> h((size_t)n);
        int64_t o = 0;
        for (auto *p : parts)
            for (int64_t i = 0; i < p->numel(); ++i) h[(size_t)o++] = p->at(i);
        DI_HIP(hipMemcpy(dst.p, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    } else {
        std::vector<uint16_t> h((size_t)n);
        int64_t o = 0;
        for (auto *p : parts) {
            if (p->t->dtype == DI_DTYPE_BF16) {
                std::memcpy(&h[(size_t)o], p->t->data, (size_t)p->numel() * 2);
                o += p->numel();
            } else {
                const float *src = static_cast<const float *>(p->t->data);
                for (int64_t i = 0; i < p->numel(); ++i) h[(size_t)o++] = f32_to_bf16_bits(src[i]);
            }
        }
        DI_HIP(hipMemcpy(dst.p, h.data(), (size_t)n * 2, hipMemcpyHostToDevice));
    }
}

// split-bf16 GEMM weight (fp32-faithful mode): each [K] row of W becomes a split row
// (enc_common.h split_col: 32 hi then 32 lo bf16 per 32 columns), hi = bf16(w),
// lo = bf16(w - hi), the layout the split GEMM's K tiles read.
void upload_split3(DevBuf &dst, const std::vector<const HostTensor *> &parts, int K) {
    int64_t rows = 0;
    for (auto *p : parts) rows += p->numel() / K;
    std::vector<uint16_t> h((size_t)(rows * 2 * K));
    int64_t r = 0;
    for (auto *p : parts) {
        const int64_t pr = p->numel() / K;
        for (int64_t i = 0; i < pr; ++i, ++r) {
            uint16_t *o = &h[(size_t)(r * 2 * K)];
            for (int k = 0; k < K; ++k) {
                const float w = p->at(i * K + k);
                const uint16_t hi = f32_to_bf16_bits(w);
                const uint16_t lo = f32_to_bf16_bits(w - bf16_bits_to_f32(hi));
                o[split_col(k)] = hi;
                o[split_col(k) + 32] = lo;
            }
        }
    }
    dst.reserve(h.size() * 2);
    DI_HIP(hipMemcpy(dst.p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
}

void ensure_workspace(di_encoder *e, int64_t M, int n_docs, int64_t n_terms) {
    const int H = e->cfg.hidden, F = e->cfg.intermediate;
    if (M > e->cap_tokens || n_docs > e->cap_docs) {
        int64_t cap = std::max<int64_t>(std::max<int64_t>(M, e->cap_tokens), 256);
        const int capd = std::max(std::max(n_docs, e->cap_docs), 16);
        const size_t es = e->esz;
        // GEMM A operands (X, X1, ctx, Hff) carry rows up to a multiple of 256 so
        // the 256-row GEMM tiles read them unclamped (GemmArgs::a_rows)
        const int64_t capr = (cap + 255) / 256 * 256;
        e->X.reserve(capr * H * es);
        e->X1.reserve(capr * H * es);
        e->ctx.reserve(capr * H * es);
        e->qk.reserve(cap * 3 * H * es);  // [M][3H] (v3 path) or [M][2H] + V^T
        e->Hff.reserve(capr * F * es);
        e->pre.reserve(cap * H * es);
        e->impact.reserve(cap * 4);
        e->ids.reserve(cap * 4);
        // V^T (doc-aligned) for the generic attention kernels; the split (bf16x3)
        // attention reads V rows, the bf16 v3 attention too
        const size_t vt_bytes = e->split ? 0 : (size_t)H * vt_ld(cap, capd) * es;
        if (!e->split) e->vcol.reserve(cap * 4);
        if (vt_bytes > e->vt.bytes) {
            e->vt.reserve(vt_bytes);
            // never-written gap columns between documents must read as finite zeros
            DI_HIP(hipMemset(e->vt.p, 0, vt_bytes));
        }
        if (e->folded) {
            const size_t sb = (size_t)(H / 128) * capr * 16;  // float4 per row and 128 (or 256) columns
            e->stats1.reserve(sb);
            e->stats2.reserve(sb);
            e->rln1.reserve((size_t)capr * 8);
            e->rln2.reserve((size_t)capr * 8);
        }
        e->cap_tokens = cap;
        e->cap_rows = capr;
        e->cap_docs = capd;
    }
    e->ld_v = vt_ld(M, n_docs);
    e->cu.reserve((size_t)(n_docs + 1) * 4);
    e->cut.reserve((size_t)(n_docs + 1) * 4);
    e->tt.reserve((size_t)std::max<int64_t>(n_terms, 1) * 4);
    e->err.reserve(16);
}

template <typename T>
void forward(di_encoder *e, const int32_t *d_ids, const int32_t *d_cu, int n_docs, int64_t M,
             int max_len, bool timing, hipStream_t s) {
    const auto &c = e->cfg;
    const int H = c.hidden, F = c.intermediate;
    const int pos_offset = (c.variant == DI_VARIANT_XLMR) ? c.pad_id + 1 : 0;
    T *X = e->X.as<T>(), *X1 = e->X1.as<T>();
    {
        TimedLaunch tl(e->timer, timing, "embed_ln", s);
        launch_embed_ln<T>(d_ids, d_cu, n_docs, (int)M, H, e->word.as<T>(), e->pos.as<T>(),
                           e->type0.as<T>(), e->emb_g.as<float>(), e->emb_b.as<float>(),
                           c.layer_norm_eps, pos_offset, c.vocab_size, c.max_positions, X,
                           e->err.as<int32_t>(), s);
    }
    // attention path: the persistent v3 kernel when it applies (bf16, max_len <= 512)
    const bool use_v3 = std::is_same<T, bf16>::value && attention_v3_ok(max_len, H);
    if (!use_v3) launch_vt_cols(d_cu, n_docs, (int)M, e->vcol.as<int32_t>(), s);
    for (size_t l = 0; l < e->layers.size(); ++l) {
        Layer &L = *e->layers[l];
        const bool last = l + 1 == e->layers.size();
        GemmArgs g{};
        g.M = (int)M;
        g.a_rows = e->cap_rows;
        g.hidden = H;
        // QKV projection + attention.  bf16 with max_len <= 320: row-major [M][3H]
        // and the persistent LDS-DMA attention (v3); otherwise Q|K row-major with V
        // written transposed (doc-aligned V^T) for the generic attention kernels.
        if (use_v3) {
            g.A = X;
            g.B = L.w_qkv.p;
            g.bias = L.b_qkv.as<float>();
            g.out = e->qk.p;
            g.N = 3 * H;
            g.K = H;
            g.ld_out = 3 * H;
            {
                TimedLaunch tl(e->timer, timing, "gemm_qkv", s);
                launch_gemm<T>(EPI_BIAS, g, s);
            }
            {
                TimedLaunch tl(e->timer, timing, "attention", s);
                launch_attention_v3(e->qk.as<bf16>(), d_cu, n_docs, max_len, H, e->ctx.as<bf16>(),
                                    s);
            }
        } else {
            g.A = X;
            g.B = L.w_qkv.p;
            g.bias = L.b_qkv.as<float>();
            g.out = e->qk.p;
            g.out2 = e->vt.p;
            g.N = 3 * H;
            g.K = H;
            g.ld_out = 2 * H;
            g.ld_v = e->ld_v;
            g.vcol = e->vcol.as<int32_t>();
            {
                TimedLaunch tl(e->timer, timing, "gemm_qkv", s);
                launch_gemm<T>(EPI_QKV, g, s);
            }
            {
                TimedLaunch tl(e->timer, timing, "attention", s);
                launch_attention<T>(e->qk.as<T>(), e->vt.as<T>(), d_cu, n_docs, max_len, H,
                                    e->ld_v, e->ctx.as<T>(), s);
            }
        }
        // attention output + residual -> LN1 (fused into the GEMM when it can be)
        g = GemmArgs{};
        g.M = (int)M;
        g.a_rows = e->cap_rows;
        g.A = e->ctx.p;
        g.B = L.w_o.p;
        g.bias = L.b_o.as<float>();
        g.resid = X;
        g.out = e->pre.p;
        g.N = H;
        g.K = H;
        g.ld_out = H;
        g.ln_eps = c.layer_norm_eps;
        {
            TimedLaunch tl(e->timer, timing, "gemm_o", s);
            launch_gemm<T>(EPI_BIAS_RESID, g, s);
        }
        {
            TimedLaunch tl(e->timer, timing, "ln", s);
            launch_ln<T>(e->pre.as<T>(), (int)M, H, L.ln1_g.as<float>(), L.ln1_b.as<float>(),
                         c.layer_norm_eps, X1, nullptr, 0.f, c.activation, nullptr, s);
        }
        // FFN
        g = GemmArgs{};
        g.M = (int)M;
        g.a_rows = e->cap_rows;
        g.A = X1;
        g.B = L.w_i.p;
        g.bias = L.b_i.as<float>();
        g.out = e->Hff.p;
        g.N = F;
        g.K = H;
        g.ld_out = F;
        {
            TimedLaunch tl(e->timer, timing, "gemm_ffn1", s);
            launch_gemm<T>(EPI_BIAS_GELU, g, s);
        }
        // FFN output + residual -> LN2; the last LayerNorm feeds only the impact head
        g = GemmArgs{};
        g.M = (int)M;
        g.a_rows = e->cap_rows;
        g.A = e->Hff.p;
        g.B = L.w_out.p;
        g.bias = L.b_out.as<float>();
        g.resid = X1;
        g.out = e->pre.p;
        g.N = H;
        g.K = F;
        g.ld_out = H;
        g.ln_eps = c.layer_norm_eps;
        {
            TimedLaunch tl(e->timer, timing, "gemm_ffn2", s);
            launch_gemm<T>(EPI_BIAS_RESID, g, s);
        }
        {
            TimedLaunch tl(e->timer, timing, "ln", s);
            launch_ln<T>(e->pre.as<T>(), (int)M, H, L.ln2_g.as<float>(), L.ln2_b.as<float>(),
                         c.layer_norm_eps, last ? nullptr : X,
                         last ? e->head_w.as<float>() : nullptr, e->head_b, c.activation,
                         last ? e->impact.as<float>() : nullptr, s);
        }
    }
}

// bf16 / bf16x3 forward with every LayerNorm after the embeddings folded into its consumers
// (EPI_FOLD* / EPI_RESID_STATS, see enc_common.h): no LayerNorm pass over the
// activations.  Buffers: X holds the layer input (the normalised embeddings, then
// the un-normalised FFN output P2 of the previous layer), X1 the attention-block
// output P1; stats2 / stats1 their row-statistics partials.
// Pruned last layer (d_tt != nullptr): the term gather reads only the rows of the
// terms' first tokens, and every operation after the last layer's QKV projection is
// row-independent (attention per query row, the GEMMs and the LayerNorms per row), so
// that layer computes the attention for those query rows only (keys: every token) and
// the O / FFN GEMMs, row statistics and head on the packed term rows -- the same
// arithmetic per kept row (bit-identical impacts), ~4/5 fewer rows at the bench shape.
void forward_folded(di_encoder *e, const int32_t *d_ids, const int32_t *d_cu, int n_docs,
                    int64_t M, int max_len, bool timing, hipStream_t s,
                    const int32_t *d_tt = nullptr, const int32_t *d_ct = nullptr,
                    int64_t n_terms = 0) {
    const auto &c = e->cfg;
    const int H = c.hidden, F = c.intermediate;
    const int pos_offset = (c.variant == DI_VARIANT_XLMR) ? c.pad_id + 1 : 0;
    // sp (bf16x3): activations are split rows (row stride 2W), GEMMs split-bf16,
    // attention attention_x3_kernel
    const bool sp = e->split;
    const int W2 = sp ? 2 : 1;
    if (!sp) DI_REQUIRE(attention_v3_ok(max_len, H), DI_EINVAL, "max_len %d > 512", max_len);
    bf16 *X = e->X.as<bf16>(), *X1 = e->X1.as<bf16>();
    float4 *st1 = e->stats1.as<float4>(), *st2 = e->stats2.as<float4>();
    float2 *rl1 = e->rln1.as<float2>(), *rl2 = e->rln2.as<float2>();
    const int ld = (int)e->cap_rows, n_part = H / gemm_stats_cols();
    {
        TimedLaunch tl(e->timer, timing, "embed_ln", s);
        if (sp)
            launch_embed_ln_split(d_ids, d_cu, n_docs, (int)M, H, e->word.as<float>(),
                                  e->pos.as<float>(), e->type0.as<float>(), e->emb_g.as<float>(),
                                  e->emb_b.as<float>(), c.layer_norm_eps, pos_offset,
                                  c.vocab_size, c.max_positions, X, e->err.as<int32_t>(), s);
        else
            launch_embed_ln<bf16>(d_ids, d_cu, n_docs, (int)M, H, e->word.as<bf16>(),
                                  e->pos.as<bf16>(), e->type0.as<bf16>(), e->emb_g.as<float>(),
                                  e->emb_b.as<float>(), c.layer_norm_eps, pos_offset,
                                  c.vocab_size, c.max_positions, X, e->err.as<int32_t>(), s);
    }
    auto gemm = [&](int epi, const GemmArgs &g) {
        if (sp)
            launch_gemm256(epi, g, s);
        else
            launch_gemm<bf16>(epi, g, s);
    };
    auto base = [&]() {
        GemmArgs g{};
        // tile-order group: 8 M-tiles (measured +4% QKV, +1% O / FFN1 over 4); FFN2
        // (K = 3072, N = 768) keeps 4
        g.tune_gm = 8;
        g.M = (int)M;
        g.a_rows = e->cap_rows;
        g.hidden = H;
        g.stats_ld = ld;
        g.n_part = n_part;
        g.ln_h = H;
        g.ln_eps = c.layer_norm_eps;
        g.split = sp ? 1 : 0;
        return g;
    };
    for (size_t l = 0; l < e->layers.size(); ++l) {
        Layer &L = *e->layers[l];
        const Layer *P = l > 0 ? e->layers[l - 1].get() : nullptr;
        const bool last = l + 1 == e->layers.size();
        const bool prune = last && d_tt != nullptr;
        const int64_t Mr = prune ? n_terms : M;  // rows from here on
        bf16 *Xr = X;                             // the O GEMM's residual rows
        const float2 *rl2r = rl2;
        auto gather_rows = [&]() {  // the terms' layer-input rows (and LN2 parameters):
            TimedLaunch tl(e->timer, timing, "gather_rows", s);  // Hff / rl1 are free
            Xr = e->Hff.as<bf16>();                               // until later
            launch_gather_term_rows(X, P ? rl2 : nullptr, d_cu, d_ct, d_tt, n_docs, H * W2, Xr,
                                    rl1, s);
            rl2r = rl1;
        };
        // Pruned last layer, split path: the queries are the terms' rows only, so Q is
        // projected from their gathered rows (a GEMM of n_terms rows) and K | V from every
        // row -- each kept element the same sum in the same order as the full QKV GEMM's;
        // the packed Q rows then go to their token rows' Q columns of qk, where the
        // attention reads them (one 3 KiB copy per term)
        const bool qc = prune && sp;
        if (qc) gather_rows();
        // QKV: layer 0 reads the normalised embeddings; later layers fold LN2(l-1)
        GemmArgs g = base();
        g.A = X;
        g.B = L.w_qkv.p;
        g.bias = L.b_qkv.as<float>();
        g.out = e->qk.p;
        g.N = 3 * H;
        g.K = H;
        g.ld_out = 3 * H * W2;
        if (P) {
            g.row_ln = rl2;
            g.col_s = L.s_qkv.as<float>();
            g.col_c = L.c_qkv.as<float>();
        }
        {
            TimedLaunch tl(e->timer, timing, "gemm_qkv", s);
            if (!qc) {
                gemm(P ? EPI_FOLD : EPI_BIAS, g);
            } else {
                GemmArgs gk = g;  // K | V: weight rows H .. 3H, output columns H .. 3H
                gk.B = static_cast<const bf16 *>(L.w_qkv.p) + (int64_t)H * 2 * H;
                gk.bias = L.b_qkv.as<float>() + H;
                if (P) {
                    gk.col_s = L.s_qkv.as<float>() + H;
                    gk.col_c = L.c_qkv.as<float>() + H;
                }
                gk.out = e->qk.as<bf16>() + 2 * H;
                gk.N = 2 * H;
                gemm(P ? EPI_FOLD : EPI_BIAS, gk);
                GemmArgs gq = g;  // Q of the terms' rows, packed (ctx: free until the attention)
                gq.A = Xr;
                gq.M = (int)n_terms;
                gq.N = H;
                gq.out = e->ctx.p;
                gq.ld_out = 2 * H;
                gq.row_ln = P ? rl1 : nullptr;
                gemm(P ? EPI_FOLD : EPI_BIAS, gq);
                launch_scatter_term_rows(e->ctx.as<bf16>(), d_cu, d_ct, d_tt, n_docs, 2 * H,
                                         6 * (int64_t)H, e->qk.as<bf16>(), s);
            }
        }
        {
            TimedLaunch tl(e->timer, timing, "attention", s);
            if (sp)
                launch_attention_x3(e->qk.as<bf16>(), d_cu, n_docs, H, e->ctx.as<bf16>(), s,
                                    prune ? d_tt : nullptr, prune ? d_ct : nullptr);
            else
                launch_attention_v3(e->qk.as<bf16>(), d_cu, n_docs, max_len, H,
                                    e->ctx.as<bf16>(), s, prune ? d_tt : nullptr,
                                    prune ? d_ct : nullptr);
        }
        if (prune && !qc) gather_rows();
        auto base_r = [&]() {
            GemmArgs gr = base();
            gr.M = (int)Mr;
            return gr;
        };
        // O: P1 = ctx W_o^T + b_o + LN2(l-1)(X)  (plain X on layer 0) -> X1, stats1
        g = base_r();
        g.A = e->ctx.p;
        g.B = L.w_o.p;
        g.bias = L.b_o.as<float>();
        g.resid = Xr;
        g.out = X1;
        g.N = H;
        g.K = H;
        g.ld_out = H * W2;
        g.stats_out = st1;
        if (P) {
            g.row_ln = rl2r;
            g.res_gamma = P->ln2_g.as<float>();
            g.res_beta = P->ln2_b.as<float>();
        }
        {
            TimedLaunch tl(e->timer, timing, "gemm_o", s);
            gemm(EPI_RESID_STATS, g);
        }
        {
            TimedLaunch tl(e->timer, timing, "row_ln", s);
            launch_row_ln(st1, ld, n_part, (int)Mr, H, c.layer_norm_eps, rl1, s);
        }
        // FFN1 on LN1(P1), folded
        g = base_r();
        g.A = X1;
        g.B = L.w_i.p;
        g.out = e->Hff.p;
        g.N = F;
        g.K = H;
        g.ld_out = F * W2;
        g.row_ln = rl1;
        g.col_s = L.s_i.as<float>();
        g.col_c = L.c_i.as<float>();
        {
            TimedLaunch tl(e->timer, timing, "gemm_ffn1", s);
            gemm(EPI_FOLD_GELU, g);
        }
        // FFN2: P2 = Hff W_out^T + b_out + LN1(P1) -> X, stats2 (+ head dot, last layer)
        g = base_r();
        g.A = e->Hff.p;
        g.B = L.w_out.p;
        g.bias = L.b_out.as<float>();
        g.resid = X1;
        g.out = X;
        g.N = H;
        g.K = F;
        g.ld_out = H * W2;
        g.tune_gm = 4;
        g.row_ln = rl1;
        g.res_gamma = L.ln1_g.as<float>();
        g.res_beta = L.ln1_b.as<float>();
        g.stats_out = st2;
        g.head_wg = last ? e->head_wg.as<float>() : nullptr;
        {
            TimedLaunch tl(e->timer, timing, "gemm_ffn2", s);
            gemm(EPI_RESID_STATS, g);
        }
        if (!last) {
            TimedLaunch tl(e->timer, timing, "row_ln", s);
            launch_row_ln(st2, ld, n_part, (int)M, H, c.layer_norm_eps, rl2, s);
        }
    }
    {
        TimedLaunch tl(e->timer, timing, "head", s);
        launch_head_from_stats(st2, ld, n_part, (int)(d_tt ? n_terms : M), H, c.layer_norm_eps,
                               e->head_sw,
                               e->head_cw, c.activation, e->impact.as<float>(), s);
    }
}

// fp32-faithful forward (DI_PREC_BF16X3): the unfolded post-LN structure of
// forward<T> with every GEMM a split-bf16 256-tile GEMM (3 bf16 MFMA products per
// fp32 product, f32 accumulate: ~2^-17 relative per product), attention with split
// bf16 products too (attention_x3_kernel; f32 softmax), LayerNorms in f32 from f32
// pre-LN rows.  Activations that feed a GEMM or the attention products are split
// rows (Q | K and V^T included); the pre-LN rows are f32.
// Pruned last layer (d_tt != nullptr), as forward_folded: after the last QKV projection
// only the terms' first-token rows are computed (attention queries, O / FFN GEMMs,
// LayerNorms, head), packed -- the same arithmetic per kept row, bit-identical impacts.
void forward_split(di_encoder *e, const int32_t *d_ids, const int32_t *d_cu, int n_docs,
                   int64_t M, int max_len, bool timing, hipStream_t s,
                   const int32_t *d_tt = nullptr, const int32_t *d_ct = nullptr,
                   int64_t n_terms = 0) {
    const auto &c = e->cfg;
    const int H = c.hidden, F = c.intermediate;
    const int pos_offset = (c.variant == DI_VARIANT_XLMR) ? c.pad_id + 1 : 0;
    bf16 *X = e->X.as<bf16>(), *X1 = e->X1.as<bf16>(), *ctx = e->ctx.as<bf16>();
    float *pre = e->pre.as<float>();
    {
        TimedLaunch tl(e->timer, timing, "embed_ln", s);
        launch_embed_ln_split(d_ids, d_cu, n_docs, (int)M, H, e->word.as<float>(),
                              e->pos.as<float>(), e->type0.as<float>(), e->emb_g.as<float>(),
                              e->emb_b.as<float>(), c.layer_norm_eps, pos_offset, c.vocab_size,
                              c.max_positions, X, e->err.as<int32_t>(), s);
    }
    auto base = [&]() {
        GemmArgs g{};
        g.M = (int)M;
        g.a_rows = e->cap_rows;
        g.hidden = H;
        g.tune_gm = 8;
        g.split = 1;
        return g;
    };
    for (size_t l = 0; l < e->layers.size(); ++l) {
        Layer &L = *e->layers[l];
        const bool last = l + 1 == e->layers.size();
        GemmArgs g = base();
        g.A = X;
        g.B = L.w_qkv.p;
        g.bias = L.b_qkv.as<float>();
        g.out = e->qk.p;  // split Q | K | V rows [M][6H]
        g.N = 3 * H;
        g.K = H;
        g.ld_out = 6 * H;
        {
            TimedLaunch tl(e->timer, timing, "gemm_qkv", s);
            launch_gemm256(EPI_BIAS, g, s);
        }
        const bool prune = last && d_tt != nullptr;
        const int64_t Mr = prune ? n_terms : M;  // rows from here on
        bf16 *Xr = X;                             // the O GEMM's residual rows
        {
            TimedLaunch tl(e->timer, timing, "attention", s);
            launch_attention_x3(e->qk.as<bf16>(), d_cu, n_docs, H, ctx, s,
                                prune ? d_tt : nullptr, prune ? d_ct : nullptr);
        }
        if (prune) {  // the terms' residual rows, packed into Hff (free until FFN1)
            TimedLaunch tl(e->timer, timing, "gather_rows", s);
            Xr = e->Hff.as<bf16>();
            launch_gather_term_rows(X, nullptr, d_cu, d_ct, d_tt, n_docs, 2 * H, Xr, nullptr, s);
        }
        auto base_r = [&]() {
            GemmArgs gr = base();
            gr.M = (int)Mr;
            return gr;
        };
        g = base_r();
        g.A = ctx;
        g.B = L.w_o.p;
        g.bias = L.b_o.as<float>();
        g.resid = Xr;
        g.out = pre;
        g.N = H;
        g.K = H;
        g.ld_out = H;
        {
            TimedLaunch tl(e->timer, timing, "gemm_o", s);
            launch_gemm256(EPI_BIAS_RESID, g, s);
        }
        {
            TimedLaunch tl(e->timer, timing, "ln", s);
            launch_ln_split(pre, (int)Mr, H, L.ln1_g.as<float>(), L.ln1_b.as<float>(),
                            c.layer_norm_eps, X1, nullptr, 0.f, c.activation, nullptr, s);
        }
        g = base_r();
        g.A = X1;
        g.B = L.w_i.p;
        g.bias = L.b_i.as<float>();
        g.out = e->Hff.p;
        g.N = F;
        g.K = H;
        g.ld_out = 2 * F;
        {
            TimedLaunch tl(e->timer, timing, "gemm_ffn1", s);
            launch_gemm256(EPI_BIAS_GELU, g, s);
        }
        g = base_r();
        g.A = e->Hff.p;
        g.B = L.w_out.p;
        g.bias = L.b_out.as<float>();
        g.resid = X1;
        g.out = pre;
        g.N = H;
        g.K = F;
        g.ld_out = H;
        g.tune_gm = 4;
        {
            TimedLaunch tl(e->timer, timing, "gemm_ffn2", s);
            launch_gemm256(EPI_BIAS_RESID, g, s);
        }
        {
            TimedLaunch tl(e->timer, timing, "ln", s);
            launch_ln_split(pre, (int)Mr, H, L.ln2_g.as<float>(), L.ln2_b.as<float>(),
                            c.layer_norm_eps, last ? nullptr : X,
                            last ? e->head_w.as<float>() : nullptr, e->head_b, c.activation,
                            last ? e->impact.as<float>() : nullptr, s);
        }
    }
}

}  // namespace

extern "C" {

int di_encoder_create(const di_encoder_cfg *cfg, const di_tensor *w, int32_t n_w, int device,
                      di_encoder **out) {
    return guard([&] {
        DI_REQUIRE(cfg && out && (n_w == 0 || w), DI_EINVAL, "null argument");
        int ndev = 0;
        DI_REQUIRE(hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0, DI_ENODEV,
                   "no HIP device");
        DI_REQUIRE(device >= 0 && device < ndev, DI_EINVAL, "bad device %d", device);
        const di_encoder_cfg &c = *cfg;
        DI_REQUIRE(c.variant == DI_VARIANT_XLMR || c.variant == DI_VARIANT_BERT, DI_EINVAL,
                   "bad variant");
        DI_REQUIRE(c.activation == DI_ACT_SOFTPLUS || c.activation == DI_ACT_RELU, DI_EINVAL,
                   "bad activation");
        DI_REQUIRE(c.precision == DI_PREC_BF16 || c.precision == DI_PREC_FP32 ||
                       c.precision == DI_PREC_BF16X3,
                   DI_EINVAL, "bad precision");
        DI_REQUIRE(c.precision != DI_PREC_BF16X3 ||
                       ((c.hidden == 768 || c.hidden == 1024) && c.intermediate % 256 == 0),
                   DI_EINVAL, "bf16x3 mode: hidden 768 / 1024 and intermediate %% 256");
        DI_REQUIRE(c.hidden > 0 && c.hidden % 64 == 0 && c.hidden <= 1024, DI_EINVAL,
                   "hidden=%d must be a multiple of 64, <= 1024", c.hidden);
        DI_REQUIRE(c.heads > 0 && c.hidden / c.heads == 64 && c.hidden % c.heads == 0,
                   DI_EINVAL, "head dim must be 64 (hidden=%d heads=%d)", c.hidden, c.heads);
        DI_REQUIRE(c.intermediate > 0 && c.intermediate % 64 == 0, DI_EINVAL,
                   "intermediate=%d must be a multiple of 64", c.intermediate);
        DI_REQUIRE(c.layers > 0 && c.vocab_size > 0 && c.max_positions > 0, DI_EINVAL,
                   "bad sizes");
        DeviceScope ds(device);
        std::unique_ptr<di_encoder> e(new di_encoder());
        e->cfg = c;
        e->device = device;
        e->esz = c.precision == DI_PREC_BF16 ? 2 : 4;
        e->split = c.precision == DI_PREC_BF16X3;
        DI_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
        e->own_stream = true;

        std::unordered_map<std::string, HostTensor> byname;
        std::vector<HostTensor> ht((size_t)n_w);
        for (int i = 0; i < n_w; ++i) {
            DI_REQUIRE(w[i].name && w[i].data, DI_EINVAL, "tensor %d has no name/data", i);
            DI_REQUIRE(w[i].dtype == DI_DTYPE_F32 || w[i].dtype == DI_DTYPE_BF16, DI_EINVAL,
                       "tensor %s: dtype must be f32 or bf16", w[i].name);
            ht[(size_t)i].t = &w[i];
            std::string k = strip_prefix(w[i].name);
            if (k == "embeddings.position_ids" || k.rfind("pooler.", 0) == 0) continue;
            byname[k] = ht[(size_t)i];
        }
        std::unordered_map<std::string, int> used;
        auto get = [&](const std::string &k, std::initializer_list<int64_t> shape)
            -> const HostTensor * {
            auto it = byname.find(k);
            DI_REQUIRE(it != byname.end(), DI_EINVAL, "missing weight %s", k.c_str());
            const di_tensor *t = it->second.t;
            DI_REQUIRE(t->ndim == (int)shape.size(), DI_EINVAL, "weight %s: ndim %d", k.c_str(),
                       t->ndim);
            int i = 0;
            for (int64_t d : shape) {
                DI_REQUIRE(d < 0 || t->shape[i] == d, DI_EINVAL,
                           "weight %s: dim %d is %lld, expected %lld", k.c_str(), i,
                           (long long)t->shape[i], (long long)d);
                ++i;
            }
            used[k] = 1;
            return &it->second;
        };
        const int64_t H = c.hidden, F = c.intermediate;
        const HostTensor *we = get("embeddings.word_embeddings.weight", {c.vocab_size, H});
        const HostTensor *pe = get("embeddings.position_embeddings.weight", {-1, H});
        DI_REQUIRE(pe->t->shape[0] >= c.max_positions, DI_EINVAL,
                   "position table has %lld rows < max_positions %d",
                   (long long)pe->t->shape[0], c.max_positions);
        const HostTensor *te = get("embeddings.token_type_embeddings.weight", {-1, H});
        upload(e->word, {we}, 0, false, e->esz);
        upload(e->pos, {pe}, 0, false, e->esz);
        {
            // token_type_ids are not passed (xlmr_original.py:73): row 0 is used
            di_tensor row0 = *te->t;
            row0.ndim = 1;
            row0.shape[0] = H;
            HostTensor r0{&row0};
            upload(e->type0, {&r0}, 0, false, e->esz);
        }
        upload(e->emb_g, {get("embeddings.LayerNorm.weight", {H})}, 0, true, 4);
        upload(e->emb_b, {get("embeddings.LayerNorm.bias", {H})}, 0, true, 4);
        // LayerNorm folding: bf16 with shapes the 256-tile GEMM takes (DI_NO_LN_FOLD: off)
        // (bf16x3 too: the GEMMs then read split rows of the un-normalised x, 2^-17
        // relative, and no LayerNorm pass runs)
        e->folded = (e->esz == 2 || e->split) && H % 256 == 0 && F % 256 == 0 && H <= 1024 &&
                    std::getenv("DI_NO_LN_FOLD") == nullptr;
        const HostTensor *prev_g2 = nullptr, *prev_b2 = nullptr;  // LN2 of layer l-1
        for (int l = 0; l < c.layers; ++l) {
            std::string p = "encoder.layer." + std::to_string(l) + ".";
            auto L = std::make_unique<Layer>();
            const std::vector<const HostTensor *> wqkv = {
                get(p + "attention.self.query.weight", {H, H}),
                get(p + "attention.self.key.weight", {H, H}),
                get(p + "attention.self.value.weight", {H, H})};
            const std::vector<const HostTensor *> bqkv = {
                get(p + "attention.self.query.bias", {H}), get(p + "attention.self.key.bias", {H}),
                get(p + "attention.self.value.bias", {H})};
            if (e->folded && l > 0)  // layer 0 reads the (normalised) embedding output
                fold_upload(L->w_qkv, L->s_qkv, L->c_qkv, wqkv, bqkv, H, prev_g2, prev_b2,
                            e->split);
            else if (e->split)
                upload_split3(L->w_qkv, wqkv, (int)H);
            else
                upload(L->w_qkv, wqkv, 0, false, e->esz);
            upload(L->b_qkv, bqkv, 0, true, 4);
            if (e->split)
                upload_split3(L->w_o, {get(p + "attention.output.dense.weight", {H, H})}, (int)H);
            else
                upload(L->w_o, {get(p + "attention.output.dense.weight", {H, H})}, 0, false,
                       e->esz);
            upload(L->b_o, {get(p + "attention.output.dense.bias", {H})}, 0, true, 4);
            upload(L->ln1_g, {get(p + "attention.output.LayerNorm.weight", {H})}, 0, true, 4);
            upload(L->ln1_b, {get(p + "attention.output.LayerNorm.bias", {H})}, 0, true, 4);
            const HostTensor *wi = get(p + "intermediate.dense.weight", {F, H});
            const HostTensor *bi = get(p + "intermediate.dense.bias", {F});
            if (e->folded)
                fold_upload(L->w_i, L->s_i, L->c_i, {wi}, {bi}, H,
                            get(p + "attention.output.LayerNorm.weight", {H}),
                            get(p + "attention.output.LayerNorm.bias", {H}), e->split);
            else if (e->split)
                upload_split3(L->w_i, {wi}, (int)H);
            else
                upload(L->w_i, {wi}, 0, false, e->esz);
            upload(L->b_i, {bi}, 0, true, 4);
            if (e->split)
                upload_split3(L->w_out, {get(p + "output.dense.weight", {H, F})}, (int)F);
            else
                upload(L->w_out, {get(p + "output.dense.weight", {H, F})}, 0, false, e->esz);
            upload(L->b_out, {get(p + "output.dense.bias", {H})}, 0, true, 4);
            prev_g2 = get(p + "output.LayerNorm.weight", {H});
            prev_b2 = get(p + "output.LayerNorm.bias", {H});
            upload(L->ln2_g, {prev_g2}, 0, true, 4);
            upload(L->ln2_b, {prev_b2}, 0, true, 4);
            e->layers.push_back(std::move(L));
        }
        const HostTensor *hw = get("impact_score_encoder.0.weight", {1, H});
        upload(e->head_w, {hw}, 0, true, 4);
        e->head_b = get("impact_score_encoder.0.bias", {1})->at(0);
        if (e->folded) {  // head on the folded last LayerNorm: w * gamma, sums
            std::vector<float> wg((size_t)H);
            double sw = 0.0, cw = e->head_b;
            for (int k = 0; k < H; ++k) {
                wg[(size_t)k] = hw->at(k) * prev_g2->at(k);
                sw += wg[(size_t)k];
                cw += (double)hw->at(k) * prev_b2->at(k);
            }
            e->head_wg.reserve((size_t)H * 4);
            DI_HIP(hipMemcpy(e->head_wg.p, wg.data(), (size_t)H * 4, hipMemcpyHostToDevice));
            e->head_sw = (float)sw;
            e->head_cw = (float)cw;
        }
        // strict, as ModelCheckpoint.load -> load_state_dict (checkpoint.py:117)
        for (auto &kv : byname)
            DI_REQUIRE(used.count(kv.first), DI_EINVAL, "unexpected weight %s",
                       kv.first.c_str());
        *out = e.release();
    });
}

int di_encode(di_encoder *e, const int32_t *tok_ids, const int32_t *cu_seqlens, int32_t n_docs,
              int64_t n_tokens, int32_t max_len, const int32_t *term_tok, const int32_t *cu_terms,
              int64_t n_terms, float *out, uint32_t flags) {
    return guard([&] {
        DI_REQUIRE(e && cu_seqlens && out && n_docs >= 0, DI_EINVAL, "bad argument");
        DeviceScope ds(e->device);
        const bool dev = flags & DI_F_DEVICE_PTRS;
        const bool timing = flags & DI_F_TIMING;
        const bool token_out = flags & DI_F_TOKEN_IMPACTS;
        hipStream_t s = e->stream;
        if (!dev) {
            DI_REQUIRE(cu_seqlens[0] == 0, DI_EINVAL, "cu_seqlens[0] must be 0");
            int32_t mx = 0;
            for (int d = 0; d < n_docs; ++d) {
                int32_t len = cu_seqlens[d + 1] - cu_seqlens[d];
                DI_REQUIRE(len >= 0, DI_EINVAL, "cu_seqlens not monotone at %d", d);
                mx = std::max(mx, len);
            }
            n_tokens = cu_seqlens[n_docs];
            max_len = mx;
            if (!token_out) {
                DI_REQUIRE(term_tok && cu_terms && cu_terms[0] == 0, DI_EINVAL,
                           "term arrays required");
                n_terms = cu_terms[n_docs];
            }
        }
        DI_REQUIRE(n_tokens >= 0 && n_tokens < (1ll << 31), DI_ERANGE, "n_tokens=%lld",
                   (long long)n_tokens);
        DI_REQUIRE(max_len <= e->cfg.max_positions, DI_ERANGE,
                   "a document has %d tokens > max_positions %d", max_len,
                   e->cfg.max_positions);
        if (n_docs == 0) return;
        ensure_workspace(e, n_tokens, n_docs, n_terms);
        const int32_t *d_ids =
            (const int32_t *)stage_in(tok_ids, (size_t)n_tokens * 4, dev, e->ids, s);
        const int32_t *d_cu =
            (const int32_t *)stage_in(cu_seqlens, (size_t)(n_docs + 1) * 4, dev, e->cu, s);
        DI_HIP(hipMemsetAsync(e->err.p, 0, 4, s));
        const int32_t *d_tt = nullptr, *d_cut = nullptr;
        if (!token_out) {
            d_tt = (const int32_t *)stage_in(term_tok, (size_t)n_terms * 4, dev, e->tt, s);
            d_cut = (const int32_t *)stage_in(cu_terms, (size_t)(n_docs + 1) * 4, dev, e->cut, s);
        }
        // pruned last layer (bf16 folded and bf16x3 paths, term output)
        const bool prune = !token_out && (e->split || (e->esz == 2 && e->folded)) &&
                           n_terms <= n_tokens;  // (packed term rows fit the row buffers)
        if (n_tokens > 0) {
            if (e->split && !e->folded)
                forward_split(e, d_ids, d_cu, n_docs, n_tokens, max_len, timing, s,
                              prune ? d_tt : nullptr, prune ? d_cut : nullptr, n_terms);
            else if (e->split)
                forward_folded(e, d_ids, d_cu, n_docs, n_tokens, max_len, timing, s,
                               prune ? d_tt : nullptr, prune ? d_cut : nullptr, n_terms);
            else if (e->esz == 2)
                if (e->folded)
                    forward_folded(e, d_ids, d_cu, n_docs, n_tokens, max_len, timing, s,
                                   prune ? d_tt : nullptr, prune ? d_cut : nullptr, n_terms);
                else
                    forward<bf16>(e, d_ids, d_cu, n_docs, n_tokens, max_len, timing, s);
            else
                forward<float>(e, d_ids, d_cu, n_docs, n_tokens, max_len, timing, s);
        }
        float *d_out = out;
        DevBuf tmp;
        if (token_out) {
            if (dev)
                DI_HIP(hipMemcpyAsync(out, e->impact.p, (size_t)n_tokens * 4,
                                      hipMemcpyDeviceToDevice, s));
            else
                DI_HIP(hipMemcpyAsync(out, e->impact.p, (size_t)n_tokens * 4,
                                      hipMemcpyDeviceToHost, s));
        } else {
            if (!dev) {
                tmp.reserve((size_t)std::max<int64_t>(n_terms, 1) * 4);
                d_out = tmp.as<float>();
            }
            {
                TimedLaunch tl(e->timer, timing, "gather_terms", s);
                launch_gather_terms(e->impact.as<float>(), d_cu, d_cut, n_docs, d_tt,
                                    (int)n_terms,
                                    ((flags & DI_F_ROUND3) ? 1 : 0) | (prune && n_tokens > 0 ? 2 : 0),
                                    d_out, e->err.as<int32_t>(), s);
            }
            if (!dev && n_terms)
                DI_HIP(hipMemcpyAsync(out, d_out, (size_t)n_terms * 4, hipMemcpyDeviceToHost,
                                      s));
        }
        if (!(flags & DI_F_ASYNC) || !dev) {
            int32_t err = 0;
            DI_HIP(hipMemcpyAsync(&err, e->err.p, 4, hipMemcpyDeviceToHost, s));
            DI_HIP(hipStreamSynchronize(s));
            e->timer.resolve();
            DI_REQUIRE(!(err & 1), DI_EINVAL,
                       "a token id is outside the vocabulary or a position exceeds the table");
            DI_REQUIRE(!(err & 2), DI_EINVAL, "a term token index is outside its document");
        }
    });
}

int di_encoder_reserve(di_encoder *e, int64_t max_tokens, int32_t max_docs, int64_t max_terms) {
    return guard([&] {
        DI_REQUIRE(e && max_tokens >= 0 && max_docs >= 0 && max_terms >= 0, DI_EINVAL,
                   "bad argument");
        DeviceScope ds(e->device);
        ensure_workspace(e, max_tokens, max_docs, max_terms);
    });
}

int di_encoder_set_stream(di_encoder *e, void *stream) {
    return guard([&] {
        DI_REQUIRE(e, DI_EINVAL, "null handle");
        DeviceScope ds(e->device);
        if (e->own_stream && e->stream) DI_HIP(hipStreamDestroy(e->stream));
        e->own_stream = stream == nullptr;
        if (stream)
            e->stream = (hipStream_t)stream;
        else
            DI_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    });
}

int di_encoder_sync(di_encoder *e) {
    return guard([&] {
        DI_REQUIRE(e, DI_EINVAL, "null handle");
        DeviceScope ds(e->device);
        DI_HIP(hipStreamSynchronize(e->stream));
        e->timer.resolve();
    });
}

int di_encoder_timing(di_encoder *e, const char *name, di_timing *out, int reset) {
    return guard([&] {
        DI_REQUIRE(e && name && out, DI_EINVAL, "null argument");
        e->timer.get(name, out, reset != 0);
    });
}

int di_encoder_destroy(di_encoder *e) {
    return guard([&] {
        if (!e) return;
        {
            DeviceScope ds(e->device);
            if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
        }
        delete e;
    });
}

}  // extern "C"
