// synthetic.cpp -- seeded MS MARCO-shaped collections at full scale (bench / test data).
//
// There is no network and no MS MARCO here: retrieval benches run on
// a collection of the same shape, made by the generator SURVEY §8d / BASELINE.md §2
// specify -- per doc the first `max_terms` unique values (ascending, as np.unique) of
// `draws` draws of min(zipf(a), V), impacts float32(softplus(N(-0.5, 1.5))), then the
// reference text path: round(., 3) (indexer.py:62-68), the 8-bit quantizer with its
// fp64 global max (quantize.py:13-47, zeros dropped) and the index order value desc /
// doc asc per term (create.py:41).  synthetic.py's numpy generator draws the same
// distribution one doc at a time (minutes at 8.8 M docs); this one runs threads over
// doc chunks (8.8 M docs in seconds) with a counter-based stream per doc, so the
// output depends on (seed, doc) only -- not on the thread count.
//
// Zipf sampling: Walker alias table over 1..V with P(k) = k^-a / zeta(a) (k < V) and
// the clamped tail P(V) = sum_{k >= V} k^-a / zeta(a) (Euler-Maclaurin), i.e. exactly
// min(zipf(a), V).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "di_common.h"
#include "pytext.h"

namespace {

inline uint64_t splitmix64(uint64_t &x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Rng {  // xoshiro256** seeded from (seed, stream) by splitmix64
    uint64_t s[4];
    Rng(uint64_t seed, uint64_t stream) {
        uint64_t x = seed * 0xD1342543DE82EF95ull + stream;
        for (auto &v : s) v = splitmix64(x);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    double uniform() { return (double)(next() >> 11) * 0x1.0p-53; }  // [0, 1)
    double normal() {  // Box-Muller (one of the pair)
        double u1 = uniform(), u2 = uniform();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

struct Alias {
    std::vector<double> prob;
    std::vector<uint32_t> alias;
    Alias(int V, double a) {
        std::vector<double> p((size_t)V);
        double head = 0.0;
        for (int k = 1; k < V; ++k) head += (p[(size_t)k - 1] = std::pow((double)k, -a));
        const double v = V;  // sum_{k >= V} k^-a, Euler-Maclaurin
        const double tail = std::pow(v, 1.0 - a) / (a - 1.0) + 0.5 * std::pow(v, -a) +
                            a / 12.0 * std::pow(v, -a - 1.0);
        p[(size_t)V - 1] = tail;
        const double z = head + tail;
        prob.assign((size_t)V, 0.0);
        alias.assign((size_t)V, 0);
        std::vector<uint32_t> small, large;
        std::vector<double> q((size_t)V);
        for (int i = 0; i < V; ++i) {
            q[(size_t)i] = p[(size_t)i] / z * V;
            (q[(size_t)i] < 1.0 ? small : large).push_back((uint32_t)i);
        }
        while (!small.empty() && !large.empty()) {
            const uint32_t s = small.back(), l = large.back();
            small.pop_back();
            prob[s] = q[s];
            alias[s] = l;
            q[l] -= 1.0 - q[s];
            if (q[l] < 1.0) {
                large.pop_back();
                small.push_back(l);
            }
        }
        for (uint32_t i : large) prob[i] = 1.0;
        for (uint32_t i : small) prob[i] = 1.0;
    }
    uint32_t sample(Rng &r) const {  // value in 1..V
        const double u = r.uniform() * (double)prob.size();
        const uint32_t i = (uint32_t)u;
        return (u - i < prob[i] ? i : alias[i]) + 1;
    }
};

// numpy's round(np.float32, 3): fl32(rint(fl32(x * 1000)) / 1000)
inline float round3(float x) {
    volatile float t = x * 1000.0f;  // (no contraction)
    return (float)(std::nearbyint(t)) / 1000.0f;
}

// Skew of the impacts (di_synth_skew, include/deepimpact.h; all off = SURVEY §8d's
// i.i.d. impacts): impact = softplus(N(-0.5, 1.5)) x term factor x doc mass.
struct Skew {
    double term_rank0 = 0.0, term_exp = 0.0;
    int32_t cluster_docs = 0;
    double cluster_sigma = 0.0, doc_sigma = 0.0, mass_max = 0.0;
    bool on() const { return term_rank0 > 0.0 || cluster_docs > 0 || doc_sigma > 0.0; }
    // the term of 0-based zipf rank t: frequent terms carry small impacts (the IDF-like
    // shape a learned impact model gives its common terms)
    double term_factor(uint32_t t) const {
        if (term_rank0 <= 0.0) return 1.0;
        return std::min(1.0, std::pow(((double)t + 1.0) / term_rank0, term_exp));
    }
    // doc d's mass: a lognormal factor shared by its cluster of consecutive doc ids
    // (passages of one source document sit together) times its own, clipped
    double mass(uint64_t seed, int64_t d, Rng &r) const {
        double z = doc_sigma > 0.0 ? doc_sigma * r.normal() : 0.0;
        if (cluster_docs > 0) {
            Rng rc(seed ^ 0x5BD1E9955BD1E995ull, (uint64_t)(d / cluster_docs));
            z += cluster_sigma * rc.normal();
        }
        const double m = std::exp(z);
        return mass_max > 0.0 ? std::min(m, mass_max) : m;
    }
};

// Doc d of the collection: its sorted unique 0-based term ids and float32 impacts
// (the stream depends on (seed, d) only).
inline void synth_doc(const Alias &zipf, uint64_t seed, int64_t d, int32_t max_terms,
                      int32_t draws, std::vector<uint32_t> &buf, std::vector<uint32_t> &terms,
                      std::vector<float> &imps, const Skew &sk = Skew()) {
    Rng r(seed, (uint64_t)d);
    buf.resize((size_t)draws);
    for (int i = 0; i < draws; ++i) buf[(size_t)i] = zipf.sample(r);
    std::sort(buf.begin(), buf.end());
    const size_t n = (size_t)(std::unique(buf.begin(), buf.end()) - buf.begin());
    const size_t m = std::min<size_t>(n, (size_t)max_terms);
    terms.clear();
    imps.clear();
    for (size_t i = 0; i < m; ++i) {
        const double x = r.normal() * 1.5 - 0.5;
        terms.push_back(buf[i] - 1);
        imps.push_back((float)std::log1p(std::exp(x)));
    }
    if (sk.on()) {  // (after the i.i.d. draws: the skew-free stream is unchanged)
        const double md = sk.mass(seed, d, r);
        for (size_t i = 0; i < m; ++i)
            imps[i] = (float)((double)imps[i] * sk.term_factor(terms[i]) * md);
    }
}

}  // namespace

// The same collection as di_synth_postings, as the impact TSV the index CLI writes
// (indexer.py:62-68: ', '.join(f'{term}: {round(impact, 3)}'), one line per doc), the
// term of id t spelled "\u2581t<t>" (an XLM-R-style Metaspace term).  Bench input of
// the quantize and index-create legs (A10 / A11).  Threads over doc chunks, written in
// order; *n_terms_out = the (doc, term) pairs written.
extern "C" int di_synth_impact_tsv(const char *path, int64_t n_docs, int32_t v_terms,
                                   uint64_t seed, int32_t max_terms, int32_t draws,
                                   double zipf_a, int64_t *n_terms_out) {
    using namespace di;
    return guard([&] {
        DI_REQUIRE(path && n_docs >= 0 && v_terms > 0 && max_terms > 0 && draws > 0 &&
                       zipf_a > 1.0,
                   DI_EINVAL, "bad argument");
        const Alias zipf(v_terms, zipf_a);
        FILE *f = std::fopen(path, "wb");
        DI_REQUIRE(f, DI_EIO, "cannot create %s", path);
        const int T = host_threads();
        const int64_t per = 65536;  // docs per chunk; T chunks formatted at a time
        int64_t total = 0;
        bool ok = true;
        std::vector<std::string> text((size_t)T);
        std::vector<int64_t> cnt((size_t)T);
        for (int64_t d0 = 0; d0 < n_docs && ok; d0 += per * T) {
            parallel_for(T, [&](int64_t lo, int64_t hi, int) {
                std::vector<uint32_t> buf, terms;
                std::vector<float> imps;
                char num[16];
                for (int64_t c = lo; c < hi; ++c) {
                    std::string &out = text[(size_t)c];
                    out.clear();
                    cnt[(size_t)c] = 0;
                    const int64_t a = std::min(n_docs, d0 + c * per), b = std::min(n_docs, a + per);
                    for (int64_t d = a; d < b; ++d) {
                        synth_doc(zipf, seed, d, max_terms, draws, buf, terms, imps);
                        for (size_t i = 0; i < terms.size(); ++i) {
                            if (i) out += ", ";
                            out += "\xe2\x96\x81t";
                            const int len = std::snprintf(num, sizeof num, "%u", terms[i]);
                            out.append(num, (size_t)len);
                            out += ": ";
                            py::repr_double((double)round3(imps[i]), out);
                        }
                        out += '\n';
                        cnt[(size_t)c] += (int64_t)terms.size();
                    }
                }
            });
            for (int c = 0; c < T; ++c) {
                ok = ok && std::fwrite(text[(size_t)c].data(), 1, text[(size_t)c].size(), f) ==
                               text[(size_t)c].size();
                total += cnt[(size_t)c];
            }
        }
        ok = (std::fclose(f) == 0) && ok;
        DI_REQUIRE(ok, DI_EIO, "short write to %s", path);
        if (n_terms_out) *n_terms_out = total;
    });
}

extern "C" int di_synth_postings_skewed(int64_t n_docs, int32_t v_terms, uint64_t seed,
                                        int32_t max_terms, int32_t draws, double zipf_a,
                                        const di_synth_skew *skew, int64_t *term_off,
                                        uint32_t *pdoc, uint8_t *pval, int64_t cap,
                                        int64_t *n_post, double *max_impact) {
    const int rc = di::guard([&] { DI_REQUIRE(term_off, DI_EINVAL, "bad argument"); });
    if (rc != DI_OK) return rc;
    return di_synth_postings_shard(0, n_docs, v_terms, seed, max_terms, draws, zipf_a, skew, 0.0,
                                   term_off, pdoc, pval, cap, n_post, max_impact);
}

extern "C" int di_synth_postings(int64_t n_docs, int32_t v_terms, uint64_t seed,
                                 int32_t max_terms, int32_t draws, double zipf_a,
                                 int64_t *term_off, uint32_t *pdoc, uint8_t *pval, int64_t cap,
                                 int64_t *n_post, double *max_impact) {
    return di_synth_postings_skewed(n_docs, v_terms, seed, max_terms, draws, zipf_a, nullptr,
                                    term_off, pdoc, pval, cap, n_post, max_impact);
}

extern "C" int di_synth_postings_shard(int64_t doc0, int64_t n_docs, int32_t v_terms,
                                       uint64_t seed, int32_t max_terms, int32_t draws,
                                       double zipf_a, const di_synth_skew *skew, double quant_max,
                                       int64_t *term_off, uint32_t *pdoc, uint8_t *pval,
                                       int64_t cap, int64_t *n_post, double *max_impact) {
    using namespace di;
    return guard([&] {
        DI_REQUIRE(n_docs >= 0 && doc0 >= 0 && doc0 + n_docs <= 0xFFFFFFFFll && v_terms > 0 &&
                       max_terms > 0 && draws > 0 && zipf_a > 1.0 && quant_max >= 0.0 &&
                       (term_off || !pdoc) && (n_post || !term_off),
                   DI_EINVAL, "bad argument");
        Skew sk;
        if (skew) {
            DI_REQUIRE(skew->term_rank0 >= 0.0 && skew->term_exp >= 0.0 &&
                           skew->cluster_docs >= 0 && skew->cluster_sigma >= 0.0 &&
                           skew->doc_sigma >= 0.0 && skew->mass_max >= 0.0,
                       DI_EINVAL, "bad skew parameters");
            sk.term_rank0 = skew->term_rank0;
            sk.term_exp = skew->term_exp;
            sk.cluster_docs = skew->cluster_docs;
            sk.cluster_sigma = skew->cluster_sigma;
            sk.doc_sigma = skew->doc_sigma;
            sk.mass_max = skew->mass_max;
        }
        const Alias zipf(v_terms, zipf_a);
        // 1. per doc: sorted unique term ids (0-based) and float32 impacts, chunked
        const int T = host_threads();
        const int64_t n_chunks = std::max<int64_t>(1, std::min<int64_t>(n_docs, 64 * T));
        std::vector<std::vector<uint32_t>> c_term((size_t)n_chunks);
        std::vector<std::vector<float>> c_imp((size_t)n_chunks);
        std::vector<std::vector<uint32_t>> c_len((size_t)n_chunks);
        std::vector<float> c_max((size_t)n_chunks, 0.0f);
        parallel_for(n_chunks, [&](int64_t lo, int64_t hi, int) {
            std::vector<uint32_t> buf((size_t)draws);
            for (int64_t c = lo; c < hi; ++c) {
                const int64_t d0 = n_docs * c / n_chunks, d1 = n_docs * (c + 1) / n_chunks;
                auto &vt = c_term[(size_t)c];
                auto &vi = c_imp[(size_t)c];
                auto &vl = c_len[(size_t)c];
                vt.reserve((size_t)(d1 - d0) * max_terms);
                vi.reserve((size_t)(d1 - d0) * max_terms);
                vl.reserve((size_t)(d1 - d0));
                float mx = 0.0f;
                std::vector<uint32_t> terms;
                std::vector<float> imps;
                for (int64_t d = d0; d < d1; ++d) {
                    synth_doc(zipf, seed, doc0 + d, max_terms, draws, buf, terms, imps, sk);
                    for (size_t i = 0; i < terms.size(); ++i) {
                        vt.push_back(terms[i]);
                        vi.push_back(imps[i]);
                        mx = std::max(mx, round3(imps[i]));
                    }
                    vl.push_back((uint32_t)terms.size());
                }
                c_max[(size_t)c] = mx;
            }
        });
        // 2. max of the 3-decimal impacts (fp64 as the quantizer) and the scale: the
        // shard's own, or quant_max (> 0: the collection's max, all shards alike)
        float mxf = 0.0f;
        for (float m : c_max) mxf = std::max(mxf, m);
        if (max_impact) *max_impact = (double)mxf;
        if (!term_off) return;  // max only
        const double m = quant_max > 0.0 ? quant_max : (double)mxf;
        DI_REQUIRE(m > 0.0 || n_docs == 0, DI_EINVAL, "max impact is 0");
        DI_REQUIRE(m >= (double)mxf, DI_EINVAL, "quant_max %g below the shard's max %g", m,
                   (double)mxf);
        const double scale = 255.0 / (m > 0.0 ? m : 1.0);
        // 3. kept postings per term (quantized value > 0)
        std::vector<int64_t> c_doc0((size_t)n_chunks + 1, 0);
        for (int64_t c = 0; c < n_chunks; ++c) c_doc0[(size_t)c + 1] = n_docs * (c + 1) / n_chunks;
        auto qval = [&](float imp) { return (int)(double)((double)round3(imp) * scale); };
        {
            std::vector<int64_t> cnt((size_t)v_terms + 1, 0);
            std::vector<std::vector<int64_t>> part((size_t)T, std::vector<int64_t>());
            parallel_for(n_chunks, [&](int64_t lo, int64_t hi, int t) {
                auto &pc = part[(size_t)t];
                pc.assign((size_t)v_terms, 0);
                for (int64_t c = lo; c < hi; ++c) {
                    const auto &vt = c_term[(size_t)c];
                    const auto &vi = c_imp[(size_t)c];
                    for (size_t i = 0; i < vt.size(); ++i)
                        if (qval(vi[i]) > 0) pc[vt[i]]++;
                }
            });
            for (auto &pc : part)
                if (!pc.empty())
                    for (int32_t v = 0; v < v_terms; ++v) cnt[(size_t)v + 1] += pc[(size_t)v];
            for (int32_t v = 0; v < v_terms; ++v) cnt[(size_t)v + 1] += cnt[(size_t)v];
            std::memcpy(term_off, cnt.data(), ((size_t)v_terms + 1) * 8);
        }
        const int64_t total = term_off[v_terms];
        *n_post = total;
        if (!pdoc || !pval) return;  // sizes only
        DI_REQUIRE(cap >= total, DI_ERANGE, "postings capacity %lld < %lld", (long long)cap,
                   (long long)total);
        // 4. place by term in doc order (chunks in order: doc ascending inside a term)
        std::vector<int64_t> cur(term_off, term_off + v_terms);
        for (int64_t c = 0; c < n_chunks; ++c) {
            const auto &vt = c_term[(size_t)c];
            const auto &vi = c_imp[(size_t)c];
            const auto &vl = c_len[(size_t)c];
            size_t i = 0;
            for (size_t k = 0; k < vl.size(); ++k) {
                const uint32_t d = (uint32_t)(c_doc0[(size_t)c] + (int64_t)k);
                for (uint32_t j = 0; j < vl[k]; ++j, ++i) {
                    const int q = qval(vi[i]);
                    if (q <= 0) continue;
                    const int64_t p = cur[vt[i]]++;
                    pdoc[p] = d;
                    pval[p] = (uint8_t)std::min(q, 255);
                }
            }
            std::vector<uint32_t>().swap(c_term[(size_t)c]);
            std::vector<float>().swap(c_imp[(size_t)c]);
        }
        // 5. per term: stable sort by value descending (doc ascending inside a value)
        parallel_for(v_terms, [&](int64_t lo, int64_t hi, int) {
            std::vector<uint32_t> d2;
            std::vector<uint8_t> v2;
            for (int64_t t = lo; t < hi; ++t) {
                const int64_t a = term_off[t], b = term_off[t + 1], n = b - a;
                if (n < 2) continue;
                int64_t cnt[256] = {0};
                for (int64_t p = a; p < b; ++p) cnt[255 - pval[p]]++;
                int64_t run = 0;
                for (int i = 0; i < 256; ++i) {
                    const int64_t c = cnt[i];
                    cnt[i] = run;
                    run += c;
                }
                d2.resize((size_t)n);
                v2.resize((size_t)n);
                for (int64_t p = a; p < b; ++p) {
                    const int64_t o = cnt[255 - pval[p]]++;
                    d2[(size_t)o] = pdoc[p];
                    v2[(size_t)o] = pval[p];
                }
                std::memcpy(pdoc + a, d2.data(), (size_t)n * 4);
                std::memcpy(pval + a, v2.data(), (size_t)n);
            }
        });
    });
}
