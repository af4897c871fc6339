/*
 * oracle.c -- CPU restatement of the reference DeeperImpact hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product path (libdeepimpact_hip.so) never
 * links, loads or calls anything under oracle/.
 *
 * Every function restates one reference function; the citation is
 * path:line relative to the reference repository root.  Parity of this
 * restatement is pinned by tests/test_oracle_golden.py against fixtures
 * produced by running the reference's own Python here
 * (tests/golden/make_golden.py).
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------
 * A9: `round(impact, 3)` on a numpy float32
 *     src/deep_impact/indexing/indexer.py:132
 * numpy rounds a float32 as fl32(rint(fl32(x * 1000)) / 1000); the text is
 * then repr(float(y)) (done by the Python side of the oracle).
 * ---------------------------------------------------------------------- */
OR_API void or_round3(const float *x, int64_t n, float *y) {
    for (int64_t i = 0; i < n; ++i) {
        volatile float t = x[i] * 1000.0f; /* one f32 rounding, no FMA */
        float r = rintf(t);
        y[i] = r / 1000.0f;
    }
}

/* ------------------------------------------------------------------------
 * A10: quantize
 *     src/deep_impact/indexing/quantize.py:13-14  quantize = int(value*scale)
 *     src/deep_impact/indexing/quantize.py:17-24  find_max_value (starts at 0)
 *     src/deep_impact/indexing/quantize.py:37     scale = 255 / max_val (fp64)
 * values: the parsed fp64 impacts; out: int(v*scale) (truncation toward 0).
 * max_val <= 0 or NaN means "not given": compute it as the reference does.
 * Returns the max actually used through *max_used.
 * ---------------------------------------------------------------------- */
OR_API void or_quantize(const double *v, int64_t n, double max_val, int bits,
                        int64_t *out, double *max_used) {
    double m = max_val;
    if (!(m > 0.0)) {
        m = 0.0;
        for (int64_t i = 0; i < n; ++i)
            if (v[i] > m) m = v[i];
    }
    double scale = (double)((1 << bits) - 1) / m;
    for (int64_t i = 0; i < n; ++i) {
        double p = v[i] * scale;
        out[i] = (int64_t)p; /* C cast truncates toward zero, as Python int() */
    }
    *max_used = m;
}

/* ------------------------------------------------------------------------
 * A11: posting lists of the on-disk index
 *     src/deep_impact/inverted_index/create.py:31-51
 * Docs are visited in line order; per term the postings are stable-sorted by
 * value descending, so equal values keep doc-id ascending order.
 * Inputs: CSR over docs (cu[n_docs+1]) of (term id into the sorted vocab,
 * int value).  Output: term_off[n_terms+1] (posting index, not bytes),
 * pdoc[], pval[] in file order.
 * ---------------------------------------------------------------------- */
OR_API int or_build_postings(int64_t n_docs, const int64_t *cu, const uint32_t *term,
                             const int64_t *val, uint32_t n_terms, int64_t *term_off,
                             uint32_t *pdoc, int64_t *pval) {
    int64_t n = cu[n_docs];
    int64_t *cnt = (int64_t *)calloc((size_t)n_terms + 1, sizeof(int64_t));
    if (!cnt) return -1;
    for (int64_t i = 0; i < n; ++i) cnt[term[i] + 1]++;
    for (uint32_t t = 0; t < n_terms; ++t) cnt[t + 1] += cnt[t];
    memcpy(term_off, cnt, ((size_t)n_terms + 1) * sizeof(int64_t));
    /* bucket postings by term in doc order */
    uint32_t *tmp_doc = (uint32_t *)malloc((size_t)(n ? n : 1) * sizeof(uint32_t));
    int64_t *tmp_val = (int64_t *)malloc((size_t)(n ? n : 1) * sizeof(int64_t));
    if (!tmp_doc || !tmp_val) { free(cnt); free(tmp_doc); free(tmp_val); return -1; }
    for (int64_t d = 0; d < n_docs; ++d)
        for (int64_t i = cu[d]; i < cu[d + 1]; ++i) {
            int64_t p = cnt[term[i]]++;
            tmp_doc[p] = (uint32_t)d;
            tmp_val[p] = val[i];
        }
    /* stable sort each term by value descending (insertion sort on runs is
     * too slow for long lists; use a merge sort per term) */
    for (uint32_t t = 0; t < n_terms; ++t) {
        int64_t a = term_off[t], b = term_off[t + 1], len = b - a;
        /* bottom-up stable merge sort into pdoc/pval */
        uint32_t *sd = tmp_doc + a; int64_t *sv = tmp_val + a;
        uint32_t *dd = pdoc + a;    int64_t *dv = pval + a;
        for (int64_t w = 1; w < len; w *= 2) {
            for (int64_t lo = 0; lo < len; lo += 2 * w) {
                int64_t mid = lo + w < len ? lo + w : len;
                int64_t hi = lo + 2 * w < len ? lo + 2 * w : len;
                int64_t i = lo, j = mid, o = lo;
                while (i < mid && j < hi) {
                    if (sv[j] > sv[i]) { dd[o] = sd[j]; dv[o++] = sv[j++]; }
                    else { dd[o] = sd[i]; dv[o++] = sv[i++]; }
                }
                while (i < mid) { dd[o] = sd[i]; dv[o++] = sv[i++]; }
                while (j < hi) { dd[o] = sd[j]; dv[o++] = sv[j++]; }
            }
            uint32_t *x = sd; sd = dd; dd = x;
            int64_t *y = sv; sv = dv; dv = y;
        }
        if (sd != pdoc + a) {
            memcpy(pdoc + a, sd, (size_t)len * sizeof(uint32_t));
            memcpy(pval + a, sv, (size_t)len * sizeof(int64_t));
        }
    }
    free(cnt); free(tmp_doc); free(tmp_val);
    return 0;
}

/* ------------------------------------------------------------------------
 * A12: InvertedIndex.score(query_terms, top_k)
 *     src/deep_impact/inverted_index/inverted_index.py:31-53 term_docs
 *       (reads (doc,val) records until `end`, stops at the first val == 0)
 *     src/deep_impact/inverted_index/inverted_index.py:55-62 score
 *       scores[doc] = scores.get(doc, 0) + val   -- dict, insertion order
 *       heapq.nlargest(top_k, items, key=score)  -- stable: ties keep
 *                                                    first-touch order
 * Query terms are given in iteration order (the reference iterates a set);
 * unknown terms are simply absent from q_terms.
 * Outputs: out_doc/out_score [n_q * k], out_n[n_q].
 * ---------------------------------------------------------------------- */
typedef struct {
    uint32_t *acc;
    uint32_t *touched;
} or_ws;

static void score_one(const int64_t *term_off, const uint32_t *pdoc, const uint8_t *pval,
                      const uint32_t *qt, int nt, int k, uint32_t *acc, uint32_t *touched,
                      uint32_t *ftk, uint32_t *od, uint32_t *os, int32_t *on, uint64_t *ok) {
    int64_t nt_touch = 0;
    uint32_t max_score = 0;
    for (int j = 0; j < nt; ++j) {
        uint32_t t = qt[j];
        for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
            uint32_t v = pval[p];
            if (v == 0) break; /* inverted_index.py:50-51 */
            uint32_t d = pdoc[p];
            if (acc[d] == 0) {
                touched[nt_touch++] = d;
                /* first touch: term index j and its value there (list order) */
                ftk[d] = ((uint32_t)j << 8) | v;
            }
            acc[d] += v;
            if (acc[d] > max_score) max_score = acc[d];
        }
    }
    /* stable descending selection: counting sort on score keeps first-touch
     * order inside a score, exactly as the stable nlargest does */
    int64_t *hist = (int64_t *)calloc((size_t)max_score + 2, sizeof(int64_t));
    for (int64_t i = 0; i < nt_touch; ++i) hist[acc[touched[i]]]++;
    /* start offset per score in descending order */
    int64_t run = 0;
    for (int64_t s = (int64_t)max_score; s >= 1; --s) {
        int64_t c = hist[s];
        hist[s] = run;
        run += c;
    }
    int kk = (int)(nt_touch < k ? nt_touch : k);
    for (int64_t i = 0; i < nt_touch; ++i) {
        uint32_t d = touched[i];
        int64_t pos = hist[acc[d]]++;
        if (pos < kk) {
            od[pos] = d;
            os[pos] = acc[d];
            /* the shard-merge key of the HIP path (include/deepimpact.h di_key_*):
             * compact up to 256 query terms, wide beyond */
            const uint64_t j = ftk[d] >> 8, v = ftk[d] & 255u;
            if (ok && nt <= 256)
                ok[pos] = ((uint64_t)acc[d] << 48) | ((255 - j) << 40) | (v << 32) |
                          (uint64_t)(0xFFFFFFFFu - d);
            else if (ok)
                ok[pos] = ((uint64_t)acc[d] << 44) | ((4095 - j) << 32) | (v << 24) |
                          (uint64_t)(0xFFFFFFu - d);
        }
    }
    *on = kk;
    for (int64_t i = 0; i < nt_touch; ++i) acc[touched[i]] = 0;
    free(hist);
}

OR_API int or_score(const int64_t *term_off, const uint32_t *pdoc, const uint8_t *pval,
                    uint32_t n_docs, const uint32_t *q_terms, const int32_t *cu_q, int n_q,
                    int k, uint32_t *out_doc, uint32_t *out_score, int32_t *out_n,
                    uint64_t *out_key, int n_threads) {
    if (n_threads < 1) n_threads = 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(n_threads)
#endif
    {
        uint32_t *acc = (uint32_t *)calloc((size_t)n_docs + 1, sizeof(uint32_t));
        uint32_t *touched = (uint32_t *)malloc(((size_t)n_docs + 1) * sizeof(uint32_t));
        uint32_t *ftk = (uint32_t *)malloc(((size_t)n_docs + 1) * sizeof(uint32_t));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int q = 0; q < n_q; ++q)
            score_one(term_off, pdoc, pval, q_terms + cu_q[q], cu_q[q + 1] - cu_q[q], k, acc,
                      touched, ftk, out_doc + (int64_t)q * k, out_score + (int64_t)q * k,
                      out_n + q, out_key ? out_key + (int64_t)q * k : NULL);
        free(acc);
        free(touched);
        free(ftk);
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * A14/A15: SparseSearch (in-memory float index)
 *     src/deep_impact/evaluation/nano_beir_evaluator.py:78-101 build:
 *       postings appended in corpus order, only `score > 0`
 *     src/deep_impact/evaluation/nano_beir_evaluator.py:113-133 search:
 *       doc_scores = defaultdict(float); += impact, terms in set order;
 *       numpy>=2: 0.0 + np.float32 -> float32 accumulation (use_f64=0);
 *       numpy 1.25 (pinned): float64 accumulation (use_f64=1);
 *       top-k = stable sort by score desc (sorted() or heapq.nlargest).
 * Postings arrive already filtered and in corpus order (CSR by term).
 * out_score is double for both modes (f32 results are exact in double).
 * ---------------------------------------------------------------------- */
typedef struct {
    double s;
    int64_t order;
    uint32_t doc;
} or_fitem;

static int cmp_fitem(const void *a, const void *b) {
    const or_fitem *x = (const or_fitem *)a, *y = (const or_fitem *)b;
    if (x->s > y->s) return -1;
    if (x->s < y->s) return 1;
    return (x->order < y->order) ? -1 : (x->order > y->order);
}

OR_API int or_sparse_search(const int64_t *term_off, const uint32_t *pdoc, const float *pimp,
                            uint32_t n_docs, const uint32_t *q_terms, const int32_t *cu_q,
                            int n_q, int k, int use_f64, uint32_t *out_doc, double *out_score,
                            int32_t *out_n) {
    float *acc32 = (float *)calloc((size_t)n_docs + 1, sizeof(float));
    double *acc64 = (double *)calloc((size_t)n_docs + 1, sizeof(double));
    uint8_t *seen = (uint8_t *)calloc((size_t)n_docs + 1, 1);
    uint32_t *touched = (uint32_t *)malloc(((size_t)n_docs + 1) * sizeof(uint32_t));
    or_fitem *items = (or_fitem *)malloc(((size_t)n_docs + 1) * sizeof(or_fitem));
    for (int q = 0; q < n_q; ++q) {
        int64_t nt_touch = 0;
        for (int j = cu_q[q]; j < cu_q[q + 1]; ++j) {
            uint32_t t = q_terms[j];
            for (int64_t p = term_off[t]; p < term_off[t + 1]; ++p) {
                uint32_t d = pdoc[p];
                if (!seen[d]) { seen[d] = 1; touched[nt_touch++] = d; }
                if (use_f64) acc64[d] = acc64[d] + (double)pimp[p];
                else acc32[d] = acc32[d] + pimp[p];
            }
        }
        for (int64_t i = 0; i < nt_touch; ++i) {
            uint32_t d = touched[i];
            items[i].s = use_f64 ? acc64[d] : (double)acc32[d];
            items[i].order = i;
            items[i].doc = d;
            acc32[d] = 0.0f; acc64[d] = 0.0; seen[d] = 0;
        }
        qsort(items, (size_t)nt_touch, sizeof(or_fitem), cmp_fitem);
        int kk = (int)(nt_touch < k ? nt_touch : k);
        for (int i = 0; i < kk; ++i) {
            out_doc[(int64_t)q * k + i] = items[i].doc;
            out_score[(int64_t)q * k + i] = items[i].s;
        }
        out_n[q] = kk;
    }
    free(acc32); free(acc64); free(seen); free(touched); free(items);
    return 0;
}
