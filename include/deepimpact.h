/*
 * deepimpact.h -- C ABI of libdeepimpact_hip.so, the MI355X-native (gfx950)
 * DeeperImpact encode-and-retrieve path.
 *
 * The reference (Tommachilez/improving-learned-index) has no FFI layer: its
 * boundary is a set of Python protocols and file formats.  Each
 * entry point below names the reference interface it replaces (path:line,
 * relative to the reference repository root).  The Python host side
 * (improving-learned-index_amd/) binds these through ctypes; INTEGRATION.md
 * shows the binding a maintainer would add to the reference itself.
 *
 * Conventions
 *   - Every function returns DI_OK (0) or a negative DI_E* code; the message of
 *     the last failure on the calling thread is di_last_error().  No C++
 *     exception crosses the ABI.
 *   - Array arguments are borrowed for the duration of the call.  Unless the
 *     DI_F_DEVICE_PTRS flag is given they are host pointers; with it they are
 *     device pointers on the handle's device (inputs already resident in HBM).
 *   - Outputs are caller-allocated; their sizes are known before the call.
 *   - One handle per device.  A handle is not thread-safe; different handles
 *     may be used concurrently.  Each handle owns one HIP stream (replaceable
 *     with di_*_set_stream); calls are synchronous at return unless
 *     DI_F_ASYNC is given together with DI_F_DEVICE_PTRS.
 */
#ifndef DEEPIMPACT_H
#define DEEPIMPACT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DI_OK 0
#define DI_EINVAL (-1)   /* bad argument                                   */
#define DI_ENOMEM (-2)   /* host or device allocation failed                */
#define DI_EHIP (-3)     /* HIP runtime error                               */
#define DI_ERANGE (-4)   /* a documented size limit was exceeded            */
#define DI_ENODEV (-5)   /* no HIP device                                   */
#define DI_EIO (-6)      /* file could not be read                          */
#define DI_EFORMAT (-7)  /* file content does not follow the reference format */

#define DI_F_DEVICE_PTRS 0x1u /* array arguments are device pointers           */
#define DI_F_ASYNC 0x2u       /* do not synchronise the stream before return   */
#define DI_F_TIMING 0x4u      /* record HIP events around every kernel         */
#define DI_F_LISTS_MAJOR 0x8u /* di_topk_merge: keys are [list][query][k]       */

/* Limits of the retrieval kernels (documented in DESIGN.md). */
#define DI_SHORT_QUERY_TERMS 256 /* queries up to this many known terms use the compact key */
#define DI_MAX_QUERY_TERMS 4096  /* known terms per query of the quantized scorer; longer
                                    than DI_SHORT_QUERY_TERMS: wide keys, shard docs < 2^24 */
#define DI_MAX_TOPK 4096
#define DI_MAX_SPARSE_QUERY_TERMS 4096 /* float search: known terms per query (chunked) */
#define DI_MAX_SPARSE_DOCS 16777215u /* float index: doc ids embedded in 24 bits   */

const char *di_last_error(void);
int di_version(void); /* (major << 16) | minor */
int di_device_count(int *n);

/* Per-kernel timing collected under DI_F_TIMING (HIP events on the launching
 * stream).  `name` is the kernel's short name, e.g. "score_blocks".  Returns the
 * summed milliseconds and the number of launches since the last reset. */
typedef struct di_timing {
    double ms;
    int64_t launches;
} di_timing;

/* ======================================================================
 * On-disk quantized index: build and score                  (A11, A12)
 * ====================================================================== */
typedef struct di_index di_index;

/* Replaces InvertedIndexCreator (src/deep_impact/inverted_index/create.py:12-55)
 * as the producer of the device index, and InvertedIndex.__init__
 * (src/deep_impact/inverted_index/inverted_index.py:18-20).
 * Input: postings in the reference file order -- term-major, value descending,
 * doc ascending -- as CSR: term_off[n_terms+1] (posting index), pdoc[], pval[].
 * Postings from the first zero value of a term on are dropped, exactly as
 * InvertedIndex.term_docs stops there (inverted_index.py:50-51).
 * Only docs in [doc_lo, doc_hi) are kept (one shard of a doc-id-sharded index);
 * doc ids stay global.  doc_hi = 0 means "max doc + 1".                        */
int di_index_create(const int64_t *term_off, int64_t n_terms, const uint32_t *pdoc,
                    const uint8_t *pval, uint32_t doc_lo, uint32_t doc_hi, int device,
                    di_index **out);

/* Native host builder of the reference files: replaces InvertedIndexCreator.run
 * (create.py:53-55) reading the collection like DeepImpactCollection
 * (src/deep_impact/indexing/deep_impact_collection.py:6-33).  Writes
 * <out_dir>/vocab.txt, inverted_index.idx, inverted_index.dat byte-identical to
 * the reference.  Malformed lines fail with DI_EFORMAT where the reference raises. */
int di_build_reference_index(const char *collection_path, const char *out_dir);

/* Reads <dir>/inverted_index.idx and <dir>/inverted_index.dat (create.py:45-51,
 * formats src/utils/defaults.py:22-37).  vocab.txt stays on the host side. */
int di_index_load_reference(const char *dir, uint32_t doc_lo, uint32_t doc_hi, int device,
                            di_index **out);

/* Replaces InvertedIndex.score (inverted_index.py:55-62) for a batch of queries.
 * q_terms: term ids of all queries in iteration order (the reference iterates a
 * Python set; its order is the tie order), CSR by cu_q[n_q+1].  For each query
 * the top-k (doc, score) pairs are written in the reference's order -- score
 * descending, ties in first-touch order -- to out_doc/out_score[q*k ...] and the
 * count to out_n[q].  out_key (may be NULL) receives the 64-bit merge keys used
 * to combine shards (di_topk_merge; wide keys for queries of more than
 * DI_SHORT_QUERY_TERMS terms, see di_key_doc_wide).  A query over a kernel limit
 * (more than DI_MAX_QUERY_TERMS terms; a long query on a shard reaching doc 2^24;
 * an unknown term id) fails the call with DI_ERANGE / DI_EINVAL for host pointers,
 * and gets out_n[q] = -1 with DI_F_DEVICE_PTRS (the caller must check).          */
int di_index_search(di_index *ix, const uint32_t *q_terms, const int32_t *cu_q, int32_t n_q,
                    int32_t k, uint32_t *out_doc, uint32_t *out_score, int32_t *out_n,
                    uint64_t *out_key, uint32_t flags);

/* Pre-allocates device workspace for batches of up to max_q queries at top-k. */
int di_index_reserve(di_index *ix, int32_t max_q, int32_t k);
int di_index_info(const di_index *ix, int64_t *n_terms, int64_t *n_postings, uint32_t *n_docs,
                  int32_t *n_blocks);
/* Query-time impact pruning (BASELINE configs[4], the QPS-vs-recall@1000 sweep): score
 * only the postings with value >= 2^floor(log2 min_impact) -- a prefix of every
 * (term, block) sublist, which the index keeps grouped by impact class.  1 (the
 * default) scores every posting: exactly InvertedIndex.score (inverted_index.py:55-62);
 * anything larger is an approximation whose recall bench tools measure.  No reference
 * counterpart (the reference scores exhaustively).                                  */
int di_index_set_min_impact(di_index *ix, int32_t min_impact);
/* Block-max skipping (BASELINE configs[4]): per (term, block) and per (long sublist, wave
 * segment of 2048 docs) the largest value is kept at build time; a segment whose bound
 * (the sum over the query terms of those maxima) stays below the query's running top-k
 * threshold is not scored.  factor 0: off (default); 1: exact -- the same ranking as
 * InvertedIndex.score (inverted_index.py:55-62); in (1, 16]: skips segments below
 * factor x threshold, an approximation (QPS vs recall@1000).  Queries of at most 64
 * terms, with the shared threshold (>= 8 blocks).  Long sublists: >= 128 postings in a
 * block.  di_index_timing("bm_segments" / "bm_segments_skipped") counts the evaluated
 * and skipped segments.  Items run block-major; DI_BLOCK_ORDER=1 (environment, at index
 * creation) runs each query's blocks in descending bound order instead. */
int di_index_set_block_max(di_index *ix, float factor);
/* Packed (block-compressed) postings -- BASELINE configs[4]: on != 0 builds (once, from
 * the device layout) a second copy of the postings in which every run (a short
 * (term, block) sublist, or one scorer wave segment's run of a long one) is sorted by doc
 * and cut into frames of up to 512 postings, each bit-packed with its own widths (doc
 * deltas in bd bits, value - vmin in bv bits, decoded in registers by the scorer), and
 * scores queries of at most 64 terms from it, alone or with block-max skipping; the
 * ranking is unchanged (same keys).  Exact scoring only: with impact pruning
 * (di_index_set_min_impact > 1) the plain layout is used.  *packed_bytes (optional)
 * receives the packed size (headers + data).  on = 0: the plain layout again. */
int di_index_set_packed(di_index *ix, int32_t on, int64_t *packed_bytes);
int di_index_set_stream(di_index *ix, void *hip_stream);
int di_index_sync(di_index *ix);
/* Per-kernel HIP-event time ("score_blocks", "merge_topk") accumulated over DI_F_TIMING
 * searches; also the block-max counters "bm_segments" (wave segments evaluated) and
 * "bm_segments_skipped" (segments not scored), returned in out->launches (ms = 0),
 * accumulated since the last reset (reading them synchronises the stream). */
int di_index_timing(di_index *ix, const char *name, di_timing *out, int reset);
int di_index_destroy(di_index *ix);

/* Combine per-shard top-k lists (from di_index_search out_key, or the sparse
 * index) into the global top-k: keys[(q*n_lists + l)*k + i], counts[q*n_lists+l]
 * (with DI_F_LISTS_MAJOR: keys[(l*n_q + q)*k + i], counts[l*n_q + q] -- the layout
 * an all-gather of per-shard results produces).
 * The keys are unique and totally ordered, so the result equals a single-shard
 * search over the whole collection.  Device pointers when DI_F_DEVICE_PTRS.
 * Replaces nothing in the reference (it has no sharded retrieval). */
int di_topk_merge(const uint64_t *keys, const int32_t *counts, int32_t n_q, int32_t n_lists,
                  int32_t k, uint64_t *out_key, int32_t *out_n, int device, void *hip_stream,
                  uint32_t flags);

/* The local steps of the pruned exact exchange of per-shard top-k lists between ranks
 * (parallel.exchange_topk; the collectives between them are the caller's all_gathers).
 * keys [n_q][k] descending merge keys (> 0), counts [n_q] (negative: rejected query).
 * Device pointers only, asynchronous on hip_stream.  Replaces nothing in the reference
 * (it has no sharded retrieval); the result feeds di_topk_merge, whose
 * output equals the merge of the full lists (ranker.py:43-48 keeps the global top-k).
 *   sample:  samples [n_q][k/g] = keys at positions g-1, 2g-1, ... (0 past counts[q]);
 *   count:   gathered_samples [world][n_q][k/g] -> T_q = the ceil(k/g)-th largest
 *            sample, ec [2][n_q] = (this rank's keys >= T_q, counts);
 *   offsets: gathered_ec [world][2][n_q] -> offsets [world][n_q] (exclusive scans of the
 *            key counts), totals [world];
 *   pack:    ec / offsets of this rank -> buf (its keys >= T_q back to back);
 *   unpack:  gathered [world][emax] -> out_keys [world][n_q][k], out_n [world][n_q]
 *            (the layout of a plain all_gather; DI_F_LISTS_MAJOR for di_topk_merge). */
int di_xchg_sample(const uint64_t *keys, const int32_t *counts, int32_t n_q, int32_t k,
                   int32_t g, uint64_t *samples, int device, void *hip_stream);
int di_xchg_count(const uint64_t *gathered_samples, int32_t world, const uint64_t *keys,
                  const int32_t *counts, int32_t n_q, int32_t k, int32_t g, int32_t *ec,
                  int device, void *hip_stream);
int di_xchg_offsets(const int32_t *gathered_ec, int32_t world, int32_t n_q, int64_t *offsets,
                    int64_t *totals, int device, void *hip_stream);
int di_xchg_pack(const uint64_t *keys, const int32_t *ec, const int64_t *offsets, int32_t n_q,
                 int32_t k, uint64_t *buf, int device, void *hip_stream);
int di_xchg_unpack(const uint64_t *gathered, int64_t emax, const int32_t *gathered_ec,
                   const int64_t *offsets, int32_t world, int32_t n_q, int32_t k,
                   uint64_t *out_keys, int32_t *out_n, int device, void *hip_stream);

/* ======================================================================
 * In-memory float index of the NanoBEIR evaluator           (A14, A15)
 * ====================================================================== */
typedef struct di_sparse di_sparse;

/* Replaces SparseSearch._build_inverted_index (nano_beir_evaluator.py:78-101):
 * per term, postings (doc = corpus position, float32 impact) in corpus order;
 * impacts <= 0 are dropped (:98).  n_docs <= DI_MAX_SPARSE_DOCS. */
int di_sparse_create(const int64_t *term_off, int64_t n_terms, const uint32_t *pdoc,
                     const float *pimp, uint32_t n_docs, int device, di_sparse **out);

/* Replaces SparseSearch.search's scoring (nano_beir_evaluator.py:113-133):
 * float32 sums formed in the reference's order (bit-exact under numpy >= 2),
 * top-k by score with ties in first-touch order.  out_key: merge keys
 * (score bits << 32 | (255 - first term) << 24 | (0xFFFFFF - doc)). */
int di_sparse_search(di_sparse *sp, const uint32_t *q_terms, const int32_t *cu_q, int32_t n_q,
                     int32_t k, uint32_t *out_doc, float *out_score, int32_t *out_n,
                     uint64_t *out_key, uint32_t flags);
/* The same search with float64 accumulation: the reference's pinned numpy 1.25.1,
 * where `0.0 + np.float32` is an np.float64 (nano_beir_evaluator.py:113-121, SURVEY
 * App. B.4).  f64 sums formed in the reference's order, top-k by f64 score with
 * ties in first-touch order; out_score: the f64 scores (the reference's float()). */
int di_sparse_search_f64(di_sparse *sp, const uint32_t *q_terms, const int32_t *cu_q,
                         int32_t n_q, int32_t k, uint32_t *out_doc, double *out_score,
                         int32_t *out_n, uint32_t flags);
int di_sparse_info(const di_sparse *sp, int64_t *n_terms, int64_t *n_postings, uint32_t *n_docs,
                   int32_t *n_blocks);
int di_sparse_timing(di_sparse *sp, const char *name, di_timing *out, int reset);
int di_sparse_destroy(di_sparse *sp);

/* ======================================================================
 * Encoder: DeepImpact forward + first-occurrence gather     (A2, A5-A9)
 * ====================================================================== */
typedef struct di_encoder di_encoder;

#define DI_VARIANT_XLMR 0 /* RoBERTa / XLM-R: positions pad_id+1+i (xlmr_original.py) */
#define DI_VARIANT_BERT 1 /* BERT / CoCondenser: absolute positions (soyuj/deeper-impact) */
#define DI_ACT_SOFTPLUS 0 /* nn.Softplus() head (xlmr_original.py:34-38)               */
#define DI_ACT_RELU 1     /* nn.ReLU() head (original.py:44-47)                        */
#define DI_PREC_BF16 0    /* bf16 MFMA, f32 accumulate/softmax/LayerNorm (fast)        */
#define DI_PREC_FP32 1    /* f32 MFMA throughout (parity with the f32 reference)       */
#define DI_PREC_BF16X3 2  /* fp32-faithful fast mode: split-bf16 GEMMs (3 bf16 MFMA
                             products per f32 product, f32 accumulate), f32 attention
                             and LayerNorm; hidden 768 / 1024                           */
#define DI_DTYPE_F32 0
#define DI_DTYPE_BF16 1

#define DI_F_ROUND3 0x10u        /* di_encode: apply round(impact, 3) (indexer.py:132)  */
#define DI_F_TOKEN_IMPACTS 0x20u /* di_encode: write per-token impacts [n_tokens]       */

typedef struct di_encoder_cfg {
    int32_t variant, activation, precision;
    int32_t vocab_size, hidden, layers, heads, intermediate, max_positions, type_vocab, pad_id;
    float layer_norm_eps;
} di_encoder_cfg;

/* One checkpoint tensor: the reference's state-dict key (ModelCheckpoint layout,
 * src/utils/checkpoint.py:72-77: "bert.embeddings...", "bert.encoder.layer.N...",
 * "impact_score_encoder.0.weight"), host data, row-major. */
typedef struct di_tensor {
    const char *name;
    const void *data;
    int32_t dtype; /* DI_DTYPE_* */
    int32_t ndim;
    int64_t shape[4];
} di_tensor;

/* Replaces DeepImpact.load + .to(cuda).eval() (xlmr_original.py:191-203,
 * indexer.py:22-24).  Strict like load_state_dict (checkpoint.py:117): a missing
 * or unexpected key is DI_EINVAL; "embeddings.position_ids" and "pooler.*" are
 * ignored.  Head dim must be 64; hidden <= 1024. */
int di_encoder_create(const di_encoder_cfg *cfg, const di_tensor *weights, int32_t n_weights,
                      int device, di_encoder **out);

/* Replaces DeepImpact.forward (xlmr_original.py:41-85) + compute_term_impacts
 * (:205-225) [+ round(.,3) of indexer.py:132 with DI_F_ROUND3] for a batch.
 * tok_ids: the documents' token ids packed without padding, CSR by
 * cu_seqlens[n_docs+1] (each doc = what the tokenizer emitted incl. <s>/</s>).
 * term_tok[cu_terms[d] .. cu_terms[d+1]): token index (within doc d) of the
 * first token of each kept term, in term order.  out[cu_terms[d] + i] = impact.
 * With DI_F_TOKEN_IMPACTS out[n_tokens] = impact of every token (no gather).
 * n_tokens/max_len/n_terms are required with DI_F_DEVICE_PTRS (no host read of
 * device arrays) and recomputed from the arrays otherwise. */
int di_encode(di_encoder *enc, const int32_t *tok_ids, const int32_t *cu_seqlens, int32_t n_docs,
              int64_t n_tokens, int32_t max_len, const int32_t *term_tok, const int32_t *cu_terms,
              int64_t n_terms, float *out, uint32_t flags);
int di_encoder_reserve(di_encoder *enc, int64_t max_tokens, int32_t max_docs, int64_t max_terms);
int di_encoder_set_stream(di_encoder *enc, void *hip_stream);
int di_encoder_sync(di_encoder *enc);
int di_encoder_timing(di_encoder *enc, const char *name, di_timing *out, int reset);
int di_encoder_destroy(di_encoder *enc);

/* ======================================================================
 * 8-bit quantizer                                          (A10)
 * ====================================================================== */
/* Replaces quantize_file's arithmetic (src/deep_impact/indexing/quantize.py:13-47):
 * max_val <= 0 means "compute max(0, impacts)"; scale = (2^bits-1)/max_val in
 * fp64; out[i] = int(impacts[i] * scale) (truncation).  impacts are the values
 * the impact TSV holds (3-decimal float32).  *max_used receives the max. */
int di_quantize(const float *impacts, int64_t n, double max_val, int32_t bits, int32_t *out,
                double *max_used, int device, void *hip_stream, uint32_t flags);

/* quantize_file (quantize.py:27-47) end to end: parse the impact TSV exactly as
 * the reference (line.strip().split(', '), t.strip().split(': '), float()),
 * quantize on the GPU in fp64, write the quantized TSV.  Empty / malformed
 * lines fail with DI_EFORMAT where the reference raises ValueError.
 * output_path NULL: only *max_used = the file's max impact (find_max_value,
 * quantize.py:17-24) -- the doc-sharded quantizer all-reduces it (MAX) across ranks. */
int di_quantize_file(const char *input_path, const char *output_path, double max_val,
                     int32_t bits, int device, double *max_used);

/* ======================================================================
 * Impact TSV text                                          (A9)
 * ====================================================================== */
/* Replaces the formatting loop of Indexer.index (indexer.py:62-68): for each doc
 * the terms (UTF-8, terms + term_off[i]..term_off[i+1]) and impacts (already
 * rounded, DI_F_ROUND3) become ', '.join(f'{term}: {impact}') + '\n', numbers
 * printed as Python's repr of the float64 value.  Writes *out_len bytes; returns
 * DI_ERANGE (with *out_len = bytes needed) if out_cap is too small. */
int di_format_impact_lines(const char *terms, const int64_t *term_off, const float *impacts,
                           const int64_t *cu_doc_terms, int32_t n_docs, char *out,
                           int64_t out_cap, int64_t *out_len);

/* Replaces RunFile.writelines (src/utils/datasets.py:305-324) over a batch: appends
 * to `path`, for each query q (its id qids[qid_off[q] .. qid_off[q+1]), UTF-8) and rank
 * i < counts[q], "qid\tpid\trank\tscore\n" with pid = docs[q*k + i], rank = i + 1,
 * score = scores[q*k + i] (integers: the quantized index). */
int di_append_run_lines(const char *path, const char *qids, const int64_t *qid_off,
                        int32_t n_q, const uint32_t *docs, const uint32_t *scores,
                        const int32_t *counts, int32_t k);

/* ======================================================================
 * Bench / test data (not a reference interface)
 * ====================================================================== */
/* Seeded MS MARCO-shaped quantized collection (SURVEY §8d generator: per doc the
 * first max_terms unique values of `draws` draws of min(zipf(zipf_a), v_terms),
 * impacts float32(softplus(N(-0.5, 1.5))), round3 + fp64 8-bit quantize, zeros
 * dropped), returned as reference-order postings (term_off[v_terms + 1], then per
 * term value desc / doc asc, create.py:41).  pdoc / pval may be null (sizes only);
 * else cap >= *n_post.  Host threads: DI_HOST_THREADS or OMP_NUM_THREADS. */
int di_synth_postings(int64_t n_docs, int32_t v_terms, uint64_t seed, int32_t max_terms,
                      int32_t draws, double zipf_a, int64_t *term_off, uint32_t *pdoc,
                      uint8_t *pval, int64_t cap, int64_t *n_post, double *max_impact);

/* Skew of a synthetic collection's impacts -- a documented deviation from SURVEY §8d's
 * i.i.d. impacts, for block-max skipping (BASELINE configs[4]): impact =
 * softplus(N(-0.5, 1.5)) x min(1, ((t + 1) / term_rank0)^term_exp) (t = the term's
 * 0-based zipf rank: frequent terms carry small impacts; term_rank0 0 = off) x the doc's
 * mass min(mass_max, exp(cluster_sigma z_c + doc_sigma z_d)) (z_c shared by the
 * cluster_docs consecutive doc ids of a cluster, z_d per doc; mass_max 0 = no clip). */
typedef struct di_synth_skew {
    double term_rank0;
    double term_exp;
    int32_t cluster_docs;
    double cluster_sigma;
    double doc_sigma;
    double mass_max;
} di_synth_skew;

/* di_synth_postings with skewed impacts (skew null: exactly di_synth_postings). */
int di_synth_postings_skewed(int64_t n_docs, int32_t v_terms, uint64_t seed, int32_t max_terms,
                             int32_t draws, double zipf_a, const di_synth_skew *skew,
                             int64_t *term_off, uint32_t *pdoc, uint8_t *pval, int64_t cap,
                             int64_t *n_post, double *max_impact);

/* Docs [doc0, doc0 + n_docs) of the seeded collection di_synth_postings_skewed generates
 * for seed (each doc depends only on (seed, doc id)): one doc-id shard of it, doc ids
 * local (0-based).  quant_max > 0 quantizes with that max (the collection's: the
 * all_reduce(MAX) of the shards' maxima, as the sharded quantize CLI does) instead of the
 * shard's own; term_off null: only *max_impact (the shard's max) is computed.  Bench and
 * test input of the multi-rank retrieve legs. */
int di_synth_postings_shard(int64_t doc0, int64_t n_docs, int32_t v_terms, uint64_t seed,
                            int32_t max_terms, int32_t draws, double zipf_a,
                            const di_synth_skew *skew, double quant_max, int64_t *term_off,
                            uint32_t *pdoc, uint8_t *pval, int64_t cap, int64_t *n_post,
                            double *max_impact);

/* The same seeded collection as the impact TSV of the index CLI (indexer.py:62-68),
 * term id t spelled "\u2581t<t>": bench input of the quantize / index-create legs.
 * *n_terms receives the (doc, term) pairs written. */
int di_synth_impact_tsv(const char *path, int64_t n_docs, int32_t v_terms, uint64_t seed,
                        int32_t max_terms, int32_t draws, double zipf_a, int64_t *n_terms);

/* Decoding of a quantized-index merge key.  A query of at most DI_SHORT_QUERY_TERMS
 * known terms: score(16) | (255 - first term)(8) | its value(8) | ~doc(32).  A longer
 * one (wide key): score(20) | (4095 - first term)(12) | its value(8) | (0xFFFFFF - doc)(24).
 * Within one query every key has the same form and keys order exactly like the
 * reference ranking (score desc, then first touch). */
static inline uint32_t di_key_doc(uint64_t key) { return 0xFFFFFFFFu - (uint32_t)key; }
static inline uint32_t di_key_score(uint64_t key) { return (uint32_t)(key >> 48); }
static inline uint32_t di_key_doc_wide(uint64_t key) { return 0xFFFFFFu - (uint32_t)(key & 0xFFFFFFu); }
static inline uint32_t di_key_score_wide(uint64_t key) { return (uint32_t)(key >> 44); }

#ifdef __cplusplus
}
#endif
#endif /* DEEPIMPACT_H */
