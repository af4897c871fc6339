"""Seeded synthetic workloads (BASELINE.md §2 / SURVEY.md §8d generators).

There is no network and no MS MARCO here: benches and large parity tests use
collections of the same shape, generated deterministically.
"""
from __future__ import annotations

import numpy as np


def round3_f32(x):
    """numpy's round(np.float32, 3): fl32(rint(fl32(x*1000)) / 1000)
    (reference src/deep_impact/indexing/indexer.py:132)."""
    x = np.asarray(x, np.float32)
    return (np.rint(x * np.float32(1000)) / np.float32(1000)).astype(np.float32)


def msmarco_like_docs(n_docs=100_000, v_terms=200_000, seed=1234, max_terms=100):
    """Per doc: first `max_terms` unique values of min(zipf(1.2, 200), V) and
    impacts float32(softplus(N(-0.5, 1.5))).  Returns (cu, term, impact_f32) CSR;
    term ids are 0-based (zipf value - 1)."""
    rng = np.random.default_rng(seed)
    cu = np.zeros(n_docs + 1, np.int64)
    terms, imps = [], []
    for d in range(n_docs):
        t = np.unique(np.minimum(rng.zipf(1.2, 200), v_terms))[:max_terms]
        imp = np.log1p(np.exp(rng.normal(-0.5, 1.5, len(t)))).astype(np.float32)
        terms.append(t - 1)
        imps.append(imp)
        cu[d + 1] = cu[d] + len(t)
    return cu, np.concatenate(terms).astype(np.uint32), np.concatenate(imps)


def quantize_like_reference(imp_f32, bits=8, max_val=None):
    """Impact TSV text -> quantize.py semantics, without the text round trip:
    the 3-decimal float32 prints as the shortest repr of its double, which
    float() reads back exactly.  max_val: the collection's max (a doc-id shard
    quantized like the whole, quantize.py:31-37), default this array's."""
    v = round3_f32(imp_f32).astype(np.float64)
    m = float(v.max()) if v.size else 0.0
    if max_val is not None:
        m = float(max_val)
    scale = ((1 << bits) - 1) / m
    return np.trunc(v * scale).astype(np.int64), m


def postings_reference_order(cu, term, val, n_terms):
    """CSR by term in the reference file order: value desc, doc asc
    (create.py:41); zero values dropped (they are dropped by quantize.py:44)."""
    n_docs = len(cu) - 1
    doc = np.repeat(np.arange(n_docs, dtype=np.uint32), np.diff(cu))
    keep = val > 0
    doc, t, v = doc[keep], term[keep], val[keep]
    order = np.lexsort((doc, -v, t))
    t_sorted = t[order]
    term_off = np.zeros(n_terms + 1, np.int64)
    np.add.at(term_off, t_sorted.astype(np.int64) + 1, 1)
    term_off = np.cumsum(term_off)
    return term_off, doc[order].astype(np.uint32), v[order].astype(np.uint8)


def msmarco_like_index(n_docs=100_000, v_terms=200_000, seed=1234):
    cu, term, imp = msmarco_like_docs(n_docs, v_terms, seed)
    q, _ = quantize_like_reference(imp)
    return postings_reference_order(cu, term, q, v_terms)


def msmarco_like_queries(n_q, v_terms=200_000, seed=1234, draws=6):
    """Each query: the set of min(zipf(1.3, draws), V) (first-occurrence order)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_q):
        z = np.minimum(rng.zipf(1.3, draws), v_terms) - 1
        out.append(list(dict.fromkeys(int(x) for x in z)))
    return out


# The skewed collection of the block-max measurements (BASELINE configs[4]; a stated
# deviation from SURVEY §8d, whose impacts are i.i.d. -- on those every 2 K-doc segment
# holds a high value of every frequent query term, so exact block-max can skip nothing,
# DESIGN.md §3).  Impacts: frequent terms small (term factor ((t + 1) / 2000)^0.5 up to
# rank 2000: the IDF-like shape of a learned impact model), and a heavy-tailed doc mass
# shared by clusters of 4096 consecutive doc ids (passages of one source document)
# times a per-doc factor, clipped at 6.
SKEW_CONFIG4 = {"term_rank0": 2000.0, "term_exp": 0.5, "cluster_docs": 4096,
                "cluster_sigma": 1.2, "doc_sigma": 0.5, "mass_max": 6.0}


def synth_postings(n_docs, v_terms=200_000, seed=1234, max_terms=100, draws=200, zipf_a=1.2,
                   skew=None, doc0=0, quant_max=0.0):
    """The same generator at full scale, in the HIP library's host code (threads over
    doc chunks, a counter-based stream per doc): reference-order postings
    (term_off, pdoc u32, pval u8) of the quantized collection and the fp64 max impact.
    Same distribution as msmarco_like_docs -> quantize_like_reference ->
    postings_reference_order; a different random stream (seconds at 8.8 M docs).
    skew: a dict of di_synth_skew fields (e.g. SKEW_CONFIG4), None = i.i.d. impacts.
    doc0 / quant_max: docs [doc0, doc0 + n_docs) of the seed's collection (local doc
    ids), quantized with quant_max (> 0: the collection's max) -- one doc-id shard; the
    returned max is the shard's own (synth_max_impact: that alone)."""
    import ctypes

    from ._lib import check, di_synth_skew, lib, ptr

    term_off = np.zeros(v_terms + 1, np.int64)
    cap = int(n_docs) * int(max_terms)
    pdoc = np.empty(max(cap, 1), np.uint32)
    pval = np.empty(max(cap, 1), np.uint8)
    n = ctypes.c_int64(0)
    m = ctypes.c_double(0.0)
    sk = ctypes.byref(di_synth_skew(**skew)) if skew else None
    if doc0 == 0 and quant_max == 0.0:  # (the whole collection: also in older builds, A/B)
        check(lib().di_synth_postings_skewed(int(n_docs), int(v_terms), int(seed), int(max_terms),
                                             int(draws), float(zipf_a), sk, ptr(term_off),
                                             ptr(pdoc), ptr(pval), cap, ctypes.byref(n),
                                             ctypes.byref(m)))
    else:
        check(lib().di_synth_postings_shard(int(doc0), int(n_docs), int(v_terms), int(seed),
                                            int(max_terms), int(draws), float(zipf_a), sk,
                                            float(quant_max), ptr(term_off), ptr(pdoc), ptr(pval),
                                            cap, ctypes.byref(n), ctypes.byref(m)))
    return term_off, pdoc[:n.value], pval[:n.value], m.value


def synth_max_impact(n_docs, v_terms=200_000, seed=1234, max_terms=100, draws=200, zipf_a=1.2,
                     skew=None, doc0=0):
    """The max 3-decimal impact of docs [doc0, doc0 + n_docs) of synth_postings' collection
    (no postings built): each shard's input to the all_reduce(MAX) of a sharded run."""
    import ctypes

    from ._lib import check, di_synth_skew, lib

    m = ctypes.c_double(0.0)
    sk = ctypes.byref(di_synth_skew(**skew)) if skew else None
    check(lib().di_synth_postings_shard(int(doc0), int(n_docs), int(v_terms), int(seed),
                                        int(max_terms), int(draws), float(zipf_a), sk, 0.0, None,
                                        None, None, 0, None, ctypes.byref(m)))
    return m.value


def synth_impact_tsv(path, n_docs, v_terms=200_000, seed=1234, max_terms=100, draws=200,
                     zipf_a=1.2) -> int:
    """The synth_postings collection as the impact TSV the index CLI writes (A9 text,
    terms "\\u2581t<id>"), generated in the library's host code.  Returns the number of
    (doc, term) pairs written."""
    import ctypes

    from ._lib import check, lib

    n = ctypes.c_int64(0)
    check(lib().di_synth_impact_tsv(str(path).encode(), int(n_docs), int(v_terms), int(seed),
                                    int(max_terms), int(draws), float(zipf_a), ctypes.byref(n)))
    return n.value
