"""Pin the oracle (oracle/) against fixtures produced by the reference's own code.

Fixtures: tests/golden/make_golden.py (ran the reference Python in the build
container).  CPU only.
"""
import json
import tempfile
from pathlib import Path

import numpy as np
import pytest
import torch

import oracle
import encoder_ref
from conftest import GOLDEN


def test_round3_format_matches_reference_expression():
    # indexer.py:132  f'{term}: {round(impact, 3)}'
    vals = np.load(GOLDEN / "round3_in.npy").view(np.float32)
    want = (GOLDEN / "round3_out.txt").read_text().split("\n")[:-1]
    got = [oracle.format_impact(v) for v in oracle.round3(vals)]
    bad = [(i, vals[i], g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad[:5] and len(got) == len(want)


def test_impact_tsv_matches_reference_indexer():
    docs = json.loads((GOLDEN / "collection.docs.json").read_text())
    lines = [oracle.impact_line(d["terms"],
                                np.array(d["impacts_f32_bits"], np.uint32).view(np.float32))
             for d in docs]
    want = (GOLDEN / "collection.index").read_text()
    assert "\n".join(lines) + "\n" == want


def test_quantize_matches_reference():
    lines = [l for l in (GOLDEN / "collection.index").read_text().split("\n")[:-1] if l.strip()]
    out, m = oracle.quantize_lines(lines)
    assert m == 20.0
    assert "\n".join(out) + "\n" == (GOLDEN / "collection.quantized").read_text()
    out7, _ = oracle.quantize_lines(lines, max_val=7.0)
    assert "\n".join(out7) + "\n" == (GOLDEN / "collection.quantized.m7").read_text()
    q254 = (GOLDEN / "q254.index").read_text().split("\n")[:-1]
    o254, _ = oracle.quantize_lines(q254)
    assert "\n".join(o254) + "\n" == (GOLDEN / "q254.quantized").read_text()
    # the reference raises on an empty line (quantize.py:22)
    with pytest.raises(ValueError):
        oracle.quantize_lines(["▁a: 1.0", ""])


@pytest.mark.parametrize("src,dirname", [("collection.quantized", "index"),
                                         ("ties.quantized", "index_ties")])
def test_index_bytes_match_reference(src, dirname):
    docs = oracle.collection_items(GOLDEN / src)
    vocab, off, pdoc, pval = oracle.build_index(docs)
    with tempfile.TemporaryDirectory() as td:
        oracle.write_index(td, vocab, off, pdoc, pval)
        for f in ("vocab.txt", "inverted_index.idx", "inverted_index.dat"):
            assert (Path(td) / f).read_bytes() == (GOLDEN / dirname / f).read_bytes(), f


def test_score_matches_reference():
    fx = json.loads((GOLDEN / "score.json").read_text())
    idx = oracle.Index(GOLDEN / "index")
    for q, w1000, w10 in zip(fx["queries"], fx["top1000"], fx["top10"]):
        assert [list(x) for x in idx.score(q, 1000)] == w1000
        assert [list(x) for x in idx.score(q, 10)] == w10
    tx = json.loads((GOLDEN / "score_ties.json").read_text())
    tidx = oracle.Index(GOLDEN / "index_ties")
    for q, w2, w1000 in zip(tx["queries"], tx["top2"], tx["top1000"]):
        assert [list(x) for x in tidx.score(q, 2)] == w2
        assert [list(x) for x in tidx.score(q, 1000)] == w1000


def test_score_multithreaded_equals_single():
    fx = json.loads((GOLDEN / "score.json").read_text())
    idx = oracle.Index(GOLDEN / "index")
    qs = [idx.term_ids(q) for q in fx["queries"]]
    assert idx.score_ids(qs, 100, n_threads=4) == idx.score_ids(qs, 100, n_threads=1)


def test_sparse_search_matches_reference():
    fx = json.loads((GOLDEN / "sparse_search.json").read_text())
    corpus_ids = list(fx["corpus"])
    items = [[(t, np.float32(v)) for t, v in fx["corpus_impacts"][fx["corpus"][c]]]
             for c in corpus_ids]
    si = oracle.SparseIndex(corpus_ids, items)
    qids = list(fx["queries"])
    qterms = [fx["query_terms"][fx["queries"][q]] for q in qids]
    use_f64 = int(fx["numpy"].split(".")[0]) < 2
    for k in (1000, 5):
        got = si.search(qterms, k, use_f64=use_f64)
        for qid, g in zip(qids, got):
            want = fx["results"][str(k)][qid]
            assert [[d, s] for d, s in g] == want, qid


def test_metrics_match_reference():
    fx = json.loads((GOLDEN / "metrics.json").read_text())
    run = []
    for line in (GOLDEN / "metrics.run.tsv").read_text().split("\n")[:-1]:
        qid, pid, rank, _ = line.split("\t")
        run.append((qid, pid, int(rank)))
    qrels = {}
    for line in (GOLDEN / "metrics.qrels.tsv").read_text().split("\n")[:-1]:
        q, _, p, _ = line.split("\t")
        qrels.setdefault(q, set()).add(p)
    mrr, rec, nq = oracle.mrr_recall(run, qrels)
    assert nq == fx["n_queries"]
    for k, v in fx["mrr_sums"].items():
        assert mrr[int(k)] == pytest.approx(v, abs=1e-12)
    for k, v in fx["recall_sums"].items():
        assert rec[int(k)] == pytest.approx(v, abs=1e-12)


@pytest.mark.parametrize("name", ["xlmr_small", "xlmr_base"])
def test_encoder_restatement_matches_reference_class(name):
    fx = json.loads((GOLDEN / f"encoder_{name}.json").read_text())
    sd = encoder_ref.seeded_state_dict(fx["state_dict_shapes"], fx["seed"], fx["std"])
    with torch.no_grad():
        imp = encoder_ref.forward(sd, fx["config"], torch.tensor(fx["input_ids"]),
                                  torch.tensor(fx["attention_mask"]), "xlmr", "softplus")
    maps = fx["term_maps"]
    got = encoder_ref.gather_terms(imp, maps)
    want = fx["term_impacts_f32_bits"]
    for g, w in zip(got, want):
        assert [t for t, _ in g] == [t for t, _ in w]
        wv = np.array([b for _, b in w], np.uint32).view(np.float32)
        gv = np.array([v for _, v in g], np.float32)
        np.testing.assert_allclose(gv, wv, rtol=2e-5, atol=2e-6)
    if fx["token_impacts_f32_bits"] is not None:
        wt = np.array(fx["token_impacts_f32_bits"], np.uint32).view(np.float32)
        m = np.array(fx["attention_mask"], bool)
        np.testing.assert_allclose(imp.numpy()[m], wt[m], rtol=2e-5, atol=2e-6)


def test_encoder_restatement_matches_bert_variant():
    fx = json.loads((GOLDEN / "encoder_bert_small.json").read_text())
    sd = encoder_ref.seeded_state_dict(fx["state_dict_shapes"], fx["seed"], fx["std"])
    with torch.no_grad():
        imp = encoder_ref.forward(sd, fx["config"], torch.tensor(fx["input_ids"]),
                                  torch.tensor(fx["attention_mask"]), "bert", "relu")
    wt = np.array(fx["token_impacts_f32_bits"], np.uint32).view(np.float32)
    m = np.array(fx["attention_mask"], bool)
    np.testing.assert_allclose(imp.numpy()[m], wt[m], rtol=2e-5, atol=2e-6)
