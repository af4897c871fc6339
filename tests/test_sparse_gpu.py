"""GPU parity of the in-memory float index (A14/A15) against the reference's own
SparseSearch output (fixture sparse_search.json: reference code run here, numpy
2.x => float32 sums).  Bit-exact scores and order, including exact float ties."""
import json

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


class FakeModel:
    def __init__(self, fx):
        self.ci, self.qt = fx["corpus_impacts"], fx["query_terms"]

    def get_impact_scores_batch(self, texts):
        return [[(t, np.float32(v)) for t, v in self.ci[x]] for x in texts]

    def process_query(self, q):
        return list(self.qt[q])


@pytest.fixture(scope="module")
def fx():
    from improving_learned_index_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible (GPU test run without a GPU)")
    return json.loads((GOLDEN / "sparse_search.json").read_text())


@pytest.mark.parametrize("k", [1000, 5])
def test_sparse_search_matches_reference(fx, k):
    from improving_learned_index_amd.nano_beir import SparseSearch

    ss = SparseSearch(FakeModel(fx), batch_size=16, encode_batch_size=7)
    got = ss.search(fx["queries"], fx["corpus"], k)
    for qid, want in fx["results"][str(k)].items():
        assert [[d, s] for d, s in got[qid].items()] == want, qid


def test_sparse_multiblock_matches_oracle(fx):
    """40k docs (3 LDS blocks of 16384) against the oracle's float32 scorer."""
    from improving_learned_index_amd import _lib

    rng = np.random.default_rng(9)
    n_docs, V = 40000, 300
    lists = {t: [] for t in range(V)}
    for d in range(n_docs):
        for t in np.unique(np.minimum(rng.zipf(1.3, 12), V) - 1):
            lists[int(t)].append((d, np.float32(rng.integers(1, 40) / 8.0)))  # many exact ties
    term_off = np.zeros(V + 1, np.int64)
    term_off[1:] = np.cumsum([len(lists[t]) for t in range(V)])
    pdoc = np.array([d for t in range(V) for d, _ in lists[t]], np.uint32)
    pimp = np.array([x for t in range(V) for _, x in lists[t]], np.float32)
    dev = _lib.DeviceSparseIndex(term_off, pdoc, pimp, n_docs)
    ora = oracle.SparseIndex.__new__(oracle.SparseIndex)
    ora.corpus_ids = list(range(n_docs))
    ora.vocab = {t: t for t in range(V)}
    ora.term_off, ora.pdoc, ora.pimp = term_off, pdoc, pimp
    qs = [list(dict.fromkeys(int(x) for x in np.minimum(rng.zipf(1.2, 5), V) - 1))
          for _ in range(50)]
    for k in (10, 1000):
        got = dev.search(qs, k)
        want = ora.search(qs, k)
        for g, w in zip(got, want):
            assert [(d, float(s)) for d, s in g] == w


def test_sparse_long_queries_match_oracle(fx):
    """Argument-style queries with more than 256 known terms (NanoArguAna-like) are
    scored in term chunks with the accumulators carried over: same scores and order as
    the oracle (continuous impacts: no exact ties among late-touched docs)."""
    from improving_learned_index_amd import _lib

    rng = np.random.default_rng(4)
    n_docs, V = 20000, 1500
    lists = {t: [] for t in range(V)}
    for d in range(n_docs):
        for t in rng.choice(V, size=40, replace=False):
            lists[int(t)].append((d, np.float32(rng.random() * 3 + 1e-3)))
    term_off = np.zeros(V + 1, np.int64)
    term_off[1:] = np.cumsum([len(lists[t]) for t in range(V)])
    pdoc = np.array([d for t in range(V) for d, _ in lists[t]], np.uint32)
    pimp = np.array([x for t in range(V) for _, x in lists[t]], np.float32)
    dev = _lib.DeviceSparseIndex(term_off, pdoc, pimp, n_docs)
    ora = oracle.SparseIndex.__new__(oracle.SparseIndex)
    ora.corpus_ids = list(range(n_docs))
    ora.vocab = {t: t for t in range(V)}
    ora.term_off, ora.pdoc, ora.pimp = term_off, pdoc, pimp
    qs = [rng.choice(V, size=n, replace=False).tolist() for n in (257, 300, 600, 1200, 5)]
    for k in (10, 1000):
        got = dev.search(qs, k)
        want = ora.search(qs, k)
        for g, w in zip(got, want):
            assert [(d, float(s)) for d, s in g] == w
    with pytest.raises(_lib.DIError):
        dev.search([list(range(V)) * 3], 10)  # 4500 terms > DI_MAX_SPARSE_QUERY_TERMS


def _random_index(seed, n_docs, V, per_doc, decimals):
    rng = np.random.default_rng(seed)
    lists = {t: [] for t in range(V)}
    for d in range(n_docs):
        for t in rng.choice(V, size=per_doc, replace=False):
            v = rng.random() * 4 + 0.1  # > 0 after rounding (zero impacts are dropped)
            lists[int(t)].append((d, np.float32(round(v, decimals) if decimals else v)))
    term_off = np.zeros(V + 1, np.int64)
    term_off[1:] = np.cumsum([len(lists[t]) for t in range(V)])
    pdoc = np.array([d for t in range(V) for d, _ in lists[t]], np.uint32)
    pimp = np.array([x for t in range(V) for _, x in lists[t]], np.float32)
    ora = oracle.SparseIndex.__new__(oracle.SparseIndex)
    ora.corpus_ids = list(range(n_docs))
    ora.vocab = {t: t for t in range(V)}
    ora.term_off, ora.pdoc, ora.pimp = term_off, pdoc, pimp
    return rng, term_off, pdoc, pimp, ora


@pytest.mark.parametrize("decimals", [1, 3, 0])
def test_sparse_f64_matches_oracle(fx, decimals):
    """f64 accumulation (the reference's pinned numpy 1.25.1) against the
    oracle's use_f64 scorer: f64 scores bit-exact, same order with first-touch ties.
    40k docs = 3 blocks (6 half-block workgroups); 1-decimal impacts make many exact
    ties, 0 = unrounded impacts (f64 and f32 sums then differ in most docs)."""
    from improving_learned_index_amd import _lib

    rng, term_off, pdoc, pimp, ora = _random_index(11 + decimals, 40000, 400, 10, decimals)
    dev = _lib.DeviceSparseIndex(term_off, pdoc, pimp, 40000)
    qs = [rng.choice(400, size=n, replace=False).tolist()
          for n in (1, 2, 3, 5, 8, 13, 40, 300)] + [[]]
    for k in (1, 10, 1000):
        got = dev.search(qs, k, accumulation="f64")
        want = ora.search(qs, k, use_f64=True)
        for g, w in zip(got, want):
            assert [(d, float(s)) for d, s in g] == w
    if decimals == 0:  # the two semantics really differ on these inputs
        f32 = dev.search(qs, 1000)
        assert any([s for _, s in a] != [float(s) for _, s in b]
                   for a, b in zip(f32, dev.search(qs, 1000, accumulation="f64")))


def test_sparse_f64_search_api(fx):
    """SparseSearch(accumulation="f64") over the reference fixture's corpus and queries
    against the oracle's f64 scorer on the same term impacts."""
    from improving_learned_index_amd.nano_beir import SparseSearch

    model = FakeModel(fx)
    got = SparseSearch(model, batch_size=16, accumulation="f64").search(
        fx["queries"], fx["corpus"], 1000)
    ids = list(fx["corpus"])
    ora = oracle.SparseIndex(ids, model.get_impact_scores_batch([fx["corpus"][i] for i in ids]))
    qids = list(fx["queries"])
    want = ora.search([model.process_query(fx["queries"][q]) for q in qids], 1000, use_f64=True)
    for qid, w in zip(qids, want):
        assert list(got[qid].items()) == w, qid
    with pytest.raises(ValueError):
        SparseSearch(model, batch_size=16, accumulation="f16")
