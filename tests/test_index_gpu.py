"""GPU parity of the quantized-index scorer (di_index_search) -- A11/A12.

Checked through the C ABI against (1) the reference's own outputs (golden
fixtures) and (2) the oracle (oracle/oracle.c, pinned to the same fixtures) on
seeded synthetic collections that cross the 32768-doc LDS blocks.  Integer work:
bit-exact, including the reference's first-touch tie order.
"""
import json

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from improving_learned_index_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible (GPU test run without a GPU)")
    return _lib


def test_golden_index_matches_reference(L):
    from improving_learned_index_amd.inverted_index import InvertedIndex

    fx = json.loads((GOLDEN / "score.json").read_text())
    ix = InvertedIndex(GOLDEN / "index")
    got1000 = ix.score_batch(fx["queries"], 1000)
    got10 = ix.score_batch(fx["queries"], 10)
    for q, g1000, g10, w1000, w10 in zip(fx["queries"], got1000, got10, fx["top1000"],
                                         fx["top10"]):
        assert [list(x) for x in g1000] == w1000, q
        assert [list(x) for x in g10] == w10, q
    # single-query interface == reference InvertedIndex.score
    assert [list(x) for x in ix.score(fx["queries"][0], top_k=1000)] == fx["top1000"][0]


def test_golden_ties_match_reference(L):
    from improving_learned_index_amd.inverted_index import InvertedIndex

    tx = json.loads((GOLDEN / "score_ties.json").read_text())
    ix = InvertedIndex(GOLDEN / "index_ties")
    for q, w2, w1000 in zip(tx["queries"], tx["top2"], tx["top1000"]):
        assert [list(x) for x in ix.score(q, 2)] == w2
        assert [list(x) for x in ix.score(q, 1000)] == w1000


def _synthetic(n_docs, v_terms, seed):
    from improving_learned_index_amd import synthetic as S

    cu, term, imp = S.msmarco_like_docs(n_docs, v_terms, seed, max_terms=60)
    q, _ = S.quantize_like_reference(imp)
    return S.postings_reference_order(cu, term, q, v_terms)


@pytest.fixture(scope="module")
def synth():
    term_off, pdoc, pval = _synthetic(70_000, 5000, seed=5)
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval = term_off, pdoc, pval
    ora.n_docs = int(pdoc.max()) + 1
    return term_off, pdoc, pval, ora


def _queries(v_terms, n, seed, long_every=0):
    rng = np.random.default_rng(seed)
    qs = []
    for i in range(n):
        nd = int(rng.integers(1, 9))
        if long_every and i % long_every == 0:
            nd = int(rng.integers(100, 300))
        z = np.minimum(rng.zipf(1.25, nd), v_terms) - 1
        q = list(dict.fromkeys(int(x) for x in z))[:256]
        qs.append(q)
    qs += [[], [v_terms - 1], [0], [0, 1], [1, 0]]
    return qs


@pytest.mark.parametrize("k", [1, 10, 1000, 2000, 4096])
def test_synthetic_matches_oracle(L, synth, k):
    # (k 1000 over 3 blocks: the register merge; 2000 and 4096: past its 4096
    # candidates, the general merge kernel)
    term_off, pdoc, pval, ora = synth
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    info = dev.info()
    assert info["n_blocks"] == 3 and info["n_docs"] == ora.n_docs
    qs = _queries(5000, 120, seed=k, long_every=40)
    got = dev.search(qs, k)
    want = ora.score_ids(qs, k, n_threads=8)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, len(g), len(w))


def test_shards_merge_equals_single(L, synth):
    term_off, pdoc, pval, ora = synth
    k = 500
    qs = _queries(5000, 60, seed=11)
    full = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    _, _, n_full, key_full = full.search_csr(*L.csr(qs), k, with_keys=True)
    cuts = [0, 20_000, 45_001, ora.n_docs]
    keys = np.zeros((len(qs), 3, k), np.uint64)
    counts = np.zeros((len(qs), 3), np.int32)
    for s in range(3):
        sh = L.DeviceIndex.from_postings(term_off, pdoc, pval, cuts[s], cuts[s + 1])
        docs, _, n, key = sh.search_csr(*L.csr(qs), k, with_keys=True)
        for i in range(len(qs)):
            assert ((docs[i, :n[i]] >= cuts[s]) & (docs[i, :n[i]] < cuts[s + 1])).all()
        keys[:, s, :] = key
        counts[:, s] = n
    mk, mn = L.topk_merge(keys, counts, k)
    assert (mn == n_full).all()
    for i in range(len(qs)):
        assert (mk[i, :mn[i]] == key_full[i, :n_full[i]]).all()
        w = ora.score_ids([qs[i]], k)[0]
        assert list(zip(L.key_doc(mk[i, :mn[i]]).tolist(),
                        L.key_score(mk[i, :mn[i]]).tolist())) == w


def _long_queries(v_terms, n, seed, lo=257, hi=1200):
    """Queries of lo..hi distinct known terms (zipf-ordered draws: the frequent terms
    come early, as in a real long query; the rest fills up with random terms)."""
    rng = np.random.default_rng(seed)
    qs = []
    for _ in range(n):
        nt = int(rng.integers(lo, hi + 1))
        z = np.minimum(rng.zipf(1.2, 2 * nt), v_terms) - 1
        q = list(dict.fromkeys(int(x) for x in z))
        seen = set(q)
        rest = [int(x) for x in rng.permutation(v_terms) if int(x) not in seen]
        qs.append((q + rest)[:nt])
    return qs


@pytest.mark.parametrize("k", [1, 10, 1000, 4096])
def test_long_queries_match_oracle(L, synth, k):
    """Queries of 257..1200 known terms (score_long_kernel: 64-bit words over half
    blocks, wide keys) in one batch with short ones: the reference's ranking exactly
    (InvertedIndex.score has no term limit, inverted_index.py:55-62)."""
    term_off, pdoc, pval, ora = synth
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    qs = _long_queries(5000, 10, seed=k) + _queries(5000, 30, seed=k)
    qs = [qs[i] for i in np.random.default_rng(k).permutation(len(qs))]
    assert max(len(q) for q in qs) > 256
    got = dev.search(qs, k)
    want = ora.score_ids(qs, k, n_threads=8)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, len(qs[i]), len(g), len(w))
    # pruned (min_impact) long queries too
    dev.set_min_impact(16)
    keep = pval >= 16
    cnt = np.array([int(keep[term_off[t]:term_off[t + 1]].sum()) for t in range(len(term_off) - 1)])
    pr = oracle.Index.__new__(oracle.Index)
    pr.term_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    pr.pdoc, pr.pval, pr.n_docs = pdoc[keep], pval[keep], ora.n_docs
    assert dev.search(qs, k) == pr.score_ids(qs, k, n_threads=8)


def test_long_query_shards_merge_equals_single(L, synth):
    """Wide keys of long queries merge across doc-id shards exactly like the compact
    ones (di_topk_merge is key-order only) and decode with key_doc/key_score(wide)."""
    term_off, pdoc, pval, ora = synth
    k = 700
    qs = _long_queries(5000, 6, seed=3, lo=257, hi=900) + _queries(5000, 6, seed=4)
    full = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    _, _, n_full, key_full = full.search_csr(*L.csr(qs), k, with_keys=True)
    _, okeys, on = ora.score_ids(qs, k, n_threads=8, with_keys=True)
    cuts = [0, 33_333, ora.n_docs]
    keys = np.zeros((len(qs), 2, k), np.uint64)
    counts = np.zeros((len(qs), 2), np.int32)
    for s in range(2):
        sh = L.DeviceIndex.from_postings(term_off, pdoc, pval, cuts[s], cuts[s + 1])
        _, _, n, key = sh.search_csr(*L.csr(qs), k, with_keys=True)
        keys[:, s, :], counts[:, s] = key, n
    mk, mn = L.topk_merge(keys, counts, k)
    assert (mn == n_full).all() and (mn == on).all()
    for i, q in enumerate(qs):
        wide = L.is_wide(len(q))
        assert (mk[i, :mn[i]] == key_full[i, :n_full[i]]).all()
        assert (mk[i, :mn[i]] == okeys[i, :on[i]]).all()  # the oracle's own keys
        w = ora.score_ids([q], k)[0]
        assert list(zip(L.key_doc(mk[i, :mn[i]], wide).tolist(),
                        L.key_score(mk[i, :mn[i]], wide).tolist())) == w


def test_device_path_flags_rejected_queries(L, synth):
    """DI_F_DEVICE_PTRS (the sharded rank CLI, bench) skips the host checks: a query
    over a kernel limit must come back as out_n = -1 -- never as keys -- and the other
    queries of the batch stay exact."""
    import torch

    term_off, pdoc, pval, ora = synth
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    qs = [[1, 2, 3], list(range(4097)), [7], list(range(300)), [5000]]  # 4097 terms; bad id
    flat, cu = L.csr(qs)
    k = 10
    d_t = torch.from_numpy(flat.astype(np.int32)).cuda()
    d_cu = torch.from_numpy(cu).cuda()
    od = torch.empty(len(qs) * k, dtype=torch.int32, device="cuda")
    osc = torch.empty_like(od)
    on = torch.empty(len(qs), dtype=torch.int32, device="cuda")
    ok = torch.empty(len(qs) * k, dtype=torch.int64, device="cuda")
    dev.search_device(d_t, d_cu, len(qs), k, od, osc, on, ok)
    n = on.cpu().numpy()
    assert n[1] == -1 and n[4] == -1
    want = ora.score_ids([qs[0], qs[2], qs[3]], k)
    od, osc = od.cpu().numpy(), osc.cpu().numpy()
    for i, w in zip((0, 2, 3), want):
        assert list(zip(od[i * k:i * k + n[i]].tolist(), osc[i * k:i * k + n[i]].tolist())) == w
    from improving_learned_index_amd import parallel

    with pytest.raises(RuntimeError):
        parallel.decode_quant_keys(ok.cpu().numpy().view(np.uint64)[k:2 * k], int(n[1]), 4097)


def test_limits_and_errors(L, synth):
    term_off, pdoc, pval, _ = synth
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    with pytest.raises(L.DIError) as e:
        dev.search([list(range(4097))], 10)  # DI_MAX_QUERY_TERMS
    assert e.value.code == -4
    assert len(dev.search([list(range(257))], 10)[0]) == 10  # no 256-term limit any more
    # a long query needs 24-bit docs (wide key): a shard reaching doc 2^24 rejects it
    far = L.DeviceIndex.from_postings(np.array([0, 1, 2], np.int64),
                                      np.array([(1 << 24) + 3, 5], np.uint32),
                                      np.array([9, 4], np.uint8))
    assert far.search([[0, 1]], 10) == [[((1 << 24) + 3, 9), (5, 4)]]
    with pytest.raises(L.DIError) as e:
        far.search([[0, 1] * 129], 10)
    assert e.value.code == -4
    with pytest.raises(L.DIError):
        dev.search([[5000]], 10)  # unknown term id
    with pytest.raises(L.DIError):
        dev.search([[1]], 0)
    assert dev.search([], 10) == []
    empty = L.DeviceIndex.from_postings(np.zeros(3, np.int64), np.zeros(0, np.uint32),
                                        np.zeros(0, np.uint8))
    assert empty.search([[0, 1]], 10) == [[]]


def test_zero_values_stop_term_lists(L):
    # inverted_index.py:50-51: a term list ends at its first 0 value
    term_off = np.array([0, 4], np.int64)
    pdoc = np.array([3, 1, 2, 0], np.uint32)
    pval = np.array([9, 5, 0, 7], np.uint8)
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    assert dev.search([[0]], 10) == [[(3, 9), (1, 5)]]


def _pruned_oracle(term_off, pdoc, pval, n_docs, min_impact):
    """The oracle over the postings a min_impact search scores (value >= 2^floor(log2 m))."""
    keep = pval >= (1 << (int(min_impact).bit_length() - 1))
    c = np.concatenate([[0], np.cumsum(keep, dtype=np.int64)])
    cnt = c[term_off[1:]] - c[term_off[:-1]]
    pr = oracle.Index.__new__(oracle.Index)
    pr.term_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    pr.pdoc, pr.pval, pr.n_docs = pdoc[keep], pval[keep], n_docs
    return pr


@pytest.mark.parametrize("k", [10, 100, 1000])
def test_sparse_items_equal_oracle(L, synth, k, monkeypatch):
    """Items (query, block) that scatter at most k postings take the one-sweep selection
    (every touched doc is a candidate) in the EXT_BM instantiation, which heavily pruned
    searches on shards of >= 8 blocks run (here forced on the 3-block shard by
    DI_PROFILE_ABLATE bit 65536): queries of rare terms, alone and next to a frequent
    one (which puts some of their items over k), equal the oracle, exhaustive and pruned."""
    term_off, pdoc, pval, ora = synth
    df = np.diff(term_off)
    rare = [int(t) for t in np.nonzero((df > 0) & (df <= 400))[0]]
    rng = np.random.default_rng(k)
    qs = [[int(t) for t in rng.choice(rare, int(rng.integers(1, 9)), replace=False)]
          for _ in range(150)]
    qs += [q + [0] for q in qs[:30]] + [[0] + q for q in qs[30:60]]
    assert sum(int(df[q].sum()) <= k for q in qs) >= 10  # (more items are, per block)
    want = ora.score_ids(qs, k, n_threads=8)
    assert L.DeviceIndex.from_postings(term_off, pdoc, pval).search(qs, k) == want
    monkeypatch.setenv("DI_PROFILE_ABLATE", "65536")
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    assert dev.search(qs, k) == want
    dev.set_min_impact(2)
    assert dev.search(qs, k) == _pruned_oracle(term_off, pdoc, pval, ora.n_docs, 2).score_ids(
        qs, k, n_threads=8)


@pytest.mark.parametrize("min_impact", [2, 5, 64])
def test_min_impact_pruning_equals_oracle_on_pruned_postings(L, synth, min_impact):
    """di_index_set_min_impact (BASELINE configs[4] sweep): scoring the postings with
    value >= 2^floor(log2 min_impact) gives exactly the oracle's ranking over those
    postings (the first-touch tie rule unchanged); 1 restores the exact search.  Short
    queries (class prefixes, per-wave runs) and 65..200-term ones (the all-wave form:
    whole sublists filtered by value)."""
    term_off, pdoc, pval, ora = synth
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    qs = _queries(5000, 60, seed=min_impact) + _long_queries(5000, 4, seed=min_impact, lo=65,
                                                                hi=200)
    thr = 1 << (int(min_impact).bit_length() - 1)
    keep = pval >= thr
    cnt = np.array([int(keep[term_off[t]:term_off[t + 1]].sum()) for t in range(len(term_off) - 1)])
    pr = oracle.Index.__new__(oracle.Index)
    pr.term_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    pr.pdoc, pr.pval, pr.n_docs = pdoc[keep], pval[keep], ora.n_docs
    dev.set_min_impact(min_impact)
    assert dev.search(qs, 1000) == pr.score_ids(qs, 1000, n_threads=8)
    dev.set_min_impact(1)
    assert dev.search(qs, 1000) == ora.score_ids(qs, 1000, n_threads=8)


def test_inverted_index_min_impact_matches_pruned_oracle(L):
    """The Python drop-in carries the config-5 knob (InvertedIndex(min_impact=...),
    rank --min_impact): on the reference-format golden index it ranks exactly like
    the oracle over the postings it keeps; set_min_impact(1) is the exact ranking."""
    from improving_learned_index_amd.inverted_index import InvertedIndex

    fx = json.loads((GOLDEN / "score.json").read_text())
    ora = oracle.Index(GOLDEN / "index")
    qids = [ora.term_ids(q) for q in fx["queries"]]
    ix = InvertedIndex(GOLDEN / "index", min_impact=6)  # -> values >= 4
    keep = ora.pval >= 4
    cnt = np.array([int(keep[ora.term_off[t]:ora.term_off[t + 1]].sum())
                    for t in range(len(ora.term_off) - 1)])
    pr = oracle.Index.__new__(oracle.Index)
    pr.term_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    pr.pdoc, pr.pval, pr.n_docs = ora.pdoc[keep], ora.pval[keep], ora.n_docs
    assert keep.sum() < keep.size  # the knob prunes something here
    assert ix.score_batch(fx["queries"], 1000) == pr.score_ids(qids, 1000)
    ix.set_min_impact(1)
    assert [[list(x) for x in g] for g in ix.score_batch(fx["queries"], 1000)] == fx["top1000"]
    with pytest.raises(Exception):
        ix.set_min_impact(0)
    # configs[4] knob of the drop-in (rank --block_max): factor 1 is the exact ranking
    ex = InvertedIndex(GOLDEN / "index", block_max=1.0)
    assert [[list(x) for x in g] for g in ex.score_batch(fx["queries"], 1000)] == fx["top1000"]
    # rank --packed: the block-compressed postings, alone and with exact block-max
    pk = InvertedIndex(GOLDEN / "index", packed=True)
    assert [[list(x) for x in g] for g in pk.score_batch(fx["queries"], 1000)] == fx["top1000"]
    pk.set_block_max(1.0)
    assert [[list(x) for x in g] for g in pk.score_batch(fx["queries"], 10)] == fx["top10"]


def test_shared_threshold_off_equals_oracle(L, synth, monkeypatch):
    """The per-query threshold shared across blocks (default) and the plain per-block
    top-k (DI_SCORE_THRESHOLD=0) both rank exactly as the oracle."""
    term_off, pdoc, pval, ora = synth
    qs = _queries(5000, 80, seed=3, long_every=20)
    want = ora.score_ids(qs, 1000, n_threads=8)
    monkeypatch.setenv("DI_SCORE_THRESHOLD", "0")
    off = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    assert off.search(qs, 1000) == want
    monkeypatch.setenv("DI_SCORE_THRESHOLD", "1")
    on = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    assert on.search(qs, 1000) == want
    assert on.search(qs, 7) == ora.score_ids(qs, 7, n_threads=8)
    assert on.search(qs, 1) == ora.score_ids(qs, 1, n_threads=8)


def test_in_kernel_setup_fallback_equals_oracle(L, synth, monkeypatch):
    """score_blocks resolves its items' sublists itself when the item_setup_kernel
    records would pass 2 GiB (e.g. rank --top_k 10 over 8.8 M docs); DI_PROFILE_ABLATE
    bit 1024 forces that path here: the same exact ranking."""
    term_off, pdoc, pval, ora = synth
    qs = _queries(5000, 80, seed=13, long_every=10)
    monkeypatch.setenv("DI_PROFILE_ABLATE", "1024")
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    for k in (10, 1000):
        assert dev.search(qs, k) == ora.score_ids(qs, k, n_threads=8)


def _two_block_skewed(n_docs, v_terms, seed):
    """A 2-block shard whose second block outscores the first: every doc holds ~12 of
    v_terms terms; block 0 impacts 1..60, block 1 impacts 90..255.  A query's block-1
    items then find more than 2 k docs above the running threshold (block 0's k-th
    score), so the emit-above sweep overflows its list and falls back to the full
    selection -- with near-full blocks (no accumulator tail) after staging keys in the
    score-histogram area."""
    from improving_learned_index_amd import synthetic as S

    rng = np.random.default_rng(seed)
    per = 12
    half = (n_docs + 1) // 2
    term = np.concatenate([np.sort(rng.choice(v_terms, per, replace=False)) for _ in range(n_docs)])
    doc = np.repeat(np.arange(n_docs), per)
    val = np.where(doc < half, rng.integers(1, 61, doc.size), rng.integers(90, 256, doc.size))
    cu = np.arange(0, (n_docs + 1) * per, per, dtype=np.int64)
    return S.postings_reference_order(cu, term.astype(np.uint32), val.astype(np.int64), v_terms)


@pytest.mark.parametrize("k", [100, 1000])
def test_emit_above_overflow_with_full_blocks_equals_oracle(L, k):
    """the few-block emit-above selection stages up to 2 k keys in the
    score-histogram area when a near-full block leaves no accumulator tail (k 1000:
    block_docs > 28768); when more than 2 k docs pass the running threshold it falls back
    to the full selection, whose histogram must be zeroed again.  2 blocks of 31 000 docs,
    skewed so the second block overflows: the exact top-k."""
    n_docs, v = 62_000, 60
    term_off, pdoc, pval = _two_block_skewed(n_docs, v, seed=k)
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n_docs)
    info = dev.info()
    assert info["n_blocks"] == 2 and info["n_docs"] == n_docs
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n_docs
    rng = np.random.default_rng(7 + k)
    # enough queries that block-major order runs most block-1 items after block 0's
    qs = [list(dict.fromkeys(int(x) for x in rng.integers(0, v, rng.integers(1, 6))))
          for _ in range(1200)]
    got = dev.search(qs, k)
    want = ora.score_ids(qs, k, n_threads=8)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, (i, qs[i], len(g), len(w))


@pytest.fixture(scope="module")
def million():
    """One 8-way shard of configs[2] (full MS MARCO: 8.8 M docs): 1.1 M docs, 34 LDS
    blocks, ~105 M postings, the SURVEY §8d generator with the vocabulary scaled with N
    (V = 2 N = 2.2 M terms, ~8.7 M (term, block) entries in the sparse table)."""
    from improving_learned_index_amd import synthetic as S

    term_off, pdoc, pval, _ = S.synth_postings(1_100_000, 2_200_000, seed=99)
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval = term_off, pdoc, pval
    ora.n_docs = 1_100_000
    return term_off, pdoc, pval, ora


@pytest.mark.parametrize("k", [10, 1000])
def test_million_doc_shard_matches_oracle(L, million, k):
    """34 blocks, scaled vocabulary, shared threshold on: the exact top-k (dev.small-
    shaped queries, longer ones, and queries of 65..300 terms: the all-wave form and
    the long-query kernel)."""
    from improving_learned_index_amd import synthetic as S

    term_off, pdoc, pval, ora = million
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, ora.n_docs)
    assert dev.info()["n_blocks"] == 34
    qs = S.msmarco_like_queries(24, 2_200_000, seed=k) + _queries(2_200_000, 8, seed=k) + \
        _long_queries(3000, 3, seed=k, lo=65, hi=300)
    assert dev.search(qs, k) == ora.score_ids(qs, k, n_threads=16)
    # min_impact 16 / 128 at 34 blocks: the EXT_BM instantiation and its one-sweep
    # selection of sparse items
    for m in (16, 128):
        dev.set_min_impact(m)
        assert dev.search(qs, k) == _pruned_oracle(term_off, pdoc, pval, ora.n_docs, m).score_ids(
            qs, k, n_threads=16), m


@pytest.mark.parametrize("every,first", [(1, 0), (2, 0), (8, 2), (1000, 1)])
def test_threshold_refresh_schedules_equal_oracle(L, million, every, first, monkeypatch):
    """score_item's threshold refresh schedule (DI_TQ_EVERY / DI_TQ_FIRST): only some
    blocks' items read the query's candidate histogram, the others the running word
    qtq -- a staler lower bound, so more of their sweeps overflow to the full selection
    (with full 32 K-doc blocks the overflowed keys sat in the histogram area, which must
    be zeroed again).  Every schedule: the exact top-k (34 blocks, k 10 and 1000; every
    1000: block 0 alone reads the histogram)."""
    from improving_learned_index_amd import synthetic as S

    term_off, pdoc, pval, ora = million
    monkeypatch.setenv("DI_TQ_EVERY", str(every))
    monkeypatch.setenv("DI_TQ_FIRST", str(first))
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, ora.n_docs)
    qs = S.msmarco_like_queries(24, 2_200_000, seed=31) + _queries(2_200_000, 8, seed=31)
    for k in (10, 1000):
        assert dev.search(qs, k) == ora.score_ids(qs, k, n_threads=16), k


def test_threshold_refresh_small_blocks_equal_oracle(L, synth, monkeypatch):
    """The same schedules on the 3-block 70 k-doc shard with the shared threshold forced
    on (blocks with an accumulator tail; long queries in the batch)."""
    term_off, pdoc, pval, ora = synth
    qs = _queries(5000, 80, seed=23, long_every=20)
    monkeypatch.setenv("DI_SCORE_THRESHOLD", "1")
    for every in (2, 3):
        monkeypatch.setenv("DI_TQ_EVERY", str(every))
        dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
        for k in (10, 1000):
            assert dev.search(qs, k) == ora.score_ids(qs, k, n_threads=8), (every, k)


def test_million_doc_merge_past_lds_capacity(L, million, monkeypatch):
    """Shared threshold off at 34 blocks: every block lists its full top-1000, 34 k
    candidates per query against the merge's 8192-key LDS array -- the two-pass
    histogram filter (a wave per list) keeps the keys at or above the 1000th key's score
    bin and selects among those: the exact top-1000."""
    from improving_learned_index_amd import synthetic as S

    term_off, pdoc, pval, ora = million
    monkeypatch.setenv("DI_SCORE_THRESHOLD", "0")
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, ora.n_docs)
    qs = S.msmarco_like_queries(24, 2_200_000, seed=5) + _queries(2_200_000, 8, seed=5)
    got = dev.search(qs, 1000)
    assert got == ora.score_ids(qs, 1000, n_threads=16)
    assert sum(len(g) == 1000 for g in got) >= 16  # (most queries past the capacity)


def test_full_msmarco_scaled_vocab_on_one_gpu(L):
    """configs[2] at full size on one GPU: 8.8 M docs (269 blocks), the vocabulary
    scaled with N (V = 2 N = 17.6 M terms: a dense term x block table would be 4.7 G
    entries; the sparse one holds only the nonempty (term, block) pairs), ~0.9 G
    postings.  It loads, and dev.small-shaped queries equal the oracle."""
    from improving_learned_index_amd import synthetic as S

    n, v = 8_800_000, 17_600_000
    term_off, pdoc, pval, _ = S.synth_postings(n, v, seed=7)
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n)
    info = dev.info()
    assert info["n_blocks"] == 269 and info["n_terms"] == v and info["n_docs"] == n
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n
    qs = S.msmarco_like_queries(16, v, seed=3)
    assert dev.search(qs, 1000) == ora.score_ids(qs, 1000, n_threads=16)


@pytest.mark.parametrize("k", [10, 1000])
def test_block_max_exact_equals_oracle(L, synth, k, monkeypatch):
    """configs[4] block-max skipping (di_index_set_block_max): factor 1 skips only wave
    segments whose upper bound is below the query's running threshold -- the exact
    ranking; a larger factor is approximate, but every doc it returns carries its full
    score (a segment is scored for all terms or not at all) in key order."""
    term_off, pdoc, pval, ora = synth
    monkeypatch.setenv("DI_SCORE_THRESHOLD", "1")  # (3 blocks: force the shared threshold)
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    qs = _queries(5000, 80, seed=k + 1) + _long_queries(5000, 2, seed=k, lo=65, hi=90)
    want = ora.score_ids(qs, k, n_threads=8)
    dev.set_block_max(1.0)
    assert dev.search(qs, k) == want
    dev.set_block_max(4.0)
    got = dev.search(qs, k)
    full = ora.score_ids(qs, ora.n_docs, n_threads=8)
    for g, f in zip(got, full):
        true = dict(f)
        assert all(true[d] == s for d, s in g)
        assert [s for _, s in g] == sorted((s for _, s in g), reverse=True)
    dev.set_block_max(0.0)
    assert dev.search(qs, k) == want
    with pytest.raises(L.DIError):
        dev.set_block_max(0.5)


def test_million_block_max_exact(L, million):
    """Block-max skipping, factor 1, at 34 blocks and the scaled vocabulary: exact."""
    from improving_learned_index_amd import synthetic as S

    term_off, pdoc, pval, ora = million
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, ora.n_docs)
    dev.set_block_max(1.0)
    qs = S.msmarco_like_queries(24, 2_200_000, seed=5) + _queries(2_200_000, 8, seed=5)
    assert dev.search(qs, 1000) == ora.score_ids(qs, 1000, n_threads=16)


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("k", [10, 1000])
def test_block_max_exact_skips_on_skewed_collection(L, k, order, monkeypatch):
    """configs[4] where skipping fires: a 1.1 M-doc shard of the skewed collection
    (synthetic.SKEW_CONFIG4: frequent terms carry small impacts, doc mass shared by
    clusters of consecutive ids -- a stated deviation from SURVEY §8d, on whose i.i.d.
    impacts exact block-max finds nothing to skip).  Factor 1 skips wave segments (the
    scorer's own counter says how many) and the ranking still equals the oracle's --
    block-major items (default) and per-query bound order (DI_BLOCK_ORDER=1)."""
    from improving_learned_index_amd import synthetic as S

    monkeypatch.setenv("DI_BLOCK_ORDER", str(order))
    n = 1_100_000
    term_off, pdoc, pval, _ = S.synth_postings(n, 2 * n, seed=4321, skew=S.SKEW_CONFIG4)
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n)
    qs = S.msmarco_like_queries(1000, 2 * n, seed=k)
    want = ora.score_ids(qs, k, n_threads=16)
    dev.set_block_max(1.0)
    dev.timing("bm_segments", reset=True)
    dev.timing("bm_segments_skipped", reset=True)
    assert dev.search(qs, k) == want
    seg = dev.timing("bm_segments")[1]
    skipped = dev.timing("bm_segments_skipped")[1]
    print(f"k={k} order={order}: {skipped} of {seg} wave segments skipped "
          f"({skipped / max(seg, 1):.3f})")
    # (the exact skip potential with the final k-th score is ~0.6 of the segments,
    # tools/skip_potential.py; the running threshold reaches less of it at k = 1000)
    assert seg > 0 and skipped > (0.3 if k == 10 else 0.1) * seg
    dev.set_block_max(0.0)
    dev.timing("bm_segments", reset=True)
    assert dev.search(qs, k) == want
    assert dev.timing("bm_segments")[1] == 0  # (off: nothing evaluated)


@pytest.mark.parametrize("k", [1, 10, 1000])
def test_packed_postings_equal_oracle(L, synth, k):
    """configs[4] block-compressed postings (di_index_set_packed): every run sorted by
    doc, bit-packed frames of <= 512 postings decoded in registers -- the same ranking
    as the reference (oracle), alone and with exact block-max skipping; queries past 64
    terms in the same batch fall back to the plain layout.  The packed copy is smaller
    than the plain 4-byte postings, and switching it off gives the plain scorer back."""
    term_off, pdoc, pval, ora = synth
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval)
    qs = _queries(5000, 120, seed=k + 7) + _long_queries(5000, 2, seed=k, lo=65, hi=90)
    want = ora.score_ids(qs, k, n_threads=8)
    plain_bytes = 4 * dev.info()["n_postings"]
    packed = dev.set_packed(True)
    assert 0 < packed < plain_bytes
    assert dev.search(qs, k) == want
    dev.set_block_max(1.0)
    assert dev.search(qs, k) == want
    dev.set_min_impact(8)  # (pruning: the plain layout serves -- the pruned oracle's ranking)
    keep = pval >= 8
    cnt = np.array([int(keep[term_off[t]:term_off[t + 1]].sum()) for t in range(len(term_off) - 1)])
    pr = oracle.Index.__new__(oracle.Index)
    pr.term_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    pr.pdoc, pr.pval, pr.n_docs = pdoc[keep], pval[keep], ora.n_docs
    assert dev.search(qs, k) == pr.score_ids(qs, k, n_threads=8)
    dev.set_min_impact(1)
    assert dev.search(qs, k) == want
    dev.set_packed(False)
    dev.set_block_max(0.0)
    assert dev.search(qs, k) == want


def test_packed_postings_edge_runs(L):
    """Frames at their limits: a term in every doc of a block (deltas of 1, one long
    run per wave segment, full 512-posting frames), a term with one posting, equal
    values (bv = 0), values 1 and 255 in one frame (bv = 8), a sparse term spread over
    a 32 K-doc block (15-bit deltas, W = 24), docs 0 and the block's last."""
    rng = np.random.default_rng(3)
    n_docs = 70_000
    lists = []
    lists.append((np.arange(0, 40_000), rng.integers(1, 256, 40_000)))      # dense, all values
    lists.append((np.array([69_999]), np.array([7])))                       # one posting
    lists.append((np.arange(0, n_docs, 3), np.full(len(range(0, n_docs, 3)), 5)))  # bv = 0
    lists.append((np.array([0, 1, 2, 32_000, 32_767]), np.array([1, 255, 1, 255, 128])))
    lists.append((np.sort(rng.choice(n_docs, 300, replace=False)), rng.integers(1, 4, 300)))
    lists.append((np.arange(5, n_docs, 2), rng.integers(200, 256, len(range(5, n_docs, 2)))))
    term_off, pd, pv = [0], [], []
    for d, v in lists:
        order = np.lexsort((d, -v))  # reference order: value desc, doc asc
        pd.append(d[order].astype(np.uint32))
        pv.append(v[order].astype(np.uint8))
        term_off.append(term_off[-1] + len(d))
    term_off = np.array(term_off, np.int64)
    pdoc, pval = np.concatenate(pd), np.concatenate(pv)
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n_docs
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n_docs)
    qs = [[0], [1], [2], [3], [4], [5], [0, 1, 2, 3, 4, 5], [5, 4, 3, 2, 1, 0], [2, 0], [3, 1]]
    for k in (1, 10, 1000, 4096):
        want = ora.score_ids(qs, k, n_threads=8)
        dev.set_packed(False)
        assert dev.search(qs, k) == want
        dev.set_packed(True)
        assert dev.search(qs, k) == want, k


def test_packed_block_max_on_skewed_collection(L):
    """Packed postings with exact block-max skipping on the skewed 1.1 M-doc collection
    (SKEW_CONFIG4): oracle-equal top-1000, segments skipped."""
    from improving_learned_index_amd import synthetic as S

    n = 1_100_000
    term_off, pdoc, pval, _ = S.synth_postings(n, 2 * n, seed=4321, skew=S.SKEW_CONFIG4)
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n)
    qs = S.msmarco_like_queries(500, 2 * n, seed=77)
    want = ora.score_ids(qs, 1000, n_threads=16)
    nbytes = dev.set_packed(True)
    print(f"packed {nbytes} B vs plain {4 * len(pdoc)} B ({nbytes / (4 * len(pdoc)):.3f})")
    assert dev.search(qs, 1000) == want
    dev.set_block_max(1.0)
    dev.timing("bm_segments_skipped", reset=True)
    dev.timing("bm_segments", reset=True)
    assert dev.search(qs, 1000) == want
    assert dev.timing("bm_segments_skipped")[1] > 0


def test_block_max_approximate_factors_on_skewed_collection(L):
    """Factors > 1 skip far more (approximate): every search still completes (every item
    writes a valid candidate count) and returns docs with their full scores in key
    order.  (The block-max skip decision is one workgroup-wide value: waves that read the
    running threshold themselves could disagree on skipping -- and on the barriers they
    reach; this ran into a selection-count error and an illegal address before.)"""
    from improving_learned_index_amd import synthetic as S

    n = 1_100_000
    term_off, pdoc, pval, _ = S.synth_postings(n, 2 * n, seed=4321, skew=S.SKEW_CONFIG4)
    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n
    dev = L.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n)
    qs = S.msmarco_like_queries(3000, 2 * n, seed=13)
    full = ora.score_ids(qs[:200], n, n_threads=16)
    for f in (1.5, 2.0, 3.0, 1.5, 2.0):
        dev.set_block_max(f)
        got = dev.search(qs, 1000)
        for g, w in zip(got[:200], full):
            true = dict(w)
            assert all(true[d] == s_ for d, s_ in g)
            assert [s_ for _, s_ in g] == sorted((s_ for _, s_ in g), reverse=True)
