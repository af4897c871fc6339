"""The per-word token cache of DeepImpact.process_documents (models._WordCache) gives
exactly the encodings of the tokenizer's own batched encode -- ids, word ids and the
extracted term maps -- including right truncation at small max_length, empty and
whitespace-only documents, punctuation-only words, repeated words and non-ASCII text
(A3, xlmr_original.py:120-189)."""
import json

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture()
def model_cls():
    from improving_learned_index_amd.models import DeepImpact

    DeepImpact.set_tokenizer(GOLDEN / "tokenizer.json")
    DeepImpact.term_mapping = "word_ids"
    yield DeepImpact
    DeepImpact.word_cache = True
    DeepImpact._wcache_tok = None


def _docs(n, seed):
    vocab = json.loads((GOLDEN / "tokenizer.json").read_text())["model"]["vocab"]
    words = [w[1:] for w, _ in vocab if w.startswith("▁") and len(w) > 1]
    extra = ["", ".", ",", "!?", "naïve", "Ünïcødé", "日本語", "x" * 40, "a,b", "--", "(x)",
             "  ", "\t", "é", "ﬁ", "１２３"]
    rng = np.random.default_rng(seed)
    out = ["", " ", "   ", ".", "a a a a"]
    for _ in range(n):
        k = int(rng.integers(0, 120))
        ws = [extra[int(rng.integers(0, len(extra)))] if rng.random() < 0.15
              else words[int(rng.integers(0, len(words)))] for _ in range(k)]
        out.append(" ".join(ws))
    return out


@pytest.mark.parametrize("max_length", [4, 16, 64, 300, 512])
def test_cache_equals_batched_encode(model_cls, max_length):
    docs = _docs(300, max_length)
    model_cls.word_cache = False
    model_cls._wcache_tok = None
    want = model_cls.process_documents(docs, max_length)
    model_cls.word_cache = True
    model_cls._wcache_tok = None
    got = []
    for i in range(0, len(docs), 37):  # several batches: misses, then hits
        got += model_cls.process_documents(docs[i:i + 37], max_length)
    assert model_cls._wcache is not None and model_cls._wcache.ok
    assert len(got) == len(want)
    for (ge, gm), (we, wm) in zip(got, want):
        assert ge.ids == we.ids
        assert ge.word_ids == we.word_ids
        assert gm == wm  # same terms, same first-token positions, same order


def test_cache_bound_keeps_the_batch_words(model_cls, monkeypatch):
    """Past MAX_ENTRIES the cache starts over before a batch's fill (not after it), so
    every word the batch looks up is present: same encodings as without the cache."""
    from improving_learned_index_amd import models

    docs = _docs(200, 7)
    model_cls.word_cache = False
    model_cls._wcache_tok = None
    want = model_cls.process_documents(docs, 64)
    model_cls.word_cache = True
    model_cls._wcache_tok = None
    monkeypatch.setattr(models._WordCache, "MAX_ENTRIES", 150)
    got = []
    for i in range(0, len(docs), 9):  # every batch brings new words past the bound
        got += model_cls.process_documents(docs[i:i + 9], 64)
    wc = model_cls._wcache
    assert wc is not None and wc.ok
    assert len(wc.first) + len(wc.other) <= 150 + 9 * 120
    for (ge, gm), (we, wm) in zip(got, want):
        assert ge.ids == we.ids and ge.word_ids == we.word_ids and gm == wm
