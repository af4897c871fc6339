"""Host hot loop #1 in worker processes, and the BERT variant's term
mapping.  The TokenizerPool (the reference's 8-process Pool, indexer.py:29,41) must
give the in-process bytes; the BERT variant maps terms with the upstream
soyuj/deeper-impact logic (reference original.py:155-177, a commented block there:
every token after [CLS] not starting with '##' opens the next term), restated on a
locally built WordPiece tokenizer -- parity unpinned beyond that restatement."""
import json

import numpy as np
import pytest

from conftest import GOLDEN


class _FakeModel:
    """process_documents of the real class; encode_processed = deterministic impacts
    (a function of the term's first token id), rounded like DI_F_ROUND3."""

    max_length = 512

    def __init__(self):
        from improving_learned_index_amd import models

        self.process_documents = models.DeepImpact.process_documents

    def encode_packed_terms(self, packed, round3=False):
        ids, cu, terms, tt, ct = packed
        out = []
        for d in range(len(ct) - 1):
            out.append([(terms[j], np.float32(np.rint(
                np.float32(ids[cu[d] + tt[j]] % 977 / 97.0) * 1000) / 1000))
                for j in range(ct[d], ct[d + 1])])
        return out

    def encode_packed_text(self, packed):
        """The real class's pool path: blob terms -> impacts -> native formatter."""
        from improving_learned_index_amd import _lib

        ids, cu, blob, term_off, tt, ct = packed
        terms = [blob[term_off[i]:term_off[i + 1]].decode("utf-8")
                 for i in range(len(term_off) - 1)]
        imp = [v for d in self.encode_packed_terms((ids, cu, terms, tt, ct)) for _, v in d]
        return _lib.format_impact_lines_packed(blob, term_off, np.array(imp, np.float32), ct)

    def encode_processed(self, proc, round3=False):
        from improving_learned_index_amd import models

        return self.encode_packed_terms(models.DeepImpact.pack_processed(proc), round3)


@pytest.fixture
def restore_class():
    from improving_learned_index_amd import models

    saved = (models.DeepImpact.tokenizer, models.DeepImpact.term_mapping)
    yield models
    models.DeepImpact.tokenizer, models.DeepImpact.term_mapping = saved


def test_pool_indexer_writes_the_in_process_bytes(tmp_path, restore_class):
    from improving_learned_index_amd import indexer

    restore_class.DeepImpact.set_tokenizer(GOLDEN / "tokenizer.json")
    texts = json.loads((GOLDEN / "encoder_xlmr_small.json").read_text())["texts"]
    batch = [texts[i % len(texts)] + f" doc{i}" for i in range(600)]  # 3 chunks of <= 256
    fake = _FakeModel()
    with open(tmp_path / "a.tsv", "w") as f:
        indexer.Indexer(fake, 32).index(batch, f)
    with indexer.TokenizerPool(2, GOLDEN / "tokenizer.json", 512) as pool:
        with open(tmp_path / "b.tsv", "w") as f:
            indexer.Indexer(fake, 32, num_processes=2, pool=pool).index(batch, f)
    a = (tmp_path / "a.tsv").read_bytes()
    assert a == (tmp_path / "b.tsv").read_bytes()
    assert a.count(b"\n") == len(batch) and b"doc599: " in a


def _bert_tokenizer():
    from tokenizers import Tokenizer, models, normalizers, pre_tokenizers, processors

    vocab = {t: i for i, t in enumerate(
        ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "hello", "world", "again", ",", "un",
         "##believ", "##able", "the"])}
    tok = Tokenizer(models.WordPiece(vocab, unk_token="[UNK]"))
    tok.normalizer = normalizers.BertNormalizer(lowercase=True)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tok.post_processor = processors.TemplateProcessing(
        single="[CLS] $A [SEP]", special_tokens=[("[CLS]", 2), ("[SEP]", 3)])
    return tok


def _legacy_restatement(tokens, terms, punct):
    """original.py:162-177 (commented block)."""
    t2t, counter = {}, 0
    for i, token in enumerate(tokens[1:], start=1):
        if token.startswith("##"):
            continue
        t2t[counter] = i
        counter += 1
    out = {}
    for i, term in enumerate(terms):
        if term not in out and term not in punct and i in t2t:
            out[term] = t2t[i]
    return out


@pytest.mark.parametrize("max_length", [4, 6, 512])
def test_bert_legacy_term_mapping(restore_class, max_length):
    M = restore_class
    tok = _bert_tokenizer()
    M.DeepImpact.tokenizer = tok
    M.DeepImpact.term_mapping = "bert_legacy"
    doc = "Hello world, unbelievable the world again!"
    (enc, tmap), = M.DeepImpact.process_documents([doc], max_length)
    tok.no_padding()
    tok.enable_truncation(max_length)
    terms = [x[0] for x in tok.pre_tokenizer.pre_tokenize_str(tok.normalizer.normalize_str(doc))]
    e = tok.encode(terms, is_pretokenized=True)
    assert tmap == _legacy_restatement(e.tokens, terms, M.PUNCTUATION)
    if max_length == 4:  # [CLS] hello world [SEP]: the legacy counter maps ',' -> [SEP]
        assert tmap == {"hello": 1, "world": 2}
    if max_length == 6:  # [CLS] hello world , un [SEP]: 'unbelievable' -> 'un', 'the' -> [SEP]
        assert tmap == {"hello": 1, "world": 2, "unbelievable": 4, "the": 5}
    M.DeepImpact.term_mapping = "word_ids"
    (_, wmap), = M.DeepImpact.process_documents([doc], max_length)
    if max_length == 6:
        assert wmap == {"hello": 1, "world": 2, "unbelievable": 4}


def test_merged_chunks_equal_one_packed_batch(restore_class):
    """The pool path merges the workers' chunks into device batches
    (DeepImpact.merge_packed_blobs): the merge must equal packing the whole batch at
    once (ids, cu_seqlens, term blob and offsets, term token indices, cu_terms)."""
    D = restore_class.DeepImpact
    D.set_tokenizer(GOLDEN / "tokenizer.json")
    texts = json.loads((GOLDEN / "encoder_xlmr_small.json").read_text())["texts"]
    docs = [texts[i % len(texts)] + f" w{i}, x:{i} é" * (i % 3) for i in range(41)] + [""]
    whole = D.pack_processed_blob(D.process_documents(docs, 512))
    parts = [D.pack_processed_blob(D.process_documents(docs[i:i + 6], 512))
             for i in range(0, len(docs), 6)]
    merged = D.merge_packed_blobs(parts)
    assert merged[2] == whole[2]
    for i in (0, 1, 3, 4, 5):
        assert merged[i].dtype == whole[i].dtype
        np.testing.assert_array_equal(merged[i], whole[i])


def test_worker_threads_follow_the_cpu_share(monkeypatch):
    """Each tokenizer worker's thread pool is sized from the process's CPU share
    (OMP_NUM_THREADS when set, as on the GPU box) over the worker count, 2..4."""
    import os

    from improving_learned_index_amd import indexer

    # a fixed CPU affinity (256 CPUs, like the GPU box): the share is then the
    # OMP_NUM_THREADS value alone, whatever machine runs the test
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)), raising=False)
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert indexer.worker_threads(16) == 2
    assert indexer.worker_threads(2) == 4
    monkeypatch.setenv("OMP_NUM_THREADS", "64")
    assert indexer.worker_threads(16) == 4
    monkeypatch.setenv("OMP_NUM_THREADS", "")
    assert indexer.worker_threads(16) == 4  # 256 // 16 = 16, capped at 4
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)), raising=False)
    assert indexer.worker_threads(8) == 2  # 8 // 8 = 1, at least 2


class _DeferredFakeModel(_FakeModel):
    """The real class's split: encode now, format later (Indexer's writer thread)."""

    def encode_packed_impacts(self, packed):
        text = self.encode_packed_text(packed)
        return lambda: text


@pytest.mark.parametrize("model_cls", [_FakeModel, _DeferredFakeModel])
def test_index_file_deferred_writes_keep_the_bytes(tmp_path, restore_class, model_cls):
    """index._index_file with a tokenizer pool: each batch's formatting and write run on
    the writer thread behind the next batch's encode (finish(wait=False)); the file must
    equal the sequential in-process loop's, empty first batch included (process batch
    size 7 over 100 docs: 15 batches)."""
    import time

    from improving_learned_index_amd import index as index_cli
    from improving_learned_index_amd import indexer

    restore_class.DeepImpact.set_tokenizer(GOLDEN / "tokenizer.json")
    texts = json.loads((GOLDEN / "encoder_xlmr_small.json").read_text())["texts"]
    coll = tmp_path / "c.tsv"
    coll.write_text("".join(f"{i}\t{texts[i % len(texts)]} doc{i}\n" for i in range(100)))
    index_cli._index_file(indexer.Indexer(_FakeModel(), 32), coll, "msmarco", tmp_path / "a",
                          7, None, time.time())
    with indexer.TokenizerPool(2, GOLDEN / "tokenizer.json", 512) as pool:
        idx = indexer.Indexer(model_cls(), 32, num_processes=2, pool=pool)
        index_cli._index_file(idx, coll, "msmarco", tmp_path / "b", 7, None, time.time())
    assert (tmp_path / "a").read_bytes() == (tmp_path / "b").read_bytes()
    assert (tmp_path / "a").read_bytes().count(b"\n") == 100
