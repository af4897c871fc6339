"""NanoBEIR evaluation path: in-memory sparse search on the GPU.

Reference: src/deep_impact/evaluation/nano_beir_evaluator.py -- SparseSearch
(:70-137) and NanoBEIREvaluator (:153-232).  The model protocol is the
reference's (``get_impact_scores_batch``, ``process_query``), so any model
object the reference accepts works here; the scores are computed by the HIP
float index (di_sparse_*): float32 sums in the reference's order, ties in
first-touch order, bit-exact with the reference under numpy >= 2.

Datasets: the reference downloads zeta-alpha-ai/Nano* from the hub (:165-167),
which is impossible offline; ``NanoBEIREvaluator`` takes local datasets
(corpus/queries/qrels dicts, or a directory of corpus.jsonl / queries.jsonl /
qrels.tsv).  nDCG follows trec_eval (metrics.ndcg_at_k) since beir/pytrec_eval
are absent (parity unpinned).
"""
from __future__ import annotations

import json
from collections import OrderedDict
from pathlib import Path
from typing import Dict, Optional

import numpy as np

from ._lib import DeviceSparseIndex, csr
from .metrics import ndcg_at_k


class SparseSearch:
    def __init__(self, model, batch_size: int, verbose: bool = False, device: int = 0,
                 encode_batch_size: Optional[int] = None):
        self.model = model
        self.batch_size = batch_size
        self.encode_batch_size = encode_batch_size or max(batch_size, 256)
        self.verbose = verbose
        self.device = device
        self.inverted_index = None  # DeviceSparseIndex once built
        self.vocab: Dict[str, int] = {}
        self.corpus_ids = []

    def _build_inverted_index(self, corpus):
        """nano_beir_evaluator.py:78-101: terms -> postings in corpus order, score > 0."""
        self.corpus_ids = list(corpus.keys())
        texts = list(corpus.values())
        lists: "OrderedDict[str, list]" = OrderedDict()
        bs = self.encode_batch_size
        for s in range(0, len(texts), bs):
            for di, emb in enumerate(self.model.get_impact_scores_batch(texts[s:s + bs]),
                                     start=s):
                for term, score in emb:
                    if score > 0:
                        lists.setdefault(term, []).append((di, np.float32(score)))
        self.vocab = {t: i for i, t in enumerate(lists)}
        term_off = np.zeros(len(lists) + 1, np.int64)
        term_off[1:] = np.cumsum([len(v) for v in lists.values()])
        pdoc = np.fromiter((d for v in lists.values() for d, _ in v), np.uint32,
                           count=int(term_off[-1]))
        pimp = np.fromiter((x for v in lists.values() for _, x in v), np.float32,
                           count=int(term_off[-1]))
        self.inverted_index = DeviceSparseIndex(term_off, pdoc, pimp, len(self.corpus_ids),
                                                self.device)

    def search(self, queries, corpus, k):
        """nano_beir_evaluator.py:103-137: {qid: {doc_id: float(score)}} in rank order."""
        if self.inverted_index is None:
            self._build_inverted_index(corpus)
        qids = list(queries.keys())
        qterms = [[self.vocab[t] for t in self.model.process_query(queries[q]) if t in self.vocab]
                  for q in qids]
        flat, cu = csr(qterms)
        docs, scores, n, _ = self.inverted_index.search_csr(flat, cu, k)
        out = {}
        for i, qid in enumerate(qids):
            out[qid] = {self.corpus_ids[d]: float(s)
                        for d, s in zip(docs[i, :n[i]].tolist(), scores[i, :n[i]].tolist())}
        return out


def _read_local(path: Path):
    corpus, queries, qrels = {}, {}, {}
    with open(path / "corpus.jsonl", encoding="utf-8") as f:
        for line in f:
            x = json.loads(line)
            if len(x["text"]) > 0:
                corpus[x["_id"]] = x["text"]
    with open(path / "queries.jsonl", encoding="utf-8") as f:
        for line in f:
            x = json.loads(line)
            if len(x["text"]) > 0:
                queries[x["_id"]] = x["text"]
    with open(path / "qrels.tsv", encoding="utf-8") as f:
        for line in f:
            p = line.rstrip("\n").split("\t")
            if p[0] == "query-id":
                continue
            qrels.setdefault(p[0], {})[p[1]] = 1
    return corpus, queries, qrels


class NanoBEIREvaluator:
    """evaluate_dataset on local data: (corpus, queries, qrels) dicts or a directory."""

    def __init__(self, batch_size=16, verbose=False, device=0):
        self.batch_size, self.verbose, self.device = batch_size, verbose, device

    def evaluate_dataset(self, model, dataset, k_values=(10, 100, 1000)):
        corpus, queries, qrels = _read_local(Path(dataset)) if isinstance(
            dataset, (str, Path)) else dataset
        searcher = SparseSearch(model, batch_size=self.batch_size, verbose=self.verbose,
                                device=self.device)
        results = searcher.search(queries, corpus, k=1000)
        return {f"NDCG@{k}": ndcg_at_k(qrels, results, k) for k in k_values}, results
