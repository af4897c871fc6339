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
from .metrics import evaluate_retrieval, ndcg_at_k  # noqa: F401


class SparseSearch:
    def __init__(self, model, batch_size: int, verbose: bool = False, device: int = 0,
                 encode_batch_size: Optional[int] = None, accumulation: str = "f32"):
        """accumulation: "f32" -- `0.0 + np.float32` under numpy >= 2; "f64" -- under the
        reference's pinned numpy 1.25.1 (f64 doc scores)."""
        if accumulation not in ("f32", "f64"):
            raise ValueError(f"accumulation must be 'f32' or 'f64', not {accumulation!r}")
        self.accumulation = accumulation
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
        docs, scores, n, _ = self.inverted_index.search_csr(flat, cu, k,
                                                            accumulation=self.accumulation)
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


# nano_beir_evaluator.py:30-60: the 13 NanoBEIR datasets (hub ids zeta-alpha-ai/Nano*)
MAPPING_DATASET_NAME_TO_HUMAN_READABLE = {
    "climatefever": "ClimateFEVER", "dbpedia": "DBPedia", "fever": "FEVER",
    "fiqa2018": "FiQA2018", "hotpotqa": "HotpotQA", "msmarco": "MSMARCO",
    "nfcorpus": "NFCorpus", "nq": "NQ", "quoraretrieval": "QuoraRetrieval",
    "scidocs": "SCIDOCS", "arguana": "ArguAna", "scifact": "SciFact",
    "touche2020": "Touche2020",
}
MAPPING_DATASET_NAME_TO_ID = {k: f"zeta-alpha-ai/Nano{v}"
                              for k, v in MAPPING_DATASET_NAME_TO_HUMAN_READABLE.items()}
K_VALUES = (10, 100, 1000)  # nano_beir_evaluator.py:231


class NanoBEIREvaluator:
    """nano_beir_evaluator.py:153-232 on local data.  A dataset is a (corpus, queries,
    qrels) tuple of dicts or a directory with corpus.jsonl / queries.jsonl / qrels.tsv
    (the hub's NanoBEIR files); ``evaluate_all`` walks ``data_dir``/Nano<Name> for the
    13 datasets (those present) and adds their average as metrics["avg"]."""

    def __init__(self, batch_size=16, verbose=False, device=0, data_dir=None,
                 accumulation="f32"):
        self.batch_size, self.verbose, self.device = batch_size, verbose, device
        self.accumulation = accumulation
        self.data_dir = Path(data_dir) if data_dir is not None else None

    def _load_dataset(self, dataset):
        if isinstance(dataset, (str, Path)):
            p = Path(dataset)
            if not p.exists() and self.data_dir is not None:
                name = MAPPING_DATASET_NAME_TO_HUMAN_READABLE.get(str(dataset), str(dataset))
                p = self.data_dir / f"Nano{name}"
            return _read_local(p)
        return dataset

    def search(self, model, dataset, k=1000):
        corpus, queries, qrels = self._load_dataset(dataset)
        searcher = SparseSearch(model, batch_size=self.batch_size, verbose=self.verbose,
                                device=self.device, accumulation=self.accumulation)
        return searcher.search(queries, corpus, k=k), qrels

    def evaluate_dataset(self, model, dataset):
        """(NDCG, MAP, Recall, P) dicts at k = 10, 100, 1000 (beir's evaluate)."""
        results, qrels = self.search(model, dataset, k=1000)
        return evaluate_retrieval(qrels, results, K_VALUES)

    def evaluate_all(self, model, data_dir=None):
        root = Path(data_dir) if data_dir is not None else self.data_dir
        if root is None:
            raise ValueError("evaluate_all needs data_dir (the hub is unreachable offline)")
        metrics = {}
        for name, human in MAPPING_DATASET_NAME_TO_HUMAN_READABLE.items():
            d = root / f"Nano{human}"
            if not d.is_dir():
                continue
            if self.verbose:
                print(f"Evaluating dataset {name}...")
            metrics[name] = self.evaluate_dataset(model, d)
            if self.verbose:
                print(f"Metrics for {name}: {metrics[name]}")
        if not metrics:
            raise FileNotFoundError(f"no Nano<Name> dataset directory under {root}")
        metrics["avg"] = tuple(
            {key: sum(metrics[n][i][key] for n in metrics) / len(metrics) for key in m}
            for i, m in enumerate(next(iter(metrics.values()))))
        return metrics


def main(argv=None):
    """nano_beir_evaluator.py:236-243 (the reference loads soyuj/deeper-impact from the
    hub; here a local checkpoint + tokenizer and local NanoBEIR directories)."""
    import argparse

    from .models import DeepImpact

    p = argparse.ArgumentParser("NanoBEIR evaluation of a DeepImpact checkpoint.")
    p.add_argument("--data_dir", type=Path, required=True,
                   help="directory holding Nano<Name>/{corpus.jsonl,queries.jsonl,qrels.tsv}")
    p.add_argument("--model_checkpoint_path", type=str, required=True)
    p.add_argument("--tokenizer_path", type=str, default=None)
    p.add_argument("--variant", choices=["xlmr", "bert"], default="bert")
    p.add_argument("--precision", choices=["bf16x3", "fp32", "bf16"], default="bf16x3")
    p.add_argument("--max_length", type=int, default=None)
    p.add_argument("--batch_size", type=int, default=16)
    p.add_argument("--device", type=int, default=0)
    p.add_argument("--dataset", type=str, default=None, help="one dataset name only")
    p.add_argument("--accumulation", choices=["f32", "f64"], default="f32",
                   help="doc-score sums: f32 (numpy >= 2) or f64 (the reference's numpy 1.25.1)")
    a = p.parse_args(argv)
    model = DeepImpact.load(a.model_checkpoint_path, tokenizer_path=a.tokenizer_path,
                            precision=a.precision, device=a.device, variant=a.variant,
                            max_length=a.max_length)
    ev = NanoBEIREvaluator(batch_size=a.batch_size, verbose=True, device=a.device,
                           data_dir=a.data_dir, accumulation=a.accumulation)
    out = ev.evaluate_dataset(model, a.dataset) if a.dataset else ev.evaluate_all(model)
    print(out)
    return out


if __name__ == "__main__":
    main()
