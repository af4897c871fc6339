"""Second-stage re-ranking of a top-k run with the DeepImpact encoder (SURVEY §8f F3;
reference src/deep_impact/evaluation/reranker.py:13-91 and src/deep_impact/rerank.py).

For every query of the top-k run, each candidate passage's term impacts are computed
once (the reference's per-pid cache, reranker.py:52-54) and the passage scores
sum(impact of each query term present) in the query-term iteration order
(reranker.py:56-57); the candidates are then sorted by score, stable, first 1000
(reranker.py:91).  The encoder is the same HIP path as indexing (di_encode, float
impacts without the 3-decimal rounding, as compute_term_impacts gives them); passages
missing from the cache are encoded in batches of `batch_size` across queries rather
than per query, which changes nothing but the batch boundaries.
"""
from __future__ import annotations

import argparse
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Union

import numpy as np

from .datasets import Collection, Queries, RunFile, TopKRunFile
from .models import DeepImpact


class ReRanker:
    def __init__(self, checkpoint_path: Union[str, Path, None], top_k_run_file_path,
                 queries_path, collection_path, output_path, batch_size: int = 128,
                 num_processes: int = 4, model: Optional[DeepImpact] = None,
                 tokenizer_path=None, precision: str = "bf16x3", device: int = 0,
                 variant: str = "xlmr", max_length: Optional[int] = None):
        self.top_k = TopKRunFile(run_file_path=top_k_run_file_path)
        self.queries = Queries(queries_path=queries_path)
        self.collection = Collection(collection_path=collection_path)
        self.batch_size = batch_size
        self.num_processes = num_processes  # tokenization runs in the Rust tokenizer
        self.model = model if model is not None else DeepImpact.load(
            checkpoint_path, tokenizer_path=tokenizer_path, precision=precision,
            device=device, variant=variant, max_length=max_length)
        self.run_file = RunFile(run_file_path=output_path)
        self.cache: Dict[str, Dict[str, np.float32]] = {}

    def save(self, pids: Sequence[str], batch_doc_term_scores) -> None:
        """reranker.py:52-54."""
        for pid, doc_term_scores in zip(pids, batch_doc_term_scores):
            self.cache[pid] = {term: score for term, score in doc_term_scores}

    def score(self, pid, query_terms):
        """reranker.py:56-57: Python sum from int 0 over the query terms' impacts
        (np.float32 adds under numpy >= 2, as in the reference's environment here)."""
        return sum(self.cache[pid].get(term, 0) for term in query_terms)

    def _encode_missing(self, pids: Sequence[str]) -> None:
        todo = list(dict.fromkeys(p for p in pids if p not in self.cache))
        for s in range(0, len(todo), self.batch_size):
            batch = todo[s:s + self.batch_size]
            self.save(batch, self.model.get_impact_scores_batch([self.collection[p] for p in batch]))

    def rerank(self, qid, pids) -> List:
        """reranker.py:59-91."""
        query_terms = DeepImpact.process_query(query=self.queries[qid])
        self._encode_missing(pids)
        scores = [self.score(pid, query_terms) for pid in pids]
        return sorted(zip(pids, scores), key=lambda x: x[1], reverse=True)[:1000]

    def run(self) -> None:
        """reranker.py:43-48."""
        for qid, pids in self.top_k:
            self.run_file.writelines(qid, self.rerank(qid, pids))


def main(argv=None):
    p = argparse.ArgumentParser(
        "Evaluate a DeepImpact model by reranking TopK dataset and computing evaluation metrics.")
    p.add_argument("--checkpoint_path", type=Path, required=True)
    p.add_argument("--top_k_run_file_path", type=Path, required=True)
    p.add_argument("--queries_path", type=Path, required=True)
    p.add_argument("--collection_path", type=Path, required=True)
    p.add_argument("--output_path", type=Path, required=True)
    p.add_argument("--batch_size", type=int, default=128)
    p.add_argument("--num_processes", type=int, default=4)
    p.add_argument("--tokenizer_path", type=str, default=None)
    p.add_argument("--precision", choices=["bf16x3", "fp32", "bf16"], default="bf16x3",
                   help="bf16x3 (default): fp32-faithful split-bf16; fp32: f32 MFMA; "
                        "bf16: throughput mode, NOT fp32-faithful (different round3 text)")
    p.add_argument("--device", type=int, default=0)
    p.add_argument("--variant", choices=["xlmr", "bert"], default="xlmr")
    p.add_argument("--max_length", type=int, default=None)
    args = p.parse_args(argv)
    ReRanker(**vars(args)).run()


if __name__ == "__main__":
    main()
