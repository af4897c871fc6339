"""MRR@k / Recall@k over a run file (reference src/deep_impact/evaluation/metrics.py:26-57,
src/deep_impact/evaluate.py) and a trec_eval-style nDCG@k for the NanoBEIR path
(replaces beir.EvaluateRetrieval, nano_beir_evaluator.py:230-231; beir/pytrec_eval
are not installed -- nDCG parity unpinned)."""
from __future__ import annotations

import argparse
import logging
import math
from collections import defaultdict
from pathlib import Path
from typing import Dict, List

from .datasets import QueryRelevanceDataset, RunFile

MRR_DEPTHS = [10]
RECALL_DEPTHS = [3, 10, 20, 50] + list(range(100, 1001, 100))
logger = logging.getLogger("metrics")


class Metrics:
    def __init__(self, run_file_path, qrels_path, mrr_depths: List[int], recall_depths: List[int]):
        self.run_file = RunFile(run_file_path=run_file_path)
        self.qrels = QueryRelevanceDataset(qrels_path=qrels_path)
        self.mrr_sums = {d: 0 for d in mrr_depths}
        self.recall_sums = {d: 0 for d in recall_depths}

    def evaluate(self):
        ranks = defaultdict(list)
        for qid, pid, rank, _ in self.run_file.read():
            if pid not in self.qrels[qid]:
                continue
            ranks[qid].append(rank)
        for qid, rs in ranks.items():
            rs.sort()
            best = rs[0]
            for d in self.mrr_sums:
                if best <= d:
                    self.mrr_sums[d] += 1.0 / best
            for d in self.recall_sums:
                self.recall_sums[d] += len([0 for i in rs if i <= d]) / len(self.qrels[qid])
        n = len(self.qrels)
        out = {}
        for d in sorted(self.mrr_sums):
            out[f"MRR@{d}"] = round(self.mrr_sums[d] / n, 3)
            logger.info(f"MRR@{d} = {out[f'MRR@{d}']}")
        for d in sorted(self.recall_sums):
            out[f"Recall@{d}"] = round(self.recall_sums[d] / n, 3)
            logger.info(f"Recall@{d} = {out[f'Recall@{d}']}")
        return out


def ndcg_at_k(qrels: Dict[str, Dict[str, int]], results: Dict[str, Dict[str, float]], k: int):
    """trec_eval ndcg_cut.k: gain = relevance, log2(rank + 1) discount; documents
    ranked by score descending, ties by doc id descending (trec_eval's order);
    mean over the queries present in qrels."""
    vals = []
    for qid, rels in qrels.items():
        run = results.get(qid, {})
        ranked = sorted(run.items(), key=lambda x: (x[1], x[0]), reverse=True)[:k]
        dcg = sum(rels.get(d, 0) / math.log2(i + 2) for i, (d, _) in enumerate(ranked))
        ideal = sorted(rels.values(), reverse=True)[:k]
        idcg = sum(g / math.log2(i + 2) for i, g in enumerate(ideal))
        vals.append(dcg / idcg if idcg > 0 else 0.0)
    return sum(vals) / len(vals) if vals else 0.0


def main(argv=None):
    p = argparse.ArgumentParser("Evaluate a DeepImpact run file.")
    p.add_argument("--run_file_path", type=Path, required=True)
    p.add_argument("--qrels_path", type=Path, required=True)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    print(Metrics(a.run_file_path, a.qrels_path, MRR_DEPTHS, RECALL_DEPTHS).evaluate())


if __name__ == "__main__":
    main()
