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


def _trec_ranked(run: Dict[str, float]):
    """trec_eval's document order: score descending, ties by doc id descending."""
    return [d for d, _ in sorted(run.items(), key=lambda x: (x[1], x[0]), reverse=True)]


def evaluate_retrieval(qrels: Dict[str, Dict[str, int]], results: Dict[str, Dict[str, float]],
                       k_values=(10, 100, 1000), ignore_identical_ids: bool = True):
    """beir EvaluateRetrieval.evaluate (called at nano_beir_evaluator.py:230-231) restated
    on trec_eval's measures (pytrec_eval is absent here -- parity unpinned):
    ndcg_cut.k (gain = relevance, log2(rank + 1) discount), map_cut.k (AP truncated at
    k over the query's relevant count), recall.k, P.k (over k); per-query values are
    averaged over the queries of `results` that have judgments, then rounded to 5
    places.  Returns the (NDCG, MAP, Recall, P) dicts beir returns; with
    ignore_identical_ids (beir's default) a doc whose id equals the query id is
    dropped first."""
    ndcg = {f"NDCG@{k}": 0.0 for k in k_values}
    _map = {f"MAP@{k}": 0.0 for k in k_values}
    recall = {f"Recall@{k}": 0.0 for k in k_values}
    prec = {f"P@{k}": 0.0 for k in k_values}
    n = 0
    for qid, run in results.items():
        rels = qrels.get(qid)
        if rels is None:
            continue
        n += 1
        if ignore_identical_ids and qid in run:
            run = {d: s for d, s in run.items() if d != qid}
        ranked = _trec_ranked(run)
        n_rel = sum(1 for g in rels.values() if g > 0)
        ideal = sorted((g for g in rels.values() if g > 0), reverse=True)
        for k in k_values:
            top = ranked[:k]
            dcg = sum(rels.get(d, 0) / math.log2(i + 2) for i, d in enumerate(top)
                      if rels.get(d, 0) > 0)
            idcg = sum(g / math.log2(i + 2) for i, g in enumerate(ideal[:k]))
            ndcg[f"NDCG@{k}"] += dcg / idcg if idcg > 0 else 0.0
            hits, ap = 0, 0.0
            for i, d in enumerate(top):
                if rels.get(d, 0) > 0:
                    hits += 1
                    ap += hits / (i + 1)
            _map[f"MAP@{k}"] += ap / n_rel if n_rel else 0.0
            recall[f"Recall@{k}"] += hits / n_rel if n_rel else 0.0
            prec[f"P@{k}"] += hits / k
    for m in (ndcg, _map, recall, prec):
        for key in m:
            m[key] = round(m[key] / n, 5) if n else 0.0
    return ndcg, _map, recall, prec


def main(argv=None):
    p = argparse.ArgumentParser("Evaluate a DeepImpact run file.")
    p.add_argument("--run_file_path", type=Path, required=True)
    p.add_argument("--qrels_path", type=Path, required=True)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    print(Metrics(a.run_file_path, a.qrels_path, MRR_DEPTHS, RECALL_DEPTHS).evaluate())


if __name__ == "__main__":
    main()
