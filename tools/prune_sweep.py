"""BASELINE configs[4] sweep: queries/s vs recall@1000 of query-time impact pruning
(di_index_set_min_impact) on the bench shard (100k docs, 6980 dev.small-shaped
queries, top-1000).  Recall@1000 = |pruned top-1000 ∩ exact top-1000| / |exact|,
averaged over queries; bytes = 4 B per posting actually scored.  One JSON line.
    python tools/prune_sweep.py > profiles/r01_prune_sweep.json
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from improving_learned_index_amd import _lib  # noqa: E402
from improving_learned_index_amd import synthetic as S  # noqa: E402


def main():
    n_docs, v_terms, nq, k = 100_000, 200_000, 6980, 1000
    cu, term, imp = S.msmarco_like_docs(n_docs, v_terms, seed=1234)
    q, _ = S.quantize_like_reference(imp)
    term_off, pdoc, pval = S.postings_reference_order(cu, term, q, v_terms)
    ix = _lib.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n_docs)
    queries = S.msmarco_like_queries(nq, v_terms, seed=1234)
    flat, cuq = _lib.csr(queries)
    ix.reserve(nq, k)
    rows, exact = [], None
    for mi in (1, 2, 4, 8, 16, 32, 64, 128):
        ix.set_min_impact(mi)
        thr = 1 << (mi.bit_length() - 1)
        posts = sum(int((pval[term_off[t]:term_off[t + 1]] >= thr).sum())
                    for qq in queries for t in qq)
        ix.search_csr(flat, cuq, k)  # warm
        ix.timing("score_blocks", reset=True)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            docs, _, n, _ = ix.search_csr(flat, cuq, k, timing=True)
        wall = (time.perf_counter() - t0) / reps
        ms_sb, n_sb = ix.timing("score_blocks")
        ms_mg, n_mg = ix.timing("merge_topk")
        kern = (ms_sb / max(n_sb, 1) + ms_mg / max(n_mg, 1)) / 1000.0
        res = [set(docs[i, :n[i]].tolist()) for i in range(nq)]
        if exact is None:
            exact = res
        rec = float(np.mean([len(a & b) / max(len(b), 1) for a, b in zip(res, exact)]))
        rows.append({"min_impact": mi, "postings_per_query": posts / nq,
                     "device_queries_per_s": nq / kern, "host_call_queries_per_s": nq / wall,
                     "score_blocks_ms": ms_sb / max(n_sb, 1), "recall_at_1000": rec})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"sweep": "query-time impact pruning (di_index_set_min_impact)",
                      "workload": "100k-doc shard, 6980 dev.small-shaped queries, top-1000",
                      "rows": rows}))


if __name__ == "__main__":
    torch.cuda.init() if torch.cuda.is_available() else None
    main()
