"""Sweep of score_item's threshold refresh schedule (DI_TQ_EVERY / DI_TQ_FIRST): device
ms per 6980-query top-1000 batch (score_blocks + merge) per schedule on one shard, the
first 20 queries checked against the oracle.  Profiling only.
    python tools/tq_sweep.py <n_docs> <iid|skew> every:first [every:first ...]
"""
import gc
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
from improving_learned_index_amd import _lib  # noqa: E402
from improving_learned_index_amd import synthetic as S  # noqa: E402

NQ, K = 6980, 1000
n_docs, skew = int(sys.argv[1]), sys.argv[2] == "skew"
term_off, pdoc, pval, _ = S.synth_postings(n_docs, 2 * n_docs, seed=4321,
                                           skew=S.SKEW_CONFIG4 if skew else None)
queries = S.msmarco_like_queries(NQ, 2 * n_docs, seed=1234)
flat, cuq = _lib.csr(queries)
import oracle  # noqa: E402

ora = oracle.Index.__new__(oracle.Index)
ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n_docs
want = ora.score_ids(queries[:20], K, n_threads=16)
rows = []
for rep in range(2):
    for sch in sys.argv[3:]:
        every, first = (int(x) for x in sch.split(":"))
        os.environ["DI_TQ_EVERY"], os.environ["DI_TQ_FIRST"] = str(every), str(first)
        ix = _lib.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n_docs)
        ix.reserve(NQ, K)
        ix.search_csr(flat, cuq, K)  # warm
        best = None
        for _ in range(3):
            ix.timing("score_blocks", reset=True)
            ix.timing("merge_topk", reset=True)
            docs, scores, n = ix.search_csr(flat, cuq, K, timing=True)[:3]
            sb, mg = ix.timing("score_blocks")[0], ix.timing("merge_topk")[0]
            if best is None or sb + mg < best[0] + best[1]:
                best = (sb, mg)
        ok = all(list(zip(docs[i, :n[i]].tolist(), scores[i, :n[i]].tolist())) == want[i]
                 for i in range(20))
        row = {"rep": rep, "every": every, "first": first, "score_blocks_ms": round(best[0], 3),
               "merge_ms": round(best[1], 3), "q_per_s": round(NQ / (best[0] + best[1]) * 1e3, 1),
               "oracle_first20": ok}
        print(json.dumps(row), file=sys.stderr, flush=True)
        rows.append(row)
        del ix
        gc.collect()
print(json.dumps({"n_docs": n_docs, "collection": "skew" if skew else "iid", "rows": rows}))
