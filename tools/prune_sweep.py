"""BASELINE configs[4] sweep: queries/s vs recall@1000 on a full-scale shard.

Two knobs of the scorer, on a full-scale collection (default: full MS MARCO-sized,
8.8M docs on one GPU; the bench's generator, V = 2 N) with 6980 dev.small-shaped
queries at top-1000:
  * query-time impact pruning (di_index_set_min_impact): score only postings of value
    >= 2^floor(log2 m) -- approximate, the recall column measures it;
  * block-max skipping (di_index_set_block_max): factor 1 exact (recall 1.0 by
    construction, checked here), > 1 approximate.
Recall@1000 = |pruned top-1000 ∩ exact top-1000| / |exact|, averaged over queries.
Device time per batch = score_blocks + merge_topk over all the batch's launches (both
reported per row).
Block-max rows also carry the scorer's skip counters (segments evaluated / skipped).
    python tools/prune_sweep.py [n_docs] [iid|skew] > profiles/<round>_prune_sweep.json
skew: synthetic.SKEW_CONFIG4 (frequent terms carry small impacts, doc mass shared by
clusters of consecutive ids -- a stated deviation from SURVEY §8d's i.i.d. impacts).
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from improving_learned_index_amd import _lib  # noqa: E402
from improving_learned_index_amd import synthetic as S  # noqa: E402


def run(ix, flat, cuq, nq, k, reps=3):
    ix.search_csr(flat, cuq, k)  # warm
    ix.timing("score_blocks", reset=True)
    ix.timing("merge_topk", reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        docs, _, n, _ = ix.search_csr(flat, cuq, k, timing=True)
    wall = (time.perf_counter() - t0) / reps
    score_ms = ix.timing("score_blocks")[0] / reps / 1000.0
    merge_ms = ix.timing("merge_topk")[0] / reps / 1000.0
    return docs, n, (score_ms + merge_ms, score_ms, merge_ms), wall


def main():
    n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else 8_800_000
    skew = len(sys.argv) > 2 and sys.argv[2] == "skew"
    v_terms, nq, k = 2 * n_docs, 6980, 1000
    term_off, pdoc, pval, _ = S.synth_postings(n_docs, v_terms, seed=4321,
                                               skew=S.SKEW_CONFIG4 if skew else None)
    queries = S.msmarco_like_queries(nq, v_terms, seed=1234)
    flat, cuq = _lib.csr(queries)
    rows, exact = [], None
    ix = _lib.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n_docs)
    ix.reserve(nq, k)
    lens = np.diff(term_off)
    rows_sel = [(m, 0.0, False) for m in (1, 2, 4, 8, 16, 32, 64, 128)] + \
        [(1, f, False) for f in (1.0, 1.25, 1.5, 2.0, 3.0, 4.0)] + \
        [(1, f, True) for f in (0.0, 1.0, 1.5, 2.0)]
    if os.environ.get("SWEEP") == "bm":  # exhaustive + the block-max rows only
        rows_sel = [(1, 0.0, False)] + [(1, f, False) for f in (1.0, 1.5, 2.0)]
    elif os.environ.get("SWEEP") == "exh":  # the exhaustive row only
        rows_sel = [(1, 0.0, False)]
    packed_bytes = None
    for mi, bm, pk in rows_sel:
        ix.set_min_impact(mi)
        ix.set_block_max(bm)
        nb = ix.set_packed(pk)
        if pk:
            packed_bytes = nb
        thr = 1 << (mi.bit_length() - 1)
        if thr == 1:
            per_term = lens
        else:  # postings of value >= thr per term (empty terms: reduceat's quirk masked)
            per_term = np.add.reduceat((pval >= thr).astype(np.int64),
                                       np.minimum(term_off[:-1], max(len(pval) - 1, 0)))
            per_term[lens == 0] = 0
        posts = int(per_term[flat.astype(np.int64)].sum())
        ix.timing("bm_segments", reset=True)
        ix.timing("bm_segments_skipped", reset=True)
        docs, n, (dev_s, score_s, merge_s), wall = run(ix, flat, cuq, nq, k)
        seg_n = ix.timing("bm_segments")[1]
        seg_s = ix.timing("bm_segments_skipped")[1]
        res = [set(docs[i, :n[i]].tolist()) for i in range(nq)]
        if exact is None:
            exact = res
        rec = float(np.mean([len(a & b) / max(len(b), 1) for a, b in zip(res, exact)]))
        ratio = packed_bytes / (4.0 * len(pval)) if pk else 1.0
        rows.append({"min_impact": mi, "block_max_factor": bm, "packed": pk,
                     # algorithmic bytes read per query: 4 B per plain posting; packed --
                     # the index's packed bytes per posting (headers included) x postings
                     "bytes_per_query": 4.0 * ratio * posts / nq,
                     "postings_per_query": posts / nq, "device_queries_per_s": nq / dev_s,
                     "host_call_queries_per_s": nq / wall, "device_ms": dev_s * 1000,
                     "score_blocks_ms": score_s * 1000, "merge_ms": merge_s * 1000,
                     "recall_at_1000": rec,
                     "bm_segments_skipped_frac": seg_s / seg_n if seg_n else None})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    del ix
    print(json.dumps({"sweep": "configs[4]: query-time impact pruning and block-max "
                               "skipping of the quantized scorer",
                      "workload": f"{n_docs}-doc shard (synth_postings seed 4321"
                                  f"{', skew SKEW_CONFIG4' if skew else ''}), {nq} "
                                  f"dev.small-shaped queries, top-{k}",
                      "skew": S.SKEW_CONFIG4 if skew else None,
                      "postings": int(len(pval)), "plain_bytes": 4 * int(len(pval)),
                      "packed_bytes": packed_bytes,
                      "rows": rows}))


if __name__ == "__main__":
    import torch

    torch.cuda.init()
    main()
