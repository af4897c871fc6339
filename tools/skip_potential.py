"""Exact block-max skip potential of a synthetic collection (CPU, no GPU needed).

For each query: the exact k-th score T (oracle C scorer), and for every scorer wave
segment (block of the shard's nb equal blocks, 16 segments each, as the device index
lays them out) the bound sum over the query's terms of the term's largest value in the
segment.  A segment with bound < T cannot hold a top-k doc: the fraction of such
(query, segment) pairs is what exact (factor 1) block-max skipping can skip at best
(the scorer compares with the running threshold, which is <= T).
    python tools/skip_potential.py [n_docs] [n_queries] [skew|iid]
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
from improving_learned_index_amd import synthetic as S  # noqa: E402


def main():
    n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else 1_100_000
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    skew = (sys.argv[3] if len(sys.argv) > 3 else "skew") == "skew"
    k = 1000
    V = 2 * n_docs
    import os

    sk = dict(S.SKEW_CONFIG4, **json.loads(os.environ.get("SKEW", "{}"))) if skew else None
    term_off, pdoc, pval, m = S.synth_postings(n_docs, V, seed=4321, skew=sk)
    queries = S.msmarco_like_queries(nq, V, seed=1234)
    import oracle

    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n_docs
    res = ora.score_ids(queries, k, n_threads=8)
    nb = (n_docs + 32767) // 32768
    bd = min(32768, ((n_docs + nb - 1) // nb + 63) // 64 * 64)
    seg = (bd + 15) // 16
    n_seg = nb * 16
    skip = tot = bskip = 0
    p_skip = p_tot = 0
    touched_frac = []
    for q, r in zip(queries, res):
        if len(r) < k:
            continue
        T = r[-1][1]
        bound = np.zeros(n_seg, np.int64)
        cnt = np.zeros(n_seg, np.int64)
        for t in q:
            a, b = term_off[t], term_off[t + 1]
            d = pdoc[a:b].astype(np.int64)
            s_id = (d // bd) * 16 + np.minimum((d % bd) // seg, 15)
            mx = np.zeros(n_seg, np.int64)
            np.maximum.at(mx, s_id, pval[a:b].astype(np.int64))
            bound += mx
            cnt += np.bincount(s_id, minlength=n_seg)
        skip += int((bound < T).sum())
        tot += n_seg
        p_skip += int(cnt[bound < T].sum())
        p_tot += int(cnt.sum())
        # whole blocks: sum over the terms of the term's largest value in the block
        bb = np.zeros(nb, np.int64)
        for t in q:
            a, b = term_off[t], term_off[t + 1]
            mx = np.zeros(nb, np.int64)
            np.maximum.at(mx, pdoc[a:b].astype(np.int64) // bd, pval[a:b].astype(np.int64))
            bb += mx
        bskip += int((bb < T).sum())
        touched_frac.append(float(np.mean(bound > 0)))
    post = float(np.mean([sum(int(term_off[t + 1] - term_off[t]) for t in q) for q in queries]))
    print(json.dumps({"n_docs": n_docs, "collection": "skewed (SKEW_CONFIG4)" if skew else "iid (§8d)",
                      "skew": sk, "queries": nq, "k": k,
                      "postings": int(len(pdoc)), "postings_per_query": post,
                      "segment_docs": seg, "segments": n_seg,
                      "skippable_segment_fraction": skip / max(tot, 1),
                      "skippable_posting_fraction": p_skip / max(p_tot, 1),
                      "skippable_block_fraction": bskip / max(tot // 16, 1),
                      "segments_with_any_posting": float(np.mean(touched_frac)),
                      "max_impact": m}))


if __name__ == "__main__":
    main()
