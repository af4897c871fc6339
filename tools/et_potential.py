"""How much could exact block-max skipping save on the synthetic collection?

For each query: the exact top-1000 threshold T (the 1000th score), and per R-doc range
the block-max upper bound UB = sum over the query terms of the range's max value.  A
range with UB < T can be skipped exactly (block-max WAND); the fraction of ranges /
postings with UB >= T must still be scored.  CPU only (numpy), one JSON line.
    python tools/et_potential.py > profiles/r02_et_potential.json
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from improving_learned_index_amd import synthetic as S  # noqa: E402


def main(n_docs=1_100_000, n_q=40, v_terms=None):
    v_terms = v_terms or 2 * n_docs  # V scales with N
    to, pd, pv, _ = S.synth_postings(n_docs, v_terms, seed=4321)
    qs = S.msmarco_like_queries(n_q, v_terms, seed=1234)
    out = {}
    for R in (64, 256, 2048, 32768):
        alive, post_alive = [], []
        for q in qs:
            sc = np.zeros(n_docs, np.int64)
            ub = np.zeros((n_docs + R - 1) // R, np.int64)
            tot = 0
            for t in q:
                d = pd[to[t]:to[t + 1]].astype(np.int64)
                v = pv[to[t]:to[t + 1]].astype(np.int64)
                sc[d] += v
                tot += len(d)
                mx = np.zeros_like(ub)
                np.maximum.at(mx, d // R, v)
                ub += mx
            T = np.sort(sc)[-1000] if (sc > 0).sum() >= 1000 else 0
            a = ub >= T
            alive.append(float(a.mean()))
            pa = sum(int(a[pd[to[t]:to[t + 1]].astype(np.int64) // R].sum()) for t in q)
            post_alive.append(pa / max(tot, 1))
        out[str(R)] = {"alive_ranges": float(np.mean(alive)),
                       "alive_postings": float(np.mean(post_alive))}
    print(json.dumps({"workload": f"{n_docs}-doc synthetic shard, V = {v_terms}, {n_q} queries, "
                                  "top-1000", "by_range_docs": out}))


if __name__ == "__main__":
    main(v_terms=int(sys.argv[1]) if len(sys.argv) > 1 else None)
