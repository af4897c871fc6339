"""Scorer phase stamps (DI_PROFILE_ABLATE=64, workgroup 0) and device ms per batch at one
impact-pruning level, to see where a pruned (query, block) item's time goes.
Profiling only (the stamps change nothing but timing).
    DI_PROFILE_ABLATE=64 python tools/phase_prune.py <n_docs> <min_impact> [skew] [bm]
(skew: synthetic.SKEW_CONFIG4; bm: block-max factor, default 0 = off)
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from improving_learned_index_amd import _lib  # noqa: E402
from improving_learned_index_amd import synthetic as S  # noqa: E402

n_docs, mi = int(sys.argv[1]), int(sys.argv[2])
skew = len(sys.argv) > 3 and sys.argv[3] == "skew"
bm = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
nq, k = 6980, 1000
def collection():
    """The synthetic collection; SYNTH_CACHE=<dir> keeps it as .npy files between runs
    (the PMC passes of tools/measure.sh run this script once per counter group)."""
    import os
    import numpy as np
    cache = os.environ.get("SYNTH_CACHE")
    tag = f"{n_docs}_{'skew' if skew else 'iid'}"
    if cache and os.path.exists(f"{cache}/{tag}_pval.npy"):
        return tuple(np.load(f"{cache}/{tag}_{n}.npy") for n in ("term_off", "pdoc", "pval"))
    t_off, pd, pv, _ = S.synth_postings(n_docs, 2 * n_docs, seed=4321,
                                        skew=S.SKEW_CONFIG4 if skew else None)
    if cache:
        os.makedirs(cache, exist_ok=True)
        for n, a in (("term_off", t_off), ("pdoc", pd), ("pval", pv)):
            np.save(f"{cache}/{tag}_{n}.npy", a)
    return t_off, pd, pv


term_off, pdoc, pval = collection()
flat, cuq = _lib.csr(S.msmarco_like_queries(nq, 2 * n_docs, seed=1234))
ix = _lib.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n_docs)
ix.reserve(nq, k)
ix.set_min_impact(mi)
ix.set_block_max(bm)
ix.search_csr(flat, cuq, k)
print("---- timed", file=sys.stderr, flush=True)
ix.timing("score_blocks", reset=True)
ix.search_csr(flat, cuq, k, timing=True)
nb = (n_docs + 32767) // 32768
ms = ix.timing("score_blocks")[0]
print(f"n_docs {n_docs} min_impact {mi} items {nq * nb} score_blocks {ms:.3f} ms "
      f"({ms * 1e3 * 256 / (nq * nb):.2f} us per item per CU)", flush=True)
