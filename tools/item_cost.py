"""Per-item cost model of score_blocks (configs[4] / verdict r5 item 6, option b).

For each shard (n_docs, collection) it times one 6980-query top-1000 batch at several
impact-pruning levels (min_impact m keeps the postings of value >= m: the items stay,
their postings shrink) and with exact block-max (f = 1), and reads workgroup 0's phase
stamps (DI_PROFILE_ABLATE=64, printed by the library on stderr).  A least-squares fit
  score_blocks_ms = n_items / 256 * (t_item + t_post * postings_per_item)
separates the per-item fixed cost from the per-posting cost; with the oracle's final
k-th score per query (tools/skip_potential.py's measure, recomputed here on a sample of
queries) it bounds what exact skipping of 2 K-doc wave segments can save:
  saving <= t_post * (postings in segments whose bound is below the final k-th score).
Profiling only.
    DI_PROFILE_ABLATE=64 python tools/item_cost.py 1100000 iid  8800000 skew  > out.json
"""
import json
import os
import re
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
from improving_learned_index_amd import _lib  # noqa: E402
from improving_learned_index_amd import synthetic as S  # noqa: E402

NQ, K = 6980, 1000
PH = re.compile(r"setup (\d+) scatter (\d+) hist (\d+) \[count (\d+)\] write (\d+) ties (\d+) "
                r"copy (\d+) tq-select (\d+) \[tq-read (\d+)\] scatter-loop slowest wave (\d+) "
                r"mean wave (\d+)")
_PREV = None
NAMES = ("setup", "scatter", "hist", "count", "write", "ties", "copy", "tq_select", "tq_read",
         "wave_max", "wave_mean")


def stamps_of(fn):
    """Run fn() with fd 2 captured; return the last phase line's counters (cumulative)."""
    with tempfile.TemporaryFile(mode="w+b") as tf:
        sys.stderr.flush()
        old = os.dup(2)
        os.dup2(tf.fileno(), 2)
        try:
            fn()
        finally:
            sys.stderr.flush()
            os.dup2(old, 2)
            os.close(old)
        tf.seek(0)
        txt = tf.read().decode(errors="replace")
    m = None
    for m in PH.finditer(txt):
        pass
    return dict(zip(NAMES, map(int, m.groups()))) if m else None


def shard(n_docs, skew):
    t_off, pd, pv, _ = S.synth_postings(n_docs, 2 * n_docs, seed=4321,
                                        skew=S.SKEW_CONFIG4 if skew else None)
    return t_off, pd, pv


def measure(n_docs, skew):
    term_off, pdoc, pval = shard(n_docs, skew)
    queries = S.msmarco_like_queries(NQ, 2 * n_docs, seed=1234)
    flat, cuq = _lib.csr(queries)
    ix = _lib.DeviceIndex.from_postings(term_off, pdoc, pval, 0, n_docs)
    ix.reserve(NQ, K)
    nb = ix.info()["n_blocks"]
    items = NQ * nb
    lens = np.diff(term_off)
    rows = []
    global _PREV
    for m, f in ((1, 0.0), (2, 0.0), (8, 0.0), (32, 0.0), (128, 0.0), (1, 1.0)):
        ix.set_min_impact(m)
        ix.set_block_max(f)
        ix.search_csr(flat, cuq, K)  # warm
        ix.timing("score_blocks", reset=True)
        ix.timing("merge_topk", reset=True)
        ix.timing("bm_segments", reset=True)
        ix.timing("bm_segments_skipped", reset=True)
        st = stamps_of(lambda: ix.search_csr(flat, cuq, K, timing=True))
        ms = ix.timing("score_blocks")[0]
        mg = ix.timing("merge_topk")[0]
        # postings scored per query at this level (values >= m)
        if m == 1:
            ppq = float(sum(int(lens[np.asarray(q, np.int64)].sum()) for q in queries)) / NQ
        else:
            keep = (pval >= m).astype(np.int64)
            cum = np.concatenate([[0], np.cumsum(keep)])
            ppq = float(sum(int((cum[term_off[np.asarray(q, np.int64) + 1]] -
                                 cum[term_off[np.asarray(q, np.int64)]]).sum()) for q in queries)) / NQ
        # stamps are cumulative over the process: this search's share
        d = None
        if st:
            # (the library's stamp counters are process-wide: previous shards included)
            d = {k: st[k] - (_PREV[k] if _PREV else 0) for k in st}
            _PREV = st
            # (the warm-up search adds as much again: halve)
            d = {k: v / 2.0 for k, v in d.items()}
        wg0_items = items / min(items, 256)
        row = {"min_impact": m, "block_max": f, "score_blocks_ms": round(ms, 3),
               "merge_ms": round(mg, 3), "postings_per_query": round(ppq, 1),
               "postings_per_item": round(ppq / nb, 1),
               "us_per_item_per_cu": round(ms * 1e3 * 256 / items, 3)}
        if d:
            tot = sum(d[k] for k in ("setup", "scatter", "hist", "write", "ties", "copy",
                                     "tq_select"))
            row["phase_cycles_per_item_wg0"] = {k: round(v / wg0_items, 1) for k, v in d.items()}
            row["phase_share_wg0"] = {k: round(d[k] / tot, 3) for k in
                                      ("setup", "scatter", "hist", "write", "ties", "copy",
                                       "tq_select") if tot}
        if f > 0:
            seg, skp = ix.timing("bm_segments")[1], ix.timing("bm_segments_skipped")[1]
            row["bm_segments_skipped_frac"] = round(skp / max(seg, 1), 4)
        print(json.dumps(row), file=sys.stderr, flush=True)
        rows.append(row)
    ix.set_min_impact(1)
    ix.set_block_max(0.0)
    # least squares over the pruning levels (block-max off): ms * 256 / items =
    # t_item + t_post * postings_per_item
    xs = np.array([r["postings_per_item"] for r in rows if r["block_max"] == 0])
    ys = np.array([r["us_per_item_per_cu"] for r in rows if r["block_max"] == 0])
    A = np.stack([np.ones_like(xs), xs], 1)
    (t_item, t_post), *_ = np.linalg.lstsq(A, ys, rcond=None)
    resid = ys - A @ np.array([t_item, t_post])
    exh = rows[0]
    # exact skipping bound: the postings of (query, wave segment) pairs whose bound is
    # below the query's final k-th score, from the oracle on a query sample
    skippable = skip_share(term_off, pdoc, pval, n_docs, queries[:200])
    post_part = t_post * exh["postings_per_item"]
    best = exh["us_per_item_per_cu"] - post_part * skippable
    model = {"t_item_us": round(float(t_item), 3), "t_post_ns": round(float(t_post) * 1e3, 4),
             "fit_max_abs_resid_us": round(float(np.abs(resid).max()), 3),
             "exhaustive_us_per_item": exh["us_per_item_per_cu"],
             "posting_part_of_exhaustive": round(post_part / exh["us_per_item_per_cu"], 3),
             "skippable_posting_share_final_kth": round(skippable, 4),
             "exact_skip_best_case_speedup": round(exh["us_per_item_per_cu"] / best, 4),
             "speedup_needed": 1.10}
    return {"n_docs": n_docs, "collection": "skew" if skew else "iid", "blocks": nb,
            "items": items, "rows": rows, "model": model}


def skip_share(term_off, pdoc, pval, n_docs, queries):
    """Share of the sample's postings lying in (query, block, wave segment) triples whose
    upper bound (sum over the query's terms of the segment's largest value) is below the
    query's final k-th score (oracle) -- what exact (f = 1) segment skipping could skip
    if its running threshold were the final one already."""
    import oracle

    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval, ora.n_docs = term_off, pdoc, pval, n_docs
    want = ora.score_ids(queries, K, n_threads=16)
    nb = (n_docs + 32767) // 32768
    bd = (n_docs + nb - 1) // nb
    wseg = (bd + 15) // 16
    tot = skip = 0
    for q, w in zip(queries, want):
        if len(w) < K:
            for t in q:
                tot += int(term_off[t + 1] - term_off[t])
            continue
        T = w[-1][1]
        segs = {}
        ub = None
        for t in q:
            lo, hi = int(term_off[t]), int(term_off[t + 1])
            d = pdoc[lo:hi].astype(np.int64)
            v = pval[lo:hi].astype(np.int64)
            sid = (d // bd) * 16 + (d % bd) // wseg
            mx = np.zeros(nb * 16, np.int64)
            np.maximum.at(mx, sid, v)
            cnt = np.bincount(sid, minlength=nb * 16)
            ub = mx if ub is None else ub + mx
            segs[t] = cnt
        below = ub < T
        for t in q:
            tot += int(segs[t].sum())
            skip += int(segs[t][below].sum())
    return skip / max(tot, 1)


def main():
    a = sys.argv[1:]
    out = []
    for i in range(0, len(a), 2):
        t0 = time.time()
        out.append(measure(int(a[i]), a[i + 1] == "skew"))
        print(f"{a[i]} {a[i + 1]} done in {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    print(json.dumps({"tool": "tools/item_cost.py", "k": K, "queries": NQ, "shards": out}))


if __name__ == "__main__":
    main()
