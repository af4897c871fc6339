"""world_size-2 gloo tests of the doc-id-sharded paths (parallel.py).

Each rank holds one contiguous doc-id shard of an index.  The shard scorer is the
oracle (CPU restatement, emitting the same unique 64-bit keys the HIP scorer
emits); the exchange is parallel.ShardedRetriever's all_gather over gloo; the
merge is a numpy restatement of di_topk_merge.  The merged ranking must equal the
unsharded oracle ranking exactly -- scores, docs and the reference's tie order.
"""
import multiprocessing as mp
import os
import socket
import traceback

import numpy as np
import pytest

import oracle
from improving_learned_index_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _random_docs(n_docs, n_vocab, seed):
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(n_docs):
        n = int(rng.integers(0, 12))
        terms = rng.choice(n_vocab, size=n, replace=False)
        # few distinct values -> many score ties across the shard boundary
        docs.append({f"t{t}": float(rng.integers(1, 6)) for t in terms})
    return docs


def _shard(ix, lo, hi):
    """Postings of docs [lo, hi) only, in the full index's per-term order."""
    keep = (ix.pdoc >= lo) & (ix.pdoc < hi)
    sh = object.__new__(oracle.Index)
    sh.vocab = ix.vocab
    counts = np.add.reduceat(keep.astype(np.int64), ix.term_off[:-1]) if keep.size else \
        np.zeros(len(ix.term_off) - 1, np.int64)
    counts[np.diff(ix.term_off) == 0] = 0
    sh.term_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    sh.pdoc = np.ascontiguousarray(ix.pdoc[keep])
    sh.pval = np.ascontiguousarray(ix.pval[keep])
    sh.n_docs = ix.n_docs
    return sh


def _numpy_merge(keys, counts, k):
    """di_topk_merge restated: union of the lists' valid keys, descending, top k."""
    w, nq, _ = keys.shape
    out = np.zeros((nq, k), np.uint64)
    n = np.zeros(nq, np.int32)
    for q in range(nq):
        allk = np.concatenate([keys[r, q, :counts[r, q]] for r in range(w)])
        allk = np.sort(allk)[::-1][:k]
        out[q, :allk.size] = allk
        n[q] = allk.size
    return out, n


def _worker(rank, world, port, index_dir, queries, k, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ix = oracle.Index(index_dir)
        lo, hi = parallel.shard_range(ix.n_docs, world, rank)
        sh = _shard(ix, lo, hi)

        def local(qs):
            _, keys, n = sh.score_ids(qs, k, with_keys=True)
            return keys, n

        res = parallel.ShardedRetriever(k, local, merge=_numpy_merge).search(queries)
        local_max = float(sh.pval.max()) if sh.pval.size else 0.0
        gmax = parallel.global_max(local_max)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res, gmax, (lo, hi)))
    except Exception:
        q.put((rank, traceback.format_exc(), None, None))


def _run(world, index_dir, queries, k):
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, index_dir, queries, k, q))
          for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r, res, gmax, rng = q.get(timeout=120)
        if isinstance(res, str):
            raise AssertionError(f"rank {r} failed:\n{res}")
        out[r] = (res, gmax, rng)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_shard_range_covers():
    for n in (0, 1, 7, 100, 8841823):
        for w in (1, 2, 3, 8):
            rs = [parallel.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


@pytest.mark.parametrize("k", [1, 7, 1000])
def test_sharded_search_matches_single_shard(tmp_path, k):
    docs = _random_docs(600, 80, seed=k)
    vocab, term_off, pdoc, pval = oracle.build_index(docs)
    oracle.write_index(tmp_path, vocab, term_off, pdoc, pval)
    ix = oracle.Index(tmp_path)
    rng = np.random.default_rng(7)
    queries = [list(rng.choice(len(vocab), size=int(rng.integers(0, 6)), replace=False))
               for _ in range(40)]
    queries = [[int(t) for t in qq] for qq in queries]
    full = ix.score_ids(queries, k)
    out = _run(2, str(tmp_path), queries, k)
    for r in range(2):
        res, gmax, _ = out[r]
        assert gmax == float(pval.max())
        assert [[(int(d), int(s)) for d, s in qq] for qq in res] == \
            [[(int(d), int(s)) for d, s in qq] for qq in full]


def test_sharded_search_golden_index():
    """The reference-built golden index (tests/golden/index), sharded over 2 ranks."""
    from conftest import GOLDEN
    import json

    ix = oracle.Index(GOLDEN / "index")
    gold = json.loads((GOLDEN / "score.json").read_text())
    queries = [ix.term_ids(qq) for qq in gold["queries"]]
    out = _run(2, str(GOLDEN / "index"), queries, 1000)
    assert out[0][0] == out[1][0]
    # the reference's own ranking (InvertedIndex.score, set-iteration tie order)
    assert [[[int(d), int(s)] for d, s in qq] for qq in out[0][0]] == gold["top1000"]


def test_sharded_long_queries_match_single_shard(tmp_path):
    """Queries of more than 256 known terms carry wide keys (include/deepimpact.h); the
    sharded exchange decodes them per query length and equals the unsharded ranking."""
    docs = _random_docs(900, 700, seed=5)
    vocab, term_off, pdoc, pval = oracle.build_index(docs)
    oracle.write_index(tmp_path, vocab, term_off, pdoc, pval)
    ix = oracle.Index(tmp_path)
    rng = np.random.default_rng(9)
    queries = [[int(t) for t in rng.choice(len(vocab), size=int(rng.integers(257, 600)),
                                           replace=False)] for _ in range(6)]
    queries += [[int(t) for t in rng.choice(len(vocab), size=3, replace=False)]]
    full = ix.score_ids(queries, 1000)
    out = _run(2, str(tmp_path), queries, 1000)
    for r in range(2):
        assert [[(int(d), int(s)) for d, s in qq] for qq in out[r][0]] == \
            [[(int(d), int(s)) for d, s in qq] for qq in full]


def test_decode_quant_keys():
    """Compact and wide key layouts; a rejected query (n < 0) raises instead of
    emitting keys (the sharded rank path used to write k - 1 garbage lines)."""
    compact = np.array([(300 << 48) | (250 << 40) | (7 << 32) | (0xFFFFFFFF - 123456789)],
                       np.uint64)
    assert parallel.decode_quant_keys(compact, 1, 5) == [(123456789, 300)]
    wide = np.array([(70000 << 44) | (4000 << 32) | (7 << 24) | (0xFFFFFF - 8_800_000)],
                    np.uint64)
    assert parallel.decode_quant_keys(wide, 1, 300) == [(8_800_000, 70000)]
    assert parallel.decode_quant_keys(wide, 0, 300) == []
    with pytest.raises(RuntimeError):
        parallel.decode_quant_keys(compact, -1, 5)


def _quant_worker(rank, world, port, src, out, max_val, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)

        def shard_max(path):
            with open(path, encoding="utf-8") as f:
                vals = [float(s) for line in f for _, s in oracle.parse_impact_line(line)]
            return max([0.0] + vals)

        m = parallel.quantize_sharded(src, out, max_val, world, rank, shard_max,
                                      lambda i, o, mm: oracle.quantize_file(i, o, mm))
        dist.destroy_process_group()
        q.put((rank, m))
    except Exception:
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world,max_val", [(2, None), (3, None), (2, 7.0)])
def test_quantize_sharded_equals_single(tmp_path, world, max_val):
    """parallel.quantize_sharded (the quantize CLI under torchrun): all_reduce(MAX) of
    the shard maxima, per-shard quantize, rank-0 join == the reference file (golden
    q254 fixture: maxima where int(max * 255 / max) = 254)."""
    from conftest import GOLDEN

    src = GOLDEN / "q254.index"
    out = tmp_path / "q.out"
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_quant_worker, args=(r, world, port, src, out, max_val, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for r, m in res:
        assert not isinstance(m, str), m
    if max_val is None:
        assert out.read_bytes() == (GOLDEN / "q254.quantized").read_bytes()
    else:
        want = tmp_path / "want"
        oracle.quantize_file(src, want, max_val)
        assert out.read_bytes() == want.read_bytes()
