"""The pruned exact top-k exchange (parallel.exchange_topk) over gloo, world 2-4.

Every rank holds sorted (descending) u64 key lists per query, as the HIP scorer emits
them; the merge of the exchanged prefixes must equal the merge of the full lists, and
for doc-id shards of one collection each rank must send well under k keys per query
(the 2-rank criterion: <= 0.6 k).
"""
import multiprocessing as mp
import os
import socket
import traceback

import numpy as np
import pytest

from improving_learned_index_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lists(world, nq, k, seed, mode):
    """Per rank [nq, k] uint64 key lists (descending, valid prefix) and counts."""
    rng = np.random.default_rng(seed)
    keys = np.zeros((world, nq, k), np.uint64)
    cnt = np.zeros((world, nq), np.int32)
    for q in range(nq):
        n_all = int(rng.integers(0, 3 * k * world)) if mode == "ragged" else 4 * k * world
        # unique keys: score in the high word (few values -> ties), doc in the low word;
        # u64 order must hold across the sign bit too (high scores)
        score = rng.integers(1, 40, n_all).astype(np.uint64)
        if mode == "ragged" and q % 3 == 0:
            score |= np.uint64(1 << 31)  # keys >= 2^63: unsigned order across the sign
        doc = rng.permutation(1 << 20)[:n_all].astype(np.uint64)
        allk = (score << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - doc)
        owner = rng.integers(0, world, n_all)
        for r in range(world):
            mine = np.sort(allk[owner == r])[::-1][:k]
            keys[r, q, :mine.size] = mine
            cnt[r, q] = mine.size
    if mode == "ragged":
        cnt[0, 1 % nq] = -1  # a rejected query stays flagged
    return keys, cnt


def _merge(keys, counts, k):
    w, nq, _ = keys.shape
    out = []
    for q in range(nq):
        if (counts[:, q] < 0).any():
            out.append(None)
            continue
        allk = np.concatenate([keys[r, q, :counts[r, q]] for r in range(w)])
        out.append(np.sort(allk)[::-1][:k].tolist())
    return out


def _worker(rank, world, port, keys, cnt, k, q, pruned):
    try:
        import torch
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        kt = torch.from_numpy(keys[rank].reshape(-1).view(np.int64).copy())
        ct = torch.from_numpy(cnt[rank].copy())
        st = {}
        gk, gn = parallel.exchange_topk(kt, ct, k, stats=st, pruned=pruned)
        dist.barrier()
        dist.destroy_process_group()
        nq = cnt.shape[1]
        q.put((rank, gk.numpy().view(np.uint64).reshape(world, nq, k), gn.numpy().reshape(world, nq),
               st))
    except Exception:
        q.put((rank, traceback.format_exc(), None, None))


def _run(world, keys, cnt, k, pruned=None):
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, keys, cnt, k, q, pruned)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r, gk, gn, st = q.get(timeout=120)
        if isinstance(gk, str):
            raise AssertionError(f"rank {r} failed:\n{gk}")
        out[r] = (gk, gn, st)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("pruned", [True, None])
@pytest.mark.parametrize("world,k,mode", [(2, 50, "iid"), (3, 40, "ragged"), (4, 3, "ragged"),
                                          (2, 1, "ragged"), (3, 64, "iid"), (1, 40, "ragged"),
                                          (1, 200, "iid")])
def test_exchange_equals_full_gather(world, k, mode, pruned):
    """Forced pruned (world 1 included: the rehearsal a 1-GPU box runs) and the default
    choice (plain below PLAIN_MAX_KEYS keys per rank and at one rank)."""
    nq = 24
    keys, cnt = _lists(world, nq, k, seed=7 + world + k, mode=mode)
    want = _merge(keys, cnt, k)
    out = _run(world, keys, cnt, k, pruned)
    for r, (gk, gn, st) in out.items():
        want_path = "pruned" if parallel.exchange_pruned(world, nq, k, pruned) else "plain"
        assert st["path"] == want_path
        if pruned and k >= 8:
            assert want_path == "pruned"
        got = _merge(gk, gn, k)
        for qi in range(nq):
            assert got[qi] == want[qi], (r, qi)
        # rejected queries keep their negative count
        assert ((gn < 0) == (cnt < 0)).all()


def test_exchange_sends_under_0p6_k_at_two_ranks():
    world, k, nq = 2, 200, 40
    keys, cnt = _lists(world, nq, k, seed=11, mode="iid")
    out = _run(world, keys, cnt, k)
    for r, (_, _, st) in out.items():
        assert st["gathered_keys_per_query"] <= 0.6 * k, st
        assert st["bytes_sent"] < 0.6 * k * 8 * nq + 8 * nq


def test_exchange_auto_choice():
    """Pruned from 2 ranks at PLAIN_MAX_KEYS keys per rank; plain at one rank or below
    it, or when the sample stride would be 1; DI_EXCHANGE overrides the default."""
    big = parallel.PLAIN_MAX_KEYS
    assert parallel.exchange_pruned(2, big // 100 + 1, 100)
    assert not parallel.exchange_pruned(2, big // 100, 100)
    assert not parallel.exchange_pruned(1, 6980, 1000)
    assert parallel.exchange_pruned(1, 6980, 1000, pruned=True)
    assert not parallel.exchange_pruned(8, 6980, 3, pruned=True)  # (g = 1: plain)
    os.environ["DI_EXCHANGE"] = "pruned"
    try:
        assert parallel.exchange_pruned(1, 10, 100)
    finally:
        del os.environ["DI_EXCHANGE"]
