"""The device steps of the pruned exact top-k exchange (exchange.hip: di_xchg_sample /
count / offsets / pack / unpack) on the GPU, with the collectives replaced by
concatenation over W virtual ranks in one process: the gathered prefixes must be
exactly the ones the exchange's definition selects (T_q = the ceil(k/g)-th largest
sample of the union, every key >= T_q), and their merge must equal the merge of the
full lists (parallel.exchange_topk; /root/reference/src/deep_impact/evaluation/
ranker.py:43-48 keeps the global top-k).  Lists as test_exchange_cpu builds them:
ragged counts, rejected queries, keys past the sign bit."""
import numpy as np
import pytest
import torch

from test_exchange_cpu import _lists, _merge

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from improving_learned_index_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible (GPU test run without a GPU)")
    return _lib


def _run_device_steps(L, keys, cnt, k, g):
    lib, P = L.lib(), L.ptr
    W, nq, _ = keys.shape
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    Ks = [torch.from_numpy(keys[r].reshape(-1).view(np.int64).copy()).to(dev) for r in range(W)]
    Cs = [torch.from_numpy(cnt[r].copy()).to(dev) for r in range(W)]
    s_n = k // g
    smp = []
    for r in range(W):
        s = torch.empty(nq * s_n, dtype=torch.int64, device=dev)
        L.check(lib.di_xchg_sample(P(Ks[r]), P(Cs[r]), nq, k, g, P(s), 0, st))
        smp.append(s)
    gs = torch.cat(smp)
    ecs = []
    for r in range(W):
        ec = torch.empty(2 * nq, dtype=torch.int32, device=dev)
        L.check(lib.di_xchg_count(P(gs), W, P(Ks[r]), P(Cs[r]), nq, k, g, P(ec), 0, st))
        ecs.append(ec)
    gec = torch.cat(ecs)
    off = torch.empty(W * nq, dtype=torch.int64, device=dev)
    tot = torch.empty(W, dtype=torch.int64, device=dev)
    L.check(lib.di_xchg_offsets(P(gec), W, nq, P(off), P(tot), 0, st))
    emax = int(tot.max().item())
    g2 = torch.zeros(W * max(emax, 1), dtype=torch.int64, device=dev)
    for r in range(W):
        if emax:
            buf = g2[r * emax:(r + 1) * emax]
            L.check(lib.di_xchg_pack(P(Ks[r]), P(ecs[r]), P(off[r * nq:]), nq, k, P(buf), 0, st))
    out = torch.zeros(W * nq * k, dtype=torch.int64, device=dev)
    g_n = torch.empty(W * nq, dtype=torch.int32, device=dev)
    L.check(lib.di_xchg_unpack(P(g2) if emax else None, emax, P(gec), P(off), W, nq, k, P(out),
                               P(g_n), 0, st))
    torch.cuda.synchronize()
    return (out.cpu().numpy().view(np.uint64).reshape(W, nq, k), g_n.cpu().numpy().reshape(W, nq),
            gs.cpu().numpy().view(np.uint64).reshape(W, nq, s_n), tot.cpu().numpy())


@pytest.mark.parametrize("world,k,mode", [(2, 200, "iid"), (3, 40, "ragged"), (8, 1000, "iid"),
                                          (8, 1000, "ragged"), (1, 100, "ragged"),
                                          (64, 4096, "iid")])
def test_device_exchange_steps_equal_definition(L, world, k, mode):
    nq = 24 if world < 64 else 4
    keys, cnt = _lists(world, nq, k, seed=3 + world + k, mode=mode)
    g = max(1, min(64, k // (4 * world)))
    out, g_n, gs, tot = _run_device_steps(L, keys, cnt, k, g)
    s_n, need = k // g, -(-k // g)
    for q in range(nq):
        # the definition, in numpy: samples, T_q, this rank's keys >= T_q
        allS = []
        for r in range(world):
            c = min(max(int(cnt[r, q]), 0), k)
            pos = np.arange(1, s_n + 1) * g - 1
            sr = np.where(pos < c, keys[r, q, np.minimum(pos, k - 1)], np.uint64(0))
            assert (gs[r, q] == sr).all()
            allS.append(sr)
        allS = np.sort(np.concatenate(allS))[::-1]
        T = allS[need - 1] if allS.size >= need else np.uint64(0)
        for r in range(world):
            c = min(max(int(cnt[r, q]), 0), k)
            e = int((keys[r, q, :c] >= T).sum())
            want_n = int(cnt[r, q]) if cnt[r, q] < 0 else e
            assert g_n[r, q] == want_n, (r, q)
            assert (out[r, q, :e] == keys[r, q, :e]).all(), (r, q)
    assert (tot == np.maximum(g_n, 0).sum(1)).all()
    # the merge of the exchanged prefixes is the merge of the full lists
    got, want = _merge(out, g_n, k), _merge(keys, cnt, k)
    for q in range(nq):
        assert got[q] == want[q], q
    if world >= 2 and mode == "iid":  # doc-id-sharded lists: well under k keys per rank
        assert tot.max() / nq < 0.6 * k + s_n
