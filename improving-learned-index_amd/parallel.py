"""Doc-id-sharded multi-GPU paths: one process per GPU.

* Encode: contiguous doc-id (line) ranges per rank -- no collective; the shard
  outputs concatenated in rank order are the single-GPU impact TSV.
* Quantize: the scale needs the global max (quantize.py:31-37): one
  all_reduce(MAX) of an fp64 scalar, then every shard quantizes with that max.
* Retrieve: every rank scores every query on its shard and keeps a local top-k
  of unique 64-bit keys; one all_gather of (keys, counts) -- RCCL over xGMI with
  the nccl backend -- and a GPU merge (di_topk_merge) give exactly the
  single-shard result, because the keys totally order (score, first touch, doc).

The exchange is written against torch.distributed so it runs over RCCL on
MI355X and over gloo in the CPU tests (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def shard_range(n_items: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) of rank `rank` among `world`."""
    return n_items * rank // world, n_items * (rank + 1) // world


def global_max(local_max: float, group=None, device=None) -> float:
    """all_reduce(MAX) of the shard's max impact (fp64)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(local_max)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def decode_quant_keys(keys: np.ndarray, n: int) -> List[Tuple[int, int]]:
    k = keys[:n].astype(np.uint64)
    docs = (np.uint64(0xFFFFFFFF) - (k & np.uint64(0xFFFFFFFF))).astype(np.int64)
    scores = (k >> np.uint64(48)).astype(np.int64)
    return list(zip(docs.tolist(), scores.tolist()))


class ShardedRetriever:
    """Global top-k over doc-id shards held by the ranks of a process group.

    local_search(queries) -> (keys uint64 [n_q, k], counts int32 [n_q]) of this
    rank's shard; merge(keys [world, n_q, k], counts [world, n_q], k) ->
    (keys [n_q, k], counts [n_q]).  Defaults: the HIP scorer and di_topk_merge.
    """

    def __init__(self, k: int, local_search: Callable, merge: Optional[Callable] = None,
                 group=None, device=None):
        self.k, self.local_search, self.group, self.device = k, local_search, group, device
        self.merge = merge or self._gpu_merge

    def _gpu_merge(self, keys, counts, k):
        from . import _lib

        w, nq, _ = keys.shape
        return _lib.topk_merge(np.ascontiguousarray(keys.transpose(1, 0, 2)),
                               np.ascontiguousarray(counts.T), k)

    def search_keys(self, queries) -> Tuple[np.ndarray, np.ndarray]:
        import torch
        import torch.distributed as dist

        keys, counts = self.local_search(queries)
        world = dist.get_world_size(self.group)
        kt = torch.from_numpy(np.ascontiguousarray(keys).view(np.int64)).to(self.device)
        ct = torch.from_numpy(np.ascontiguousarray(counts, np.int32)).to(self.device)
        # rank-major concatenation along dim 0 (the layout both RCCL and gloo take)
        gk = torch.empty((world * kt.shape[0],) + tuple(kt.shape[1:]), dtype=kt.dtype,
                         device=kt.device)
        gc = torch.empty((world * ct.shape[0],), dtype=ct.dtype, device=ct.device)
        dist.all_gather_into_tensor(gk, kt, group=self.group)
        dist.all_gather_into_tensor(gc, ct, group=self.group)
        gk = gk.cpu().numpy().view(np.uint64).reshape((world,) + tuple(kt.shape))
        gc = gc.cpu().numpy().reshape(world, -1)
        return self.merge(gk, gc, self.k)

    def search(self, queries) -> List[List[Tuple[int, int]]]:
        mk, mn = self.search_keys(queries)
        return [decode_quant_keys(mk[i], int(mn[i])) for i in range(len(mn))]


def device_shard_search(index, k: int):
    """local_search for ShardedRetriever over a DeviceIndex shard (HIP)."""
    from . import _lib

    def run(queries):
        flat, cu = _lib.csr(queries)
        _, _, n, keys = index.search_csr(flat, cu, k, with_keys=True)
        return keys, n

    return run
