"""Doc-id-sharded multi-GPU paths: one process per GPU.

* Encode: contiguous doc-id (line) ranges per rank -- no collective; the shard
  outputs concatenated in rank order are the single-GPU impact TSV.
* Quantize: the scale needs the global max (quantize.py:31-37): one
  all_reduce(MAX) of an fp64 scalar, then every shard quantizes with that max.
* Retrieve: every rank scores every query on its shard and keeps a local top-k
  of unique 64-bit keys; a pruned two-round all_gather of them (exchange_topk: a
  sample of every list, then each rank's keys above the bound the samples give)
  -- RCCL over xGMI with the nccl backend -- and a GPU merge
  (di_topk_merge) give exactly the single-shard result, because the keys totally
  order (score, first touch, doc).

The exchange is written against torch.distributed so it runs over RCCL on
MI355X and over gloo in the CPU tests (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

import os
import shutil
from pathlib import Path
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def dist_env() -> Tuple[int, int, int]:
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 without it)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def force_dist() -> bool:
    """DI_FORCE_DIST=1 under a launcher: the multi-rank path (process group, exchange,
    merge) even at one rank -- how a 1-GPU box runs the RCCL branch."""
    return os.environ.get("DI_FORCE_DIST") == "1" and "MASTER_ADDR" in os.environ


def _kfd_gpu_nodes(root="/sys/class/kfd/kfd/topology/nodes", dri="/dev/dri") -> Optional[int]:
    """GPU nodes of the KFD topology (nodes with SIMDs) whose render node this process
    can open, or None without a topology."""
    root = Path(root)
    if not root.is_dir():
        return None
    n = 0
    for node in root.iterdir():
        try:
            props = dict(line.split() for line in (node / "properties").read_text().splitlines()
                         if len(line.split()) == 2)
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue
        # a GPU this process may open (a container can list every GPU of the host in the
        # topology yet expose only some render nodes): a plain open() of its render node,
        # no HIP call
        minor = props.get("drm_render_minor")
        if minor is not None:
            try:
                os.close(os.open(f"{dri}/renderD{minor}", os.O_RDWR))
            except OSError:
                continue
        n += 1
    return n


def _env_device_list(name: str) -> Optional[int]:
    v = os.environ.get(name)
    if v is None:
        return None
    v = v.strip()
    return 0 if v in ("", "-1") else len([x for x in v.split(",") if x.strip()])


def visible_gpus() -> int:
    """GPUs this process sees, counted without the HIP runtime: a parent that spawns
    ranks must not bring HIP up (torch.cuda.device_count() may fall back to
    hipGetDeviceCount when amdsmi is missing).  HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES restrict the KFD topology's GPU nodes
    (sysfs); without a topology, torch's count."""
    n = _kfd_gpu_nodes()
    if n is None:
        import torch

        return torch.cuda.device_count()
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        m = _env_device_list(var)
        if m is not None:
            n = min(n, m)
    return n


def ranks_to_spawn(requested: Optional[int]) -> int:
    """How many per-GPU ranks a CLI started without a launcher should fan out to: the
    reference's Indexer wraps the model in DataParallel whenever
    torch.cuda.device_count() > 1 (indexer.py:25-26), so by default every visible
    GPU; `requested` (--gpus) overrides, and 1 keeps one process.  Under torchrun
    (WORLD_SIZE set) the launcher already decided: 1."""
    if "WORLD_SIZE" in os.environ:
        return 1
    n = max(1, visible_gpus()) if requested is None else int(requested)
    if n < 1:
        raise ValueError(f"--gpus must be >= 1 (got {n})")
    return n


def spawn_ranks(module: str, argv: Sequence[str], n: int) -> int:
    """Run `python -m improving_learned_index_amd.<module> argv` as n ranks of a child
    torchrun (one process per GPU, doc-id shards, rank 0 joins the outputs) and
    return its exit status.  The parent has made no HIP call and never execs."""
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = str(Path(__file__).resolve().parent.parent)
    env = dict(os.environ)
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # one hash seed for every rank: rank 0's query-term order is broadcast anyway, but
    # the children then also agree with one another on everything set-ordered
    env.setdefault("PYTHONHASHSEED", str(int.from_bytes(os.urandom(2), "little")))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           "-m", f"improving_learned_index_amd.{module}"] + list(argv)
    return subprocess.call(cmd, env=env)


def init_group(backend: str, local_rank: int = 0):
    """Process group of a torchrun-launched CLI: "nccl" (RCCL over xGMI; every rank
    owns GPU local_rank) for the retrieval exchange, "gloo" for the host-only
    barriers / scalars of the sharded index and quantize CLIs."""
    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group("gloo")


def rank_device(local_rank: int) -> int:
    """GPU of a local rank: one per GPU on an 8-GPU node; ranks share the devices when
    there are more ranks than GPUs (the 1-GPU test box)."""
    import torch

    # (torch's count: it does not initialise the GPU; torch's HIP runtime must come up
    # before the library's, see Ranker)
    return local_rank % max(1, torch.cuda.device_count())


def exchange_backend(world: int) -> str:
    """RCCL (nccl) when every rank owns its GPU, else gloo over host tensors
    (DI_DIST_BACKEND overrides)."""
    import torch

    return os.environ.get("DI_DIST_BACKEND") or (
        "nccl" if world <= torch.cuda.device_count() else "gloo")


def concat_parts(parts: Sequence[Path], out_path: Path) -> None:
    """Rank 0: the shard outputs in rank order -> the single-process file."""
    with open(out_path, "wb") as out:
        for p in parts:
            with open(p, "rb") as f:
                shutil.copyfileobj(f, out, 1 << 24)
    for p in parts:
        os.unlink(p)


def part_path(path, rank: int) -> Path:
    path = Path(path)
    return path.with_name(f"{path.name}.part{rank:05d}")


def count_lines(path) -> int:
    """Lines as Python's text-mode file iteration sees them -- universal newlines
    (\\n, \\r\\n and a lone \\r end a line; index.py and the reference read the
    collection with open(path), index.py:32) and a last line without a terminator."""
    n, prev_cr, last = 0, False, b""
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            # terminators = \n + \r - \r\n pairs (one split across blocks included)
            n += blk.count(b"\n") + blk.count(b"\r") - blk.count(b"\r\n")
            if prev_cr and blk[:1] == b"\n":
                n -= 1
            prev_cr = blk[-1:] == b"\r"
            last = blk[-1:]
    return n + (last not in (b"", b"\n", b"\r"))


def line_offsets(path, lines: Sequence[int], block: int = 1 << 24) -> List[int]:
    """Byte offsets where the given 0-based lines start (ascending; a line index past
    the end -> the file size), with the universal-newline line ends of count_lines.
    Streams the file: whole blocks are skipped by counting their terminators."""
    import re

    want = list(lines)
    assert want == sorted(want)
    out: List[int] = []
    term = re.compile(rb"\r\n|\r|\n")
    line, pos, carry_cr = 0, 0, False  # line index at byte pos (the start of a block)
    with open(path, "rb") as f:
        k = 0
        while k < len(want) and want[k] <= 0:
            out.append(0)
            k += 1
        for blk in iter(lambda: f.read(block), b""):
            if k == len(want) and not carry_cr:  # (a pending \r may take the next \n)
                break
            start = 0
            if carry_cr and blk[:1] == b"\n":  # the \n of a \r\n split across blocks
                start = 1
                # the line began after the \n: fix the offsets recorded for that line
                j = len(out) - 1
                while j >= 0 and out[j] == pos and want[j] == line:
                    out[j] = pos + 1
                    j -= 1
            n_here = (blk.count(b"\n") + blk.count(b"\r") - blk.count(b"\r\n")
                      - (1 if start else 0))
            if k == len(want):
                break
            if line + n_here < want[k]:  # no wanted line starts inside this block
                line += n_here
                carry_cr = blk[-1:] == b"\r"
                pos += len(blk)
                continue
            for m in term.finditer(blk, start):
                line += 1
                while k < len(want) and want[k] == line:
                    out.append(pos + m.end())
                    k += 1
                if k == len(want):
                    break
            carry_cr = blk[-1:] == b"\r"
            pos += len(blk)
        size = pos + sum(len(b) for b in iter(lambda: f.read(block), b""))
    out += [size] * (len(want) - len(out))
    return out


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


def decode_quant_keys(keys: np.ndarray, n: int, n_terms: int = 0) -> List[Tuple[int, int]]:
    """(doc, score) list of one query's merged keys.  n < 0 is a query the scorer
    rejected on some shard (a kernel limit, include/deepimpact.h): raise, never emit
    the keys.  n_terms: the query's known terms (wide keys above DI_SHORT_QUERY_TERMS)."""
    if n < 0:
        raise RuntimeError("DI_ERANGE: the scorer rejected a query (out_n = -1: more than "
                           "DI_MAX_QUERY_TERMS terms, or a long query on a shard past doc 2^24)")
    k = keys[:n].astype(np.uint64)
    wide = n_terms > 256  # DI_SHORT_QUERY_TERMS
    m, sh = (np.uint64(0xFFFFFF), np.uint64(44)) if wide else (np.uint64(0xFFFFFFFF), np.uint64(48))
    docs = (m - (k & m)).astype(np.int64)
    scores = (k >> sh).astype(np.int64)
    return list(zip(docs.tolist(), scores.tolist()))


def decode_quant_key_arrays(keys: np.ndarray, counts: np.ndarray, n_terms) -> Tuple[np.ndarray, np.ndarray]:
    """decode_quant_keys over a batch: keys uint64 [n_q, k], counts [n_q], the queries'
    known-term counts -> (docs, scores) uint32 [n_q, k] (valid up to counts[q]).
    Raises on a rejected query (a negative count) like decode_quant_keys."""
    counts = np.asarray(counts)
    if counts.size and int(counts.min()) < 0:
        decode_quant_keys(keys[0], int(counts.min()))  # (raises the same error)
    k = keys.astype(np.uint64)
    wide = (np.asarray(n_terms, np.int64) > 256)[:, None]  # DI_SHORT_QUERY_TERMS
    m = np.where(wide, np.uint64(0xFFFFFF), np.uint64(0xFFFFFFFF))
    sh = np.where(wide, np.uint64(44), np.uint64(48))
    docs = (m - (k & m)).astype(np.uint32)
    scores = (k >> sh).astype(np.uint32)
    return docs, scores


def quantize_sharded(input_path, output_path, max_val, world: int, rank: int,
                     shard_max: Callable, shard_quantize: Callable) -> float:
    """Doc-sharded quantize (quantize.py:27-47 over `world` ranks): every rank takes a
    contiguous line range of the impact TSV, the global max is the all_reduce(MAX) of
    the shard maxima (find_max_value, quantize.py:17-24), every rank quantizes its
    lines with it, and rank 0 joins the parts: the single-process bytes.
    shard_max(path) -> float and shard_quantize(in, out, max) are the per-shard
    kernels (the HIP di_quantize_file by default in quantize.py)."""
    import torch.distributed as dist

    # the shard's lines by byte offsets (universal newlines, as the reference's text-mode
    # iteration): streamed, never the whole file in memory
    lo, hi = shard_range(count_lines(input_path), world, rank)
    b_lo, b_hi = line_offsets(input_path, [lo, hi])
    part_in = Path(f"{part_path(output_path, rank)}.in")
    with open(input_path, "rb") as src, open(part_in, "wb") as f:
        src.seek(b_lo)
        left = b_hi - b_lo
        while left > 0:
            blk = src.read(min(left, 1 << 24))
            if not blk:
                break
            f.write(blk)
            left -= len(blk)
    if max_val is None:
        m = global_max(shard_max(part_in) if hi > lo else 0.0)
        if not m > 0.0:
            raise ZeroDivisionError("float division by zero")  # quantize.py:37
    else:
        m = float(max_val)
    shard_quantize(part_in, part_path(output_path, rank), m)
    os.unlink(part_in)
    dist.barrier()
    if rank == 0:
        concat_parts([part_path(output_path, r) for r in range(world)], Path(output_path))
    dist.barrier()
    return m


_SIGN = -(1 << 63)  # int64 view of a u64 key XOR this = the keys' unsigned order

# Below this many keys per rank (n_q * k; 32 KB) the plain all_gather (two collectives,
# no host synchronisation) costs less than the pruned exchange's three collectives and
# its one device -> host read of the round-2 size.
PLAIN_MAX_KEYS = 4096


def exchange_pruned(world: int, nq: int, k: int, pruned: Optional[bool] = None) -> bool:
    """Whether exchange_topk takes the pruned two-round path.  pruned True / False forces
    it (DI_EXCHANGE=pruned / plain likewise); by default pruned from 2 ranks when a rank
    holds at least PLAIN_MAX_KEYS keys.  Forcing it at one rank is how a 1-GPU box runs
    the device / RCCL branch of the multi-GPU retrieve."""
    if pruned is None:
        pruned = {"pruned": True, "plain": False}.get(os.environ.get("DI_EXCHANGE", "auto"))
    if pruned is None:
        pruned = world > 1 and nq * k >= PLAIN_MAX_KEYS
    return bool(pruned) and max(1, min(64, k // (4 * world))) > 1


def exchange_topk(key, cnt, k: int, group=None, stats: Optional[dict] = None,
                  pruned: Optional[bool] = None):
    """Exact, pruned all-gather of every rank's top-k key lists (SURVEY §8e retrieve).

    key: [n_q * k] int64 tensor (u64 merge keys; each query's list sorted descending, its
    first cnt[q] valid), cnt: [n_q] int32 (negative: the scorer rejected the query).
    Returns (g_key [world * n_q * k], g_n [world * n_q]) in a plain all_gather's rank-
    major layout, holding per rank and query a prefix of its list that contains every
    key able to reach the global top-k: di_topk_merge over it gives exactly the merge of
    the full lists.

    Round 1 gathers a sample of every list: the keys at positions g-1, 2g-1, ... (g keys
    apart).  A rank whose j-th sample is >= t holds >= j g keys >= t, so with s = ceil(k/g)
    samples >= T_q across the ranks at least k keys are >= T_q: T_q, the s-th largest
    sample, is a lower bound of the global k-th key.  Round 2 gathers each rank's keys
    >= T_q: their counts together with the scorer's counts (one collective), then the
    keys padded to the largest rank's total.  A plain gather moves k keys per query and
    rank; this one k / g samples + the rank's share of the keys >= T_q (k + O(world g)
    of them over all ranks).  The keys are unique (they carry the doc), so the pruning
    is exact: /root/reference/src/deep_impact/evaluation/ranker.py:43-48 keeps the top
    1000 per query, which the merge reproduces.

    Three collectives and one host synchronisation (the round-2 size): packing and
    unpacking are device scatters (no boolean indexing, no per-rank loop).
    pruned: see exchange_pruned.  stats (optional dict): path ("pruned" / "plain"),
    gathered_keys_per_query (sent by this rank, padding included), bytes_sent.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    nq = cnt.numel()
    dev = key.device
    K = key.view(nq, k)
    if not exchange_pruned(world, nq, k, pruned):
        gk = torch.empty(world * nq * k, dtype=torch.int64, device=dev)
        gc = torch.empty(world * nq, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(gk, K.reshape(-1).contiguous(), group=group)
        dist.all_gather_into_tensor(gc, cnt.contiguous(), group=group)
        if stats is not None:
            stats["path"] = "plain"
            stats["gathered_keys_per_query"] = float(k)
            stats["bytes_sent"] = 8 * nq * k + 4 * nq
        return gk, gc
    g = max(1, min(64, k // (4 * world)))
    if dev.type == "cuda":
        return _exchange_pruned_hip(K, cnt, k, g, world, group, stats)
    c = cnt.to(torch.int64).clamp(0, k)
    lo = torch.iinfo(torch.int64).min
    s_n = k // g  # samples per list (positions g-1, ..., s_n g - 1 < k)
    pos = torch.arange(1, s_n + 1, device=dev) * g - 1
    smp = torch.where(pos[None, :] < c[:, None], K[:, pos] ^ _SIGN,
                      torch.full((nq, s_n), lo, dtype=torch.int64, device=dev))
    g1 = torch.empty(world * nq * s_n, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(g1, smp.reshape(-1).contiguous(), group=group)
    allS = g1.view(world, nq, s_n).permute(1, 0, 2).reshape(nq, world * s_n)
    need = -(-k // g)
    if world * s_n >= need and nq:
        T = torch.topk(allS, need, dim=1).values[:, need - 1]  # (lo when too few samples)
    else:
        T = torch.full((nq,), lo, dtype=torch.int64, device=dev)
    # round 2: this rank's keys >= T_q (a prefix of each list: lists are sorted)
    ar_k = torch.arange(k, device=dev)
    sel = (ar_k[None, :] < c[:, None]) & ((K ^ _SIGN) >= T[:, None])
    e = sel.sum(1)
    # the prefix counts and the scorer's counts in one collective: [world, 2, nq]
    ec = torch.stack([e.to(torch.int32), cnt.to(torch.int32)]).reshape(-1)
    gec = torch.empty(world * 2 * nq, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(gec, ec, group=group)
    gec = gec.view(world, 2, nq)
    gew = gec[:, 0].to(torch.int64)
    gcw = gec[:, 1]
    tot = gew.sum(1)
    emax = int(tot.max().item()) if nq else 0  # (the one host synchronisation)
    # one slot past the rank-major lists takes every padding write
    out = torch.empty(world * nq * k + 1, dtype=torch.int64, device=dev)
    if emax:
        # pack: key j < e[q] of query q -> off[q] + j (the rest -> the dump slot emax)
        off = torch.cumsum(e, 0) - e
        dst = torch.where(sel, off[:, None] + ar_k[None, :], torch.full_like(K, emax))
        buf = torch.zeros(emax + 1, dtype=torch.int64, device=dev)
        buf.scatter_(0, dst.reshape(-1), K.reshape(-1))
        g2 = torch.empty(world * emax, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(g2, buf[:emax].contiguous(), group=group)
        # unpack every rank at once: position p of rank r belongs to the query whose
        # inclusive prefix count first exceeds p
        cum = torch.cumsum(gew, 1)  # [world, nq]
        p = torch.arange(emax, device=dev).expand(world, emax).contiguous()
        qi = torch.searchsorted(cum, p, right=True)  # [world, emax]; nq past tot[r]
        ok = p < tot[:, None]
        qc = qi.clamp(max=nq - 1)
        col = p - (torch.gather(cum, 1, qc) - torch.gather(gew, 1, qc))
        r_ix = torch.arange(world, device=dev)[:, None]
        dst2 = torch.where(ok, (r_ix * nq + qc) * k + col,
                           torch.full_like(p, world * nq * k))
        out.scatter_(0, dst2.reshape(-1), g2)
    g_n = torch.where(gcw < 0, gcw, gew.to(torch.int32))
    if stats is not None:
        stats["path"] = "pruned"
        stats["gathered_keys_per_query"] = (s_n + emax / max(nq, 1)) if nq else 0.0
        stats["bytes_sent"] = 8 * (nq * s_n + emax) + 4 * 2 * nq
    return out[:world * nq * k], g_n.reshape(-1)


def _exchange_pruned_hip(K, cnt, k: int, g: int, world: int, group, stats):
    """exchange_topk's pruned rounds on device tensors: the local steps are the
    library's di_xchg_* kernels (exchange.hip) on the current stream, around three
    all_gathers and one device -> host read (the round-2 padded size).  Same output as
    the tensor-operation form below it, which the CPU (gloo) rehearsals run."""
    import torch
    import torch.distributed as dist

    from . import _lib

    nq = cnt.numel()
    dev = K.device
    if nq == 0:  # (every rank has the same queries: all return here together)
        if stats is not None:
            stats.update(path="pruned", gathered_keys_per_query=0.0, bytes_sent=0)
        return (torch.empty(0, dtype=torch.int64, device=dev),
                torch.empty(0, dtype=torch.int32, device=dev))
    d = dev.index if dev.index is not None else torch.cuda.current_device()
    st = torch.cuda.current_stream(dev).cuda_stream
    L = _lib.lib()
    P = _lib.ptr
    cnt = cnt.to(torch.int32).contiguous()
    K = K.contiguous()
    s_n = k // g
    smp = torch.empty(nq * s_n, dtype=torch.int64, device=dev)
    _lib.check(L.di_xchg_sample(P(K), P(cnt), nq, k, g, P(smp), d, st))
    g1 = torch.empty(world * nq * s_n, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(g1, smp, group=group)
    ec = torch.empty(2 * nq, dtype=torch.int32, device=dev)
    _lib.check(L.di_xchg_count(P(g1), world, P(K), P(cnt), nq, k, g, P(ec), d, st))
    gec = torch.empty(world * 2 * nq, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(gec, ec, group=group)
    off = torch.empty(world * nq, dtype=torch.int64, device=dev)
    tot = torch.empty(world, dtype=torch.int64, device=dev)
    _lib.check(L.di_xchg_offsets(P(gec), world, nq, P(off), P(tot), d, st))
    emax = int(tot.max().item()) if nq else 0  # (the one host synchronisation)
    me = dist.get_rank(group)
    out = torch.empty(world * nq * k, dtype=torch.int64, device=dev)
    g_n = torch.empty(world * nq, dtype=torch.int32, device=dev)
    g2 = None
    if emax:
        buf = torch.zeros(emax, dtype=torch.int64, device=dev)
        _lib.check(L.di_xchg_pack(P(K), P(ec), P(off[me * nq:]), nq, k, P(buf), d, st))
        g2 = torch.empty(world * emax, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(g2, buf, group=group)
    _lib.check(L.di_xchg_unpack(P(g2), emax, P(gec), P(off), world, nq, k, P(out), P(g_n), d, st))
    if stats is not None:
        stats["path"] = "pruned"
        stats["gathered_keys_per_query"] = (s_n + emax / max(nq, 1)) if nq else 0.0
        stats["bytes_sent"] = 8 * (nq * s_n + emax) + 4 * 2 * nq
    return out, g_n


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
        mk, mn, _ = self._search_keys(queries)
        return mk, mn

    def _search_keys(self, queries):
        import torch
        import torch.distributed as dist

        res = self.local_search(queries)
        # local_search may drop terms (unknown words): it then returns the term counts it
        # actually submitted, which decide the key layout (wide above 256 terms)
        keys, counts = res[0], res[1]
        n_terms = res[2] if len(res) > 2 else [len(q) for q in queries]
        world = dist.get_world_size(self.group)
        kt = torch.from_numpy(np.ascontiguousarray(keys).view(np.int64)).to(self.device)
        ct = torch.from_numpy(np.ascontiguousarray(counts, np.int32)).to(self.device)
        # the pruned exact exchange, in the rank-major layout of a plain all_gather
        gk, gc = exchange_topk(kt.reshape(-1), ct, self.k, group=self.group)
        gk = gk.cpu().numpy().view(np.uint64).reshape((world,) + tuple(kt.shape))
        gc = gc.cpu().numpy().reshape(world, -1)
        mk, mn = self.merge(gk, gc, self.k)
        return mk, mn, n_terms

    def search(self, queries) -> List[List[Tuple[int, int]]]:
        mk, mn, n_terms = self._search_keys(queries)
        return [decode_quant_keys(mk[i], int(mn[i]), int(n_terms[i])) for i in range(len(mn))]


def exchange_merge_device(index, queries, k: int, device: int, flags: int = 0):
    """The rank CLI's retrieval step on one doc-id shard: score every query
    on this rank's DeviceIndex shard into device tensors, all_gather the (key, count)
    lists -- RCCL over xGMI under the nccl backend; host tensors under gloo -- and merge
    them on the GPU with di_topk_merge (DI_F_LISTS_MAJOR: the gathered rank-major
    layout, no transpose).  Returns host (keys [n_q, k] uint64, counts [n_q])."""
    import torch
    import torch.distributed as dist

    from . import _lib

    dev = torch.device("cuda", device)
    # one real stream for the scorer, the collectives and the merge (torch's default
    # stream has the null handle, which di_index_set_stream takes as "own stream": the
    # all_gather would then not be ordered after the scorer)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        index.set_stream(stream.cuda_stream)
        return _exchange_merge(index, queries, k, device, dev, stream, flags)


def _exchange_merge(index, queries, k, device, dev, stream, flags):
    import torch
    import torch.distributed as dist

    from . import _lib

    world = dist.get_world_size()
    gpu_exchange = dist.get_backend() == "nccl"
    flat, cu = _lib.csr(queries)
    nq = len(queries)
    f = _lib.DI_F_DEVICE_PTRS | _lib.DI_F_ASYNC | flags
    d_terms = torch.from_numpy(flat.astype(np.int32)).to(dev)
    d_cu = torch.from_numpy(cu).to(dev)
    out_doc = torch.empty(max(nq * k, 1), dtype=torch.int32, device=dev)
    out_score = torch.empty_like(out_doc)
    out_n = torch.empty(max(nq, 1), dtype=torch.int32, device=dev)
    out_key = torch.empty(max(nq * k, 1), dtype=torch.int64, device=dev)
    if nq:
        index.search_device(d_terms, d_cu, nq, k, out_doc, out_score, out_n, out_key, f)
    key, cnt = (out_key, out_n) if gpu_exchange else (out_key.cpu(), out_n.cpu())
    if not gpu_exchange:
        torch.cuda.synchronize(dev)
    # the pruned exact exchange (a plain all_gather's layout, only the keys that can
    # reach the global top-k filled in)
    g_key, g_n = exchange_topk(key[:nq * k], cnt[:nq], k)
    if nq == 0:
        return np.zeros((0, k), np.uint64), np.zeros(0, np.int32)
    m_key = torch.empty(nq * k, dtype=torch.int64, device=dev)
    m_n = torch.empty(nq, dtype=torch.int32, device=dev)
    if not gpu_exchange:  # gathered on the host: back to the device for the merge
        g_key, g_n = g_key.to(dev), g_n.to(dev)
    _lib.topk_merge_device(g_key, g_n, nq, world, k, m_key, m_n, device=device,
                           stream=stream.cuda_stream, flags=f | _lib.DI_F_LISTS_MAJOR)
    keys = m_key.cpu().numpy().view(np.uint64).reshape(nq, k)
    return keys, m_n.cpu().numpy()


def device_shard_search(index, k: int):
    """local_search for ShardedRetriever over a DeviceIndex shard (HIP): queries are
    term-id lists, submitted whole (the counts returned are theirs)."""
    from . import _lib

    def run(queries):
        flat, cu = _lib.csr(queries)
        _, _, n, keys = index.search_csr(flat, cu, k, with_keys=True)
        return keys, n, np.diff(cu)

    return run
