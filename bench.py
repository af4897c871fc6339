#!/usr/bin/env python3
"""bench.py -- DeeperImpact encode-and-retrieve on MI355X (BASELINE.json metric).

Workload = BASELINE.json configs[1]: an MS MARCO-passage-shaped 100k-doc slice
(synthetic, seeded generator of BASELINE.md §2 -- no network, no dataset) and
6,980 dev.small-sized queries at top-1000, on 1 GPU; with --gpus N each rank
holds its own 100k-doc shard (weak scaling), every query is scored on every
shard, and the per-shard top-1000 lists are all-gathered over RCCL and merged
on the GPU.

One JSON line on rank 0 (contract in the task statement), with a "roofline"
object for the dominant kernel (HIP-event timed inside the library on the
launching stream) and a "cpu_baseline" object (the oracle's C scorer on host
cores, bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from improving_learned_index_amd import _lib  # noqa: E402
from improving_learned_index_amd import synthetic as S  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.3 TB/s measured copy
DOCS_PER_SHARD = 100_000
V_TERMS = 200_000
N_QUERIES = 6980  # MS MARCO dev.small


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_pmc_traffic(name):
    """Per-launch HBM bytes of kernel `name` from the committed rocprofv3 PMC
    summary (profiles/*pmc*.json, produced by tools/pmc_summary.py), or None."""
    for p in sorted((ROOT / "profiles").glob("*pmc*.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        k = d.get("kernels", {}).get(name)
        if k and k.get("hbm_bytes_per_launch"):
            return k["hbm_bytes_per_launch"], p.name
    return None, None


def retrieve_leg(args, rank, world, dev):
    t0 = time.time()
    cu, term, imp = S.msmarco_like_docs(DOCS_PER_SHARD, V_TERMS, seed=1234 + rank)
    q, _ = S.quantize_like_reference(imp)
    term_off, pdoc, pval = S.postings_reference_order(cu, term, q, V_TERMS)
    doc_lo = rank * DOCS_PER_SHARD
    pdoc = pdoc + np.uint32(doc_lo)
    ix = _lib.DeviceIndex.from_postings(term_off, pdoc, pval, doc_lo, doc_lo + DOCS_PER_SHARD,
                                        device=dev)
    queries = S.msmarco_like_queries(args.queries, V_TERMS, seed=1234)
    flat, cuq = _lib.csr(queries)
    log(f"[rank {rank}] shard index: {ix.info()} built in {time.time() - t0:.1f}s")

    stream = torch.cuda.current_stream()
    ix.set_stream(stream.cuda_stream)
    k, nq = args.k, len(queries)
    d_terms = torch.from_numpy(flat.astype(np.int32)).cuda()
    d_cu = torch.from_numpy(cuq).cuda()
    out_doc = torch.empty(nq * k, dtype=torch.int32, device="cuda")
    out_score = torch.empty(nq * k, dtype=torch.int32, device="cuda")
    out_n = torch.empty(nq, dtype=torch.int32, device="cuda")
    out_key = torch.empty(nq * k, dtype=torch.int64, device="cuda")
    ix.reserve(nq, k)
    if world > 1:
        g_key = torch.empty(world * nq * k, dtype=torch.int64, device="cuda")
        g_n = torch.empty(world * nq, dtype=torch.int32, device="cuda")
        m_key = torch.empty(nq * k, dtype=torch.int64, device="cuda")
        m_n = torch.empty(nq, dtype=torch.int32, device="cuda")
    flags = _lib.DI_F_DEVICE_PTRS | _lib.DI_F_ASYNC

    def step(timing):
        ix.search_device(d_terms, d_cu, nq, k, out_doc, out_score, out_n, out_key,
                         flags | (_lib.DI_F_TIMING if timing else 0))
        if world > 1:
            dist.all_gather_into_tensor(g_key, out_key)
            dist.all_gather_into_tensor(g_n, out_n)
            _lib.topk_merge_device(g_key, g_n, nq, world, k, m_key, m_n, device=dev,
                                   stream=stream.cuda_stream,
                                   flags=flags | _lib.DI_F_LISTS_MAJOR)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    ix.sync()
    ix.timing("score_blocks", reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ix.sync()
    ms_sb, n_sb = ix.timing("score_blocks")
    ms_mg, n_mg = ix.timing("merge_topk")
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # correctness spot check of the timed outputs against the oracle (rank 0, N=1)
    lens = np.diff(term_off)
    post_per_launch = int(sum(int(lens[t].sum()) for t in
                              (np.asarray(qq, np.int64) for qq in queries)))
    res = {
        "value": nq * args.steps / el,
        "ms_per_step": 1000.0 * el / args.steps,
        "postings_per_query": post_per_launch / nq,
        "kernel_ms": {"score_blocks": ms_sb / max(n_sb, 1), "merge_topk": ms_mg / max(n_mg, 1)},
    }
    bytes_per_launch = 4.0 * post_per_launch  # packed u32 posting: (doc_in_block << 8) | value
    avg_s = (ms_sb / max(n_sb, 1)) / 1000.0
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    traffic, src = load_pmc_traffic("score_blocks_kernel")
    res["roofline"] = {
        "kernel": "score_blocks_kernel",
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "algorithmic_bytes_per_launch": bytes_per_launch,
        "avg_launch_ms": round(avg_s * 1000.0, 4),
        "launches": n_sb,
        "traffic_source": src,
    }
    return res, (term_off, pdoc - np.uint32(doc_lo), pval, queries,
                 out_doc, out_score, out_n)


def cpu_baseline_retrieve(args, term_off, pdoc, pval, queries, out_doc, out_score, out_n):
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle

    ora = oracle.Index.__new__(oracle.Index)
    ora.term_off, ora.pdoc, ora.pval = term_off, pdoc, pval
    ora.n_docs = int(pdoc.max()) + 1
    # parity spot check of the GPU result (first 50 queries)
    k = args.k
    want = ora.score_ids(queries[:50], k, n_threads=8)
    od, osc, on = out_doc.cpu().numpy(), out_score.cpu().numpy(), out_n.cpu().numpy()
    for i in range(50):
        got = list(zip(od[i * k:i * k + on[i]].tolist(), osc[i * k:i * k + on[i]].tolist()))
        if got != want[i]:
            raise SystemExit(f"bench parity check failed on query {i}")
    threads = min(8, os.cpu_count() or 1)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        i = done % len(queries)
        chunk = queries[i:i + 256]
        ora.score_ids(chunk, k, n_threads=threads)
        done += len(chunk)
    el = time.perf_counter() - t0
    return {"value": round(done / el, 2), "unit": "queries/s", "cores": threads,
            "kind": "port",
            "sample": f"{done} queries (cycling the {len(queries)} dev.small-shaped queries), "
                      f"top-{k}, same 100k-doc shard, oracle/oracle.c or_score "
                      f"(OpenMP over queries), {el:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--queries", type=int, default=N_QUERIES)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    res, ctx = retrieve_leg(args, rank, world, dev)
    out = {
        "metric": "queries/sec@top-1000 (MS MARCO passage shape, 100k docs per GPU)",
        "value": round(res["value"], 2),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(res["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (BASELINE.md §2 generator, seeded); quantized 8-bit impacts",
        "config": {"workload": "configs[1] retrieve: 100k-doc MS MARCO-shaped slice per GPU, "
                               f"{args.queries} dev.small-shaped queries, top-{args.k}",
                   "docs_per_gpu": DOCS_PER_SHARD, "queries": args.queries, "k": args.k,
                   "postings_per_query": round(res["postings_per_query"], 1),
                   "parallelism": f"doc-sharded x{world}, RCCL all-gather of top-k"},
        "kernel_ms": res["kernel_ms"],
        "roofline": res["roofline"],
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_retrieve(args, *ctx)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
