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
import hashlib
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
from improving_learned_index_amd import parallel  # noqa: E402
from improving_learned_index_amd import synthetic as S  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.3 TB/s measured copy
DOCS_PER_SHARD = 100_000
N_QUERIES = 6980  # MS MARCO dev.small
REF_QUANTIZE_DOCS_S = 7003.0  # reference quantize_file, 1 core (SURVEY §6 / BASELINE.md)
REF_CREATE_DOCS_S = 4726.0    # reference InvertedIndexCreator.run, 1 core (same)


def v_terms(n_docs):
    """the vocabulary scales with the collection, V = 2 N (the 100k-doc
    slice keeps BASELINE.md's V = 200k)."""
    return 2 * n_docs


def _gloo():
    return dist.is_initialized() and dist.get_backend() == "gloo"


def all_gather_dev(out, inp):
    """all_gather_into_tensor on device tensors (host-staged under gloo)."""
    if _gloo():
        o = torch.empty(out.shape, dtype=out.dtype)
        torch.cuda.synchronize()
        dist.all_gather_into_tensor(o, inp.cpu())
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp)


def max_over_ranks(x: float) -> float:
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if _gloo() else "cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_pmc_traffic(name, leg=None):
    """Per-launch HBM bytes of kernel `name` from the committed rocprofv3 PMC
    summaries (tools/pmc_legs.sh -> profiles/<round>_pmc_<leg>.json for a bench leg;
    profiles/*pmc_summary*.json from tools/pmc.sh), newest first, or None."""
    pats = ([f"*pmc_{leg}.json"] if leg else []) + ["*pmc_summary*.json"]
    for p in [q for pat in pats for q in sorted((ROOT / "profiles").glob(pat), reverse=True)]:
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        ks = d.get("kernels", {})
        k = ks.get(name) or ks.get(name.split("<")[0])  # (summaries before the template split)
        if k and k.get("hbm_bytes_per_launch"):
            return k["hbm_bytes_per_launch"], p.name
    return None, None


def load_pmc_counters(name, leg):
    """(counter dict, file name) of kernel `name` in the leg's newest PMC summary."""
    for p in sorted((ROOT / "profiles").glob(f"*pmc_{leg}.json"), reverse=True):
        try:
            ks = json.loads(p.read_text()).get("kernels", {})
            k = ks.get(name) or ks.get(name.split("<")[0])
        except Exception:
            continue
        if k:
            return k, p.name
    return None


LDS_CUS = 256
LDS_CLOCK_HZ = 2.4e9
LDS_CYCLES_PER_64_POSTINGS = 6.0


def retrieve_leg(args, rank, world, dev, n_docs=DOCS_PER_SHARD, check_queries=20):
    """One doc-id shard of n_docs per rank.  100k docs: the numpy generator
    (synthetic.msmarco_like_docs, one doc at a time); larger shards: the same
    distribution from the library's threaded generator (synthetic.synth_postings).
    check_queries > 0: the first that many queries are checked against the oracle's
    C scorer right after the timed loop."""
    t0 = time.time()
    V = v_terms(n_docs)
    # Multi-rank: the shards of one collection, quantized with the collection's max (the
    # all_reduce(MAX) of the shards' maxima, as the sharded quantize CLI does); per-shard
    # maxima would give every shard its own scale, and one shard's scores would dominate
    # the global top-k (and the exchange)
    sharded = dist.is_initialized()
    if n_docs == DOCS_PER_SHARD:
        cu, term, imp = S.msmarco_like_docs(DOCS_PER_SHARD, V, seed=1234 + rank)
        gmax = None
        if sharded:
            gmax = max_over_ranks(float(S.round3_f32(imp).astype(np.float64).max()))
        q, _ = S.quantize_like_reference(imp, max_val=gmax)
        term_off, pdoc, pval = S.postings_reference_order(cu, term, q, V)
        del cu, term, imp, q
    elif sharded:  # docs [rank n, (rank + 1) n) of the seed's collection
        gmax = max_over_ranks(S.synth_max_impact(n_docs, V, seed=4321, doc0=rank * n_docs))
        term_off, pdoc, pval, _ = S.synth_postings(n_docs, V, seed=4321, doc0=rank * n_docs,
                                                   quant_max=gmax)
    else:
        term_off, pdoc, pval, _ = S.synth_postings(n_docs, V, seed=4321)
    t_gen = time.time() - t0
    doc_lo = rank * n_docs
    if doc_lo:
        pdoc = pdoc + np.uint32(doc_lo)
    ix = _lib.DeviceIndex.from_postings(term_off, pdoc, pval, doc_lo, doc_lo + n_docs,
                                        device=dev)
    queries = S.msmarco_like_queries(args.queries, V, seed=1234)
    flat, cuq = _lib.csr(queries)
    log(f"[rank {rank}] shard index: {ix.info()} generated in {t_gen:.1f}s, built in "
        f"{time.time() - t0 - t_gen:.1f}s")

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
    if dist.is_initialized():
        g_key = torch.empty(world * nq * k, dtype=torch.int64, device="cuda")
        g_n = torch.empty(world * nq, dtype=torch.int32, device="cuda")
        m_key = torch.empty(nq * k, dtype=torch.int64, device="cuda")
        m_n = torch.empty(nq, dtype=torch.int32, device="cuda")
    flags = _lib.DI_F_DEVICE_PTRS | _lib.DI_F_ASYNC

    xch = {"ms": 0.0, "keys_per_query": 0.0, "bytes": 0, "n": 0, "path": None}

    def exchange(pruned=None, st=None):
        """parallel.exchange_topk of this step's lists into g_key / g_n; returns its
        device-synchronised host time in ms (the scorer's tail is synchronised first)."""
        torch.cuda.synchronize()
        t_x = time.perf_counter()
        st = {} if st is None else st
        if _gloo():
            gk, gn = parallel.exchange_topk(out_key.cpu(), out_n.cpu(), k, stats=st, pruned=pruned)
        else:
            gk, gn = parallel.exchange_topk(out_key, out_n, k, stats=st, pruned=pruned)
        g_key.copy_(gk)
        g_n.copy_(gn)
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t_x)

    def step(timing):
        ix.search_device(d_terms, d_cu, nq, k, out_doc, out_score, out_n, out_key,
                         flags | (_lib.DI_F_TIMING if timing else 0))
        if dist.is_initialized():
            # the exact exchange (parallel.exchange_topk: pruned two rounds from 2 ranks,
            # DI_EXCHANGE=pruned forces them at one rank); its time is the collective_ms line
            st = {}
            ms = exchange(None, st)
            if timing:
                xch["ms"] += ms
                xch["keys_per_query"] += st["gathered_keys_per_query"]
                xch["bytes"] += st["bytes_sent"]
                xch["n"] += 1
                xch["path"] = st["path"]
            _lib.topk_merge_device(g_key, g_n, nq, world, k, m_key, m_n, device=dev,
                                   stream=stream.cuda_stream,
                                   flags=flags | _lib.DI_F_LISTS_MAJOR)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    ix.sync()
    ix.timing("score_blocks", reset=True)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    el = time.perf_counter() - t0
    ix.sync()
    # a query the scorer rejected (out_n < 0: a kernel limit) invalidates the leg
    n_min = int((m_n if dist.is_initialized() else out_n).min().item()) if nq else 0
    if n_min < 0:
        raise SystemExit(f"scorer rejected a query (out_n = {n_min}): the leg is invalid")
    ms_sb, n_sb = ix.timing("score_blocks")
    ms_mg, n_mg = ix.timing("merge_topk")
    alt = None
    if dist.is_initialized():
        # the merged lists of the last timed step: at one rank they must be the scorer's
        # own (the exchange + GPU merge of one shard is the identity) -- checks the
        # device path of a forced pruned exchange end to end
        same = None
        if world == 1:
            valid = torch.arange(k, device=out_n.device)[None, :] < out_n[:, None].long()
            same = bool(torch.equal(m_n, out_n)) and bool(torch.equal(
                m_key.view(nq, k)[valid], out_key.view(nq, k)[valid]))
            if not same:
                raise SystemExit("exchange + merge at one rank changed the scorer's lists")
        # the other exchange path on the same lists (advice r5: both paths' times)
        alt_pruned = xch["path"] != "pruned"
        if parallel.exchange_pruned(world, nq, k, alt_pruned) == alt_pruned:
            st_alt = {}
            ms_alt = [exchange(alt_pruned, st_alt) for _ in range(3)]
            alt = {"path": st_alt["path"], "collective_ms_per_step": sorted(ms_alt)[1],
                   "gathered_keys_per_query": st_alt["gathered_keys_per_query"]}
    if check_queries and rank == 0:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle

        ora = oracle.Index.__new__(oracle.Index)
        ora.term_off, ora.pdoc, ora.pval = term_off, pdoc - np.uint32(doc_lo), pval
        ora.n_docs = n_docs
        want = ora.score_ids(queries[:check_queries], k, n_threads=min(16, os.cpu_count() or 1))
        od, osc, on = out_doc.cpu().numpy(), out_score.cpu().numpy(), out_n.cpu().numpy()
        for i in range(check_queries):
            got = list(zip((od[i * k:i * k + on[i]] - doc_lo).tolist(),
                           osc[i * k:i * k + on[i]].tolist()))
            if got != want[i]:
                raise SystemExit(f"bench parity check failed on query {i} ({n_docs} docs)")
        log(f"[rank 0] {n_docs}-doc shard: the first {check_queries} queries equal the oracle")
    if dist.is_initialized():
        el = max_over_ranks(el)

    # correctness spot check of the timed outputs against the oracle (rank 0, N=1)
    lens = np.diff(term_off)
    post_per_launch = int(sum(int(lens[t].sum()) for t in
                              (np.asarray(qq, np.int64) for qq in queries)))
    res = {
        "value": nq * args.steps / el,
        "ms_per_step": 1000.0 * el / args.steps,
        "postings_per_query": post_per_launch / nq,
        "docs": n_docs, "v_terms": V, "postings": int(ix.info()["n_postings"]),
        "blocks": ix.info()["n_blocks"],
        "kernel_ms": {"score_blocks": ms_sb / max(n_sb, 1), "merge_topk": ms_mg / max(n_mg, 1)},
        "kernel_ms_per_step": {"score_blocks": ms_sb / max(args.steps, 1),
                               "merge_topk": ms_mg / max(args.steps, 1)},
        "launches_per_step": n_sb / max(args.steps, 1),
    }
    if dist.is_initialized():
        n_x = max(xch["n"], 1)
        res["exchange"] = {
            # device-synchronised host time of the two-round exchange per step (the
            # scorer's tail included: the rounds need its counts), max over ranks
            "collective_ms_per_step": max_over_ranks(xch["ms"] / n_x),
            # keys this rank sent per query (a plain all_gather: k) and bytes per step
            "gathered_keys_per_query": xch["keys_per_query"] / n_x,
            "gathered_bytes_per_query": 8.0 * xch["keys_per_query"] / n_x,
            "plain_all_gather_bytes_per_query": 8.0 * k,
            "bytes_sent_per_step": xch["bytes"] / n_x,
            "path": xch["path"],
            "merged_equals_local_at_one_rank": same,
        }
        if alt is not None:
            alt["collective_ms_per_step"] = max_over_ranks(alt["collective_ms_per_step"])
            res["exchange"]["other_path"] = alt
    # algorithmic bytes of one step (every query's postings, 4 B each: the packed u32
    # posting (doc_in_block << 8) | value) over the score_blocks time of one step -- a
    # step is several launches when the candidate workspace splits the queries into
    # chunks (nb * k * 8 bytes per query, <= 4 GiB per chunk: one launch per step at
    # 100 k and 1.1 M docs, 4 at 8.8 M)
    bytes_per_launch = 4.0 * post_per_launch
    avg_s = (ms_sb / max(args.steps, 1)) / 1000.0  # score_blocks time per step
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    # PMC traffic (beyond-L2 bytes: FETCH_SIZE counts Infinity-Cache hits too) of the
    # leg's own summary, per launch -> per step
    leg = {DOCS_PER_SHARD: "retrieve", 1_100_000: "retrieve_shard",
           8_800_000: "retrieve_full"}.get(n_docs)
    # the scorer instantiation this shard runs: shards of 2..7 blocks take the emit-above
    # selection (score_blocks_kernel<4>, EXT_FEW), larger ones the plain kernel
    nb = ix.info()["n_blocks"]
    # (di_index::few_blocks: 2..7 blocks, 2 k <= 2048, the shared threshold not forced on)
    sb_kernel = ("score_blocks_kernel<4>" if 2 <= nb < 8 and 2 * k <= 2048 and
                 os.environ.get("DI_SCORE_THRESHOLD", "")[:1] != "1"
                 else "score_blocks_kernel<0>")
    traffic, src = load_pmc_traffic(sb_kernel, leg) if leg else (None, None)
    if traffic is not None:
        traffic *= n_sb / max(args.steps, 1)
    # HBM pricing by the algorithmic bytes (a side figure: the counters show the popular
    # lists served from L2 / MALL -- PMC traffic below -- so this ceiling does not bind):
    # 4 B per posting (the device word (doc_in_block << 10 | value) ^ X) and the 5 B of
    # the reference's on-disk record (inverted_index.py:18-29)
    # (not a roofline fraction: the postings are L2-reused across queries, so the
    # algorithmic byte rate can pass the HBM peak -- verdict r5; the beyond-L2 ratio
    # beside it is what the kernel really fetches per algorithmic byte)
    hbm = {
        "kernel": sb_kernel,
        "bound": "not_binding (postings L2-reused across queries)",
        "algorithmic_rate_GBps": round(achieved, 1),
        "algorithmic_rate_GBps_at_5B_per_posting": round(achieved * 1.25, 1),
        "hbm_peak_GBps": HBM_PEAK_GBS,
        "traffic": traffic,
        "beyond_l2_over_algorithmic": (round(traffic / bytes_per_launch, 4)
                                       if traffic and bytes_per_launch else None),
        "algorithmic_bytes_per_step": bytes_per_launch,
        "algorithmic_bytes_per_step_5B": 5.0 * post_per_launch,
        "traffic_source": src,
    }
    # the scatter's own ceiling (the headline roofline of the retrieve legs): one
    # conflict-free ds_read_b32 (2 LDS cycles per wave) + ds_write_b32 (4) per 64
    # postings on each CU (MI355X_MICROARCH.md "LDS" table)
    lds_peak = LDS_CUS * LDS_CLOCK_HZ / LDS_CYCLES_PER_64_POSTINGS * 64.0
    posts_per_s = post_per_launch / avg_s if avg_s > 0 else 0.0
    lds = {"kernel": sb_kernel, "bound": "lds",
           "achieved": round(posts_per_s / 1e12, 4), "peak": round(lds_peak / 1e12, 4),
           "unit": "Tpostings/s", "frac": round(posts_per_s / lds_peak, 4),
           "traffic": traffic,
           "model": f"{LDS_CYCLES_PER_64_POSTINGS:g} LDS cycles per 64 postings (ds_read_b32 2 + "
                    f"ds_write_b32 4) x {LDS_CUS} CUs x {LDS_CLOCK_HZ / 1e9:g} GHz",
           "postings_per_step": post_per_launch,
           "score_blocks_ms_per_step": round(avg_s * 1000.0, 4),
           "launches": n_sb,
           "hbm_priced": hbm}
    pmc = load_pmc_counters(sb_kernel, leg) if leg else None
    if pmc:
        for c in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE"):
            if c in pmc[0]:
                lds[c.lower() + "_per_launch"] = pmc[0][c]
        if "SQ_LDS_BANK_CONFLICT" in pmc[0] and "SQ_LDS_IDX_ACTIVE" in pmc[0]:
            lds["bank_conflict_share"] = round(pmc[0]["SQ_LDS_BANK_CONFLICT"] /
                                               max(pmc[0]["SQ_LDS_IDX_ACTIVE"], 1.0), 4)
        lds["counters_source"] = pmc[1]
    res["roofline"] = lds
    return res, (term_off, pdoc - np.uint32(doc_lo), pval, queries,
                 out_doc, out_score, out_n)


MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md; no sparsity)
MFMA_F32_PEAK_TFLOPS = 157.3  # f32 MFMA (the fp32 leg)
NOMINAL_CLOCK_GHZ = 2.4  # the clock the peaks are quoted at


def synthetic_state_dict(cfg, seed=0):
    """Random-init weights of the named architecture (no checkpoints offline):
    N(0, 0.02) matrices/biases, LayerNorm gamma 1 + N(0, 0.02)."""
    rng = np.random.default_rng(seed)
    H, F, V, P = cfg.hidden, cfg.intermediate, cfg.vocab_size, cfg.max_positions

    def n(*shape):
        return torch.from_numpy((0.02 * rng.standard_normal(shape, dtype=np.float32)))

    sd = {"bert.embeddings.word_embeddings.weight": n(V, H),
          "bert.embeddings.position_embeddings.weight": n(P, H),
          "bert.embeddings.token_type_embeddings.weight": n(cfg.type_vocab, H),
          "bert.embeddings.LayerNorm.weight": 1 + n(H), "bert.embeddings.LayerNorm.bias": n(H)}
    for l in range(cfg.layers):
        p = f"bert.encoder.layer.{l}."
        for m in ("query", "key", "value"):
            sd[p + f"attention.self.{m}.weight"] = n(H, H)
            sd[p + f"attention.self.{m}.bias"] = n(H)
        sd[p + "attention.output.dense.weight"] = n(H, H)
        sd[p + "attention.output.dense.bias"] = n(H)
        sd[p + "attention.output.LayerNorm.weight"] = 1 + n(H)
        sd[p + "attention.output.LayerNorm.bias"] = n(H)
        sd[p + "intermediate.dense.weight"] = n(F, H)
        sd[p + "intermediate.dense.bias"] = n(F)
        sd[p + "output.dense.weight"] = n(H, F)
        sd[p + "output.dense.bias"] = n(H)
        sd[p + "output.LayerNorm.weight"] = 1 + n(H)
        sd[p + "output.LayerNorm.bias"] = n(H)
    sd["impact_score_encoder.0.weight"] = n(1, H)
    sd["impact_score_encoder.0.bias"] = n(1)
    return sd


def synthetic_docs_tokens(n_docs, vocab, seed, max_len=300):
    """n_i = clip(round(N(200, 60)), 8, max_len); ids uniform [5, V);
    <s> first; words = runs of 1+Geom(0.3) tokens, unique terms ~0.7 of words."""
    rng = np.random.default_rng(seed)
    lens = np.clip(np.rint(rng.normal(200, 60, n_docs)), 8, max_len).astype(np.int32)
    cu = np.zeros(n_docs + 1, np.int32)
    cu[1:] = np.cumsum(lens)
    ids = rng.integers(5, vocab, int(cu[-1])).astype(np.int32)
    ids[cu[:-1]] = 0
    term_tok, cu_terms = [], [0]
    for n in lens:
        starts = [1]
        while True:
            nxt = starts[-1] + int(rng.geometric(0.3))  # word = 1 + Geom(0.3) tokens
            if nxt >= n - 1:
                break
            starts.append(nxt)
        keep = [s for s in starts if rng.random() < 0.7]
        term_tok += keep
        cu_terms.append(cu_terms[-1] + len(keep))
    return ids, cu, lens, np.array(term_tok, np.int32), np.array(cu_terms, np.int32)


def flops_per_doc(n, H=768, L=12, t=None, q_pruned=False):
    """sum over layers (24 n H^2 + 4 n^2 H) + 2 n H (real tokens only).
    With t (kept terms per doc): the FLOPs executed when the last layer runs its
    attention queries and its O / FFN GEMMs on the t term rows only (the pruned last
    layer; the K / V projections still cover every row, and the Q projection too unless
    q_pruned -- the bf16x3 path projects Q from the term rows only)."""
    n = np.asarray(n, np.float64)
    f = L * (24.0 * n * H * H + 4.0 * n * n * H) + 2.0 * n * H
    if t is not None:
        t = np.asarray(t, np.float64)
        f = f - ((20.0 if q_pruned else 18.0) * H * H * (n - t) + 4.0 * (n - t) * n * H)
    return f


def prune_last_layer():
    """The term-output encode (bf16 and bf16x3) computes the last layer on the kept
    terms' rows only (bit-identical impacts)."""
    return True


def peak_of(precision):
    """Dense MFMA peak of a precision's arithmetic: bf16x3 is priced against its own
    scheme (three bf16 products per fp32 product, 2500 / 3 TF/s of fp32-equivalent
    work); fp32 against the f32 MFMA peak."""
    return (MFMA_F32_PEAK_TFLOPS if precision == "fp32" else
            MFMA_BF16_PEAK_TFLOPS / 3.0 if precision == "bf16x3" else MFMA_BF16_PEAK_TFLOPS)


def encode_leg(args, rank, world, dev, precision="bf16", steps=None):
    """precision "bf16": the throughput mode configs[1] names; "bf16x3": the
    fp32-faithful mode (split-bf16 GEMMs, f32 attention / LayerNorm; impacts within
    1e-3 of the fp32 reference -- tests/test_encoder_bf16x3_gpu.py); "fp32": f32 MFMA
    throughout (the exactness side leg).  steps: timed steps (default: --steps)."""
    n_steps = args.steps if steps is None else steps
    from improving_learned_index_amd.encoder import DeviceEncoder, EncoderConfig

    t0 = time.time()
    cfg = EncoderConfig.xlmr_base()
    sd = synthetic_state_dict(cfg, seed=0)
    enc = DeviceEncoder(sd, cfg, precision=precision, device=dev)
    ids, cu, lens, tt, ct = synthetic_docs_tokens(args.docs, cfg.vocab_size, seed=100 + rank,
                                                  max_len=args.max_len)
    log(f"[rank {rank}] {precision} encoder ready in {time.time() - t0:.1f}s: {args.docs} docs, "
        f"{int(cu[-1])} tokens, {int(ct[-1])} terms per step")
    stream = torch.cuda.current_stream()
    enc.set_stream(stream.cuda_stream)
    d_ids = torch.from_numpy(ids).cuda()
    d_cu = torch.from_numpy(cu).cuda()
    d_tt = torch.from_numpy(tt).cuda()
    d_ct = torch.from_numpy(ct).cuda()
    out = torch.empty(max(1, int(ct[-1])), dtype=torch.float32, device="cuda")
    enc.reserve(int(cu[-1]), args.docs, int(ct[-1]))
    flags = _lib.DI_F_DEVICE_PTRS | _lib.DI_F_ASYNC | 0x10  # DI_F_ROUND3

    def step(timing):
        enc.encode_device(d_ids, d_cu, args.docs, int(cu[-1]), int(lens.max()), d_tt, d_ct,
                          int(ct[-1]), out, flags | (_lib.DI_F_TIMING if timing else 0))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    enc.sync()
    enc.timing("gemm_qkv", reset=True)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(n_steps):
        step(True)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    el = time.perf_counter() - t1
    enc.sync()
    if dist.is_initialized():
        el = max_over_ranks(el)
    kernels = {}
    for name in ("embed_ln", "gemm_qkv", "attention", "gemm_o", "ln", "gemm_ffn1", "gemm_ffn2",
                 "row_ln", "head", "gather_terms"):
        ms, n = enc.timing(name)
        kernels[name] = {"ms_per_step": ms / max(n_steps, 1), "launches": n}
    M, H, F, L = float(cu[-1]), cfg.hidden, cfg.intermediate, cfg.layers
    # rows per launch, averaged over the L launches of a step: the pruned last layer runs
    # O / FFN1 / FFN2 on the T term rows (QKV on all M)
    T = float(ct[-1])
    split = precision == "bf16x3"
    f32 = precision == "fp32"
    prune = prune_last_layer() and not f32  # (the fp32 mode computes every row)
    Mp = ((L - 1) * M + T) / L if prune else M
    # (bf16x3: the pruned last layer's Q projection runs on the T term rows too)
    qkv_rows = ((L - 1) * 3 * M + 2 * M + T) / L if prune and split else 3 * M
    gemm_flops = {"gemm_qkv": 2 * qkv_rows * H * H, "gemm_o": 2 * Mp * H * H,
                  "gemm_ffn1": 2 * Mp * H * F, "gemm_ffn2": 2 * Mp * F * H}
    per_launch = {}
    for k, f in gemm_flops.items():
        ms, n = enc.timing(k)
        avg = ms / max(n, 1) / 1000.0
        per_launch[k] = (f, avg, f / avg / 1e12 if avg > 0 else 0.0)
    dom = max(per_launch, key=lambda k: per_launch[k][1])
    f, avg, tf = per_launch[dom]
    # PMC names (bf16 xlm-roberta-base runs the LayerNorm-folded forward): EPI 5 = folded
    # QKV, 6 = folded FFN1 + GELU, 7 = residual + row statistics (O and FFN2 share it)
    # gemm256_kernel<EPI, SPLIT>: EPI 5 = LN-folded, 6 = folded + GELU, 7 = residual +
    # statistics; bf16x3 folds its LayerNorms the same way (SPLIT = true)
    pmc_name = {"gemm_qkv": "gemm256_kernel<5,%s>", "gemm_ffn1": "gemm256_kernel<6,%s>",
                "gemm_o": "gemm256_kernel<7,%s>",
                "gemm_ffn2": "gemm256_kernel<7,%s>"}[dom] % ("true" if split else "false")
    if f32:
        pmc_name = "gemm_nt_kernel<f32>"  # (the 128-tile f32 MFMA GEMM)
    traffic, src = load_pmc_traffic(pmc_name, "encode_x3" if split else "encode")
    pmc = load_pmc_counters(pmc_name, "encode_x3" if split else "encode")
    # the PMC run's own clock: GRBM_GUI_ACTIVE (busy cycles summed over the 8 XCDs) over
    # each profiled dispatch's own duration (tools/pmc_summary.py), never over this run's
    # time; with it that run's achieved rate and its fraction at the clock it held
    eff_ghz = pmc_run = None
    if pmc and pmc[0].get("effective_clock_ghz") and pmc[0].get("duration_ns_avg"):
        eff_ghz = pmc[0]["effective_clock_ghz"]
        pmc_tf = f / (pmc[0]["duration_ns_avg"] * 1e-9) / 1e12
        pmc_run = {"source": pmc[1], "avg_launch_ms": round(pmc[0]["duration_ns_avg"] / 1e6, 4),
                   "achieved": round(pmc_tf, 1), "effective_clock_ghz": round(eff_ghz, 3),
                   "frac_at_effective_clock": round(pmc_tf / (peak_of(precision) * eff_ghz /
                                                              NOMINAL_CLOCK_GHZ), 4)}
    # bf16x3: algorithmic (fp32) FLOPs against the split scheme's own peak -- three
    # bf16 MFMA products per fp32 product, 2500 / 3 TF/s (the f32 MFMA peak is 157.3)
    peak = peak_of(precision)
    # executed FLOPs (the pruned last layer skips the rows no output reads)
    model_flops = float(flops_per_doc(lens, t=np.diff(ct) if prune else None,
                                      q_pruned=prune and split).sum())
    docs_per_s = world * args.docs * n_steps / el
    res = {
        "value": docs_per_s,
        "ms_per_step": 1000.0 * el / n_steps,
        "steps": n_steps,
        "tokens_per_step": int(cu[-1]),
        "kernels": kernels,
        "gemm_tflops": {k: round(v[2], 1) for k, v in per_launch.items()},
        # digest of the last step's impacts: kernel changes that claim bit-identical
        # outputs are checked by comparing it across builds (seeded weights and docs)
        "out_sha1": hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest(),
        "model_tflops": round(model_flops * n_steps / el / 1e12 * 1.0, 1),
        "model_flops_frac": round(model_flops * n_steps / el / 1e12 / peak, 4),
        "roofline": {"kernel": f"{pmc_name} ({dom})", "bound": "mfma",
                     "achieved": round(tf, 1), "peak": round(peak, 1), "unit": "TFLOP/s",
                     "frac": round(tf / peak, 4), "traffic": traffic,
                     "peak_clock_ghz": NOMINAL_CLOCK_GHZ,
                     # (counters, durations and clock of one rocprofv3 --pmc run of this
                     # tree's kernels; the headline achieved / frac are this run's)
                     "pmc_run": pmc_run,
                     "traffic_source": src, "algorithmic_flops_per_launch": f, "avg_launch_ms": round(avg * 1000, 4),
                     "launches": enc.timing(dom)[1]},
    }
    return res, (sd, cfg, ids, cu, lens, tt, ct, out)


# bf16x3 against the torch fp32 oracle (oracle/encoder_ref.py, CPU, padded batches):
# tests/test_encoder_bf16x3_gpu.py::test_flip_rates_vs_torch_fp32_oracle, 512
# bench-shaped docs (21 409 terms), GPUTEST_r04 / profiles/round4_z9_pytest_gpu.log
ORACLE_FLIPS = {"text_flip_rate": 2.48e-3, "quantized_flip_rate": 2.80e-4, "max_rel": 2.5e-5,
                "fp32_mode_text_flip_rate": 3.3e-4, "fp32_mode_quantized_flip_rate": 4.7e-5,
                "source": "tests/test_encoder_bf16x3_gpu.py::test_flip_rates_vs_torch_fp32_oracle "
                          "(512 bench-shaped docs vs oracle/encoder_ref.py fp32; DESIGN.md §0 row 8)"}


def flip_rates(out_x3, out_f32):
    """bf16x3 vs the fp32 mode over one bench step's impacts (same seeded docs and
    weights): the 3-decimal texts (A9: the round3 f32 values print differently iff they
    differ) and the 8-bit integers quantize.py writes (int(v * 255 / max), fp64, each
    run quantized by its own max; indexing/quantize.py:31-44)."""
    a = out_x3.cpu().numpy().astype(np.float64)
    b = out_f32.cpu().numpy().astype(np.float64)
    n = min(a.size, b.size)
    a, b = a[:n], b[:n]
    qa = np.trunc(a * (255.0 / a.max())) if n and a.max() > 0 else a
    qb = np.trunc(b * (255.0 / b.max())) if n and b.max() > 0 else b
    return {"terms": int(n), "text_flip_rate": float((a != b).mean()) if n else 0.0,
            "quantized_flip_rate": float((qa != qb).mean()) if n else 0.0,
            # (the impacts are the round3 values: a text flip is one 1e-3 step)
            "max_abs_diff": float(np.abs(a - b).max()) if n else 0.0,
            "vs_torch_fp32_oracle": ORACLE_FLIPS}


def cpu_baseline_encode(args, sd, cfg, ids, cu, lens, tt, ct, out):
    sys.path.insert(0, str(ROOT / "oracle"))
    import encoder_ref

    c = {"hidden_size": cfg.hidden, "num_attention_heads": cfg.heads,
         "num_hidden_layers": cfg.layers, "layer_norm_eps": cfg.layer_norm_eps,
         "pad_token_id": cfg.pad_id}
    threads = torch.get_num_threads()
    done, toks, t0 = 0, 0, time.perf_counter()
    bs = 8
    while time.perf_counter() - t0 < args.cpu_seconds and done < len(lens):
        b = range(done, min(done + bs, len(lens)))
        S_ = int(max(lens[i] for i in b))
        pad = np.full((len(b), S_), cfg.pad_id, np.int64)
        mask = np.zeros((len(b), S_), np.int64)
        for r, i in enumerate(b):
            pad[r, :lens[i]] = ids[cu[i]:cu[i + 1]]
            mask[r, :lens[i]] = 1
        with torch.no_grad():
            encoder_ref.forward(sd, c, torch.from_numpy(pad), torch.from_numpy(mask), "xlmr",
                                "softplus")
        done += len(b)
        toks += int(sum(lens[i] for i in b))
    el = time.perf_counter() - t0
    return {"value": round(done / el, 3), "unit": "docs/s", "cores": threads, "kind": "port",
            "sample": f"{done} of the step's docs ({toks} tokens, batches of {bs} padded to "
                      f"the batch max), fp32 PyTorch-CPU restatement oracle/encoder_ref.py, "
                      f"{el:.1f}s"}


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


def index_e2e_leg(args, dev, rank=0, world=1):
    """A1-A9 end to end through the drop-in CLI's own code path (index.py: collection
    file -> CollectionParser -> TokenizerPool workers -> HIP encoder -> native TSV
    writer), bf16x3 (the CLI default, fp32-faithful).  The collection is synthetic
    MS MARCO-shaped text over the repo's local XLM-R-style tokenizer vocabulary
    (tests/golden/tokenizer.json: the hub tokenizer does not exist offline), word counts
    clip(N(150, 45), 6, 230); the checkpoint is random-init xlm-roberta-base.  Setup
    (checkpoint load, weight upload, worker start) is timed apart from the indexing."""
    import tempfile

    from improving_learned_index_amd import index as index_cli
    from improving_learned_index_amd.encoder import EncoderConfig
    from improving_learned_index_amd.indexer import Indexer, TokenizerPool, resolve_tokenizer
    from improving_learned_index_amd.models import DeepImpact

    tok_path = ROOT / "tests" / "golden" / "tokenizer.json"
    vocab = json.loads(tok_path.read_text())["model"]["vocab"]
    words = np.array([w[1:] for w, _ in vocab if w.startswith("\u2581") and len(w) > 2])
    rng = np.random.default_rng(7 + rank)
    n_docs = args.e2e_docs
    lens = np.clip(rng.normal(150, 45, n_docs), 6, 230).astype(int)
    procs = max(1, min(args.e2e_procs, os.cpu_count() or 1))
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        td = Path(td)
        coll = td / "collection.tsv"
        with open(coll, "w") as f:
            for i, n in enumerate(lens):
                f.write(f"{i}\t{' '.join(words[rng.integers(0, len(words), n)])}\n")
        cfg = EncoderConfig.xlmr_base()
        ckpt = td / "DeepImpact.pt"
        torch.save({"model_state_dict": synthetic_state_dict(cfg, seed=0)}, ckpt)
        t0 = time.perf_counter()
        tok = resolve_tokenizer(str(ckpt), tok_path)
        pool = TokenizerPool(procs, tok, 300, "word_ids")
        try:
            model = DeepImpact.load(str(ckpt), tokenizer_path=tok_path, precision="bf16x3",
                                    device=dev, max_length=300)
            indexer = Indexer(model, model_batch_size=args.e2e_model_batch, num_processes=procs,
                              pool=pool)
            with open(os.devnull, "w") as dn:  # warm the workers (imports, tokenizer)
                with open(coll) as f:
                    indexer.index([next(f).split("\t", 1)[1] for _ in range(4 * procs)], dn)
            t_setup = time.perf_counter() - t0
            # one worker's tokenize rate on 1000 of the collection's docs (the host budget:
            # N ranks x workers x this rate against N x the device encode rate)
            with open(coll) as f:
                sample = [next(f).split("\t", 1)[1] for _ in range(min(1000, n_docs))]
            per_worker = pool.worker_rate(sample)
            if dist.is_initialized():  # every rank's workers start together (host cores shared)
                dist.barrier()
            t1 = time.perf_counter()
            n = index_cli._index_file(indexer, coll, "msmarco", td / "collection.index",
                                      args.e2e_process_batch, None, t1)
            el = time.perf_counter() - t1
            out_bytes = (td / "collection.index").stat().st_size
        finally:
            pool.close()
    log(f"[rank {rank}] index e2e: {n} docs in {el:.2f}s after {t_setup:.1f}s setup ({procs} "
        f"tokenizer workers)")
    if dist.is_initialized():  # all ranks' documents over the slowest rank's time (host tokenization of
        el = max_over_ranks(el)  # N ranks x their workers on the node's shared cores)
    return {"value": round(world * n / el, 1), "unit": "docs/s", "docs": int(world * n),
            "ranks": world, "seconds": round(el, 3),
            "setup_seconds": round(t_setup, 2), "tokenizer_workers": procs,
            # host budget (verdict r5 #7): the node's CPUs, this process's share, the
            # workers per rank and one worker's rate; at N ranks the host side offers about
            # N x workers x rate docs/s (while cores last) against N x the device encode
            "host_cpus": os.cpu_count(),
            "cpu_affinity": (len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                             else None),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "tokenizer_workers_per_rank": procs,
            "tokenize_docs_per_s_per_worker": round(per_worker, 1),
            "host_tokenize_docs_per_s_per_rank": round(procs * per_worker, 1),
            "precision": "bf16x3", "output_bytes": int(out_bytes),
            "model_batch_size": args.e2e_model_batch, "process_batch_size": args.e2e_process_batch,
            "path": "index.py _index_file: CollectionParser -> TokenizerPool -> di_encode "
                    "(bf16x3, ROUND3) -> di_format_impact_lines (model batches below 256 "
                    "docs run as 256-doc device chunks)"}


def rank_e2e_leg(args, dev):
    """A11-A13 end to end through the drop-in `rank` CLI's own code path: a synthetic
    100 k-doc impact TSV (the retrieve leg's generator, native writer) -> quantize_file
    -> create_index (reference-format files) -> Ranker(index, queries.tsv) -> run file:
    query text tokenized by the repo's local tokenizer (terms '▁t<id>', the generator's
    names), one batched GPU search per 8192 queries, the run file written natively.
    Timed: Ranker construction (vocabulary + index load to the GPU) and run() apart."""
    import shutil
    import tempfile

    from improving_learned_index_amd.inverted_index import create_index
    from improving_learned_index_amd.quantize import quantize_file
    from improving_learned_index_amd.ranker import Ranker

    n = DOCS_PER_SHARD
    V = v_terms(n)
    td = Path(tempfile.mkdtemp(dir="/tmp"))
    try:
        S.synth_impact_tsv(td / "collection.index", n, V, seed=4321)
        quantize_file(td / "collection.index", td / "collection.quantized", sharded=False)
        create_index(td / "collection.quantized", td / "index")
        queries = S.msmarco_like_queries(args.queries, V, seed=1234)
        with open(td / "queries.tsv", "w") as f:
            for i, q in enumerate(queries):
                f.write(f"{1048576 + i}\t{' '.join(f't{t}' for t in q)}\n")
        t0 = time.perf_counter()
        r = Ranker(td / "index", td / "queries.tsv", td / "run.tsv",
                   tokenizer_path=ROOT / "tests" / "golden" / "tokenizer.json", device=dev,
                   top_k=args.k, sharded=False)  # (rank 0 alone: no collectives)
        t_load = time.perf_counter() - t0
        t1 = time.perf_counter()
        r.run()
        el = time.perf_counter() - t1
        lines = sum(1 for _ in open(td / "run.tsv", "rb"))
        size = (td / "run.tsv").stat().st_size
    finally:
        shutil.rmtree(td, ignore_errors=True)
    log(f"rank e2e: {len(queries)} queries in {el:.2f}s after {t_load:.2f}s load, {lines} lines")
    return {"value": round(len(queries) / el, 1), "unit": "queries/s", "queries": len(queries),
            "k": args.k, "seconds": round(el, 3), "load_seconds": round(t_load, 2),
            "run_file_lines": lines, "run_file_bytes": int(size), "docs": n, "v_terms": V,
            "path": "ranker.Ranker.run: query text -> process_query (local tokenizer) -> "
                    "term ids -> di_index_search (one batch) -> di_format_run_lines -> run file"}


def text_legs(args):
    """A10 + A11 at one 8-way shard of configs[2] (1.1 M docs, V = 2 N): the impact TSV
    the index CLI writes (synthetic, the retrieve legs' generator, native writer) ->
    quantize_file (di_quantize_file: threaded parse, fp64 GPU quantize, threaded
    format) -> InvertedIndexCreator.run (di_build_reference_index: threaded parse /
    vocabulary / bucketing / per-term value sort, byte-identical files).  Each timed
    region is the whole call, file read and write included, as the reference's rates
    (7.0 k / 4.7 k docs/s, 1 core) are.  Host threads: DI_HOST_THREADS or
    OMP_NUM_THREADS (16 on the GPU box).  Checked: the index holds exactly the
    generator's postings (di_synth_postings, same seed)."""
    import ctypes
    import shutil
    import tempfile

    from improving_learned_index_amd.inverted_index import create_index
    from improving_learned_index_amd.quantize import quantize_file

    n = args.text_docs
    V = v_terms(n)
    log(f"text legs: {n} docs (rank 0)")
    td = Path(tempfile.mkdtemp(dir="/tmp"))
    try:
        t0 = time.perf_counter()
        n_pairs = S.synth_impact_tsv(td / "collection.index", n, V, seed=4321)
        t_gen = time.perf_counter() - t0
        in_bytes = (td / "collection.index").stat().st_size
        t0 = time.perf_counter()
        # (rank 0 alone runs these legs: the single-process quantizer, never the
        # torchrun-sharded one, whose collectives the other ranks would never join)
        quantize_file(td / "collection.index", td / "collection.quantized", sharded=False)
        t_q = time.perf_counter() - t0
        (td / "collection.index").unlink()
        q_bytes = (td / "collection.quantized").stat().st_size
        t0 = time.perf_counter()
        create_index(td / "collection.quantized", td / "index")
        t_c = time.perf_counter() - t0
        dat = (td / "index" / "inverted_index.dat").stat().st_size
        term_off = np.zeros(V + 1, np.int64)
        n_post = ctypes.c_int64(0)
        _lib.check(_lib.lib().di_synth_postings(n, V, 4321, 100, 200, 1.2,
                                                term_off.ctypes.data_as(ctypes.c_void_p), None,
                                                None, 0, ctypes.byref(n_post), None))
        if dat != 5 * n_post.value:
            raise SystemExit(f"text legs: index holds {dat // 5} postings, the generator "
                             f"{n_post.value}")
    finally:
        shutil.rmtree(td, ignore_errors=True)
    threads = int(os.environ.get("DI_HOST_THREADS") or os.environ.get("OMP_NUM_THREADS") or
                  (os.cpu_count() or 1))
    log(f"text legs: {n} docs, gen {t_gen:.1f}s, quantize {t_q:.2f}s, create {t_c:.2f}s")
    common = {"docs": n, "v_terms": V, "terms": int(n_pairs), "host_threads": min(threads, 64)}
    return {
        "quantize": {"value": round(n / t_q, 1), "unit": "docs/s", "seconds": round(t_q, 3),
                     "input_bytes": int(in_bytes), "output_bytes": int(q_bytes),
                     "reference_cpu_docs_s": REF_QUANTIZE_DOCS_S,
                     "vs_reference_cpu": round(n / t_q / REF_QUANTIZE_DOCS_S, 1), **common},
        "index_create": {"value": round(n / t_c, 1), "unit": "docs/s", "seconds": round(t_c, 3),
                         "postings": int(dat // 5), "reference_cpu_docs_s": REF_CREATE_DOCS_S,
                         "vs_reference_cpu": round(n / t_c / REF_CREATE_DOCS_S, 1), **common},
    }


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N ranks as a
    child torchrun, one process per GPU, and forward its JSON line.  The reference's
    multi-GPU encode needs no launcher either (`Indexer` wraps the model in
    DataParallel whenever device_count() > 1, indexer.py:25-26).  Runs before any GPU
    call in this process and never execs: the parent only waits on the child."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", str(ROOT / "bench.py")] + argv
    log(f"bench: launching {n} ranks: {' '.join(cmd[1:])}")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
        "HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    p = subprocess.Popen(cmd, cwd=str(ROOT), env=env, stdout=subprocess.PIPE, text=True)
    n_lines = 0
    for line in p.stdout:
        if line.startswith("{"):
            n_lines += 1
        print(line, end="", flush=True)
    rc = p.wait()
    if rc == 0 and n_lines != 1:
        log(f"bench: the {n}-rank run printed {n_lines} JSON lines, expected 1")
        return 3
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--queries", type=int, default=N_QUERIES)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--docs", type=int, default=8192, help="docs encoded per step per GPU (1024: -3%%, 4096: -1%%: the 256-row GEMM tiles quantize less on 256 CUs with more rows)")
    ap.add_argument("--max-len", type=int, default=300)
    ap.add_argument("--e2e-docs", type=int, default=16000, help="index_e2e leg: documents")
    ap.add_argument("--e2e-procs", type=int, default=16, help="index_e2e leg: tokenizer workers")
    ap.add_argument("--e2e-model-batch", type=int, default=32,
                    help="index_e2e leg: --model_batch_size (reference default 32)")
    ap.add_argument("--e2e-process-batch", type=int, default=1600,
                    help="index_e2e leg: --process_batch_size (reference default 1600)")
    ap.add_argument("--text-docs", type=int, default=1_100_000,
                    help="text legs (quantize, index_create): docs of the impact TSV")
    ap.add_argument("--legs", default="encode_x3,encode,encode_fp32,retrieve,retrieve_shard,text,"
                                      "index_e2e,rank_e2e",
                    help="encode_x3 (fp32-faithful bf16x3: the headline), encode (bf16 throughput "
                         "mode), encode_fp32 (f32 MFMA: the exactness side leg, with the bf16x3 "
                         "flip rates against it), retrieve (100k-doc shard, configs[1]), "
                         "retrieve_shard (1.1M docs: "
                         "one 8-way shard of configs[2]), retrieve_full (8.8M docs on one GPU, "
                         "configs[2]), text (quantize + index_create of a 1.1M-doc impact TSV), "
                         "index_e2e (index.py's path end to end, tokenizer workers included), "
                         "rank_e2e (the rank CLI's path end to end on a 100k-doc index)")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}: "
                         f"launch one rank per GPU (--nproc-per-node {args.gpus}) or drop the "
                         f"launcher and let bench.py start the ranks")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    ranks_seen = 1
    # DI_FORCE_DIST=1 under a launcher: the process group and every collective of the
    # multi-rank path even at one rank (a 1-GPU box rehearses the RCCL path that way)
    if world > 1 or (os.environ.get("DI_FORCE_DIST") == "1" and "MASTER_ADDR" in os.environ):
        # one rank per GPU over RCCL; more ranks than GPUs (a 1-GPU rehearsal of the
        # multi-rank path) share the devices over gloo with host-staged collectives
        n_dev = max(1, torch.cuda.device_count())
        torch.cuda.set_device(local % n_dev)
        if world <= n_dev:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        backend = dist.get_backend()
        # every rank contributes a 1: the count the collective actually saw
        one = torch.ones(1, dtype=torch.int64, device="cpu" if _gloo() else "cuda")
        seen = torch.zeros(world, dtype=torch.int64, device=one.device)
        dist.all_gather_into_tensor(seen, one)
        ranks_seen = int(seen.sum().item())
        if ranks_seen != world:
            raise SystemExit(f"bench: all_gather saw {ranks_seen} ranks of {world}")
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    # every leg runs on one real torch stream (torch's default stream has the null
    # handle, which the library's set_stream takes as "own stream": RCCL collectives
    # and the merge would not be ordered after the scorer)
    main_stream = torch.cuda.Stream()
    torch.cuda.set_stream(main_stream)
    legs = set(args.legs.split(","))
    enc_res = ret_res = None
    x3_res = None
    if "encode_x3" in legs:
        x3_res, x3_ctx = encode_leg(args, rank, world, dev, precision="bf16x3")
    if "encode" in legs:
        enc_res, enc_ctx = encode_leg(args, rank, world, dev)
    f32_res = None
    if "encode_fp32" in legs:
        # the exactness side leg: f32 MFMA throughout (fewer timed steps: ~5x the bf16x3
        # step time), and the bf16x3 flips against it on the same docs
        f32_res, f32_ctx = encode_leg(args, rank, world, dev, precision="fp32",
                                      steps=max(1, args.steps // 4))
        if x3_res is not None:
            f32_res["exactness"] = flip_rates(x3_ctx[-1], f32_ctx[-1])
    # (profiling ablations of the scorer, DI_PROFILE_ABLATE, change its results)
    n_check = 0 if os.environ.get("DI_PROFILE_ABLATE") else 20
    if "retrieve" in legs:
        ret_res, ret_ctx = retrieve_leg(args, rank, world, dev, check_queries=n_check)
    e2e_res = index_e2e_leg(args, dev, rank, world) if "index_e2e" in legs else None
    # (rank 0 alone: the single-process CLI, as the text legs)
    rank_res = rank_e2e_leg(args, dev) if "rank_e2e" in legs and rank == 0 else None
    text_res = text_legs(args) if "text" in legs and rank == 0 else None
    big = {}
    for leg, nd in (("retrieve_shard", 1_100_000), ("retrieve_full", 8_800_000)):
        if leg in legs:
            big[leg], _ = retrieve_leg(args, rank, world, dev, n_docs=nd, check_queries=n_check)
            torch.cuda.empty_cache()
    # the headline is the fp32-faithful encode (bf16x3: the reference computes in fp32,
    # indexer.py:46); the bf16 throughput mode is a side line (it flips a third of the
    # quantized integers)
    primary = next((r for r in (x3_res, enc_res, ret_res) + tuple(big.values()) +
                    (e2e_res, rank_res) if r is not None), None)
    if primary is None:
        raise SystemExit("no bench leg selected")
    out = {
        "metric": "docs/sec encoded + queries/sec@top-1000, MS MARCO passage, 1/2/4/8 MI355X",
        "value": round(primary["value"], 2),
        "unit": "docs/s" if primary in (enc_res, x3_res, e2e_res) else "queries/s",
        "n_gpus": world,
        "backend": backend,
        "ranks_seen": ranks_seen,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(primary.get("ms_per_step") or 1e3 * primary.get("seconds", 0), 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16x3" if primary is x3_res else ("bf16" if primary is enc_res else "u8"),
        "data": "synthetic (seeded generators of BASELINE.md §2 / SURVEY §8d); random-init "
                "xlm-roberta-base weights",
        "config": {"workload": "configs[1]: MS MARCO passage 100k-doc slice shape, encode "
                               "(xlm-roberta-base DeepImpact, fp32-faithful split-bf16 "
                               "'bf16x3'; bf16 beside it) + top-1000 retrieve of 6980 "
                               "dev.small-shaped queries",
                   "docs_per_step_per_gpu": args.docs, "max_length": args.max_len,
                   "docs_per_shard": DOCS_PER_SHARD, "queries": args.queries, "k": args.k,
                   "parallelism": f"doc-sharded x{world} (encode: no collective; retrieve: "
                                  f"pruned exact two-round RCCL all-gather of per-shard top-k, "
                                  f"parallel.exchange_topk)",
                   "encode_output": "term impacts (A8/A9 gather + round3); the last layer "
                                    "computes only the rows the gather reads -- bit-identical "
                                    "impacts, DESIGN.md §3" if prune_last_layer() else
                                    "term impacts (A8/A9 gather + round3), every row computed"},
        "roofline": primary.get("roofline"),
        "cpu_baseline": None,
    }
    if enc_res is not None:
        out["encode_bf16"] = {
            "value": round(enc_res["value"], 2), "unit": "docs/s", "dtype": "bf16",
            "precision": "bf16 MFMA, LayerNorms folded: NOT fp32-faithful -- it flips a third "
                         "of the 8-bit quantized integers of the fp32 reference "
                         "(tests/test_encoder_bf16x3_gpu.py::test_flip_rates_at_bench_scale)",
            "ms_per_step": round(enc_res["ms_per_step"], 4),
            **{k: enc_res[k] for k in ("tokens_per_step", "kernels", "gemm_tflops", "model_tflops",
                                       "model_flops_frac", "roofline", "out_sha1")}}
    if f32_res is not None:
        out["encode_fp32"] = {
            "value": round(f32_res["value"], 2), "unit": "docs/s", "dtype": "f32",
            "precision": "f32 MFMA GEMMs and attention, f32 LayerNorm, every row of the last "
                         "layer: the library's fp32 mode (index --precision fp32), the price of "
                         "exactness beside the bf16x3 default",
            "steps": f32_res["steps"], "ms_per_step": round(f32_res["ms_per_step"], 4),
            **{k: f32_res[k] for k in ("kernels", "gemm_tflops", "model_tflops",
                                       "model_flops_frac", "roofline", "out_sha1")}}
        if "exactness" in f32_res:
            out["encode_fp32"]["bf16x3_vs_fp32"] = f32_res["exactness"]
    if x3_res is not None:
        out["encode_fp32_faithful"] = {
            "value": round(x3_res["value"], 2), "unit": "docs/s", "dtype": "bf16x3",
            "precision": "split-bf16 GEMMs (A_hi W_hi + A_hi W_lo + A_lo W_hi, f32 accumulate), "
                         "split-bf16 attention products with f32 softmax, LayerNorms folded into the GEMMs "
                         "(f32 row statistics of the split residual rows), last layer on the kept terms' rows: "
                         "impacts within 1e-3 relative of the fp32 reference (max 8.3e-6 measured, "
                         "tests/test_encoder_bf16x3_gpu.py)",
            "ms_per_step": round(x3_res["ms_per_step"], 4),
            **{k: x3_res[k] for k in ("kernels", "gemm_tflops", "model_tflops",
                                      "model_flops_frac", "roofline", "out_sha1")}}
    if ret_res is not None:
        out["retrieve"] = {"value": round(ret_res["value"], 2), "unit": "queries/s",
                           "ms_per_step": round(ret_res["ms_per_step"], 4),
                           "postings_per_query": round(ret_res["postings_per_query"], 1),
                           "kernel_ms": ret_res["kernel_ms"], "roofline": ret_res["roofline"],
                           "cpu_baseline": None}
        if "exchange" in ret_res:
            out["retrieve"]["exchange"] = ret_res["exchange"]
    if e2e_res is not None:
        out["index_e2e"] = e2e_res
    if rank_res is not None:
        out["rank_e2e"] = rank_res
    if text_res is not None:
        out.update(text_res)
    for leg, r in big.items():
        out[leg] = {"value": round(r["value"], 2), "unit": "queries/s",
                    "docs_per_shard": r["docs"], "postings": r["postings"], "blocks": r["blocks"],
                    "ms_per_step": round(r["ms_per_step"], 4),
                    "postings_per_query": round(r["postings_per_query"], 1),
                    "kernel_ms": r["kernel_ms"], "kernel_ms_per_step": r["kernel_ms_per_step"],
                    "launches_per_step": r["launches_per_step"], "roofline": r["roofline"]}
        if "exchange" in r:
            out[leg]["exchange"] = r["exchange"]
    if rank == 0 and world == 1 and not args.no_cpu:
        if x3_res is not None or enc_res is not None:
            cb = cpu_baseline_encode(args, *(x3_ctx if x3_res is not None else enc_ctx))
            out["cpu_baseline"] = cb
        if ret_res is not None:
            cb = cpu_baseline_retrieve(args, *ret_ctx)
            out["retrieve"]["cpu_baseline"] = cb
            if x3_res is None and enc_res is None:
                out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
