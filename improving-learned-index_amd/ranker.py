"""Query driver over the on-disk index (reference src/deep_impact/evaluation/ranker.py
and src/deep_impact/rank.py).

The reference scores one query per Pool task (pickling the whole index each
time, ranker.py:44-46); here every query of the file is scored by one batched
GPU launch sequence (di_index_search).  The run file holds the same lines; the
reference writes queries in imap_unordered completion order, this writes them
in input order (a valid completion order of the reference).

Multi-GPU (torchrun --nproc-per-node N -m improving_learned_index_amd.rank ...): rank r
loads doc-id shard r of the index on its GPU, every rank scores every query, the
per-shard top-k keys are all-gathered over RCCL and merged on the GPU
(parallel.exchange_merge_device); rank 0 writes the run file -- the same lines as one
process (the keys totally order score, first touch and doc).
"""
from __future__ import annotations

import argparse
import os
import sys
from itertools import product
from pathlib import Path
from typing import Optional, Union

from . import parallel
from .datasets import COLLECTION_TYPES, Queries, QueryRelevanceDataset, RunFile
from .inverted_index import InvertedIndex, reference_n_docs
from .models import DeepImpact


class Ranker:
    def __init__(self, index_path: Union[str, Path], queries_path: Union[str, Path],
                 output_path: Union[str, Path], num_workers: int = 4,
                 qrels_path: Optional[Union[str, Path]] = None, pairwise: bool = False,
                 dataset_type: Optional[str] = COLLECTION_TYPES[0], tokenizer_path=None,
                 device: int = 0, top_k: int = 1000, batch_queries: int = 8192,
                 min_impact: int = 1, block_max: float = 0.0, packed: bool = False,
                 sharded: Optional[bool] = None):
        # pairwise (F4): every query also scores the ordered pair terms 't1|t2' of its
        # distinct terms (ranker.py:53-58), the keys a pairwise impact collection holds
        # (deep_impact_collection.py:36-45).  The reference takes the query terms from
        # its PhoBERT / VnCoreNLP class for this mode (out of scope); here
        # they come from the configured tokenizer, like the plain mode.
        self.pairwise = pairwise
        if tokenizer_path is not None:
            DeepImpact.set_tokenizer(tokenizer_path)
        self.queries = Queries(queries_path=queries_path, dataset_type=dataset_type)
        self.query_iterator = list(self.queries.keys())
        if qrels_path is not None:  # ranker.py:34-35
            self.query_iterator = list(QueryRelevanceDataset(qrels_path=qrels_path).keys())
        # sharded: None = from the torchrun environment; False = this process alone even
        # under a launcher (bench.py's rank-0-only leg: the other ranks never join)
        self.world, self.rank, local = parallel.dist_env()
        if sharded is False:
            self.world, self.rank, local = 1, 0, local
        lo = hi = 0
        self.dist = sharded is not False and (self.world > 1 or parallel.force_dist())
        if self.dist:
            import torch

            device = parallel.rank_device(local)
            # torch's HIP runtime first: the exchange uses torch device tensors, and torch
            # cannot initialise the GPU after the library's (newer) runtime has
            torch.cuda.set_device(device)
            parallel.init_group(parallel.exchange_backend(self.world), device)
            # the collection size: one scan of inverted_index.dat on rank 0, broadcast
            import torch.distributed as dist

            n = [reference_n_docs(index_path) if self.rank == 0 else 0]
            dist.broadcast_object_list(n, src=0)
            lo, hi = parallel.shard_range(n[0], self.world, self.rank)
        self.device = device
        self.index = InvertedIndex(index_path=index_path, device=device, doc_lo=lo, doc_hi=hi,
                                   min_impact=min_impact, block_max=block_max, packed=packed)
        self.run_file = RunFile(run_file_path=output_path) if self.rank == 0 else None
        self.top_k = top_k
        self.batch_queries = batch_queries

    def get_query_terms(self, qid):
        terms = DeepImpact.process_query(query=self.queries[qid])
        if self.pairwise:  # (product materialises both operands before the adds)
            for term1, term2 in product(terms, terms):
                if term1 != term2:
                    terms.add(f"{term1}|{term2}")
        return terms

    def run(self):
        qids = self.query_iterator
        for s in range(0, len(qids), self.batch_queries):
            chunk = qids[s:s + self.batch_queries]
            terms = [self.get_query_terms(q) for q in chunk]
            if self.dist:
                # every shard must apply the terms in one order (the first-touch tie key):
                # process_query returns a set whose iteration order follows the process's
                # hash seed, so rank 0's order is broadcast to all ranks
                import torch.distributed as dist

                ids = [[self.index.term_ids(t) for t in terms]]
                dist.broadcast_object_list(ids, src=0)
                keys, n = parallel.exchange_merge_device(
                    self.index.device_index, ids[0], self.top_k, self.device)
                # (raises on a query some shard rejected, out_n < 0)
                docs, scores = parallel.decode_quant_key_arrays(
                    keys, n, [len(q) for q in ids[0]])
            else:
                docs, scores, n, _ = self.index.search_ids(
                    [self.index.term_ids(t) for t in terms], self.top_k)
            if self.run_file is None:
                continue
            if os.environ.get("DI_RANK_PY_WRITES") == "1":  # (the per-query form, A/B)
                for i, qid in enumerate(chunk):
                    self.run_file.writelines(qid, list(zip(docs[i, :n[i]].tolist(),
                                                           scores[i, :n[i]].tolist())))
            else:
                # (the chunk's lines formatted natively and appended in one write: the
                # bytes of RunFile.writelines per query, datasets.py:305-324)
                self.run_file.write_batch(chunk, docs, scores, n)


def main(argv=None):
    p = argparse.ArgumentParser("Evaluate a DeepImpact by ranking qrels docs & computing evaluation metrics.")
    p.add_argument("--index_path", type=Path, required=True)
    p.add_argument("--queries_path", type=Path, required=True)
    p.add_argument("--output_path", type=Path, required=True)
    p.add_argument("--num_workers", type=int, default=4)
    p.add_argument("--qrels_path", type=Path, default=None)
    p.add_argument("--dataset_type", type=str, default=COLLECTION_TYPES[0], choices=COLLECTION_TYPES)
    p.add_argument("--pairwise", action="store_true")
    p.add_argument("--tokenizer_path", type=str, required=True)
    p.add_argument("--device", type=int, default=None,
                   help="score on this GPU only (default: every visible GPU, see --gpus)")
    p.add_argument("--gpus", type=int, default=None,
                   help="without torchrun: shard the index over this many GPUs, one child rank "
                        "each (default: every visible GPU; 1 = this process only)")
    p.add_argument("--top_k", type=int, default=1000)
    p.add_argument("--min_impact", type=int, default=1,
                   help="query-time pruning: score postings with value >= this (rounded down "
                        "to a power of two); 1 = exact")
    p.add_argument("--block_max", type=float, default=0.0,
                   help="block-max skipping: 0 off, 1 exact, > 1 approximate (skip block "
                        "segments whose bound is below this factor x the running k-th score)")
    p.add_argument("--packed", action="store_true",
                   help="score from the block-compressed postings (configs[4]; exact)")
    argv = list(sys.argv[1:] if argv is None else argv)
    a = p.parse_args(argv)
    if a.device is None:
        n = parallel.ranks_to_spawn(a.gpus)
        if n > 1:
            rc = parallel.spawn_ranks("rank", argv, n)
            if rc:
                raise SystemExit(rc)
            return
    Ranker(a.index_path, a.queries_path, a.output_path, a.num_workers, a.qrels_path, a.pairwise,
           a.dataset_type, a.tokenizer_path, a.device or 0, top_k=a.top_k,
           min_impact=a.min_impact, block_max=a.block_max, packed=a.packed).run()


if __name__ == "__main__":
    main()
