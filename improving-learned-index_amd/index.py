"""CLI: create a DeepImpact impact TSV (drop-in for `python -m src.deep_impact.index`,
reference src/deep_impact/index.py:12-68).

    python -m improving_learned_index_amd.index --collection_path c.tsv \\
        --output_file_path collection.index --model_checkpoint_path ckpt.pt \\
        --tokenizer_path xlm-roberta-base/tokenizer.json [--max_length 300]

Same flags as the reference plus --tokenizer_path / --max_length / --precision /
--device / --variant (the reference hard-wires a hub tokenizer and 512 tokens).
Output bytes are those of the reference (one line per input line, in order).
Multi-GPU: --doc_range start:end encodes one doc-id shard; concatenating the
shard outputs in order gives the single-GPU file.  Under torchrun
(--nproc-per-node N) every rank encodes doc-id shard r on its GPU and rank 0 joins
the parts into --output_file_path (the reference's DataParallel over every visible
GPU, indexer.py:25-26, as one process per GPU).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import time
from pathlib import Path

from . import parallel
from .datasets import COLLECTION_TYPES, CollectionParser
from .indexer import Indexer, TokenizerPool, pool_supported, resolve_tokenizer
from .models import DeepImpact

BATCH_SIZE = 32  # src/utils/defaults.py:15

logger = logging.getLogger("index")


def run(collection_path, collection_type, output_file_path, model_checkpoint_path,
        num_processes=8, process_batch_size=50 * BATCH_SIZE, model_batch_size=BATCH_SIZE,
        tokenizer_path=None, max_length=None, precision="bf16x3", device=0, variant="xlmr",
        doc_range=None, pairwise=False, first_shard=True):
    if pairwise:
        raise NotImplementedError("DeepPairwiseImpact is outside this build (SURVEY §8f F4)")
    start = time.time()
    # the tokenizer workers start before the GPU is initialised (DeepImpact.load)
    tok = resolve_tokenizer(model_checkpoint_path, tokenizer_path)
    pool = None
    if num_processes > 1 and tok is not None and pool_supported():
        pool = TokenizerPool(num_processes, tok, max_length or DeepImpact.max_length,
                             "bert_legacy" if variant == "bert" else "word_ids")
    try:
        model = DeepImpact.load(model_checkpoint_path, tokenizer_path=tokenizer_path,
                                precision=precision, device=device, variant=variant,
                                max_length=max_length)
        indexer = Indexer(model, model_batch_size=model_batch_size,
                          num_processes=num_processes, pool=pool)
        return _index_file(indexer, collection_path, collection_type, output_file_path,
                           process_batch_size, doc_range, start, first_shard)
    finally:
        if pool is not None:
            pool.close()


def _index_file(indexer, collection_path, collection_type, output_file_path,
                process_batch_size, doc_range, start, first_shard=True):
    """index.py:31-44.  Batches are tokenized one ahead (Indexer.submit) while the
    previous one encodes and writes; they are written in order, so the bytes are the
    sequential loop's.

    A doc-id shard (doc_range) writes its docs' lines only: the joined shards are the
    single-process file.  The reference's one empty batch -- at line 1 when
    process_batch_size is 1 (the flush comes before the append), or the final flush of
    an empty collection -- writes an empty line; the shard holding line 1 (resp. the
    first shard) writes it."""
    lo, hi = (0, None) if doc_range is None else doc_range
    pending = None  # submitted, not yet written
    # (DI_INDEX_SYNC_WRITES=1: format and write each batch before the next encode, A/B)
    defer = os.environ.get("DI_INDEX_SYNC_WRITES") != "1"

    def flush(batch):
        nonlocal pending
        if not hasattr(indexer, "submit"):  # any object with the reference's index()
            indexer.index(batch, out)
            return
        handle = indexer.submit(batch)
        if pending is not None:
            # (its formatting and write overlap the next batch's encode)
            indexer.finish(pending, out, wait=not defer)
        pending = handle

    with open(collection_path) as f, open(output_file_path, "w") as out:
        batch = []
        n = 0
        any_line = False
        for i, passage in enumerate(f, start=1):
            any_line = True
            if hi is not None and i - 1 >= hi:
                break
            if i - 1 < lo:
                continue
            # index.py:35 (first batch one short).  A shard flushes an empty batch only
            # where the single process does (line 1, process_batch_size 1): its other
            # flush points may fall on another shard's batch
            if i % process_batch_size == 0 and (doc_range is None or batch or i == 1):
                flush(batch)
                logger.info(f"Indexed {i} passages [Rate: {i / (time.time() - start):.2f} "
                            f"passages/s]")
                batch = []
            doc_id, passage = CollectionParser.parse(passage, collection_type)
            batch.append(passage)
            n += 1
        if doc_range is None or batch or (first_shard and not any_line):
            flush(batch)
        if pending is not None:
            indexer.finish(pending, out)
        if hasattr(indexer, "drain"):
            indexer.drain()
    return n


def main(argv=None):
    p = argparse.ArgumentParser("Create a DeepImpact index by computing impacts of all document terms.")
    p.add_argument("--collection_path", type=Path, required=True)
    p.add_argument("--collection_type", type=str, default="msmarco", choices=COLLECTION_TYPES)
    p.add_argument("--output_file_path", type=Path, required=True)
    p.add_argument("--model_checkpoint_path", type=str, required=True)
    p.add_argument("--num_processes", type=int, default=8)
    p.add_argument("--process_batch_size", type=int, default=50 * BATCH_SIZE)
    p.add_argument("--model_batch_size", type=int, default=BATCH_SIZE)
    p.add_argument("--pairwise", action="store_true")
    p.add_argument("--tokenizer_path", type=str, default=None)
    p.add_argument("--max_length", type=int, default=None)
    p.add_argument("--precision", choices=["bf16x3", "fp32", "bf16"], default="bf16x3",
                   help="bf16x3 (default): fp32-faithful split-bf16; fp32: f32 MFMA; "
                        "bf16: throughput mode, NOT fp32-faithful (different round3 text)")
    p.add_argument("--device", type=int, default=None,
                   help="encode on this GPU only (default: every visible GPU, see --gpus)")
    p.add_argument("--gpus", type=int, default=None,
                   help="without torchrun: encode on this many GPUs, one child rank each, "
                        "doc-id shards joined in order (default: every visible GPU, as the "
                        "reference's DataParallel, indexer.py:25-26; 1 = this process only)")
    p.add_argument("--variant", choices=["xlmr", "bert"], default="xlmr")
    p.add_argument("--doc_range", type=str, default=None, help="start:end line range (shard)")
    argv = list(sys.argv[1:] if argv is None else argv)
    a = p.parse_args(argv)
    if a.doc_range is None and a.device is None:
        n = parallel.ranks_to_spawn(a.gpus)
        if n > 1:
            rc = parallel.spawn_ranks("index", argv, n)
            if rc:
                raise SystemExit(rc)
            return
    dr = tuple(int(x) for x in a.doc_range.split(":")) if a.doc_range else None
    logging.basicConfig(level=logging.INFO)
    world, rank, local = parallel.dist_env()
    out, device = a.output_file_path, (a.device or 0)
    if world > 1:
        import torch.distributed as dist

        parallel.init_group("gloo")  # host barriers only: encode needs no collective
        dr = parallel.shard_range(parallel.count_lines(a.collection_path), world, rank)
        out, device = parallel.part_path(a.output_file_path, rank), parallel.rank_device(local)
    run(a.collection_path, a.collection_type, out, a.model_checkpoint_path,
        a.num_processes, a.process_batch_size, a.model_batch_size, a.tokenizer_path,
        a.max_length, a.precision, device, a.variant, dr, a.pairwise, first_shard=rank == 0)
    if world > 1:
        dist.barrier()
        if rank == 0:
            parallel.concat_parts([parallel.part_path(a.output_file_path, r) for r in range(world)],
                                  a.output_file_path)
        dist.barrier()


if __name__ == "__main__":
    main()
