"""Encode loop: documents -> impact TSV (reference src/deep_impact/indexing/indexer.py
and src/deep_impact/index.py).

Indexer.index(batch, file) writes exactly the reference's bytes: one line per
document, ', '.join(f'{term}: {round(impact, 3)}'), terms in first-occurrence
order.  The forward, head, gather and 3-decimal rounding run on the GPU (di_encode
with DI_F_ROUND3); the text is produced by the native formatter
(di_format_impact_lines).

Tokenization and term extraction (A3, host hot loop #1) run either in-process (the
Rust tokenizer's batched call) or, like the reference's 8-process Pool
(indexer.py:29, :41), in a TokenizerPool of worker processes: the batch goes out in
chunks, and the GPU encodes chunk i while the workers tokenize the chunks after it.
Chunking never changes the output bytes.
"""
from __future__ import annotations

import multiprocessing as mp
from pathlib import Path
from typing import List, Optional, Sequence

from . import _lib
from .models import DeepImpact

# --------------------------------------------------------------------------- workers
_W = {}


def _tok_init(tok_json: str, max_length: int, term_mapping: str,
              rayon_threads: Optional[int] = None) -> None:
    import os

    if rayon_threads and "RAYON_NUM_THREADS" not in os.environ:
        # before the first batched call starts the tokenizers' thread pool
        os.environ["RAYON_NUM_THREADS"] = str(rayon_threads)
    from tokenizers import Tokenizer

    DeepImpact.tokenizer = Tokenizer.from_str(tok_json)
    DeepImpact.term_mapping = term_mapping
    _W["max_length"] = max_length


def _tok_chunk(docs: Sequence[str]):
    # packed numpy arrays + the terms as one UTF-8 blob: cheap to pickle back to the
    # parent, and the parent formats the lines without per-term Python objects
    return DeepImpact.pack_processed_blob(DeepImpact.process_documents(docs, _W["max_length"]))


def _tok_rate(docs: Sequence[str]) -> float:
    """One worker's tokenize + term-extraction rate (docs/s) over `docs` (the bench's
    host budget of the index CLI: indexer.py:28-33 is the reference loop it replaces)."""
    import time

    t0 = time.perf_counter()
    _tok_chunk(docs)
    return len(docs) / max(time.perf_counter() - t0, 1e-9)


def pool_supported() -> bool:
    """Spawned workers re-import the parent's __main__: impossible when it is not a
    file or module (stdin, -c); callers then tokenize in-process."""
    import os
    import sys

    main = sys.modules.get("__main__")
    if getattr(main, "__spec__", None) is not None:
        return True
    f = getattr(main, "__file__", None)
    return f is None or os.path.isfile(f)


def worker_threads(num_processes: int) -> int:
    """Threads of each worker's batched tokenizer call.  The tokenizers' pool defaults
    to every CPU the process may run on: on a share of a large machine (OMP_NUM_THREADS
    names the share) N workers would each start that many.  Measured with 16 workers on
    the GPU box (16 of 256 CPUs): default 7.7 k, 1-4 threads 9.8-9.9 k docs/s end to end;
    8 workers on 8 CPUs here: 2-4 threads 4.3-4.4 k, default 4.0 k docs/s."""
    import os

    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp))
    return max(2, min(4, share // max(1, num_processes)))


class TokenizerPool:
    """Worker processes running DeepImpact.process_documents (xlmr_original.py:120-189)
    with the parent's tokenizer, max_length and term mapping.

    Start it BEFORE the GPU is initialised (index.run does): the workers are spawned
    interpreters that never touch the GPU."""

    def __init__(self, num_processes: int, tokenizer, max_length: int,
                 term_mapping: str = "word_ids"):
        from .models import load_tokenizer

        tok = load_tokenizer(tokenizer)
        ctx = mp.get_context("spawn")
        self.n = num_processes
        self.pool = ctx.Pool(num_processes, initializer=_tok_init,
                             initargs=(tok.to_str(), max_length, term_mapping,
                                       worker_threads(num_processes)))

    def imap(self, chunks):
        return self.pool.imap(_tok_chunk, chunks)

    def worker_rate(self, docs: Sequence[str]) -> float:
        """docs/s of one worker over `docs` (the pool otherwise idle)."""
        return self.pool.apply(_tok_rate, (list(docs),))

    def close(self) -> None:
        self.pool.close()
        self.pool.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


DEVICE_DOCS = 4096  # documents per device call when tokenizer chunks are merged


class _Writer:
    """One background thread that formats and writes batches in submission order, so
    that a batch's formatting (native, the GIL released) and its file write overlap the
    next batch's device encode.  An exception in a job is raised at the next put /
    drain."""

    def __init__(self):
        import queue
        import threading

        self.q = queue.Queue(maxsize=4)
        self.err = None
        self.t = threading.Thread(target=self._run, name="di-index-writer", daemon=True)
        self.t.start()

    def _run(self):
        while True:
            job = self.q.get()
            try:
                if job is None:
                    return
                if self.err is None:
                    job()
            except BaseException as e:  # (re-raised in the caller's thread)
                self.err = e
            finally:
                self.q.task_done()

    def _check(self):
        if self.err is not None:
            err, self.err = self.err, None
            raise err

    def put(self, job):
        self._check()
        self.q.put(job)

    def drain(self):
        self.q.join()
        self._check()

    def close(self):
        self.q.put(None)
        self.t.join()
        self._check()


class Indexer:
    def __init__(self, model: DeepImpact, model_batch_size: int = 32, num_processes: int = 8,
                 pool: Optional[TokenizerPool] = None):
        self.model = model
        # the GPU takes far bigger batches than the reference's DataParallel default;
        # batch sizes never change the output bytes
        self.batch_size = max(model_batch_size, 256)
        self.num_processes = num_processes
        self.pool = pool  # None: tokenize in this process
        self._writer = None  # (pool path: formatting + writes behind the next encode)

    def _chunks(self, batch: Sequence[str]):
        # with a pool: enough chunks to keep every worker busy (down to 64 docs each)
        step = self.batch_size
        if self.pool is not None and batch:
            step = max(64, min(step, -(-len(batch) // self.pool.n)))
        return [batch[s:s + step] for s in range(0, len(batch), step)]

    def encode(self, batch: Sequence[str]):
        out: List = []
        if self.pool is not None:
            for ids, cu, blob, term_off, tt, ct in self.pool.imap(self._chunks(batch)):
                terms = [blob[term_off[i]:term_off[i + 1]].decode("utf-8")
                         for i in range(len(term_off) - 1)]
                out += self.model.encode_packed_terms((ids, cu, terms, tt, ct), round3=True)
        else:
            for c in self._chunks(batch):
                out += self.model.encode_processed(
                    self.model.process_documents(c, self.model.max_length), round3=True)
        return out

    def submit(self, batch: Sequence[str]):
        """Start tokenizing `batch` in the pool (returns at once); finish() encodes and
        writes it.  One submitted batch ahead keeps the workers busy while the GPU
        encodes the current one."""
        if self.pool is None:
            return (batch, None)
        return (batch, self.pool.imap(self._chunks(batch)))

    def finish(self, handle, file, wait: bool = True) -> None:
        """indexer.py:31-68: file.write('\\n'.join(lines) + '\\n').  wait=False (the
        pool path): return once the batch is encoded; its formatting and write run on
        the writer thread, in order, while the caller encodes the next batch --
        drain() (or a later finish with wait=True) completes them."""
        batch, it = handle
        if it is None:
            impacts = self.encode(batch)
            text = _lib.format_impact_lines([[t for t, _ in d] for d in impacts],
                                            [[v for _, v in d] for d in impacts])
            self.drain()  # (earlier deferred writes first)
            file.write(text if batch else "\n")
            file.flush()
            return
        # the workers' chunks are merged into device batches of up to DEVICE_DOCS
        # documents (a 100-doc chunk leaves most of the GPU idle), in order
        enc = getattr(self.model, "encode_packed_impacts", None)
        parts, n, jobs = [], 0, []

        def encode(parts):
            packed = DeepImpact.merge_packed_blobs(parts)
            if enc is not None:
                jobs.append(enc(packed))
            else:
                text = self.model.encode_packed_text(packed)
                jobs.append(lambda: text)

        for p in it:
            parts.append(p)
            n += len(p[1]) - 1
            if n >= DEVICE_DOCS:
                encode(parts)
                parts, n = [], 0
        if parts:
            encode(parts)

        def write():
            text = "".join(j() for j in jobs)
            # '\\n'.join(lines) + '\\n' == every line + '\\n', except for an empty batch
            file.write(text if batch else "\n")
            file.flush()

        if self._writer is None:
            self._writer = _Writer()
        self._writer.put(write)
        if wait:
            self._writer.drain()

    def drain(self) -> None:
        """Wait for the deferred formatting and writes (re-raises their errors)."""
        if self._writer is not None:
            self._writer.drain()

    def index(self, batch: Sequence[str], file) -> None:
        """indexer.py:31-68: file.write('\\n'.join(lines) + '\\n')."""
        self.finish(self.submit(batch), file)


def resolve_tokenizer(model_checkpoint_path, tokenizer_path):
    """The tokenizer DeepImpact.load would pick (explicit path, else the checkpoint
    directory's tokenizer.json)."""
    if tokenizer_path is not None:
        return tokenizer_path
    p = Path(model_checkpoint_path) if model_checkpoint_path is not None else None
    if p is not None and p.is_dir() and (p / "tokenizer.json").exists():
        return p / "tokenizer.json"
    return None
