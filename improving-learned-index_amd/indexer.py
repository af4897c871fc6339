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


def _tok_init(tok_json: str, max_length: int, term_mapping: str) -> None:
    from tokenizers import Tokenizer

    DeepImpact.tokenizer = Tokenizer.from_str(tok_json)
    DeepImpact.term_mapping = term_mapping
    _W["max_length"] = max_length


def _tok_chunk(docs: Sequence[str]):
    # packed numpy arrays + one flat term list: cheap to pickle back to the parent
    return DeepImpact.pack_processed(DeepImpact.process_documents(docs, _W["max_length"]))


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
                             initargs=(tok.to_str(), max_length, term_mapping))

    def imap(self, chunks):
        return self.pool.imap(_tok_chunk, chunks)

    def close(self) -> None:
        self.pool.close()
        self.pool.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Indexer:
    def __init__(self, model: DeepImpact, model_batch_size: int = 32, num_processes: int = 8,
                 pool: Optional[TokenizerPool] = None):
        self.model = model
        # the GPU takes far bigger batches than the reference's DataParallel default;
        # batch sizes never change the output bytes
        self.batch_size = max(model_batch_size, 256)
        self.num_processes = num_processes
        self.pool = pool  # None: tokenize in this process

    def encode(self, batch: Sequence[str]):
        chunks = [batch[s:s + self.batch_size] for s in range(0, len(batch), self.batch_size)]
        out: List = []
        if self.pool is not None:
            for packed in self.pool.imap(chunks):
                out += self.model.encode_packed_terms(packed, round3=True)
        else:
            for c in chunks:
                out += self.model.encode_processed(
                    self.model.process_documents(c, self.model.max_length), round3=True)
        return out

    def index(self, batch: Sequence[str], file) -> None:
        """indexer.py:31-68: file.write('\\n'.join(lines) + '\\n')."""
        impacts = self.encode(batch)
        text = _lib.format_impact_lines([[t for t, _ in d] for d in impacts],
                                        [[v for _, v in d] for d in impacts])
        # '\\n'.join(lines) + '\\n' == every line + '\\n', except for an empty batch
        file.write(text if batch else "\n")
        file.flush()


def resolve_tokenizer(model_checkpoint_path, tokenizer_path):
    """The tokenizer DeepImpact.load would pick (explicit path, else the checkpoint
    directory's tokenizer.json)."""
    if tokenizer_path is not None:
        return tokenizer_path
    p = Path(model_checkpoint_path) if model_checkpoint_path is not None else None
    if p is not None and p.is_dir() and (p / "tokenizer.json").exists():
        return p / "tokenizer.json"
    return None
