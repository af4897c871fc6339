"""Encode loop: documents -> impact TSV (reference src/deep_impact/indexing/indexer.py
and src/deep_impact/index.py).

Indexer.index(batch, file) writes exactly the reference's bytes: one line per
document, ', '.join(f'{term}: {round(impact, 3)}'), terms in first-occurrence
order.  Tokenization runs in the Rust tokenizer (batched, multi-threaded); the
forward, head, gather and 3-decimal rounding run on the GPU (di_encode with
DI_F_ROUND3); the text is produced by the native formatter
(di_format_impact_lines).
"""
from __future__ import annotations

from typing import List, Sequence

from . import _lib
from .models import DeepImpact


class Indexer:
    def __init__(self, model: DeepImpact, model_batch_size: int = 32, num_processes: int = 8):
        self.model = model
        # the GPU takes far bigger batches than the reference's DataParallel default;
        # batch sizes never change the output bytes
        self.batch_size = max(model_batch_size, 256)
        self.num_processes = num_processes  # tokenizers threads (RAYON_NUM_THREADS)

    def encode(self, batch: Sequence[str]):
        out = []
        for s in range(0, len(batch), self.batch_size):
            out += self.model.encode_documents(batch[s:s + self.batch_size], round3=True)
        return out

    def index(self, batch: Sequence[str], file) -> None:
        """indexer.py:31-68: file.write('\\n'.join(lines) + '\\n')."""
        impacts = self.encode(batch)
        text = _lib.format_impact_lines([[t for t, _ in d] for d in impacts],
                                        [[v for _, v in d] for d in impacts])
        # '\\n'.join(lines) + '\\n' == every line + '\\n', except for an empty batch
        file.write(text if batch else "\n")
        file.flush()
