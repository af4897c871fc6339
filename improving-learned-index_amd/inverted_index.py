"""On-disk quantized inverted index: host-side mirror of the reference interface.

Reference: src/deep_impact/inverted_index/inverted_index.py (InvertedIndex) and
src/deep_impact/inverted_index/create.py (InvertedIndexCreator, CLI ``-i/-o``).
File formats (src/utils/defaults.py:22-37): vocab.txt (sorted terms, line = id),
inverted_index.idx (u64 start, u64 end byte offsets per term), inverted_index.dat
(u32 doc, u8 value records, value-desc/doc-asc per term).

Scoring runs on the GPU (libdeepimpact_hip.so, di_index_search); building the
files runs in the library's native host code (di_build_reference_index).
"""
from __future__ import annotations

import argparse
import ctypes
from pathlib import Path
from typing import Iterable, List, Sequence, Tuple, Union

import numpy as np

from . import _lib
from ._lib import DeviceIndex, check, lib

INVERTED_INDEX_VOCAB = "vocab.txt"
INVERTED_INDEX_INDEX = "inverted_index.idx"
INVERTED_INDEX_DATA = "inverted_index.dat"


class InvertedIndex:
    """Drop-in for the reference InvertedIndex (inverted_index.py:18-62).

    ``score(query_terms, top_k)`` returns the same list of (doc_id, score) tuples
    as the reference, in the same order -- ties in first-touch order given the
    iteration order of ``query_terms`` -- computed by the HIP scorer.  A doc-id
    range [doc_lo, doc_hi) loads one shard of the index onto ``device``.
    """

    def __init__(self, index_path: Union[str, Path], device: int = 0, doc_lo: int = 0,
                 doc_hi: int = 0, min_impact: int = 1, block_max: float = 0.0,
                 packed: bool = False):
        self.index_path = Path(index_path)
        self.vocab = self._load_vocab()
        self.device = device
        self.doc_lo, self.doc_hi = doc_lo, doc_hi
        self._dev = DeviceIndex.from_reference_dir(self.index_path, doc_lo, doc_hi, device)
        self.set_min_impact(min_impact)
        self.set_block_max(block_max)
        self.packed = False
        self.packed_bytes = self.set_packed(packed) if packed else 0

    def set_min_impact(self, min_impact: int) -> None:
        """Query-time impact pruning (config 5): score only postings of value >= the
        largest power of two <= min_impact (1 = every posting = the reference's exact
        ranking).  Recall trade-off: DESIGN.md §4."""
        self.min_impact = int(min_impact)
        self._dev.set_min_impact(self.min_impact)

    def set_block_max(self, factor: float) -> None:
        """Block-max skipping (configs[4]): 0 off; 1 skips only wave segments of a block
        whose impact upper bound is below the query's running k-th score (the exact
        ranking); f > 1 skips those below f times it (approximate)."""
        self.block_max = float(factor)
        self._dev.set_block_max(self.block_max)

    def set_packed(self, on: bool) -> int:
        """Score from the block-compressed postings (configs[4]; built on first use,
        exact scoring only -- DESIGN.md §3 "Packed postings").  Returns their bytes."""
        self.packed = bool(on)
        return self._dev.set_packed(self.packed)

    def _load_vocab(self):
        vocab = dict()
        with open(self.index_path / INVERTED_INDEX_VOCAB, encoding="utf-8") as f:
            for i, line in enumerate(f):
                vocab[line.strip()] = i
        return vocab

    def term_ids(self, query_terms: Iterable[str]) -> List[int]:
        """Known terms in iteration order (unknown terms score nothing,
        inverted_index.py:25-27)."""
        v = self.vocab
        return [v[t] for t in query_terms if t in v]

    def score(self, query_terms, top_k=1000) -> List[Tuple[int, int]]:
        return self.score_batch([query_terms], top_k)[0]

    def score_batch(self, queries: Sequence[Iterable[str]], top_k=1000):
        """One GPU launch sequence for a whole batch of queries."""
        return self._dev.search([self.term_ids(q) for q in queries], top_k)

    def search_ids(self, queries_ids, top_k=1000, with_keys=False):
        flat, cu = _lib.csr(queries_ids)
        return self._dev.search_csr(flat, cu, top_k, with_keys=with_keys)

    @property
    def device_index(self) -> DeviceIndex:
        return self._dev


def reference_n_docs(index_path: Union[str, Path]) -> int:
    """Docs of a reference-format index: the largest doc id in inverted_index.dat + 1
    (doc id = collection line index, create.py:41-47)."""
    dat = Path(index_path) / INVERTED_INDEX_DATA
    if dat.stat().st_size == 0:
        return 0
    rec = np.memmap(dat, dtype=[("doc", "<u4"), ("val", "u1")], mode="r")
    m = 0
    for s in range(0, rec.shape[0], 1 << 26):
        m = max(m, int(rec["doc"][s:s + (1 << 26)].max()))
    return m + 1


def create_index(deep_impact_collection_path: Union[str, Path],
                 output_path: Union[str, Path]) -> None:
    """InvertedIndexCreator.run (create.py:53-55), byte-identical output."""
    out = Path(output_path)
    out.mkdir(parents=True, exist_ok=True)
    check(lib().di_build_reference_index(str(deep_impact_collection_path).encode("utf-8"),
                                         str(out).encode("utf-8")))


class InvertedIndexCreator:
    """Drop-in for create.py:12-55."""

    def __init__(self, deep_impact_collection_path, output_path):
        self.deep_impact_collection_path = Path(deep_impact_collection_path)
        self.output_path = Path(output_path)
        self.output_path.mkdir(parents=True, exist_ok=True)

    def run(self):
        create_index(self.deep_impact_collection_path, self.output_path)


if __name__ == "__main__":
    args = argparse.ArgumentParser()
    args.add_argument("-i", "--deep_impact_collection_path", type=Path, required=True)
    args.add_argument("-o", "--output_path", type=Path, required=True)
    args = args.parse_args()
    InvertedIndexCreator(args.deep_impact_collection_path, args.output_path).run()
