"""Collection / query / qrels / run-file formats -- mirror of the reference's
src/utils/datasets.py pieces on the hot path (Appendix A of SURVEY.md)."""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, Iterable, Iterator, Optional, Set, Tuple, Union

COLLECTION_TYPES = ["msmarco", "beir"]


class CollectionParser:
    """datasets.py:350-367."""

    @staticmethod
    def get_msmarco_item(passage: str):
        return passage.strip().split("\t")

    @staticmethod
    def get_beir_item(passage: str):
        item = json.loads(passage)
        return item["_id"], item["title"] + " " + item["text"]

    @staticmethod
    def parse(item: str, collection_type: str):
        f = {"msmarco": CollectionParser.get_msmarco_item,
             "beir": CollectionParser.get_beir_item}[collection_type]
        return f(item)


class QueryParser:
    """datasets.py:370-389."""

    @staticmethod
    def get_msmarco_item(query: str):
        qid, q = query.strip().split("\t")
        return str(qid), q

    @staticmethod
    def get_beir_item(query: str):
        item = json.loads(query)
        return item["_id"], item["text"]

    @staticmethod
    def parse(item: str, collection_type: str):
        f = {"msmarco": QueryParser.get_msmarco_item, "beir": QueryParser.get_beir_item}[
            collection_type]
        return f(item)


class Queries:
    """datasets.py:17-47."""

    def __init__(self, queries_path: Union[str, Path], dataset_type: str = COLLECTION_TYPES[0]):
        self.dataset_type = dataset_type
        self.queries: Dict[str, str] = {}
        with open(queries_path, encoding="utf-8") as f:
            for line in f:
                qid, q = QueryParser.parse(line, dataset_type)
                self.queries[str(qid)] = q

    def __len__(self):
        return len(self.queries)

    def __getitem__(self, qid):
        return self.queries[str(qid)]

    def __iter__(self):
        return iter(self.queries.items())

    def keys(self):
        return self.queries.keys()


class QueryRelevanceDataset:
    """datasets.py:138-175: qid \\t 0 \\t pid \\t 1."""

    def __init__(self, qrels_path: Union[str, Path]):
        self.qrels: Dict[str, Set[str]] = {}
        with open(qrels_path, "r", encoding="utf-8") as f:
            for line in f:
                parts = line.strip().split("\t")
                qid, x, pid, y = parts[0], int(parts[1]), parts[2], int(parts[3])
                assert x == 0 and y == 1, "Qrels file is not in the expected format"
                self.qrels.setdefault(str(qid), set()).add(str(pid))

    def __len__(self):
        return len(self.qrels)

    def __getitem__(self, qid) -> Set[str]:
        return self.qrels[str(qid)]

    def keys(self):
        return self.qrels.keys()


class Collection:
    """datasets.py:50-95: pid (str) -> passage of an MS MARCO collection, lines
    [offset, offset + limit)."""

    def __init__(self, collection_path: Union[str, Path], offset: Optional[int] = None,
                 limit: Optional[int] = None):
        offset = 0 if offset is None else offset
        limit = float("inf") if limit is None else limit
        self.collection: Dict[str, str] = {}
        with open(collection_path, encoding="utf-8") as f:
            for idx, line in enumerate(f):
                if idx < offset:
                    continue
                if idx >= offset + limit:
                    break
                pid, passage, = line.strip().split("\t")
                self.collection[str(pid)] = passage

    def __len__(self):
        return len(self.collection)

    def __getitem__(self, pid):
        return self.collection[str(pid)]

    def __iter__(self):
        return iter(self.collection.items())


class RunFile:
    """datasets.py:305-324: qid \\t pid \\t rank \\t score."""

    def __init__(self, run_file_path: Union[str, Path]):
        self.run_file_path = run_file_path

    def writelines(self, qid, scores):
        with open(self.run_file_path, "a", encoding="utf-8") as f:
            f.write("".join(f"{qid}\t{pid}\t{rank}\t{score}\n"
                            for rank, (pid, score) in enumerate(scores, start=1)))

    def write_batch(self, qids, docs, scores, counts):
        """writelines for a batch of queries in order, from arrays (docs / scores
        [n_q, k] integers, counts [n_q]): the same bytes, formatted and appended
        natively (di_append_run_lines)."""
        from . import _lib

        _lib.append_run_lines(self.run_file_path, qids, docs, scores, counts)

    def read(self) -> Iterator[Tuple[str, str, int, float]]:
        with open(self.run_file_path, "r", encoding="utf-8") as f:
            for line in f:
                qid, pid, rank, score = line.strip().split("\t")
                yield str(qid), str(pid), int(rank), float(score)


class TopKRunFile(RunFile):
    """datasets.py:327-347: qid -> its first k pids by rank."""

    def __init__(self, run_file_path: Union[str, Path], k: int = 2000):
        super().__init__(run_file_path)
        top_k: Dict[str, list] = {}
        for qid, pid, rank, _ in self.read():
            top_k.setdefault(qid, []).append((rank, pid))
        for qid in top_k:
            top_k[qid].sort()
            top_k[qid] = [v for _, v in top_k[qid][:k]]
        self.top_k = top_k

    def __len__(self):
        return len(self.top_k)

    def __getitem__(self, qid):
        return self.top_k[str(qid)]

    def __iter__(self):
        for qid in self.top_k:
            yield qid, self.top_k[qid]
