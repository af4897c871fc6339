"""MaxP aggregation of a passage-level run into a document-level run (SURVEY §8f F4;
reference src/deep_impact/aggregate_run.py:5-58).

The index's doc ids are line numbers of the split collection; `--mapping` holds, per
line, the passage id `docid#k` (or a plain id).  Each (query, document) keeps the
maximum score of its passages -- over a defaultdict(float), so a document whose every
passage scores <= 0 keeps 0.0 (aggregate_run.py:45-47) -- and each query's documents
are written sorted by score (stable: first-seen order on ties), top_k of them, with
`score:.6f`; queries in numeric order, non-numeric ids after as strings
(aggregate_run.py:51-58).  Same flags, same bytes.
"""
from __future__ import annotations

import argparse
from collections import defaultdict


def load_mapping(path):
    """aggregate_run.py:14-18: line index (str) -> passage id."""
    with open(path, "r", encoding="utf-8") as f:
        return {str(idx): line.strip() for idx, line in enumerate(f)}


def aggregate(run_file, index_to_real_id):
    """aggregate_run.py:20-47: qid -> {doc id -> max passage score}."""
    results = defaultdict(lambda: defaultdict(float))
    with open(run_file, "r", encoding="utf-8") as f:
        for line in f:
            parts = line.strip().split("\t")
            if len(parts) < 4:
                continue
            qid, int_pid, score = parts[0], parts[1], float(parts[3])
            real = index_to_real_id.get(int_pid)
            if real is None:
                continue
            doc = real.split("#")[0] if "#" in real else real
            if score > results[qid][doc]:
                results[qid][doc] = score
    return results


def write_run(results, output, top_k=1000):
    """aggregate_run.py:49-58."""
    with open(output, "w", encoding="utf-8") as f:
        for qid in sorted(results.keys(), key=lambda x: int(x) if x.isdigit() else x):
            docs = sorted(results[qid].items(), key=lambda x: x[1], reverse=True)[:top_k]
            f.write("".join(f"{qid}\t{doc}\t{rank}\t{score:.6f}\n"
                            for rank, (doc, score) in enumerate(docs, start=1)))


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--run_file", required=True, help="The raw output from rank.py (integers)")
    p.add_argument("--mapping", required=True, help="The pid_mapping.txt file")
    p.add_argument("--output", required=True, help="The final run file for evaluation")
    p.add_argument("--top_k", type=int, default=1000)
    args = p.parse_args(argv)
    write_run(aggregate(args.run_file, load_mapping(args.mapping)), args.output, args.top_k)


if __name__ == "__main__":
    main()
