"""Impact TSV -> Anserini JsonVectorCollection, the hand-off to Anserini/PISA/CIFF
(reference src/deep_impact/indexing/convert_to_anserini.py:9-37).

Output is byte-compatible with the reference, including its lossy parsing: a line
is cut at every ',' and each piece at every ':', and pieces that do not split into
exactly two parts are dropped (so XLM-R terms such as '▁world,' disappear).  That
behaviour is reproduced on purpose, not fixed.
"""
from __future__ import annotations

import json
from argparse import ArgumentParser
from pathlib import Path


def line_vector(line: str) -> dict:
    vec = {}
    for piece in line.strip().split(","):
        parts = piece.strip().split(":")
        if len(parts) != 2:
            continue
        vec[parts[0]] = float(parts[1])
    return vec


def process(input_file_path, output_file_path):
    with open(input_file_path) as src, open(output_file_path, "w+") as dst:
        for n, line in enumerate(src):
            dst.write(json.dumps({"id": n, "contents": "", "vector": line_vector(line)}) + "\n")


def main(argv=None):
    ap = ArgumentParser(description="Convert a DeepImpact collection into an Anserini "
                                    "JsonVectorCollection.")
    ap.add_argument("-i", "--input_file_path", type=Path, required=True)
    ap.add_argument("-o", "--output_file_path", type=Path, required=True)
    args = ap.parse_args(argv)
    process(args.input_file_path, args.output_file_path)


if __name__ == "__main__":
    main()
