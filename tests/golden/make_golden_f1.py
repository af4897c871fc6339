"""F1 fixtures: run the reference's own convert_to_anserini.process
(src/deep_impact/indexing/convert_to_anserini.py:9-24, imported by file path from
/root/reference) on committed impact / quantized TSVs and keep its outputs.

    python tests/golden/make_golden_f1.py      (here only; needs /root/reference)

Inputs: the golden impact TSV (tests/golden/collection.index), its quantized form,
and an edge-case TSV written below (terms holding ',' / ':', empty lines, spacing).
Outputs: tests/golden/anserini/<input>.jsonl.
"""
import importlib.util
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference")
sys.dont_write_bytecode = True

EDGE = ("▁hello: 1.5, ▁world,: 2.0, ▁a:b: 3.0, ▁x: 0.0\n"
        "\n"
        "▁only: 7\n"
        "  ▁sp:  4.25 ,▁t: 1e-05, ▁dup: 1.0, ▁dup: 2.0\n"
        "▁num: 3\n")


def main():
    spec = importlib.util.spec_from_file_location(
        "ref_convert_to_anserini", REF / "src/deep_impact/indexing/convert_to_anserini.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = HERE / "anserini"
    out.mkdir(exist_ok=True)
    (out / "edge.tsv").write_text(EDGE, encoding="utf-8")
    for src in (HERE / "collection.index", HERE / "collection.quantized", out / "edge.tsv"):
        mod.process(src, out / f"{src.name}.jsonl")
        print("wrote", out / f"{src.name}.jsonl")


if __name__ == "__main__":
    main()
