"""Golden vectors for the MaxP aggregation: writes a seeded passage-level
run file and pid mapping under tests/golden/maxp/ and runs the reference's own
src/deep_impact/aggregate_run.py on them (in this container, where /root/reference is
mounted) to produce the expected document-level run.  Re-run:
    python tests/golden/make_golden_f4.py
"""
import os
import random
import subprocess
import sys
from pathlib import Path

OUT = Path(__file__).resolve().parent / "maxp"
REF = Path("/root/reference/src/deep_impact/aggregate_run.py")


def main():
    OUT.mkdir(exist_ok=True)
    rng = random.Random(7)
    # (the reference sorts query ids with int(x) if x.isdigit() else x: a mix of
    # numeric and non-numeric ids raises TypeError there, so the ids are numeric)
    # 300 passages of 60 documents (1-8 passages each), some without '#'
    mapping = []
    for d in range(60):
        for k in range(rng.randint(1, 8)):
            mapping.append(f"doc{d}" if rng.random() < 0.1 else f"doc{d}#{k}")
    (OUT / "pid_mapping.txt").write_text("".join(m + "\n" for m in mapping))
    lines = []
    for qid in ["3", "10", "2", "27", "1"]:
        n = rng.randint(20, 120)
        for rank in range(1, n + 1):
            pid = str(rng.randrange(len(mapping) + 5))  # a few ids outside the mapping
            score = rng.choice([round(rng.uniform(-2, 30), 4), float(rng.randint(0, 40))])
            lines.append(f"{qid}\t{pid}\t{rank}\t{score}\n")
        lines.append(f"{qid}\tshort\n")  # fewer than 4 fields: skipped
    (OUT / "run.tsv").write_text("".join(lines))
    for top_k in (1000, 7):
        out = OUT / f"expected_top{top_k}.tsv"
        subprocess.run([sys.executable, str(REF), "--run_file", str(OUT / "run.tsv"),
                        "--mapping", str(OUT / "pid_mapping.txt"), "--output", str(out),
                        "--top_k", str(top_k)], check=True, capture_output=True,
                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))


if __name__ == "__main__":
    main()
