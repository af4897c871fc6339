"""Doc-id sharded CLIs on CPU: shard outputs joined in rank order must
equal the single-process output byte for byte."""
import io

import pytest

from improving_learned_index_amd import index as index_cli


class FakeIndexer:
    """Indexer.index's output contract (indexer.py:62-68): one line per doc of the batch,
    '\\n'-joined plus a final '\\n' (an empty batch would write a lone '\\n')."""

    def index(self, batch, out):
        out.write("\n".join(f"impact-of {d.strip()}" for d in batch) + "\n")


def _run(tmp_path, n_docs, pbs, doc_range):
    coll = tmp_path / "c.tsv"
    coll.write_text("".join(f"{i}\tdoc {i}\n" for i in range(n_docs)))
    out = tmp_path / f"o_{doc_range}.tsv"
    index_cli._index_file(FakeIndexer(), coll, "msmarco", out, pbs, doc_range, 0.0)
    return out.read_text()


@pytest.mark.parametrize("n_docs,pbs,cuts", [(10, 4, [0, 3, 10]), (10, 4, [0, 7, 10]),
                                             (12, 4, [0, 3, 7, 11, 12]), (9, 3, [0, 2, 5, 9]),
                                             (10, 4, [0, 10, 12])])
def test_index_shards_join_to_the_whole_run(tmp_path, n_docs, pbs, cuts):
    whole = _run(tmp_path, n_docs, pbs, None)
    assert whole.count("\n") == n_docs
    parts = [_run(tmp_path, n_docs, pbs, (lo, hi)) for lo, hi in zip(cuts, cuts[1:])]
    assert "".join(parts) == whole
