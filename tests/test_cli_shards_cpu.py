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


def _run_text(tmp_path, text, pbs, doc_range, first_shard=True, tag=""):
    coll = tmp_path / f"c{tag}.tsv"
    coll.write_bytes(text.encode())
    out = tmp_path / f"o{tag}_{doc_range}.tsv"
    index_cli._index_file(FakeIndexer(), coll, "msmarco", out, pbs, doc_range, 0.0,
                          first_shard=first_shard)
    return out.read_text()


@pytest.mark.parametrize("n_docs,cuts", [(5, [0, 2, 5]), (5, [0, 1, 3, 5]), (3, [0, 0, 3])])
def test_process_batch_size_one_keeps_the_leading_empty_line(tmp_path, n_docs, cuts):
    """process_batch_size 1: the reference flushes an empty batch at line 1 (the flush
    precedes the append, index.py:34-41), writing a leading empty line; the joined
    shards must carry it too (the shard holding line 1 writes it)."""
    text = "".join(f"{i}\tdoc {i}\n" for i in range(n_docs))
    whole = _run_text(tmp_path, text, 1, None)
    assert whole.startswith("\n") and whole.count("\n") == n_docs + 1
    parts = [_run_text(tmp_path, text, 1, (lo, hi), first_shard=r == 0)
             for r, (lo, hi) in enumerate(zip(cuts, cuts[1:]))]
    assert "".join(parts) == whole


def test_empty_collection_shards(tmp_path):
    """An empty collection: the reference writes one empty line (its final flush of an
    empty batch); under sharding only the first shard writes it."""
    whole = _run_text(tmp_path, "", 4, None, tag="e")
    parts = [_run_text(tmp_path, "", 4, (0, 0), first_shard=r == 0, tag="e") for r in range(3)]
    assert whole == "\n" and "".join(parts) == whole


def test_count_lines_universal_newlines(tmp_path):
    """parallel.count_lines counts the lines text-mode iteration yields (the shard
    ranges index.py's sharded run splits): \\n, \\r\\n and a lone \\r end a line; a last
    line without a terminator counts; a \\r\\n pair split across read blocks counts once."""
    from improving_learned_index_amd import parallel

    cases = ["", "a", "a\n", "a\nb", "a\r\nb\r\n", "a\rb\rc", "x\tone\rtwo\n3\r", "\n\n\r\r\n"]
    for i, t in enumerate(cases):
        p = tmp_path / f"l{i}"
        p.write_bytes(t.encode())
        with open(p) as f:
            want = sum(1 for _ in f)
        assert parallel.count_lines(p) == want, repr(t)
    # a \r\n pair across the 16 MiB read blocks
    p = tmp_path / "big"
    p.write_bytes(b"x" * ((1 << 24) - 1) + b"\r\n" + b"y\rz")
    with open(p) as f:
        want = sum(1 for _ in f)
    assert parallel.count_lines(p) == want == 3


def test_bare_cr_passage_shards_join(tmp_path):
    """A passage with a bare \\r inside splits into two lines for Python (and the
    reference); the sharded ranges from count_lines cover every line."""
    from improving_learned_index_amd import parallel

    text = "0\tdoc zero\n1\tdoc\r9\tone\n2\tdoc two\n3\tlast"
    whole = _run_text(tmp_path, text, 4, None, tag="cr")
    n = parallel.count_lines(tmp_path / "ccr.tsv")
    assert n == 5 and whole.count("\n") == 5
    parts = [_run_text(tmp_path, text, 4, parallel.shard_range(n, 2, r), first_shard=r == 0,
                       tag="cr") for r in range(2)]
    assert "".join(parts) == whole


def test_line_offsets_match_text_mode_lines(tmp_path):
    """parallel.line_offsets (the sharded quantize CLI's byte ranges): the byte offset
    of each line's start, universal newlines, against a brute-force scan -- random
    texts of \\n / \\r\\n / \\r terminators with tiny read blocks, so terminators (and
    \\r\\n pairs) straddle block boundaries."""
    import random
    import re

    from improving_learned_index_amd import parallel

    rng = random.Random(5)
    for it in range(300):
        parts = [rng.choice(["ab", "c", "", "\t", "é"]) + rng.choice(["\n", "\r\n", "\r", ""])
                 for _ in range(rng.randint(0, 12))]
        data = "".join(parts).encode()
        p = tmp_path / f"t{it}"
        p.write_bytes(data)
        starts = [0] + [m.end() for m in re.finditer(rb"\r\n|\r|\n", data)]
        n = parallel.count_lines(p)
        if starts and starts[-1] == len(data) and len(starts) > 1:
            starts = starts[:-1]  # (a final terminator starts no line)
        want_lines = sorted(rng.randint(0, n + 1) for _ in range(3))
        want = [starts[i] if i < len(starts) and i < n else len(data) for i in want_lines]
        for blk in (1, 2, 3, 7, 1 << 20):
            assert parallel.line_offsets(p, want_lines, block=blk) == want, (data, want_lines, blk)


def test_quantize_file_sharded_false_stays_local(tmp_path, monkeypatch):
    """Under a torchrun environment (WORLD_SIZE > 1) quantize_file shards by default, and
    every rank must call it; sharded=False (bench.py's rank-0-only text legs) quantizes
    the whole file in this process and starts no collective."""
    from improving_learned_index_amd import parallel, quantize

    calls = []
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setattr(quantize, "_quantize_one",
                        lambda i, o, m, d: calls.append(("local", m)) or _Used(3.0))
    monkeypatch.setattr(parallel, "quantize_sharded",
                        lambda *a, **k: calls.append(("sharded",)) or 3.0)
    monkeypatch.setattr(parallel, "init_group", lambda *a, **k: calls.append(("group",)))
    assert quantize.quantize_file(tmp_path / "in", tmp_path / "out", sharded=False) == 3.0
    assert calls == [("local", None)]
    calls.clear()
    quantize.quantize_file(tmp_path / "in", tmp_path / "out")
    assert calls[0] == ("group",) and ("sharded",) in calls


class _Used:
    def __init__(self, v):
        self.value = v


def test_plain_cli_fans_out_to_every_visible_gpu(monkeypatch, tmp_path):
    """index / rank started without torchrun on a multi-GPU box start one child rank per
    visible GPU (the reference's DataParallel whenever device_count() > 1,
    indexer.py:25-26); --gpus overrides; --device or --doc_range keep one process; under
    torchrun (WORLD_SIZE) nothing is spawned."""
    from improving_learned_index_amd import parallel, ranker

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(parallel, "visible_gpus", lambda: 8)
    spawned = []
    monkeypatch.setattr(parallel, "spawn_ranks",
                        lambda mod, argv, n: spawned.append((mod, list(argv), n)) or 0)
    common = ["--collection_path", "c.tsv", "--output_file_path", "o", "--model_checkpoint_path",
              "m.pt"]
    index_cli.main(common)
    assert spawned == [("index", common, 8)]
    index_cli.main(common + ["--gpus", "2"])
    assert spawned[-1] == ("index", common + ["--gpus", "2"], 2)
    rargs = ["--index_path", "i", "--queries_path", "q", "--output_path", "o",
             "--tokenizer_path", "t"]
    ranker.main(rargs)
    assert spawned[-1] == ("rank", rargs, 8)
    n = len(spawned)
    # one process: --device, --doc_range, --gpus 1, or a launcher already running
    monkeypatch.setattr(index_cli, "run", lambda *a, **k: spawned.append("run"))
    index_cli.main(common + ["--device", "3"])
    index_cli.main(common + ["--doc_range", "0:5"])
    index_cli.main(common + ["--gpus", "1"])
    monkeypatch.setenv("WORLD_SIZE", "1")
    index_cli.main(common)
    assert spawned[n:] == ["run"] * 4
    assert parallel.ranks_to_spawn(None) == 1
    monkeypatch.delenv("WORLD_SIZE")
    monkeypatch.setattr(parallel, "visible_gpus", lambda: 0)
    assert parallel.ranks_to_spawn(None) == 1  # (no GPU: one process, which fails loudly)
    with pytest.raises(ValueError):
        parallel.ranks_to_spawn(0)
