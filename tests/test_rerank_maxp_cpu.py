"""Next rows of SURVEY §8f on CPU: the MaxP aggregation (F4) against the reference's own
aggregate_run.py outputs (tests/golden/make_golden_f4.py), and the re-ranker's host
logic (F3) against a restatement of reference reranker.py:52-91 with a fake encoder
(the reference class imports the models package, whose class bodies fetch a
tokenizer from the hub: not importable offline -- parity unpinned beyond that
restatement; the encoder it calls is pinned by tests/test_encoder_gpu.py)."""
import random

import numpy as np
import pytest

from conftest import GOLDEN

MAXP = GOLDEN / "maxp"


@pytest.mark.parametrize("top_k", [1000, 7])
def test_maxp_matches_reference(tmp_path, top_k):
    from improving_learned_index_amd import aggregate_run

    out = tmp_path / "out.tsv"
    aggregate_run.main(["--run_file", str(MAXP / "run.tsv"), "--mapping",
                        str(MAXP / "pid_mapping.txt"), "--output", str(out),
                        "--top_k", str(top_k)])
    assert out.read_bytes() == (MAXP / f"expected_top{top_k}.tsv").read_bytes()


def test_maxp_mixed_query_ids_fail_like_reference(tmp_path):
    from improving_learned_index_amd import aggregate_run

    run = tmp_path / "run.tsv"
    run.write_text("1\t0\t1\t2.0\nq\t0\t1\t1.0\n")
    (tmp_path / "map.txt").write_text("d#0\n")
    with pytest.raises(TypeError):  # aggregate_run.py:52 sorts int and str keys
        aggregate_run.main(["--run_file", str(run), "--mapping", str(tmp_path / "map.txt"),
                            "--output", str(tmp_path / "o.tsv")])


class _FakeModel:
    """Deterministic term impacts per passage (np.float32), counting encoder calls."""

    def __init__(self, vocab):
        self.vocab = vocab
        self.calls = 0

    def get_impact_scores_batch(self, docs):
        from improving_learned_index_amd import models

        self.calls += 1
        out = []
        for d, (_, tmap) in zip(docs, models.DeepImpact.process_documents(docs)):
            rng = random.Random(d)
            out.append([(t, np.float32(rng.uniform(0, 5))) for t in tmap])  # real terms
        return out


def _reference_rerank(cache_fn, query_terms, pids):
    """Restatement of reranker.py:56-57,91."""
    scores = [sum(cache_fn(pid).get(t, 0) for t in query_terms) for pid in pids]
    return sorted(zip(pids, scores), key=lambda x: x[1], reverse=True)[:1000]


def test_reranker_matches_reference_logic(tmp_path):
    from improving_learned_index_amd import models, reranker

    models.DeepImpact.set_tokenizer(GOLDEN / "tokenizer.json")
    rng = random.Random(3)
    words = [f"w{i}" for i in range(40)]
    coll = {str(p): " ".join(rng.choice(words) for _ in range(rng.randint(1, 12)))
            for p in range(200)}
    (tmp_path / "coll.tsv").write_text("".join(f"{p}\t{t}\n" for p, t in coll.items()))
    queries = {str(q): " ".join(rng.choice(words) for _ in range(rng.randint(1, 5)))
               for q in range(12)}
    (tmp_path / "q.tsv").write_text("".join(f"{q}\t{t}\n" for q, t in queries.items()))
    lines = []
    for q in queries:
        pids = rng.sample(sorted(coll), 60)
        lines += [f"{q}\t{p}\t{r}\t{100 - r}\n" for r, p in enumerate(pids, start=1)]
    (tmp_path / "topk.tsv").write_text("".join(lines))
    fake = _FakeModel(words)
    rr = reranker.ReRanker(None, tmp_path / "topk.tsv", tmp_path / "q.tsv",
                           tmp_path / "coll.tsv", tmp_path / "out.tsv", batch_size=16, model=fake)
    rr.run()
    got = [l.split("\t") for l in (tmp_path / "out.tsv").read_text().splitlines()]

    def impacts(pid):
        return {t: s for t, s in fake.get_impact_scores_batch([coll[pid]])[0]}

    want = []
    for q, pids in rr.top_k:
        terms = models.DeepImpact.process_query(queries[q])
        for rank, (pid, score) in enumerate(_reference_rerank(impacts, terms, pids), start=1):
            want.append([q, pid, str(rank), f"{score}"])
    assert got == want
    assert sum(float(r[3]) > 0 for r in got) > len(got) // 5  # the query terms do match
    # every passage encoded once (the per-pid cache, reranker.py:52-54)
    assert len(rr.cache) == len({p for _, ps in rr.top_k for p in ps})
