"""Host-side product logic on CPU: term extraction (A3), query terms, formats
(A9 text, run files), the Anserini hand-off -- checked against fixtures made by
the reference's own code (tests/golden/make_golden.py)."""
import json
import tempfile
from pathlib import Path

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def M():
    from improving_learned_index_amd import models

    models.DeepImpact.set_tokenizer(GOLDEN / "tokenizer.json")
    return models


def test_process_document_matches_reference(M):
    fx = json.loads((GOLDEN / "encoder_xlmr_small.json").read_text())
    got = M.DeepImpact.process_documents(fx["texts"], max_length=fx["max_length"])
    for (enc, tmap), ids, mask, want in zip(got, fx["input_ids"], fx["attention_mask"],
                                            fx["term_maps"]):
        n = sum(mask)
        assert enc.ids == ids[:n]
        assert list(tmap.items()) == [tuple(x) for x in want]


def test_process_document_truncation_matches_reference(M):
    fx = json.loads((GOLDEN / "encoder_xlmr_base.json").read_text())
    got = M.DeepImpact.process_documents(fx["texts"], max_length=fx["max_length"])
    for (enc, tmap), ids, mask, want in zip(got, fx["input_ids"], fx["attention_mask"],
                                            fx["term_maps"]):
        assert enc.ids == ids[:sum(mask)]
        assert list(tmap.items()) == [tuple(x) for x in want]


def test_process_query_matches_reference(M):
    fx = json.loads((GOLDEN / "encoder_xlmr_small.json").read_text())
    for t, want in zip(fx["texts"], fx["query_terms_sorted"]):
        assert sorted(M.DeepImpact.process_query(t)) == want


def test_native_formatter_matches_reference_text():
    from improving_learned_index_amd import _lib, synthetic

    docs = json.loads((GOLDEN / "collection.docs.json").read_text())
    terms = [d["terms"] for d in docs]
    imps = [synthetic.round3_f32(np.array(d["impacts_f32_bits"], np.uint32).view(np.float32))
            for d in docs]
    assert _lib.format_impact_lines(terms, imps) == (GOLDEN / "collection.index").read_text()
    vals = np.load(GOLDEN / "round3_in.npy").view(np.float32)
    want = (GOLDEN / "round3_out.txt").read_text().split("\n")[:-1]
    text = _lib.format_impact_lines([["t"] * len(vals)], [synthetic.round3_f32(vals)])
    got = [p.split(": ")[1] for p in text.rstrip("\n").split(", ")]
    assert got == want


def test_anserini_conversion_is_lossy_like_the_reference():
    from improving_learned_index_amd.convert_to_anserini import process

    with tempfile.TemporaryDirectory() as td:
        src = Path(td) / "c.tsv"
        src.write_text("▁a: 1, ▁world,: 2, ▁x:y: 3\n\n")
        process(src, Path(td) / "o.jsonl")
        lines = (Path(td) / "o.jsonl").read_text().split("\n")
        # '▁world,: 2' -> pieces ' ▁world' (dropped) and ': 2' (term '' !), '▁x:y: 3' dropped
        assert json.loads(lines[0]) == {"id": 0, "contents": "", "vector": {"▁a": 1.0, "": 2.0}}
        assert json.loads(lines[1]) == {"id": 1, "contents": "", "vector": {}}


def test_run_file_and_metrics_match_reference():
    from improving_learned_index_amd.metrics import Metrics, MRR_DEPTHS, RECALL_DEPTHS

    fx = json.loads((GOLDEN / "metrics.json").read_text())
    m = Metrics(GOLDEN / "metrics.run.tsv", GOLDEN / "metrics.qrels.tsv", MRR_DEPTHS,
                RECALL_DEPTHS)
    out = m.evaluate()
    for k, v in fx["mrr"].items():
        assert out[f"MRR@{k}"] == v
    for k, v in fx["recall"].items():
        assert out[f"Recall@{k}"] == v


def test_ndcg_trec_eval_conventions():
    from improving_learned_index_amd.metrics import ndcg_at_k

    qrels = {"q": {"a": 1, "b": 1}}
    assert ndcg_at_k(qrels, {"q": {"a": 2.0, "c": 1.0, "b": 0.5}}, 10) == pytest.approx(
        (1 + 1 / np.log2(4)) / (1 + 1 / np.log2(3)))
    assert ndcg_at_k(qrels, {}, 10) == 0.0


@pytest.mark.parametrize("name", ["collection.index", "collection.quantized", "edge.tsv"])
def test_convert_to_anserini_matches_reference_output(tmp_path, name):
    """F1: byte-identical to the reference's own convert_to_anserini.process output
    (fixtures made by tests/golden/make_golden_f1.py, which ran the reference)."""
    from improving_learned_index_amd import convert_to_anserini

    src = GOLDEN / name if name != "edge.tsv" else GOLDEN / "anserini" / name
    out = tmp_path / "out.jsonl"
    convert_to_anserini.process(src, out)
    assert out.read_bytes() == (GOLDEN / "anserini" / f"{name}.jsonl").read_bytes()


def test_native_run_lines_equal_runfile_writelines(tmp_path):
    """di_format_run_lines (RunFile.write_batch) writes the bytes of the reference's
    per-query RunFile.writelines (datasets.py:305-324): unicode and numeric qids, empty
    and full lists, pids and scores up to 2^32 - 1."""
    import numpy as np

    from improving_learned_index_amd.datasets import RunFile

    rng = np.random.default_rng(3)
    qids = ["1048585", "q-ß", "", "42", "x" * 40] * 30
    k = 17
    docs = rng.integers(0, 2 ** 32, (len(qids), k), dtype=np.uint64).astype(np.uint32)
    scores = rng.integers(0, 2 ** 32, (len(qids), k), dtype=np.uint64).astype(np.uint32)
    counts = rng.integers(0, k + 1, len(qids)).astype(np.int32)
    counts[0], counts[1] = 0, k
    a, b = RunFile(tmp_path / "a"), RunFile(tmp_path / "b")
    for i, q in enumerate(qids):
        a.writelines(q, list(zip(docs[i, :counts[i]].tolist(), scores[i, :counts[i]].tolist())))
    b.write_batch(qids[:70], docs[:70], scores[:70], counts[:70])
    b.write_batch(qids[70:], docs[70:], scores[70:], counts[70:])
    assert (tmp_path / "a").read_bytes() == (tmp_path / "b").read_bytes()


def test_decode_key_arrays_equal_per_query_decode():
    """parallel.decode_quant_key_arrays == decode_quant_keys per query, narrow and wide
    (more than 256 known terms) keys; a rejected query raises."""
    import numpy as np
    import pytest

    from improving_learned_index_amd import parallel

    rng = np.random.default_rng(5)
    nq, k = 12, 9
    keys = rng.integers(0, 2 ** 63, (nq, k), dtype=np.uint64) * np.uint64(2)
    counts = rng.integers(0, k + 1, nq).astype(np.int32)
    n_terms = [3, 300, 1, 257, 256, 6, 900, 2, 2, 2, 400, 5]
    docs, scores = parallel.decode_quant_key_arrays(keys, counts, n_terms)
    for q in range(nq):
        want = parallel.decode_quant_keys(keys[q], int(counts[q]), n_terms[q])
        assert list(zip(docs[q, :counts[q]].tolist(), scores[q, :counts[q]].tolist())) == want
    counts[4] = -1
    with pytest.raises(RuntimeError):
        parallel.decode_quant_key_arrays(keys, counts, n_terms)
