"""configs[0] plumbing on the GPU (NanoBEIR evaluation, reference
nano_beir_evaluator.py:70-243): HIP encode -> in-memory float index (SparseSearch)
-> top-1000 -> beir-style (NDCG, MAP, Recall, P) at 10/100/1000, through
NanoBEIREvaluator.evaluate_all over a local Nano<Name> directory (the hub is offline).

Checked against the oracle chain on the same inputs: the fp32 torch encoder
(oracle/encoder_ref.py) -> the oracle's float sparse search (oracle.c, the
reference's SparseSearch semantics) -> the same metric function.  The fp32 mode
matches the oracle's impacts within 1e-6, so the rankings and metrics are identical.
"""
import json

import numpy as np
import pytest
import torch

import encoder_ref
import oracle
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _dataset(tmp_path, texts):
    rng = np.random.default_rng(0)
    d = tmp_path / "NanoNFCorpus"
    d.mkdir()
    docs = [(f"doc{i}", t) for i, t in enumerate(texts) if t.strip()]
    with open(d / "corpus.jsonl", "w") as f:
        for did, t in docs:
            f.write(json.dumps({"_id": did, "title": "", "text": t}) + "\n")
    queries, qrels = {}, {}
    for qi in range(24):
        did, t = docs[int(rng.integers(0, len(docs)))]
        words = t.split()
        k = min(len(words), int(rng.integers(1, 5)))
        queries[f"q{qi}"] = " ".join(rng.choice(words, size=k, replace=False).tolist())
        qrels[f"q{qi}"] = {did: 1}
        if qi % 3 == 0:  # a second relevant doc
            qrels[f"q{qi}"][docs[(qi * 7) % len(docs)][0]] = 1
    with open(d / "queries.jsonl", "w") as f:
        for q, t in queries.items():
            f.write(json.dumps({"_id": q, "text": t}) + "\n")
    with open(d / "qrels.tsv", "w") as f:
        f.write("query-id\tcorpus-id\tscore\n")
        for q, rel in qrels.items():
            for did in rel:
                f.write(f"{q}\t{did}\t1\n")
    return docs, queries, qrels


def test_nano_beir_evaluate_all_matches_oracle_chain(tmp_path):
    from improving_learned_index_amd import _lib
    from improving_learned_index_amd.encoder import EncoderConfig
    from improving_learned_index_amd.metrics import evaluate_retrieval
    from improving_learned_index_amd.models import DeepImpact
    from improving_learned_index_amd.nano_beir import NanoBEIREvaluator

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible (GPU test run without a GPU)")
    fx = json.loads((GOLDEN / "encoder_xlmr_small.json").read_text())
    sd = encoder_ref.seeded_state_dict(fx["state_dict_shapes"], fx["seed"], fx["std"])
    ckpt = tmp_path / "ckpt.pt"
    torch.save({"model_state_dict": sd, "optimizer_state_dict": {}, "step": 0,
                "batch_size": 0}, ckpt)
    cfg = EncoderConfig.from_hf({**fx["config"], "model_type": "xlm-roberta"})
    model = DeepImpact.load(ckpt, config=cfg, tokenizer_path=GOLDEN / "tokenizer.json",
                            precision="fp32", max_length=fx["max_length"])
    texts = [t for t in fx["texts"] if t.strip()]
    texts = texts + [" ".join(reversed(t.split())) for t in texts] + \
        [" ".join(t.split()[::2]) for t in texts if len(t.split()) > 3]
    docs, queries, qrels = _dataset(tmp_path, texts)
    metrics = NanoBEIREvaluator(batch_size=16, data_dir=tmp_path).evaluate_all(model)
    assert set(metrics) == {"nfcorpus", "avg"}
    got = metrics["nfcorpus"]
    assert metrics["avg"] == got
    assert [set(m) for m in got] == [{f"{n}@{k}" for k in (10, 100, 1000)}
                                     for n in ("NDCG", "MAP", "Recall", "P")]

    # oracle chain: fp32 torch encoder -> term impacts -> oracle float sparse search
    proc = [DeepImpact.process_document(t, fx["max_length"]) for _, t in docs]
    S = max(len(e.ids) for e, _ in proc)
    ids = np.ones((len(proc), S), np.int64)
    mask = np.zeros_like(ids)
    for i, (e, _) in enumerate(proc):
        ids[i, :len(e.ids)] = e.ids
        mask[i, :len(e.ids)] = 1
    with torch.no_grad():
        tok = encoder_ref.forward(sd, fx["config"], torch.from_numpy(ids),
                                  torch.from_numpy(mask), "xlmr", "softplus").numpy()
    term_imps = [[(t, np.float32(tok[i, j])) for t, j in m.items()]
                 for i, (_, m) in enumerate(proc)]
    ora = oracle.SparseIndex([d for d, _ in docs], term_imps)
    qids = list(queries)
    res = ora.search([list(DeepImpact.process_query(queries[q])) for q in qids], 1000)
    results = {q: {d: float(s) for d, s in r} for q, r in zip(qids, res)}
    want = evaluate_retrieval(qrels, results, (10, 100, 1000))
    assert got == want
    assert want[0]["NDCG@10"] > 0.3  # the queries are answerable
