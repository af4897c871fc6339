"""beir-style retrieval metrics (metrics.evaluate_retrieval, replacing
beir.EvaluateRetrieval at nano_beir_evaluator.py:230-231; pytrec_eval is absent, so
the values are pinned here by hand-computed trec_eval definitions -- parity with
pytrec_eval itself is unpinned)."""
import math

from improving_learned_index_amd.metrics import evaluate_retrieval


def test_hand_computed_trec_measures():
    qrels = {"q1": {"a": 1, "c": 1, "z": 1}, "q2": {"b": 1}, "q3": {"x": 1}}
    results = {"q1": {"a": 3.0, "b": 2.0, "c": 1.0, "d": 0.5},
               "q2": {"a": 1.0, "b": 1.0},      # tie: doc id descending -> b first
               "q4": {"x": 1.0}}                # no judgments: not averaged
    ndcg, _map, rec, p = evaluate_retrieval(qrels, results, (1, 3))
    # q1: rel at ranks 1 and 3 of 3 relevant; q2: rel at rank 1 (tie order)
    idcg3 = 1 + 1 / math.log2(3) + 1 / math.log2(4)
    q1_ndcg3 = (1 + 1 / math.log2(4)) / idcg3
    assert ndcg["NDCG@1"] == round((1 + 1) / 2, 5)
    assert ndcg["NDCG@3"] == round((q1_ndcg3 + 1) / 2, 5)
    assert _map["MAP@3"] == round(((1 + 2 / 3) / 3 + 1) / 2, 5)
    assert rec["Recall@3"] == round((2 / 3 + 1) / 2, 5)
    assert p["P@3"] == round((2 / 3 + 1 / 3) / 2, 5)
    assert p["P@1"] == 1.0


def test_identical_ids_are_ignored():
    qrels = {"q": {"d": 1}}
    assert evaluate_retrieval(qrels, {"q": {"q": 9.0, "d": 1.0}}, (1,))[0]["NDCG@1"] == 1.0
    assert evaluate_retrieval(qrels, {"q": {"q": 9.0, "d": 1.0}}, (1,),
                              ignore_identical_ids=False)[0]["NDCG@1"] == 0.0
