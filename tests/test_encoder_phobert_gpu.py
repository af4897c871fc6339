"""GPU parity of the fork's own DeepImpact class (src/deep_impact/models/original.py:18-48):
RoBERTa / PhoBERT -- RoBERTa positions (pad id + cumulative non-pad count), token
type 0, LayerNorm eps 1e-5, erf GELU -- with a Linear(768, 1) + ReLU head and
max_length 256 (original.py:20, :46), the class nano_beir_evaluator.__main__ loads
(nano_beir_evaluator.py:236-238).  vinai/phobert-base-v2's weights are not in the
container, so the model is a seeded PhoBERT-base-shaped one (V = 64,001, H = 768,
12 layers, 12 heads, F = 3072, 258 positions, type vocab 1, pad id 1) against the plain
PyTorch fp32 restatement oracle/encoder_ref.py (variant "xlmr" positions, act "relu").

Tolerances: bf16x3 -- rtol 1e-3 (north star) with atol 5e-5, the ReLU-head bar of
test_encoder_bert_gpu (the head's dot product cancels near 0); fp32 -- rtol 1e-3.
"""
import numpy as np
import pytest
import torch

import encoder_ref
from test_encoder_bert_gpu import _shapes

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-3, 5e-5
PHOBERT_BASE = {"vocab_size": 64001, "hidden_size": 768, "num_hidden_layers": 12,
                "num_attention_heads": 12, "intermediate_size": 3072,
                "max_position_embeddings": 258, "type_vocab_size": 1, "pad_token_id": 1,
                "layer_norm_eps": 1e-5}
MAX_LENGTH = 256  # original.py:20


@pytest.fixture(scope="module")
def E():
    from improving_learned_index_amd import _lib, encoder

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible (GPU test run without a GPU)")
    return encoder


@pytest.fixture(scope="module")
def pho():
    sd = encoder_ref.seeded_state_dict(_shapes(PHOBERT_BASE), seed=84, std=0.02)
    sd["impact_score_encoder.0.bias"] = torch.tensor([0.05])  # ~half the ReLU outputs > 0
    return PHOBERT_BASE, sd


def _cfg(E, c=PHOBERT_BASE):
    return E.EncoderConfig.from_hf({**c, "model_type": "roberta"}, variant="xlmr",
                                   activation="relu")


def _batch(rng, lens, vocab):
    """<s>-first ragged batch (ids in [5, V)), pad id 1, lengths <= max_length."""
    assert max(lens) <= MAX_LENGTH
    pad = np.ones((len(lens), max(lens)), np.int64)
    mask = np.zeros_like(pad)
    for i, n in enumerate(lens):
        pad[i, :n] = rng.integers(5, vocab, n)
        pad[i, 0] = 0
        mask[i, :n] = 1
    ids, cu = [], [0]
    for row, n in zip(pad, lens):
        ids += row[:n].tolist()
        cu.append(cu[-1] + n)
    return pad, mask, np.array(ids, np.int32), np.array(cu, np.int32)


def _oracle(sd, c, pad, mask):
    with torch.no_grad():
        return encoder_ref.forward(sd, c, torch.from_numpy(pad), torch.from_numpy(mask),
                                   "xlmr", "relu").numpy()


@pytest.mark.parametrize("precision", ["bf16x3", "fp32"])
@pytest.mark.parametrize("lens", [[256, 200, 131, 64, 9, 2], [256, 256, 255, 100, 1]])
def test_phobert_shape_matches_fp32_oracle(E, pho, precision, lens):
    c, sd = pho
    rng = np.random.default_rng(sum(lens))
    pad, mask, ids, cu = _batch(rng, lens, c["vocab_size"])
    want = _oracle(sd, c, pad, mask)[mask.astype(bool)]
    enc = E.DeviceEncoder(sd, _cfg(E), precision=precision)
    got = enc.encode_packed(ids, cu, token_impacts=True)
    assert 0.2 < float(np.mean(want > 0)) < 0.8  # both sides of the ReLU exercised
    assert float(np.mean(want == 0)) > 0.1  # the ReLU's exact zeros (notebook: 15 of 132)
    np.testing.assert_allclose(got, want, rtol=RTOL, atol=ATOL)


def test_phobert_shape_term_output_round3(E, pho):
    """Term output (first-occurrence gather, pruned last layer) with the reference's
    3-decimal rounding: equal to the oracle's per-token impacts gathered at the term
    rows and rounded the same way, except where the two fp32-close values straddle a
    rounding boundary (at most 1 step of 1e-3)."""
    import oracle

    c, sd = pho
    rng = np.random.default_rng(3)
    lens = [256, 190, 77, 12, 3]
    pad, mask, ids, cu = _batch(rng, lens, c["vocab_size"])
    tok = _oracle(sd, c, pad, mask)
    tt, ct = [], [0]
    for n in lens:
        pos = np.sort(rng.choice(np.arange(1, n), size=min(n - 1, 40), replace=False)) \
            if n > 1 else np.zeros(0, np.int64)
        tt += pos.tolist()
        ct.append(len(tt))
    tt, ct = np.array(tt, np.int32), np.array(ct, np.int32)
    want = np.array([tok[d, tt[j]] for d in range(len(lens)) for j in range(ct[d], ct[d + 1])],
                    np.float32)
    enc = E.DeviceEncoder(sd, _cfg(E), precision="bf16x3")
    got = enc.encode_packed(ids, cu, tt, ct, round3=True)
    want3 = oracle.round3(want)
    step = np.abs(got.astype(np.float64) - want3.astype(np.float64))
    assert float(step.max()) <= 1.0000001e-3, float(step.max())
    assert float(np.mean(got == want3)) > 0.98
