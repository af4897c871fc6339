"""GPU parity of the fp32-faithful fast encode mode (precision "bf16x3", DI_PREC_BF16X3).

Every GEMM runs as split-bf16 (A = A_hi + A_lo, W = W_hi + W_lo; three bf16 MFMA
products A_hi W_hi + A_hi W_lo + A_lo W_hi, f32 accumulate, ~2^-17 relative per
product); the attention products QK^T and PV are split-bf16 the same way with an f32
softmax; the LayerNorms are folded into the GEMMs (f32 row statistics of the split
residual rows; DI_NO_LN_FOLD=1 runs them as f32 passes) -- the reference computes in
fp32 (src/deep_impact/indexing/indexer.py:46, no autocast).  Checked against:
  * the reference's own DeepImpact (XLM-R) forward on the full xlm-roberta-base shape
    (tests/golden/encoder_xlmr_base.json, made by tests/golden/make_golden.py);
  * the plain PyTorch fp32 restatement oracle/encoder_ref.py on ragged batches up to
    512 tokens, and with outlier LayerNorm channels (large |mean| / sigma rows, the
    regime of trained RoBERTa-family checkpoints);
  * end to end through the reference's text path: round(., 3) (indexer.py:62-68) ->
    quantize (quantize.py:13-47) -> index (create.py) -> top-1000 (inverted_index.py:55-62)
    -> MRR@10 / Recall (metrics.py:26-57), against the fp32 oracle's impacts.
Tolerance (north star): float impacts within 1e-3 relative of the fp32 reference.
"""
import json

import numpy as np
import pytest
import torch

import encoder_ref
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

RTOL = 1e-3  # north star: float scores within 1e-3 relative


@pytest.fixture(scope="module")
def E():
    from improving_learned_index_amd import _lib, encoder

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible (GPU test run without a GPU)")
    return encoder


@pytest.fixture(scope="module")
def base():
    fx = json.loads((GOLDEN / "encoder_xlmr_base.json").read_text())
    sd = encoder_ref.seeded_state_dict(fx["state_dict_shapes"], fx["seed"], fx["std"])
    return fx, sd


def _cfg(E, fx):
    c = fx["config"]
    return E.EncoderConfig(variant="xlmr", activation="softplus", vocab_size=c["vocab_size"],
                           hidden=c["hidden_size"], layers=c["num_hidden_layers"],
                           heads=c["num_attention_heads"], intermediate=c["intermediate_size"],
                           max_positions=c["max_position_embeddings"],
                           type_vocab=c["type_vocab_size"], pad_id=c["pad_token_id"],
                           layer_norm_eps=c["layer_norm_eps"])


def _pack(input_ids, mask):
    ids, cu = [], [0]
    for row, m in zip(input_ids, mask):
        n = int(sum(m))
        ids += list(row[:n])
        cu.append(cu[-1] + n)
    return np.array(ids, np.int32), np.array(cu, np.int32)


def _random_batch(rng, lens, vocab):
    ids = [rng.integers(5, vocab, n).astype(np.int64) for n in lens]
    for a in ids:
        a[0] = 0
    pad = np.ones((len(lens), max(lens)), np.int64)
    mask = np.zeros_like(pad)
    for i, a in enumerate(ids):
        pad[i, :len(a)] = a
        mask[i, :len(a)] = 1
    return pad, mask


def _oracle(sd, fx, pad, mask):
    with torch.no_grad():
        return encoder_ref.forward(sd, fx["config"], torch.from_numpy(pad),
                                   torch.from_numpy(mask), "xlmr", "softplus").numpy()


def test_bf16x3_term_impacts_match_reference_class(E, base):
    fx, sd = base
    enc = E.DeviceEncoder(sd, _cfg(E, fx), precision="bf16x3")
    ids, cu = _pack(fx["input_ids"], fx["attention_mask"])
    maps = fx["term_maps"]
    tt = np.array([tok for m in maps for _, tok in m], np.int32)
    ct = np.cumsum([0] + [len(m) for m in maps]).astype(np.int32)
    got = enc.encode_packed(ids, cu, tt, ct)
    want = np.array([b for d in fx["term_impacts_f32_bits"] for _, b in d],
                    np.uint32).view(np.float32)
    np.testing.assert_allclose(got, want, rtol=RTOL, atol=1e-6)


# (the attention's pass and tile edges: 16-query tiles, three per wave, 384-query passes --
# 256 / 257 and 384 / 385 tokens put the first query into a wave's third tile / a second pass)
@pytest.mark.parametrize("lens", [[300, 250, 180, 64, 9, 120], [512, 400, 321, 40, 3, 1],
                                  [385, 384, 257, 256, 17, 16]])
def test_bf16x3_ragged_batches_match_torch_oracle(E, base, lens):
    fx, sd = base
    enc = E.DeviceEncoder(sd, _cfg(E, fx), precision="bf16x3")
    rng = np.random.default_rng(sum(lens))
    pad, mask = _random_batch(rng, lens, 250002)
    want = _oracle(sd, fx, pad, mask)[mask.astype(bool)]
    ids, cu = _pack(pad.tolist(), mask.tolist())
    got = enc.encode_packed(ids, cu, token_impacts=True)
    np.testing.assert_allclose(got, want, rtol=RTOL, atol=1e-6)


def test_bf16x3_pruned_last_layer_is_bitexact(E, base):
    """Term output computes the last layer only for the terms' first-token rows (queries
    of the attention, O / FFN GEMMs, LayerNorms, head); each kept row's arithmetic is
    unchanged, so the impacts must equal the full per-token forward gathered at those
    rows, bit for bit -- ragged documents past one 384-query pass, a document without
    terms, terms in any order and repeated."""
    fx, sd = base
    enc = E.DeviceEncoder(sd, _cfg(E, fx), precision="bf16x3")
    rng = np.random.default_rng(12)
    lens = [512, 300, 2, 64, 9, 180, 120, 33]
    pad, mask = _random_batch(rng, lens, 250002)
    ids, cu = _pack(pad.tolist(), mask.tolist())
    tok = enc.encode_packed(ids, cu, token_impacts=True)
    tt, ct = [], [0]
    for d, n in enumerate(lens):
        k = 0 if d == 2 else (n if d == 0 else int(rng.integers(1, n + 1)))
        pos = rng.choice(n, size=k, replace=False)
        if d == 3:
            pos = np.concatenate([pos, pos[:2]])  # repeated token positions
        tt += pos.tolist()
        ct.append(len(tt))
    tt, ct = np.array(tt, np.int32), np.array(ct, np.int32)
    want = np.array([tok[cu[d] + tt[j]] for d in range(len(lens)) for j in range(ct[d], ct[d + 1])],
                    np.float32)
    np.testing.assert_array_equal(enc.encode_packed(ids, cu, tt, ct), want)


def _outlier_sd(sd):
    """Outlier LayerNorm channels in every LayerNorm: large beta and gamma on three
    channels, so the residual stream carries rows with |mean| / sigma >> 1."""
    sd = dict(sd)
    ch = [5, 77, 300]
    beta = torch.tensor([6.0, -8.0, 12.0])
    for k in list(sd):
        if k.endswith("LayerNorm.bias"):
            v = sd[k].clone()
            v[ch] = beta
            sd[k] = v
        elif k.endswith("LayerNorm.weight"):
            v = sd[k].clone()
            v[ch] = 4.0
            sd[k] = v
    return sd


def test_layernorm_outlier_channels(E, base, monkeypatch):
    """bf16x3 (LayerNorms folded, and unfolded with DI_NO_LN_FOLD) stays inside the
    1e-3 bar with outlier channels; the bf16 throughput
    mode with LayerNorm folding (residual rounded to bf16 before normalisation) is
    compared with the unfolded bf16 path (DI_NO_LN_FOLD) against the same oracle, and
    folding must not be materially worse than not folding."""
    fx, sd = base
    sd = _outlier_sd(sd)
    rng = np.random.default_rng(5)
    lens = [200, 150, 77, 31]
    pad, mask = _random_batch(rng, lens, 250002)
    want = _oracle(sd, fx, pad, mask)[mask.astype(bool)]
    ids, cu = _pack(pad.tolist(), mask.tolist())
    enc = E.DeviceEncoder(sd, _cfg(E, fx), precision="bf16x3")
    got = enc.encode_packed(ids, cu, token_impacts=True)
    np.testing.assert_allclose(got, want, rtol=RTOL, atol=1e-6)
    rel = lambda y: np.abs(y - want) / np.maximum(np.abs(want), 1e-3)  # noqa: E731
    folded = E.DeviceEncoder(sd, _cfg(E, fx), precision="bf16")
    r_fold = rel(folded.encode_packed(ids, cu, token_impacts=True))
    del folded
    monkeypatch.setenv("DI_NO_LN_FOLD", "1")
    plain = E.DeviceEncoder(sd, _cfg(E, fx), precision="bf16")
    r_plain = rel(plain.encode_packed(ids, cu, token_impacts=True))
    del plain
    # bf16x3 folds its LayerNorms too (split rows of the un-normalised residual, no
    # LayerNorm pass); the unfolded bf16x3 path must meet the bar as well
    plain3 = E.DeviceEncoder(sd, _cfg(E, fx), precision="bf16x3")
    got3 = plain3.encode_packed(ids, cu, token_impacts=True)
    np.testing.assert_allclose(got3, want, rtol=RTOL, atol=1e-6)
    print(f"bf16x3 max rel folded {rel(got).max():.2e} unfolded {rel(got3).max():.2e}; "
          f"bf16 folded max/median rel {r_fold.max():.2e}/{np.median(r_fold):.2e}; "
          f"unfolded {r_plain.max():.2e}/{np.median(r_plain):.2e}")
    assert np.median(r_fold) <= 2.0 * np.median(r_plain) + 1e-3
    assert r_fold.max() <= 2.0 * r_plain.max() + 1e-2


def _pipeline(impacts_per_doc, terms_per_doc, queries, max_val=None):
    """Reference text path: round3 + repr text -> quantize -> index -> top-1000."""
    import oracle

    lines = [oracle.impact_line(t, v) for t, v in zip(terms_per_doc, impacts_per_doc)]
    q, used = oracle.quantize_lines(lines, max_val)
    docs = [dict((p.split(": ")[0], float(p.split(": ")[1])) for p in l.split(", ")) if l else {}
            for l in q]
    vocab, term_off, pdoc, pval = oracle.build_index(docs)
    ix = oracle.Index.__new__(oracle.Index)
    ix.vocab = {t: i for i, t in enumerate(vocab)}
    ix.term_off, ix.pdoc, ix.pval = term_off, pdoc, pval
    ix.n_docs = len(docs)
    runs = ix.score_ids([ix.term_ids(sorted(qq)) for qq in queries], 1000)
    return lines, q, runs, used


def test_bf16x3_end_to_end_quantized_and_metrics(E, base):
    """Impacts -> impact TSV text -> 8-bit quantized integers -> index -> top-1000 ->
    MRR@10 / Recall: the bf16x3 run must give the fp32 oracle's metrics, with
    quantized-integer flips (terms whose integer differs) at most 2e-3 of all terms;
    the bf16 throughput mode's flip rate is reported beside it."""
    import oracle

    fx, sd = base
    rng = np.random.default_rng(7)
    lens = rng.integers(24, 128, 32).tolist()
    pad, mask = _random_batch(rng, lens, 250002)
    ids, cu = _pack(pad.tolist(), mask.tolist())
    # terms: first occurrence of each token id (term string = "t<id>"), every 2nd token
    terms, toks = [], []
    for d, n in enumerate(lens):
        seen, tt, tk = set(), [], []
        for i in range(1, n - 1, 2):
            t = f"t{int(pad[d, i])}"
            if t not in seen:
                seen.add(t)
                tt.append(t)
                tk.append(i)
        terms.append(tt)
        toks.append(tk)
    tt = np.array([i for tk in toks for i in tk], np.int32)
    ct = np.cumsum([0] + [len(tk) for tk in toks]).astype(np.int32)
    want_tok = _oracle(sd, fx, pad, mask)
    want = [want_tok[d, toks[d]].astype(np.float32) for d in range(len(lens))]
    queries, qrels = [], {}
    for qi in range(64):
        d = int(rng.integers(0, len(lens)))
        k = min(len(terms[d]), int(rng.integers(2, 7)))
        queries.append(set(rng.choice(terms[d], size=k, replace=False).tolist()))
        qrels[qi] = {d}
    l_ref, q_ref, run_ref, _ = _pipeline(want, terms, queries)

    def evaluate(run):
        trip = [(qi, doc, r + 1) for qi, res in enumerate(run) for r, (doc, _) in enumerate(res)]
        return oracle.mrr_recall(trip, qrels)

    m_ref = evaluate(run_ref)
    res = {}
    for prec in ("bf16x3", "bf16"):
        enc = E.DeviceEncoder(sd, _cfg(E, fx), precision=prec)
        got = enc.encode_packed(ids, cu, tt, ct)
        del enc
        per_doc = [got[ct[d]:ct[d + 1]] for d in range(len(lens))]
        l_got, q_got, run_got, _ = _pipeline(per_doc, terms, queries)
        qa = [p for l in q_ref for p in (l.split(", ") if l else [])]
        qb = [p for l in q_got for p in (l.split(", ") if l else [])]
        text_flip = np.mean([a != b for a, b in zip(
            [p for l in l_ref for p in l.split(", ")], [p for l in l_got for p in l.split(", ")])])
        q_flip = (sum(a != b for a, b in zip(qa, qb)) + abs(len(qa) - len(qb))) / max(len(qa), 1)
        res[prec] = (text_flip, q_flip, evaluate(run_got))
    print({k: (f"text flips {v[0]:.2e}", f"quantized flips {v[1]:.2e}", v[2][0]) for k, v in
           res.items()})
    text_flip, q_flip, m = res["bf16x3"]
    assert q_flip <= 2e-3, q_flip
    assert m == m_ref


def _bench_batch(n_docs, seed, max_len=300, vocab=250002):
    """The bench's configs[1] encode batch: n_i = clip(round(N(200, 60)),
    8, 300), ids uniform [5, V) with <s> first, words of 1 + Geom(0.3) tokens, ~0.7 of
    them kept as terms (their first tokens)."""
    rng = np.random.default_rng(seed)
    lens = np.clip(np.rint(rng.normal(200, 60, n_docs)), 8, max_len).astype(np.int32)
    cu = np.zeros(n_docs + 1, np.int32)
    cu[1:] = np.cumsum(lens)
    ids = rng.integers(5, vocab, int(cu[-1])).astype(np.int32)
    ids[cu[:-1]] = 0
    tt, ct = [], [0]
    for n in lens:
        starts = [1]
        while True:
            nxt = starts[-1] + int(rng.geometric(0.3))
            if nxt >= n - 1:
                break
            starts.append(nxt)
        keep = [s for s in starts if rng.random() < 0.7]
        tt += keep
        ct.append(ct[-1] + len(keep))
    return ids, cu, np.array(tt, np.int32), np.array(ct, np.int32)


@pytest.mark.parametrize("precision", ["bf16x3", "bf16"])
def test_full_size_batch_is_batch_invariant(E, base, precision):
    """Size-independent property at the bench's full size (8192 docs, ~1.6 M tokens,
    round3 term output): every row's arithmetic is independent of the other documents
    (GEMM rows, per-document attention, per-row LayerNorm statistics), so 64 documents
    re-encoded on their own give bit-identical impacts to their slices of the full batch."""
    fx, sd = base
    enc = E.DeviceEncoder(sd, _cfg(E, fx), precision=precision)
    ids, cu, tt, ct = _bench_batch(8192, 7)
    full = enc.encode_packed(ids, cu, tt, ct, round3=True)
    assert full.shape[0] == ct[-1] and np.isfinite(full).all()
    pick = np.sort(np.random.default_rng(3).choice(8192, 64, replace=False))
    sids, scu, stt, sct = [], [0], [], [0]
    want = []
    for d in pick:
        sids.append(ids[cu[d]:cu[d + 1]])
        scu.append(scu[-1] + int(cu[d + 1] - cu[d]))
        stt.append(tt[ct[d]:ct[d + 1]])
        sct.append(sct[-1] + int(ct[d + 1] - ct[d]))
        want.append(full[ct[d]:ct[d + 1]])
    got = enc.encode_packed(np.concatenate(sids), np.array(scu, np.int32), np.concatenate(stt),
                            np.array(sct, np.int32), round3=True)
    np.testing.assert_array_equal(got, np.concatenate(want))


def test_flip_rates_at_bench_scale(E, base):
    """The bench's full configs[1] batch (8192 docs, ~1.6 M tokens, ~344 k terms):
    bf16x3 (and bf16) against the library's fp32 mode -- itself within ~1e-5 of the fp32
    oracle (test_encoder_gpu) -- through the reference's text path: round(., 3)
    (indexer.py:62-68; a "text flip" = the impact text differs) and the 8-bit quantizer
    (quantize.py:27-47, each run with its own max like quantize_file; a "quantized
    flip" = the integer differs, 0 = dropped included).  Bar: bf16x3 quantized flips
    <= 1e-3 of the terms.  The rates are printed for DESIGN.md."""
    fx, sd = base
    ids, cu, tt, ct = _bench_batch(8192, 7)
    r = {}
    for prec in ("fp32", "bf16x3", "bf16"):
        enc = E.DeviceEncoder(sd, _cfg(E, fx), precision=prec)
        r[prec] = enc.encode_packed(ids, cu, tt, ct, round3=True)
        del enc
    assert r["fp32"].shape[0] == ct[-1] > 300_000

    def quant(v):
        d = v.astype(np.float64)
        return np.trunc(d * (255.0 / float(d.max()))).astype(np.int64)

    q32 = quant(r["fp32"])
    rates = {}
    for prec in ("bf16x3", "bf16"):
        text = float(np.mean(r[prec].view(np.uint32) != r["fp32"].view(np.uint32)))
        qf = float(np.mean(quant(r[prec]) != q32))
        rel = np.abs(r[prec].astype(np.float64) - r["fp32"]) / np.maximum(np.abs(r["fp32"]), 1e-3)
        rates[prec] = (text, qf, float(rel.max()))
    print(f"flip rates over {int(ct[-1])} terms (vs fp32 mode): " + "; ".join(
        f"{p}: text {t:.3e} quantized {q:.3e} max rel (rounded) {m:.2e}"
        for p, (t, q, m) in rates.items()))
    assert rates["bf16x3"][1] <= 1e-3, rates


def test_flip_rates_vs_torch_fp32_oracle(E, base):
    """512 bench-shaped documents (configs[1]: n = clip(N(200, 60), 8, 300), ~100 k
    tokens, ~21 k terms) against the plain PyTorch fp32 oracle (oracle/encoder_ref.py,
    CPU, padded batches as the reference runs them) -- not against the library's own
    fp32 mode: the term impacts through the reference's text path, round(., 3) (a "text
    flip" = the 3-decimal text differs) and the 8-bit quantizer
    (a "quantized flip" = the integer differs; each side quantized with its own max, as
quantize_file does).  The library's fp32 mode is measured the
    same way: two fp32 summation orders already disagree on values within ~1e-6 of a
    rounding boundary, the floor any implementation other than the reference's own
    BLAS has.  Bars: bf16x3 quantized flips <= 1e-3 of the terms and max relative
    error <= 1e-3 (north star)."""
    import oracle

    fx, sd = base
    ids, cu, tt, ct = _bench_batch(512, 11)
    lens = np.diff(cu)
    # the oracle: batches of 16 documents sorted by length (little padding)
    order = np.argsort(lens, kind="stable")
    tok = [None] * len(lens)
    for s0 in range(0, len(order), 16):
        b = order[s0:s0 + 16]
        S_ = int(lens[b].max())
        pad = np.ones((len(b), S_), np.int64)
        mask = np.zeros((len(b), S_), np.int64)
        for r, d in enumerate(b):
            pad[r, :lens[d]] = ids[cu[d]:cu[d + 1]]
            mask[r, :lens[d]] = 1
        out = _oracle(sd, fx, pad, mask)
        for r, d in enumerate(b):
            tok[d] = out[r, :lens[d]]
    want = np.concatenate([tok[d][tt[ct[d]:ct[d + 1]]] for d in range(len(lens))]).astype(np.float32)
    want3 = oracle.round3(want)

    def quant(v, m):
        return np.trunc(v.astype(np.float64) * (255.0 / m)).astype(np.int64)

    m_ref = float(want3.astype(np.float64).max())
    q_ref = quant(want3, m_ref)
    rates = {}
    for prec in ("bf16x3", "fp32"):
        enc = E.DeviceEncoder(sd, _cfg(E, fx), precision=prec)
        raw = enc.encode_packed(ids, cu, tt, ct)
        got3 = enc.encode_packed(ids, cu, tt, ct, round3=True)
        del enc
        np.testing.assert_array_equal(got3, oracle.round3(raw))  # (the kernel's A9 rounding)
        rel = np.abs(raw.astype(np.float64) - want) / np.maximum(np.abs(want), 1e-3)
        rates[prec] = (float(np.mean(got3.view(np.uint32) != want3.view(np.uint32))),
                       float(np.mean(quant(got3, float(got3.astype(np.float64).max())) != q_ref)),
                       float(rel.max()))
    print(f"flip rates over {int(ct[-1])} terms vs the torch fp32 oracle: " + "; ".join(
        f"{p}: text {t:.3e} quantized {q:.3e} max rel {m:.2e}" for p, (t, q, m) in rates.items()))
    assert int(ct[-1]) > 20_000
    assert rates["bf16x3"][2] <= RTOL, rates
    assert rates["bf16x3"][1] <= 1e-3, rates
