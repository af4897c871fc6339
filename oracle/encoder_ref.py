"""Plain PyTorch fp32 restatement of the DeeperImpact encoder -- TEST INFRASTRUCTURE ONLY.

The reference's encoder arithmetic is HF transformers (pinned 4.30.2,
requirements.txt:72) called at src/deep_impact/models/xlmr_original.py:70-75
(XLMRobertaModel; token_type_ids NOT passed, :73) followed by the impact head
``Sequential(Linear(H,1), Softplus())`` (xlmr_original.py:34-38, :77-85).  The
upstream BERT variant (soyuj/deeper-impact; original.py:10,19,21 commented) is
BertModel + ``Linear(H,1)`` + ReLU.

This file restates that math in a few lines of torch so the HIP encoder has an
fp32 checker that needs neither the reference nor transformers.  It is pinned to
the reference class itself by tests/test_oracle_golden.py (fixtures made by
tests/golden/make_golden.py, which ran the reference's DeepImpact forward).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def seeded_state_dict(shapes, seed, std):
    """Regenerates the weights the golden fixtures were made with (make_golden.py
    seeded_state_dict): numpy default_rng(seed), keys in the recorded order."""
    rng = np.random.default_rng(seed)
    sd = {}
    for k, shape, dtype in shapes:
        if "float" not in dtype:
            continue
        if k.endswith("LayerNorm.weight"):
            a = 1.0 + 0.1 * rng.standard_normal(shape)
        else:
            a = std * rng.standard_normal(shape)
        sd[k] = torch.from_numpy(a.astype(np.float32))
    return sd


def position_ids(ids, variant, pad_id):
    if variant == "bert":
        return torch.arange(ids.shape[1]).unsqueeze(0).expand_as(ids)
    # RoBERTa/XLM-R: create_position_ids_from_input_ids (padding_idx = pad id)
    m = ids.ne(pad_id).int()
    return (torch.cumsum(m, dim=1).type_as(m) * m).long() + pad_id


def layer_norm(x, w, b, eps):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


def forward(sd, cfg, ids, mask, variant="xlmr", act="softplus", prefix="bert."):
    """ids/mask: [B,S] int64.  Returns per-token impacts [B,S] float32."""
    p = prefix
    H = cfg["hidden_size"]
    nh = cfg["num_attention_heads"]
    dh = H // nh
    eps = cfg["layer_norm_eps"]
    pad = cfg.get("pad_token_id", 1)
    ids = torch.as_tensor(ids)
    mask = torch.as_tensor(mask)
    pos = position_ids(ids, variant, pad)
    x = (sd[p + "embeddings.word_embeddings.weight"][ids]
         + sd[p + "embeddings.position_embeddings.weight"][pos]
         + sd[p + "embeddings.token_type_embeddings.weight"][0])
    x = layer_norm(x, sd[p + "embeddings.LayerNorm.weight"], sd[p + "embeddings.LayerNorm.bias"],
                   eps)
    B, S, _ = x.shape
    neg = (1.0 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    for i in range(cfg["num_hidden_layers"]):
        L = f"{p}encoder.layer.{i}."

        def lin(t, name):
            return t @ sd[L + name + ".weight"].T + sd[L + name + ".bias"]

        q = lin(x, "attention.self.query").view(B, S, nh, dh).transpose(1, 2)
        k = lin(x, "attention.self.key").view(B, S, nh, dh).transpose(1, 2)
        v = lin(x, "attention.self.value").view(B, S, nh, dh).transpose(1, 2)
        s = q @ k.transpose(-1, -2) / math.sqrt(dh) + neg
        ctx = (torch.softmax(s, dim=-1) @ v).transpose(1, 2).reshape(B, S, H)
        x = layer_norm(x + lin(ctx, "attention.output.dense"),
                       sd[L + "attention.output.LayerNorm.weight"],
                       sd[L + "attention.output.LayerNorm.bias"], eps)
        h = torch.nn.functional.gelu(lin(x, "intermediate.dense"))
        x = layer_norm(x + lin(h, "output.dense"), sd[L + "output.LayerNorm.weight"],
                       sd[L + "output.LayerNorm.bias"], eps)
    z = x @ sd["impact_score_encoder.0.weight"][0] + sd["impact_score_encoder.0.bias"][0]
    if act == "softplus":
        return torch.nn.functional.softplus(z)  # beta=1, threshold=20 (nn.Softplus default)
    return torch.relu(z)


def gather_terms(impacts, term_maps):
    """compute_term_impacts (xlmr_original.py:205-225): first-token gather."""
    imp = impacts.detach().cpu().numpy()
    return [[(t, imp[i][tok]) for t, tok in m] for i, m in enumerate(term_maps)]
