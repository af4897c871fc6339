"""Device-resident DeeperImpact encoder (ctypes over di_encoder_* / di_encode).

Replaces the reference's model forward + term gather for a batch
(src/deep_impact/models/xlmr_original.py:41-85, :205-225).  PyTorch is used
only to read checkpoints into host tensors.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Mapping, Optional

import numpy as np

from . import _lib
from ._lib import check, lib, ptr

DI_VARIANT_XLMR, DI_VARIANT_BERT = 0, 1
DI_ACT_SOFTPLUS, DI_ACT_RELU = 0, 1
DI_PREC_BF16, DI_PREC_FP32, DI_PREC_BF16X3 = 0, 1, 2
# "bf16": bf16 MFMA (throughput mode, not fp32-faithful); "fp32": f32 MFMA throughout;
# "bf16x3": split-bf16 GEMMs (3 bf16 products per fp32 product) + f32 attention /
# LayerNorm -- fp32-faithful (impacts within 1e-3 relative of the reference) and fast
PRECISIONS = {"bf16": DI_PREC_BF16, "fp32": DI_PREC_FP32, "bf16x3": DI_PREC_BF16X3}
DI_DTYPE_F32, DI_DTYPE_BF16 = 0, 1
DI_F_ROUND3 = 0x10
DI_F_TOKEN_IMPACTS = 0x20


class di_encoder_cfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "variant", "activation", "precision", "vocab_size", "hidden", "layers", "heads",
        "intermediate", "max_positions", "type_vocab", "pad_id")] + [
        ("layer_norm_eps", ctypes.c_float)]


class di_tensor(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("dtype", ctypes.c_int32),
                ("ndim", ctypes.c_int32), ("shape", ctypes.c_int64 * 4)]


@dataclass
class EncoderConfig:
    """Architecture of the checkpoint.  Defaults: xlm-roberta-base, the config
    the reference loads by name (xlmr_original.py:193)."""
    variant: str = "xlmr"          # "xlmr" (RoBERTa positions) | "bert"
    activation: str = "softplus"   # "softplus" (xlmr_original.py:37) | "relu" (original.py:46)
    vocab_size: int = 250002
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_positions: int = 514
    type_vocab: int = 1
    pad_id: int = 1
    layer_norm_eps: float = 1e-5

    @classmethod
    def xlmr_base(cls):
        return cls()

    @classmethod
    def bert_base(cls):
        """bert-base-uncased / CoCondenser / soyuj/deeper-impact (ReLU head)."""
        return cls(variant="bert", activation="relu", vocab_size=30522, max_positions=512,
                   type_vocab=2, pad_id=0, layer_norm_eps=1e-12)

    @classmethod
    def from_hf(cls, cfg: Mapping, variant=None, activation=None):
        """From a transformers config dict (config.json)."""
        mt = cfg.get("model_type", "xlm-roberta")
        v = variant or ("bert" if mt == "bert" else "xlmr")
        return cls(variant=v, activation=activation or ("relu" if v == "bert" else "softplus"),
                   vocab_size=cfg["vocab_size"], hidden=cfg["hidden_size"],
                   layers=cfg["num_hidden_layers"], heads=cfg["num_attention_heads"],
                   intermediate=cfg["intermediate_size"],
                   max_positions=cfg["max_position_embeddings"],
                   type_vocab=cfg.get("type_vocab_size", 1),
                   pad_id=cfg.get("pad_token_id", 1 if v == "xlmr" else 0),
                   layer_norm_eps=cfg.get("layer_norm_eps", 1e-5 if v == "xlmr" else 1e-12))

    @classmethod
    def infer(cls, state_dict: Mapping, variant="xlmr", activation=None):
        """Shapes from the state dict, the rest from the variant's base config."""
        base = cls.xlmr_base() if variant == "xlmr" else cls.bert_base()
        if activation:
            base.activation = activation

        def shp(k):
            for p in ("bert.", "roberta.", ""):
                if p + k in state_dict:
                    return tuple(state_dict[p + k].shape)
            raise KeyError(k)

        V, H = shp("embeddings.word_embeddings.weight")
        P = shp("embeddings.position_embeddings.weight")[0]
        T = shp("embeddings.token_type_embeddings.weight")[0]
        F = shp("encoder.layer.0.intermediate.dense.weight")[0]
        L = 0
        while any(f"{p}encoder.layer.{L}.output.dense.weight" in state_dict
                  for p in ("bert.", "roberta.", "")):
            L += 1
        base.vocab_size, base.hidden, base.max_positions = V, H, P
        base.type_vocab, base.intermediate, base.layers = T, F, L
        base.heads = H // 64
        return base

    def to_c(self, precision: str) -> di_encoder_cfg:
        c = di_encoder_cfg()
        c.variant = DI_VARIANT_XLMR if self.variant == "xlmr" else DI_VARIANT_BERT
        c.activation = DI_ACT_SOFTPLUS if self.activation == "softplus" else DI_ACT_RELU
        if precision not in PRECISIONS:
            raise ValueError(f"precision {precision!r}: one of {sorted(PRECISIONS)}")
        c.precision = PRECISIONS[precision]
        for f in ("vocab_size", "hidden", "layers", "heads", "intermediate", "max_positions",
                  "type_vocab", "pad_id"):
            setattr(c, f, getattr(self, f))
        c.layer_norm_eps = self.layer_norm_eps
        return c


def _host_array(t):
    """torch tensor / numpy array -> (contiguous numpy array, DI dtype)."""
    if hasattr(t, "detach"):
        import torch

        t = t.detach().cpu().contiguous()
        if t.dtype == torch.bfloat16:
            return t.view(torch.int16).numpy().view(np.uint16), DI_DTYPE_BF16
        return t.to(torch.float32).numpy(), DI_DTYPE_F32
    a = np.ascontiguousarray(t)
    if a.dtype == np.uint16:
        return a, DI_DTYPE_BF16
    return np.ascontiguousarray(a, np.float32), DI_DTYPE_F32


class DeviceEncoder:
    """Weights resident on one GPU; encode() runs the whole forward there."""

    def __init__(self, state_dict: Mapping, cfg: EncoderConfig, precision="bf16", device=0):
        if precision == "bf16x3" and not (cfg.hidden in (768, 1024) and cfg.intermediate % 256 == 0):
            precision = "fp32"  # split-bf16 kernels take base / large shapes; f32 MFMA otherwise
        self.cfg, self.precision, self.device = cfg, precision, device
        keep, tens = [], []
        for k, v in state_dict.items():
            if not (hasattr(v, "shape") and len(v.shape) <= 4):
                continue
            if hasattr(v, "is_floating_point") and not v.is_floating_point():
                continue  # e.g. embeddings.position_ids (int64 buffer)
            a, dt = _host_array(v)
            name = k.encode("utf-8")
            keep += [a, name]
            t = di_tensor()
            t.name, t.data, t.dtype, t.ndim = name, a.ctypes.data, dt, a.ndim
            for i, d in enumerate(a.shape):
                t.shape[i] = d
            tens.append(t)
        arr = (di_tensor * max(1, len(tens)))(*tens)
        h = ctypes.c_void_p()
        c = cfg.to_c(precision)
        check(lib().di_encoder_create(ctypes.byref(c), arr, len(tens), device, ctypes.byref(h)))
        self._h = h

    def encode_packed(self, ids, cu_seqlens, term_tok=None, cu_terms=None, round3=False,
                      token_impacts=False, timing=False):
        """Host arrays in, host float32 impacts out (per term, or per token)."""
        ids = np.ascontiguousarray(ids, np.int32)
        cu = np.ascontiguousarray(cu_seqlens, np.int32)
        n_docs = len(cu) - 1
        flags = (DI_F_ROUND3 if round3 else 0) | (_lib.DI_F_TIMING if timing else 0)
        if token_impacts:
            flags |= DI_F_TOKEN_IMPACTS
            out = np.zeros(max(1, int(cu[-1])), np.float32)
            tt = np.zeros(1, np.int32)
            ct = np.zeros(n_docs + 1, np.int32)
        else:
            tt = np.ascontiguousarray(term_tok, np.int32)
            ct = np.ascontiguousarray(cu_terms, np.int32)
            out = np.zeros(max(1, int(ct[-1])), np.float32)
            if tt.size == 0:
                tt = np.zeros(1, np.int32)
        if ids.size == 0:
            ids = np.zeros(1, np.int32)
        check(lib().di_encode(self._h, ptr(ids), ptr(cu), n_docs, 0, 0, ptr(tt), ptr(ct), 0,
                              ptr(out), flags))
        n = int(cu[-1]) if token_impacts else int(ct[-1])
        return out[:n]

    def encode_device(self, ids, cu_seqlens, n_docs, n_tokens, max_len, term_tok, cu_terms,
                      n_terms, out, flags=_lib.DI_F_DEVICE_PTRS):
        check(lib().di_encode(self._h, ptr(ids), ptr(cu_seqlens), n_docs, n_tokens, max_len,
                              ptr(term_tok), ptr(cu_terms), n_terms, ptr(out), flags))

    def reserve(self, max_tokens, max_docs, max_terms):
        check(lib().di_encoder_reserve(self._h, max_tokens, max_docs, max_terms))

    def set_stream(self, stream_ptr):
        check(lib().di_encoder_set_stream(self._h, ctypes.c_void_p(stream_ptr)))

    def sync(self):
        check(lib().di_encoder_sync(self._h))

    def timing(self, name, reset=False):
        t = _lib.di_timing()
        check(lib().di_encoder_timing(self._h, name.encode(), ctypes.byref(t), int(reset)))
        return t.ms, t.launches

    def close(self):
        if getattr(self, "_h", None):
            lib().di_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def quantize(impacts, max_val=None, bits=8, device=0):
    """di_quantize: int(v * (2^bits-1)/max) with the reference's fp64 arithmetic."""
    v = np.ascontiguousarray(impacts, np.float32)
    out = np.zeros(max(1, v.size), np.int32)
    used = ctypes.c_double(0.0)
    check(lib().di_quantize(ptr(v if v.size else np.zeros(1, np.float32)), v.size,
                            float(max_val) if max_val is not None else -1.0, bits, ptr(out),
                            ctypes.byref(used), device, None, 0))
    return out[:v.size], used.value
