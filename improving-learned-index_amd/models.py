"""DeepImpact model protocol on MI355X -- host-side mirror of the reference class.

Reference: src/deep_impact/models/xlmr_original.py (DeepImpact, XLM-R + Softplus)
and the upstream BERT/CoCondenser variant (src/deep_impact/models/original.py:10,
19,21,155-177, commented there; soyuj/deeper-impact: BertModel + ReLU).

Same names and argument meaning as the reference protocol used by Indexer
(indexer.py:22,33,46,57) and SparseSearch (nano_beir_evaluator.py:93,114):
``load``, ``process_document``, ``process_query``, ``compute_term_impacts``,
``__call__``, ``get_impact_scores``, ``get_impact_scores_batch``.  Tokenization
and term extraction stay on the host (HF ``tokenizers``, batched in Rust); the
forward, the impact head and the first-occurrence gather run in
libdeepimpact_hip.so.  There is no CPU compute fallback.

Not covered: the PhoBERT variant's VnCoreNLP word segmentation
(original.py:29-39,182-194) needs a Java runtime and models that are not part of
this build; its encoder math is the RoBERTa kernel path here.
"""
from __future__ import annotations

import json
import os
import string
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple, Union

import numpy as np

from . import _lib
from .encoder import DeviceEncoder, EncoderConfig

PUNCTUATION = set(string.punctuation)


class Encoding:
    """What process_document returns in place of the reference's MockEncoding
    (xlmr_original.py:16-23): ids / attention_mask / type_ids / word_ids of the
    document (unpadded: the device path packs documents without padding)."""

    __slots__ = ("ids", "attention_mask", "type_ids", "word_ids")

    def __init__(self, ids, word_ids):
        self.ids = list(ids)
        self.attention_mask = [1] * len(self.ids)
        self.type_ids = [0] * len(self.ids)
        self.word_ids = list(word_ids)


def load_tokenizer(path_or_obj):
    """A `tokenizers.Tokenizer` from tokenizer.json (or a directory holding one,
    e.g. a local xlm-roberta-base snapshot), or passed through."""
    if path_or_obj is None:
        return None
    if not isinstance(path_or_obj, (str, Path)):
        return path_or_obj
    from tokenizers import Tokenizer

    p = Path(path_or_obj)
    if p.is_dir():
        p = p / "tokenizer.json"
    return Tokenizer.from_file(str(p))


def _normalize(tok, text: str) -> str:
    n = tok.normalizer
    return n.normalize_str(text) if n is not None else text


def _pre_tokenize(tok, text: str) -> List[str]:
    pt = tok.pre_tokenizer
    if pt is None:
        return text.split()
    return [x[0] for x in pt.pre_tokenize_str(text)]


def _first_token_map(word_ids) -> Dict[int, int]:
    """word index -> index of its first token (xlmr_original.py:153-164)."""
    out, prev = {}, None
    for i, w in enumerate(word_ids):
        if w is None:
            continue
        if w != prev:
            out[w] = i
            prev = w
    return out


def _legacy_bert_map(tokens) -> Dict[int, int]:
    """Upstream BERT logic (original.py:162-170, commented there): every token
    after [CLS] that does not start with '##' opens the next term."""
    out, counter = {}, 0
    for i, t in enumerate(tokens[1:], start=1):
        if t.startswith("##"):
            continue
        out[counter] = i
        counter += 1
    return out


class _WordCache:
    """Per-word token cache for the pre-tokenized document encode.  A pre-tokenized
    input is normalized, pre-tokenized and modelled one word at a time, so a word's
    tokens do not depend on its neighbours (except, for a Metaspace pre-tokenizer with
    prepend_scheme "first", on whether it is the first word: two tables); a document's
    encoding is then the template's prefix specials, its words' cached tokens cut to
    max_length - #specials (the tokenizer's right truncation of a single sequence) and
    the suffix specials.  Misses are encoded in one batched call per document batch.
    Checked against encode_batch (tests/test_host_cpu.py) and self-checked on the first
    batch of each process: any difference turns the cache off."""

    MAX_ENTRIES = 1 << 20
    ANCHOR = "a"

    def __init__(self, tok):
        self.tok = tok
        self.first: Dict[str, List[int]] = {}
        self.other: Dict[str, List[int]] = {}
        e = tok.encode([self.ANCHOR], is_pretokenized=True, add_special_tokens=True)
        wid = e.word_ids
        lo = next(i for i, w in enumerate(wid) if w is not None)
        hi = max(i for i, w in enumerate(wid) if w is not None) + 1
        self.prefix, self.suffix = list(e.ids[:lo]), list(e.ids[hi:])
        self.checked = False
        self.ok = True

    def _fill(self, terms_list: Sequence[Sequence[str]]) -> None:
        mf = {t[0] for t in terms_list if t and t[0] not in self.first}
        mo = {w for t in terms_list for w in t[1:] if w not in self.other}
        if not mf and not mo:
            return
        if len(self.first) + len(self.other) + len(mf) + len(mo) > self.MAX_ENTRIES:
            # bounded memory: start over before this batch's fill, which then holds
            # every word the batch looks up
            self.first.clear()
            self.other.clear()
            mf = {t[0] for t in terms_list if t}
            mo = {w for t in terms_list for w in t[1:]}
        tok = self.tok
        trunc = tok.truncation
        tok.no_truncation()  # (a cached word keeps all its tokens)
        try:
            if mf:
                mf = list(mf)
                for w, e in zip(mf, tok.encode_batch([[w] for w in mf], is_pretokenized=True,
                                                     add_special_tokens=False)):
                    self.first[w] = [i for i, x in zip(e.ids, e.word_ids) if x == 0]
            if mo:
                mo = list(mo)
                for w, e in zip(mo, tok.encode_batch([[self.ANCHOR, w] for w in mo],
                                                     is_pretokenized=True,
                                                     add_special_tokens=False)):
                    self.other[w] = [i for i, x in zip(e.ids, e.word_ids) if x == 1]
        finally:
            if trunc is not None:
                tok.enable_truncation(**trunc)

    def encode(self, terms_list: Sequence[Sequence[str]], max_length: int):
        """[(ids, word_ids)] of each document, as encode_batch(..., is_pretokenized=True,
        add_special_tokens=True) under enable_truncation(max_length)."""
        self._fill(terms_list)
        budget = max(max_length - len(self.prefix) - len(self.suffix), 0)
        out = []
        first, other = self.first, self.other
        for terms in terms_list:
            ids = list(self.prefix)
            wids: List[Optional[int]] = [None] * len(ids)
            room = budget
            for i, w in enumerate(terms):
                if room <= 0:
                    break
                tk = first[w] if i == 0 else other[w]
                if len(tk) > room:
                    tk = tk[:room]
                ids.extend(tk)
                wids.extend([i] * len(tk))
                room -= len(tk)
            ids.extend(self.suffix)
            wids.extend([None] * len(self.suffix))
            out.append((ids, wids))
        return out


def _filter_terms(terms: Sequence[str], idx_map: Dict[int, int]) -> Dict[str, int]:
    """Unique, non-punctuation terms whose tokens survived truncation, in
    first-occurrence order (xlmr_original.py:181-187)."""
    out: Dict[str, int] = {}
    for i, t in enumerate(terms):
        if t not in out and t not in PUNCTUATION and i in idx_map:
            out[t] = idx_map[i]
    return out


class DeepImpact:
    """The DeeperImpact model on one MI355X."""

    max_length = 512
    tokenizer = None  # tokenizers.Tokenizer (class-level, like the reference)
    punctuation = PUNCTUATION
    term_mapping = "word_ids"  # or "bert_legacy" (original.py:162-170)

    def __init__(self, encoder: DeviceEncoder, tokenizer=None, max_length: Optional[int] = None):
        self.encoder = encoder
        if tokenizer is not None:
            type(self).set_tokenizer(tokenizer)
        if max_length is not None:
            self.max_length = max_length

    # ------------------------------------------------------------------ tokenizer
    @classmethod
    def set_tokenizer(cls, tok):
        cls.tokenizer = load_tokenizer(tok)

    @classmethod
    def _tok(cls, max_length):
        tok = cls.tokenizer
        if tok is None:
            raise RuntimeError("no tokenizer: call DeepImpact.set_tokenizer(path/to/tokenizer.json)")
        tok.no_padding()
        tok.enable_truncation(max_length)
        return tok

    @classmethod
    def process_query(cls, query: str) -> Set[str]:
        """xlmr_original.py:114-118."""
        tok = cls.tokenizer
        if tok is None:
            raise RuntimeError("no tokenizer set")
        return set(filter(lambda x: x not in cls.punctuation,
                          _pre_tokenize(tok, _normalize(tok, query))))

    @classmethod
    def process_document(cls, document: str, max_length: Optional[int] = None
                         ) -> Tuple[Encoding, Dict[str, int]]:
        """xlmr_original.py:120-189 (unpadded encoding)."""
        return cls.process_documents([document], max_length)[0]

    @classmethod
    def process_documents(cls, documents: Sequence[str], max_length: Optional[int] = None
                          ) -> List[Tuple[Encoding, Dict[str, int]]]:
        """Batched process_document: one multi-threaded tokenizers call."""
        ml = max_length or cls.max_length
        tok = cls._tok(ml)
        terms = [_pre_tokenize(tok, _normalize(tok, d)) for d in documents]
        wc = cls._word_cache(tok) if cls.term_mapping == "word_ids" else None
        if wc is not None:
            enc = wc.encode(terms, ml)
            if not wc.checked:  # first batch of this process: the same as encode_batch?
                wc.checked = True
                ref = tok.encode_batch(terms, is_pretokenized=True, add_special_tokens=True)
                wc.ok = all(list(e.ids) == ids and list(e.word_ids) == wids
                            for e, (ids, wids) in zip(ref, enc))
                if not wc.ok:
                    cls._wcache = None
                    enc = [(e.ids, e.word_ids) for e in ref]
            return [(Encoding(ids, wids), _filter_terms(t, _first_token_map(wids)))
                    for t, (ids, wids) in zip(terms, enc)]
        encs = tok.encode_batch(terms, is_pretokenized=True, add_special_tokens=True)
        out = []
        for t, e in zip(terms, encs):
            if cls.term_mapping == "bert_legacy":
                m = _legacy_bert_map(e.tokens)
            else:
                m = _first_token_map(e.word_ids)
            out.append((Encoding(e.ids, e.word_ids), _filter_terms(t, m)))
        return out

    _wcache = None
    _wcache_tok = None
    word_cache = os.environ.get("DI_TOKEN_CACHE", "1") != "0"

    @classmethod
    def _word_cache(cls, tok):
        """The process's per-word token cache for `tok` (None when disabled or found
        unequal to encode_batch)."""
        if not cls.word_cache:
            return None
        if cls._wcache_tok is not tok:
            cls._wcache_tok = tok
            cls._wcache = _WordCache(tok)
        return cls._wcache if cls._wcache is not None and cls._wcache.ok else None

    @staticmethod
    def compute_term_impacts(documents_term_to_token_index_map: List[Dict[str, int]],
                             outputs) -> List[List[Tuple[str, float]]]:
        """xlmr_original.py:205-225 for [B, S(,1)] per-token impacts."""
        if hasattr(outputs, "detach"):
            outputs = outputs.detach().cpu().numpy()
        imp = np.asarray(outputs)
        if imp.ndim == 3:
            imp = imp[..., 0]
        return [[(t, imp[i][tok]) for t, tok in m.items()]
                for i, m in enumerate(documents_term_to_token_index_map)]

    # ------------------------------------------------------------------ loading
    @classmethod
    def load(cls, checkpoint_path: Optional[Union[str, Path]] = None, *,
             config: Optional[EncoderConfig] = None, tokenizer_path=None,
             precision: str = "bf16x3", device: int = 0, variant: str = "xlmr",
             max_length: Optional[int] = None) -> "DeepImpact":
        """Replaces DeepImpact.load (xlmr_original.py:191-203) + .to(cuda).eval().

        checkpoint_path: a ModelCheckpoint .pt ({'model_state_dict': ...},
        checkpoint.py:72-77), or a local HF model directory (config.json +
        model.safetensors / pytorch_model.bin).  Hub names cannot be fetched
        offline."""
        sd, cfg = _load_weights(checkpoint_path, config, variant)
        enc = DeviceEncoder(sd, cfg, precision=precision, device=device)
        tok = tokenizer_path
        if tok is None and checkpoint_path is not None and Path(checkpoint_path).is_dir() and \
                (Path(checkpoint_path) / "tokenizer.json").exists():
            tok = Path(checkpoint_path) / "tokenizer.json"
        model = cls(enc, tok, max_length)
        # class-level, like the tokenizer: process_document(s) are classmethods
        cls.term_mapping = "bert_legacy" if variant == "bert" else "word_ids"
        return model

    # ------------------------------------------------------------------ forward
    def __call__(self, input_ids, attention_mask, token_type_ids=None):
        """Reference forward protocol (xlmr_original.py:41-54): padded [B, S]
        batch in, per-token impacts [B, S, 1] (float32, host) out.  Padding
        positions (which the reference never reads) are 0."""
        import torch

        ids = np.asarray(input_ids.cpu() if hasattr(input_ids, "cpu") else input_ids)
        mask = np.asarray(attention_mask.cpu() if hasattr(attention_mask, "cpu")
                          else attention_mask).astype(bool)
        lens = mask.sum(1)
        cu = np.zeros(len(lens) + 1, np.int32)
        cu[1:] = np.cumsum(lens)
        packed = ids[mask].astype(np.int32)
        tok = self.encoder.encode_packed(packed, cu, token_impacts=True)
        out = np.zeros(ids.shape, np.float32)
        out[mask] = tok
        return torch.from_numpy(out).unsqueeze(-1)

    def encode_documents(self, documents: Sequence[str], round3: bool = False,
                         max_length: Optional[int] = None) -> List[List[Tuple[str, np.float32]]]:
        """Tokenize, encode and gather a batch: per document the (term, impact)
        list of compute_term_impacts, optionally with round(impact, 3)."""
        proc = self.process_documents(documents, max_length or self.max_length)
        return self.encode_processed(proc, round3)

    @staticmethod
    def pack_processed(proc):
        """process_documents output -> the packed batch of the C ABI: token ids and
        their offsets, the kept terms (flat) with their first-token index and offsets."""
        lens = np.array([len(e.ids) for e, _ in proc], np.int64)
        cu = np.zeros(len(proc) + 1, np.int32)
        cu[1:] = np.cumsum(lens)
        ids = np.fromiter((i for e, _ in proc for i in e.ids), np.int32, count=int(cu[-1]))
        terms = [t for _, m in proc for t in m]
        tt = np.fromiter((t for _, m in proc for t in m.values()), np.int32, count=len(terms))
        ct = np.zeros(len(proc) + 1, np.int32)
        ct[1:] = np.cumsum([len(m) for _, m in proc])
        return ids, cu, terms, tt, ct

    @staticmethod
    def pack_processed_blob(proc):
        """pack_processed with the kept terms as one UTF-8 blob + byte offsets (what a
        tokenizer worker sends back: no per-term objects to unpickle)."""
        ids, cu, terms, tt, ct = DeepImpact.pack_processed(proc)
        enc = [t.encode("utf-8") for t in terms]
        term_off = np.zeros(len(enc) + 1, np.int64)
        if enc:
            term_off[1:] = np.cumsum([len(b) for b in enc])
        return ids, cu, b"".join(enc), term_off, tt, ct

    @staticmethod
    def merge_packed_blobs(parts):
        """Concatenate pack_processed_blob batches (in order) into one: the tokenizer
        workers' small chunks become one device batch (batch sizes never change the
        impacts: every row's arithmetic is independent of the other documents)."""
        if len(parts) == 1:
            return parts[0]
        ids = np.concatenate([p[0] for p in parts])
        tt = np.concatenate([p[4] for p in parts])
        cu, term_off, ct = [np.zeros(1, np.int32)], [np.zeros(1, np.int64)], [np.zeros(1, np.int32)]
        o_tok = o_byte = o_term = 0
        for p in parts:
            cu.append(p[1][1:] + np.int32(o_tok))
            term_off.append(p[3][1:] + np.int64(o_byte))
            ct.append(p[5][1:] + np.int32(o_term))
            o_tok += int(p[1][-1])
            o_byte += int(p[3][-1])
            o_term += int(p[5][-1])
        return (ids, np.concatenate(cu).astype(np.int32), b"".join(p[2] for p in parts),
                np.concatenate(term_off).astype(np.int64), tt, np.concatenate(ct).astype(np.int32))

    def encode_packed_text(self, packed) -> str:
        """A pack_processed_blob batch -> its impact-TSV lines (round3, native
        formatter), without per-term Python objects."""
        return self.encode_packed_impacts(packed)()

    def encode_packed_impacts(self, packed):
        """Encode a pack_processed_blob batch on the device now; return the formatting
        step as a callable (the native formatter, run later -- Indexer overlaps it with
        the next batch's encode)."""
        ids, cu, blob, term_off, tt, ct = packed
        imp = self.encoder.encode_packed(ids, cu, tt, ct, round3=True)
        return lambda: _lib.format_impact_lines_packed(blob, term_off, imp, ct)

    def encode_packed_terms(self, packed, round3=False):
        """Encode a pack_processed batch: per document its (term, impact) list."""
        ids, cu, terms, tt, ct = packed
        imp = self.encoder.encode_packed(ids, cu, tt, ct, round3=round3)
        return [list(zip(terms[ct[i]:ct[i + 1]], imp[ct[i]:ct[i + 1]]))
                for i in range(len(ct) - 1)]

    def encode_processed(self, proc, round3=False):
        return self.encode_packed_terms(self.pack_processed(proc), round3)

    def get_impact_scores(self, document: str) -> List[Tuple[str, np.float32]]:
        """xlmr_original.py:227-241."""
        return self.get_impact_scores_batch([document])[0]

    def get_impact_scores_batch(self, documents: List[str]) -> List[List[Tuple[str, np.float32]]]:
        """xlmr_original.py:243-267 (no rounding)."""
        return self.encode_documents(documents, round3=False)


# --------------------------------------------------------------------------- weights
def _load_weights(checkpoint_path, config, variant):
    import torch

    if checkpoint_path is None:
        raise ValueError("a checkpoint path is required (hub downloads are unavailable)")
    p = Path(checkpoint_path)
    if not p.exists():
        raise FileNotFoundError(f"{p} does not exist (hub names cannot be fetched offline)")
    if p.is_dir():
        cfg_json = p / "config.json"
        hf_cfg = json.loads(cfg_json.read_text()) if cfg_json.exists() else None
        if (p / "model.safetensors").exists():
            from safetensors.torch import load_file

            sd = load_file(str(p / "model.safetensors"))
        else:
            sd = torch.load(p / "pytorch_model.bin", map_location="cpu", weights_only=True)
        if config is None and hf_cfg is not None:
            config = EncoderConfig.from_hf(hf_cfg, variant=variant)
    else:
        ck = torch.load(p, map_location="cpu", weights_only=True)
        sd = ck["model_state_dict"] if isinstance(ck, dict) and "model_state_dict" in ck else ck
    if config is None:
        config = EncoderConfig.infer(sd, variant=variant)
    return sd, config
