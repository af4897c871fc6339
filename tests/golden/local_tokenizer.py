"""A locally constructed XLM-R-style tokenizer (test fixture builder).

The reference tokenizes with ``AutoTokenizer.from_pretrained('xlm-roberta-base')``
(src/deep_impact/models/xlmr_original.py:28), a hub download that does not
exist offline.  This module builds a small SentencePiece-Unigram tokenizer with
the same pipeline shape -- NFKC normalizer + collapse of repeated spaces,
Metaspace pre-tokenizer ('▁' prefix on every word), ``<s> $A </s>``
template, ids <s>=0 <pad>=1 </s>=2 <unk>=3 -- so the reference's term
extraction (xlmr_original.py:114-189) can be run on it and the build's host
tokenization checked against it.  The vocabulary is synthetic; the term
extraction LOGIC is what the fixtures pin.
"""
from __future__ import annotations

import json
import string

WORDS = (
    "the of and to a in is that for on with as was at by an be this are from or have "
    "it not but what all were when we there can which their if do will each about how up "
    "out them then she many some so these would other into has more her two like him see "
    "time could no make than first been its who now people my made over did down only way "
    "find use may water long little very after words called just where most know get through "
    "back much before go good new write our used me man too any day same right look think "
    "also around another came come work three word must because does part even place well "
    "such here take why things help put years different away again off went old number "
    "great tell men say small every found still between name should home big give air line "
    "set own under read last never us left end along while might next sound below saw "
    "something thought both few those always looked show large often together asked house "
    "world going want school important until form food keep children feet land side without "
    "boy once animals life enough took sometimes four head above kind began almost live page "
    "got earth need far hand high year mother light parts country father let night following "
    "picture being study second eyes soon times story boys since white days ever paper hard "
    "near sentence better best across during today others however sure means knew its try "
    "told young miles sun ways thing whole hear example heard several change answer room sea "
    "against top turned learn point city play toward five using himself usually money seen "
    "car morning body upon family later turn move face door cut done group true leave color "
    "red friends pages black within person hello ok retrieval index impact passage query "
    "document term score model learned sparse neural ranking search engine vector"
).split()

SUBWORDS = ["ing", "ed", "er", "es", "ly", "tion", "al", "ment", "ness", "re", "un", "in",
            "th", "an", "on", "en", "at", "st", "ou", "ar", "or", "le", "it", "is"]


def build_vocab():
    vocab = [("<s>", 0.0), ("<pad>", 0.0), ("</s>", 0.0), ("<unk>", 0.0)]
    seen = {v for v, _ in vocab}

    def add(piece, score):
        if piece not in seen:
            seen.add(piece)
            vocab.append((piece, score))

    for i, w in enumerate(WORDS):
        add("▁" + w, -4.0 - 0.001 * i)
        add("▁" + w.capitalize(), -6.0 - 0.001 * i)
    for i, s in enumerate(SUBWORDS):
        add(s, -7.0 - 0.01 * i)
        add("▁" + s, -7.5 - 0.01 * i)
    for c in string.ascii_letters + string.digits + string.punctuation:
        add(c, -10.0)
        add("▁" + c, -10.5)
    add("▁", -9.0)
    return vocab


def build_tokenizer():
    from tokenizers import Regex, Tokenizer, models, normalizers, pre_tokenizers, processors

    tok = Tokenizer(models.Unigram(build_vocab(), unk_id=3, byte_fallback=False))
    tok.normalizer = normalizers.Sequence(
        [normalizers.NFKC(), normalizers.Replace(Regex(" {2,}"), " ")])
    tok.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="always")
    tok.post_processor = processors.TemplateProcessing(
        single="<s> $A </s>", pair="<s> $A </s> </s> $B </s>",
        special_tokens=[("<s>", 0), ("</s>", 2)])
    return tok


def build_hf_tokenizer():
    """transformers wrapper with the attributes the reference reads."""
    from transformers import PreTrainedTokenizerFast

    ft = PreTrainedTokenizerFast(
        tokenizer_object=build_tokenizer(), bos_token="<s>", eos_token="</s>",
        pad_token="<pad>", unk_token="<unk>", cls_token="<s>", sep_token="</s>")
    return ft


def save(path):
    build_tokenizer().save(str(path))


if __name__ == "__main__":
    import sys

    save(sys.argv[1] if len(sys.argv) > 1 else "tokenizer.json")
    print(json.dumps({"vocab": len(build_vocab())}))
