"""The host float parser of the native text passes (pytext.h parse_float: Clinger's fast
path, the x87 80-bit path for 17-19-digit mantissas, strtod) against Python's float()
-- the reference's parser (quantize.py:22, :43; deep_impact_collection.py:25) -- on
random 15-19-digit decimals and on decimals within a few units of the last digit of
a midpoint between two adjacent doubles, where a double rounding would go wrong.
Compiled here with g++ (CPU only)."""
import random
import struct
import subprocess
from decimal import Decimal, getcontext

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = tmp_path_factory.mktemp("pf") / "parse_float_check"
    src = ROOT / "tests" / "native" / "parse_float_check.cpp"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), str(src)], check=True)

    def run(texts):
        out = subprocess.run([str(exe)], input="\n".join(texts) + "\n", capture_output=True,
                             text=True, check=True).stdout.split()
        assert len(out) == len(texts)
        return out

    return run


def _bits(x):
    return "%016x" % struct.unpack("<Q", struct.pack("<d", x))[0]


def test_random_long_decimals(checker):
    rng = random.Random(11)
    texts = []
    for _ in range(20000):
        nd = rng.randint(15, 19)
        digits = "".join(rng.choice("0123456789") for _ in range(nd)).lstrip("0") or "7"
        k = rng.randint(0, min(22, len(digits)))
        t = digits if k == 0 else (digits[:-k] or "0") + "." + digits[-k:]
        texts.append(t)
    got = checker(texts)
    bad = [(t, g, _bits(float(t))) for t, g in zip(texts, got) if g != _bits(float(t))]
    assert not bad, bad[:5]


def test_near_midpoint_decimals(checker):
    """Decimals at, just below and just above the exact midpoint of two adjacent doubles
    (truncated to 19 significant digits): the x87 quotient rounds to the midpoint
    pattern there, and the parser must defer to strtod."""
    getcontext().prec = 60
    rng = random.Random(5)
    texts = []
    for _ in range(3000):
        x = rng.uniform(0.001, 300.0)
        y = float.fromhex(x.hex())
        nxt = struct.unpack("<d", struct.pack("<Q", struct.unpack("<Q", struct.pack("<d", y))[0] + 1))[0]
        mid = (Decimal(y) + Decimal(nxt)) / 2
        for eps in (0, 1, -1, 3, -3):
            q = mid.quantize(Decimal(1).scaleb(mid.adjusted() - 18))  # 19 significant digits
            q += Decimal(eps).scaleb(mid.adjusted() - 18)
            t = format(q, "f")
            if len(t.split(".")[-1]) > 22 or len(t.replace(".", "").lstrip("0")) > 19:
                continue
            texts.append(t)
    assert len(texts) > 5000
    got = checker(texts)
    bad = [(t, g, _bits(float(t))) for t, g in zip(texts, got) if g != _bits(float(t))]
    assert not bad, bad[:5]


def test_rejects_what_python_rejects(checker):
    texts = ["1_000.5", "_1", "1__0", "0x1p3", "1e5", " 2.5 ", "nan", "-inf", "", "1.2.3"]
    got = checker([t if t else " " for t in texts])
    for t, g in zip(texts, got):
        try:
            want = _bits(float(t)) if t.strip() else "ERR"
        except ValueError:
            want = "ERR"
        if want != "ERR" and t.strip().lower() == "nan":
            assert g != "ERR"
            continue
        assert g == want, (t, g, want)
