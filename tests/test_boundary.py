"""The C-ABI boundary: libdeepimpact_hip.so loads and exports every entry point
include/deepimpact.h declares (no compute calls -- runs without a GPU), and the
native host-side builders are byte-identical to the reference (CPU only)."""
import ctypes
import re
import tempfile
from pathlib import Path

import pytest

from conftest import GOLDEN, ROOT


def declared_symbols():
    text = (ROOT / "include" / "deepimpact.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set()
    for m in re.finditer(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(di_[a-z0-9_]+)\s*\(", text,
                         re.M):
        names.add(m.group(1))
    inline = set(re.findall(r"static inline [a-z0-9_]+ (di_[a-z0-9_]+)\(", text))
    return sorted(names - inline)


def test_library_exports_every_declared_symbol():
    from improving_learned_index_amd import _lib

    syms = declared_symbols()
    assert len(syms) >= 10
    L = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # and the ctypes binding covers exactly the declared set
    assert sorted(_lib.SIGNATURES) == syms


def test_library_reports_no_device_cleanly_or_counts():
    from improving_learned_index_amd import _lib

    n = _lib.device_count()
    assert n >= 0
    assert _lib.version() >= (0, 1)


@pytest.mark.parametrize("src,dirname", [("collection.quantized", "index"),
                                         ("ties.quantized", "index_ties")])
def test_native_index_builder_is_byte_identical(src, dirname):
    from improving_learned_index_amd.inverted_index import InvertedIndexCreator

    with tempfile.TemporaryDirectory() as td:
        InvertedIndexCreator(GOLDEN / src, td).run()
        for f in ("vocab.txt", "inverted_index.idx", "inverted_index.dat"):
            assert (Path(td) / f).read_bytes() == (GOLDEN / dirname / f).read_bytes(), f


def test_native_index_builder_rejects_what_the_reference_rejects():
    from improving_learned_index_amd import _lib
    from improving_learned_index_amd.inverted_index import create_index

    with tempfile.TemporaryDirectory() as td:
        bad = Path(td) / "bad.tsv"
        bad.write_text("▁a: 1: 2\n")
        with pytest.raises(_lib.DIError) as e:
            create_index(bad, Path(td) / "out")
        assert e.value.code == -7
        bad.write_text("▁a: 300\n")  # struct.pack('B', 300) fails in the reference
        with pytest.raises(_lib.DIError):
            create_index(bad, Path(td) / "out")
