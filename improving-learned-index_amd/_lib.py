"""ctypes binding of libdeepimpact_hip.so (the C ABI in include/deepimpact.h).

The HIP library is the product path: there is no CPU fallback.  If the shared
object is missing or cannot be loaded this module raises ImportError-like
errors at first use, loudly.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("DEEPIMPACT_HIP_LIB", _HERE / "libdeepimpact_hip.so"))

DI_OK = 0
DI_F_DEVICE_PTRS = 0x1
DI_F_ASYNC = 0x2
DI_F_TIMING = 0x4
DI_F_LISTS_MAJOR = 0x8
DI_SHORT_QUERY_TERMS = 256  # longer queries: wide merge keys (include/deepimpact.h)
DI_MAX_QUERY_TERMS = 4096
DI_MAX_TOPK = 4096

_ERRNAMES = {-1: "DI_EINVAL", -2: "DI_ENOMEM", -3: "DI_EHIP", -4: "DI_ERANGE",
             -5: "DI_ENODEV", -6: "DI_EIO", -7: "DI_EFORMAT"}


class DIError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class di_timing(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double), ("launches", ctypes.c_int64)]


class di_synth_skew(ctypes.Structure):
    _fields_ = [("term_rank0", ctypes.c_double), ("term_exp", ctypes.c_double),
                ("cluster_docs", ctypes.c_int32), ("cluster_sigma", ctypes.c_double),
                ("doc_sigma", ctypes.c_double), ("mass_max", ctypes.c_double)]


P = ctypes.c_void_p
I32, I64, U32, U64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64

# name -> (restype, argtypes); every symbol include/deepimpact.h declares
SIGNATURES = {
    "di_last_error": (ctypes.c_char_p, []),
    "di_version": (ctypes.c_int, []),
    "di_device_count": (ctypes.c_int, [P]),
    "di_index_create": (ctypes.c_int, [P, I64, P, P, U32, U32, ctypes.c_int, P]),
    "di_index_load_reference": (ctypes.c_int, [ctypes.c_char_p, U32, U32, ctypes.c_int, P]),
    "di_build_reference_index": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "di_index_search": (ctypes.c_int, [P, P, P, I32, I32, P, P, P, P, U32]),
    "di_index_reserve": (ctypes.c_int, [P, I32, I32]),
    "di_index_info": (ctypes.c_int, [P, P, P, P, P]),
    "di_index_set_min_impact": (ctypes.c_int, [P, I32]),
    "di_index_set_block_max": (ctypes.c_int, [P, ctypes.c_float]),
    "di_index_set_packed": (ctypes.c_int, [P, I32, P]),
    "di_index_set_stream": (ctypes.c_int, [P, P]),
    "di_index_sync": (ctypes.c_int, [P]),
    "di_index_timing": (ctypes.c_int, [P, ctypes.c_char_p, P, ctypes.c_int]),
    "di_index_destroy": (ctypes.c_int, [P]),
    "di_topk_merge": (ctypes.c_int, [P, P, I32, I32, I32, P, P, ctypes.c_int, P, U32]),
    "di_xchg_sample": (ctypes.c_int, [P, P, I32, I32, I32, P, ctypes.c_int, P]),
    "di_xchg_count": (ctypes.c_int, [P, I32, P, P, I32, I32, I32, P, ctypes.c_int, P]),
    "di_xchg_offsets": (ctypes.c_int, [P, I32, I32, P, P, ctypes.c_int, P]),
    "di_xchg_pack": (ctypes.c_int, [P, P, P, I32, I32, P, ctypes.c_int, P]),
    "di_xchg_unpack": (ctypes.c_int, [P, I64, P, P, I32, I32, I32, P, P, ctypes.c_int, P]),
    "di_encoder_create": (ctypes.c_int, [P, P, I32, ctypes.c_int, P]),
    "di_encode": (ctypes.c_int, [P, P, P, I32, I64, I32, P, P, I64, P, U32]),
    "di_encoder_reserve": (ctypes.c_int, [P, I64, I32, I64]),
    "di_encoder_set_stream": (ctypes.c_int, [P, P]),
    "di_encoder_sync": (ctypes.c_int, [P]),
    "di_encoder_timing": (ctypes.c_int, [P, ctypes.c_char_p, P, ctypes.c_int]),
    "di_encoder_destroy": (ctypes.c_int, [P]),
    "di_quantize": (ctypes.c_int, [P, I64, ctypes.c_double, I32, P, P, ctypes.c_int, P, U32]),
    "di_quantize_file": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_double, I32,
                                        ctypes.c_int, P]),
    "di_format_impact_lines": (ctypes.c_int, [P, P, P, P, I32, P, I64, P]),
    "di_append_run_lines": (ctypes.c_int, [ctypes.c_char_p, P, P, I32, P, P, P, I32]),
    "di_sparse_create": (ctypes.c_int, [P, I64, P, P, U32, ctypes.c_int, P]),
    "di_sparse_search": (ctypes.c_int, [P, P, P, I32, I32, P, P, P, P, U32]),
    "di_sparse_search_f64": (ctypes.c_int, [P, P, P, I32, I32, P, P, P, U32]),
    "di_sparse_info": (ctypes.c_int, [P, P, P, P, P]),
    "di_sparse_timing": (ctypes.c_int, [P, ctypes.c_char_p, P, ctypes.c_int]),
    "di_sparse_destroy": (ctypes.c_int, [P]),
    "di_synth_postings": (ctypes.c_int, [I64, I32, U64, I32, I32, ctypes.c_double, P, P, P, I64,
                                         P, P]),
    "di_synth_postings_skewed": (ctypes.c_int, [I64, I32, U64, I32, I32, ctypes.c_double, P, P,
                                                P, P, I64, P, P]),
    "di_synth_postings_shard": (ctypes.c_int, [I64, I64, I32, U64, I32, I32, ctypes.c_double,
                                               P, ctypes.c_double, P, P, P, I64, P, P]),
    "di_synth_impact_tsv": (ctypes.c_int, [ctypes.c_char_p, I64, I32, U64, I32, I32,
                                           ctypes.c_double, P]),
}

_LIB = None


def hip_runtimes_mapped():
    """Real paths of every libamdhip64 mapped into this process (/proc/self/maps)."""
    found = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split(maxsplit=5)
                if len(p) == 6 and "libamdhip64.so" in p[5]:
                    found.add(os.path.realpath(p[5].strip()))
    except OSError:
        pass
    return found


def _torch_lib_dir():
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return None
    return os.path.realpath(os.path.join(os.path.dirname(spec.origin), "lib"))


def _guard_hip_runtime():
    """torch bundles its own libamdhip64.so (SONAME libamdhip64.so.7, like
    /opt/rocm's this library links), and whichever loads first serves both.  So
    when torch is importable, torch's runtime must be the one mapped: import torch
    before loading the library, and refuse if a different HIP runtime is already in
    the process (an embedder that loaded /opt/rocm's first would break torch)."""
    import sys

    tdir = _torch_lib_dir()
    if tdir is None:
        return  # no torch: the library's own runtime (RUNPATH /opt/rocm) serves alone
    if "torch" not in sys.modules:
        foreign = [p for p in hip_runtimes_mapped() if not p.startswith(tdir + os.sep)]
        if foreign:
            raise RuntimeError(
                f"a HIP runtime other than torch's is already loaded ({', '.join(foreign)}); "
                f"torch ({tdir}) would bind to it. Import torch before loading any HIP "
                f"library, or before importing improving_learned_index_amd")
        import torch  # noqa: F401  (maps torch's libamdhip64 first)


def _check_one_runtime():
    rts = hip_runtimes_mapped()
    if len(rts) > 1:
        raise RuntimeError(f"two HIP runtimes are mapped into this process: {sorted(rts)}")


def lib():
    """Load the HIP library (raises if it is missing -- no fallback)."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"{LIB_PATH} is missing: the HIP extension must be built "
                f"(python -c 'import __graft_entry__; __graft_entry__.build()')")
        _guard_hip_runtime()
        L = ctypes.CDLL(str(LIB_PATH))
        _check_one_runtime()
        # (DI_LIB_ALLOW_MISSING=1: an older build for an A/B run, tools/ab_scorer.sh)
        allow_missing = os.environ.get("DI_LIB_ALLOW_MISSING") == "1"
        for name, (res, args) in SIGNATURES.items():
            if allow_missing and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(rc):
    if rc != DI_OK:
        raise DIError(rc, lib().di_last_error().decode("utf-8", "replace"))
    return rc


def ptr(a):
    """ctypes pointer of a numpy array or a torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return ctypes.c_void_p(a.ctypes.data)
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    raise TypeError(type(a))


def device_count():
    n = ctypes.c_int(0)
    check(lib().di_device_count(ctypes.byref(n)))
    return n.value


def version():
    v = lib().di_version()
    return (v >> 16, v & 0xFFFF)


def csr(queries):
    """list of term-id lists -> (uint32 terms, int32 cu)."""
    cu = np.zeros(len(queries) + 1, np.int32)
    for i, q in enumerate(queries):
        cu[i + 1] = cu[i] + len(q)
    flat = np.fromiter((t for q in queries for t in q), np.uint32, count=int(cu[-1]))
    return flat, cu


class DeviceIndex:
    """Device-resident quantized index (one shard [doc_lo, doc_hi) of doc ids)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def from_postings(cls, term_off, pdoc, pval, doc_lo=0, doc_hi=0, device=0):
        term_off = np.ascontiguousarray(term_off, np.int64)
        pdoc = np.ascontiguousarray(pdoc, np.uint32)
        pval = np.ascontiguousarray(pval, np.uint8)
        if pdoc.size == 0:
            pdoc = np.zeros(1, np.uint32)
            pval = np.zeros(1, np.uint8)
        h = ctypes.c_void_p()
        check(lib().di_index_create(ptr(term_off), len(term_off) - 1, ptr(pdoc), ptr(pval),
                                    doc_lo, doc_hi, device, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def from_reference_dir(cls, path, doc_lo=0, doc_hi=0, device=0):
        h = ctypes.c_void_p()
        check(lib().di_index_load_reference(str(path).encode(), doc_lo, doc_hi, device,
                                            ctypes.byref(h)))
        return cls(h)

    def info(self):
        nt, npo, nd, nb = I64(), I64(), U32(), I32()
        check(lib().di_index_info(self._h, ctypes.byref(nt), ctypes.byref(npo),
                                  ctypes.byref(nd), ctypes.byref(nb)))
        return {"n_terms": nt.value, "n_postings": npo.value, "n_docs": nd.value,
                "n_blocks": nb.value}

    def search_csr(self, q_terms, cu_q, k, with_keys=False, timing=False):
        q_terms = np.ascontiguousarray(q_terms, np.uint32)
        if q_terms.size == 0:
            q_terms = np.zeros(1, np.uint32)
        cu_q = np.ascontiguousarray(cu_q, np.int32)
        n_q = len(cu_q) - 1
        docs = np.zeros((max(n_q, 1), k), np.uint32)
        scores = np.zeros((max(n_q, 1), k), np.uint32)
        n = np.zeros(max(n_q, 1), np.int32)
        keys = np.zeros((max(n_q, 1), k), np.uint64) if with_keys else None
        flags = DI_F_TIMING if timing else 0
        check(lib().di_index_search(self._h, ptr(q_terms), ptr(cu_q), n_q, k, ptr(docs),
                                    ptr(scores), ptr(n), ptr(keys), flags))
        return docs[:n_q], scores[:n_q], n[:n_q], (keys[:n_q] if with_keys else None)

    def search(self, queries, k=1000):
        """queries: list of term-id lists (iteration order = tie order)."""
        flat, cu = csr(queries)
        docs, scores, n, _ = self.search_csr(flat, cu, k)
        return [list(zip(docs[i, :n[i]].tolist(), scores[i, :n[i]].tolist()))
                for i in range(len(queries))]

    def search_device(self, q_terms, cu_q, n_q, k, out_doc, out_score, out_n, out_key=None,
                      flags=DI_F_DEVICE_PTRS):
        """All pointers are device pointers (torch tensors or ints)."""
        check(lib().di_index_search(self._h, ptr(q_terms), ptr(cu_q), n_q, k, ptr(out_doc),
                                    ptr(out_score), ptr(out_n), ptr(out_key), flags))

    def reserve(self, max_q, k):
        check(lib().di_index_reserve(self._h, max_q, k))

    def set_min_impact(self, min_impact=1):
        """Score only postings with value >= 2^floor(log2 min_impact) (1 = exact)."""
        check(lib().di_index_set_min_impact(self._h, int(min_impact)))

    def set_block_max(self, factor=0.0):
        """Block-max skipping: 0 off, 1 exact, > 1 approximate (di_index_set_block_max)."""
        check(lib().di_index_set_block_max(self._h, float(factor)))

    def set_packed(self, on=True):
        """Block-compressed postings (di_index_set_packed, configs[4]); returns the packed
        size in bytes."""
        b = I64(0)
        check(lib().di_index_set_packed(self._h, int(bool(on)), ctypes.byref(b)))
        return b.value

    def set_stream(self, stream_ptr):
        check(lib().di_index_set_stream(self._h, ctypes.c_void_p(stream_ptr)))

    def sync(self):
        check(lib().di_index_sync(self._h))

    def timing(self, name, reset=False):
        t = di_timing()
        check(lib().di_index_timing(self._h, name.encode(), ctypes.byref(t), int(reset)))
        return t.ms, t.launches

    def close(self):
        if self._h:
            lib().di_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def topk_merge(keys, counts, k, device=0, stream=None, flags=0):
    """keys: [n_q, n_lists, k] uint64, counts: [n_q, n_lists] int32 (host numpy, or device
    tensors with DI_F_DEVICE_PTRS).  Returns (keys [n_q,k], n [n_q]) for host inputs."""
    if flags & DI_F_DEVICE_PTRS:
        raise ValueError("use topk_merge_device for device pointers")
    keys = np.ascontiguousarray(keys, np.uint64)
    counts = np.ascontiguousarray(counts, np.int32)
    n_q, n_lists = counts.shape
    assert keys.shape == (n_q, n_lists, k)
    out = np.zeros((max(n_q, 1), k), np.uint64)
    n = np.zeros(max(n_q, 1), np.int32)
    check(lib().di_topk_merge(ptr(keys), ptr(counts), n_q, n_lists, k, ptr(out), ptr(n),
                              device, ctypes.c_void_p(stream or 0), flags))
    return out[:n_q], n[:n_q]


def topk_merge_device(keys, counts, n_q, n_lists, k, out_key, out_n, device=0, stream=0,
                      flags=DI_F_DEVICE_PTRS):
    check(lib().di_topk_merge(ptr(keys), ptr(counts), n_q, n_lists, k, ptr(out_key),
                              ptr(out_n), device, ctypes.c_void_p(stream), flags))


def key_doc(keys, wide=False):
    """Doc of quantized-index merge keys (di_key_doc / di_key_doc_wide); wide: the
    keys of a query of more than DI_SHORT_QUERY_TERMS known terms."""
    if wide:
        return (np.uint64(0xFFFFFF) - (keys & np.uint64(0xFFFFFF))).astype(np.uint32)
    return (np.uint64(0xFFFFFFFF) - (keys & np.uint64(0xFFFFFFFF))).astype(np.uint32)


def key_score(keys, wide=False):
    return (keys >> np.uint64(44 if wide else 48)).astype(np.uint32)


def is_wide(n_terms: int) -> bool:
    """Does a query of n_terms known terms get wide merge keys?"""
    return n_terms > DI_SHORT_QUERY_TERMS


def append_run_lines(path, qids, docs, scores, counts) -> None:
    """Native RunFile.writelines over a batch (di_append_run_lines): qids (str list),
    docs / scores uint32 [n_q, k], counts [n_q] -> those queries' lines appended to path."""
    n_q = len(qids)
    if n_q == 0:
        open(path, "ab").close()
        return
    enc = [str(q).encode("utf-8") for q in qids]
    blob = b"".join(enc) + b"\0"
    off = np.zeros(n_q + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in enc])
    docs = np.ascontiguousarray(docs, np.uint32).reshape(n_q, -1)
    scores = np.ascontiguousarray(scores, np.uint32).reshape(docs.shape)
    cnt = np.ascontiguousarray(counts, np.int32)
    check(lib().di_append_run_lines(str(path).encode("utf-8"), blob, ptr(off), n_q, ptr(docs),
                                    ptr(scores), ptr(cnt), docs.shape[1]))


def format_impact_lines_packed(blob: bytes, term_off, impacts, cu_terms) -> str:
    """format_impact_lines on the packed form: the terms' UTF-8 bytes back to back
    (term_off [T+1] int64 byte offsets), their float32 impacts and the per-document
    term offsets cu_terms [n_docs+1]."""
    n_docs = len(cu_terms) - 1
    term_off = np.ascontiguousarray(term_off, np.int64)
    imp = np.ascontiguousarray(impacts, np.float32)
    if imp.size == 0:
        imp = np.zeros(1, np.float32)
    cu = np.ascontiguousarray(cu_terms, np.int64)
    n_terms = len(term_off) - 1
    cap = len(blob) + 30 * (n_terms + 1) + n_docs + 16
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64(0)
    tb = ctypes.create_string_buffer(blob, len(blob) + 1)
    check(lib().di_format_impact_lines(tb, ptr(term_off), ptr(imp), ptr(cu), n_docs, out, cap,
                                       ctypes.byref(n)))
    return out.raw[:n.value].decode("utf-8")


def format_impact_lines(doc_terms, doc_impacts):
    """Native A9 formatter: list (per doc) of term lists + float32 impact arrays
    (already rounded) -> the impact-TSV text of those docs (one line each)."""
    n_docs = len(doc_terms)
    enc = [t.encode("utf-8") for terms in doc_terms for t in terms]
    blob = b"".join(enc)
    term_off = np.zeros(len(enc) + 1, np.int64)
    if enc:
        term_off[1:] = np.cumsum([len(b) for b in enc])
    cu = np.zeros(n_docs + 1, np.int64)
    cu[1:] = np.cumsum([len(t) for t in doc_terms])
    imp = np.ascontiguousarray(np.concatenate([np.asarray(x, np.float32) for x in doc_impacts])
                               if n_docs else np.zeros(0, np.float32), np.float32)
    if imp.size == 0:
        imp = np.zeros(1, np.float32)
    cap = len(blob) + 30 * (len(enc) + 1) + n_docs + 16
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64(0)
    tb = ctypes.create_string_buffer(blob, len(blob) + 1)
    check(lib().di_format_impact_lines(tb, ptr(term_off), ptr(imp), ptr(cu), n_docs, out, cap,
                                       ctypes.byref(n)))
    return out.raw[:n.value].decode("utf-8")


class DeviceSparseIndex:
    """Device-resident float index (di_sparse_*), NanoBEIR's SparseSearch path."""

    def __init__(self, term_off, pdoc, pimp, n_docs, device=0):
        term_off = np.ascontiguousarray(term_off, np.int64)
        pdoc = np.ascontiguousarray(pdoc, np.uint32)
        pimp = np.ascontiguousarray(pimp, np.float32)
        if pdoc.size == 0:
            pdoc, pimp = np.zeros(1, np.uint32), np.zeros(1, np.float32)
        h = ctypes.c_void_p()
        check(lib().di_sparse_create(ptr(term_off), len(term_off) - 1, ptr(pdoc), ptr(pimp),
                                     n_docs, device, ctypes.byref(h)))
        self._h = h

    def search_csr(self, q_terms, cu_q, k, with_keys=False, accumulation="f32"):
        """accumulation "f32" (numpy >= 2) or "f64" (the reference's pinned numpy 1.25:
        f64 scores; no keys)."""
        q_terms = np.ascontiguousarray(q_terms, np.uint32)
        if q_terms.size == 0:
            q_terms = np.zeros(1, np.uint32)
        cu_q = np.ascontiguousarray(cu_q, np.int32)
        n_q = len(cu_q) - 1
        docs = np.zeros((max(n_q, 1), k), np.uint32)
        if accumulation == "f64":
            if with_keys:
                raise ValueError("f64 search has no 64-bit merge keys")
            scores = np.zeros((max(n_q, 1), k), np.float64)
            n = np.zeros(max(n_q, 1), np.int32)
            check(lib().di_sparse_search_f64(self._h, ptr(q_terms), ptr(cu_q), n_q, k, ptr(docs),
                                             ptr(scores), ptr(n), 0))
            return docs[:n_q], scores[:n_q], n[:n_q], None
        if accumulation != "f32":
            raise ValueError(f"accumulation must be 'f32' or 'f64', not {accumulation!r}")
        scores = np.zeros((max(n_q, 1), k), np.float32)
        n = np.zeros(max(n_q, 1), np.int32)
        keys = np.zeros((max(n_q, 1), k), np.uint64) if with_keys else None
        check(lib().di_sparse_search(self._h, ptr(q_terms), ptr(cu_q), n_q, k, ptr(docs),
                                     ptr(scores), ptr(n), ptr(keys), 0))
        return docs[:n_q], scores[:n_q], n[:n_q], (keys[:n_q] if with_keys else None)

    def search(self, queries, k, accumulation="f32"):
        flat, cu = csr(queries)
        docs, scores, n, _ = self.search_csr(flat, cu, k, accumulation=accumulation)
        return [list(zip(docs[i, :n[i]].tolist(), scores[i, :n[i]].tolist()))
                for i in range(len(queries))]

    def close(self):
        if getattr(self, "_h", None):
            lib().di_sparse_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
