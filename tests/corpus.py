"""Deterministic synthetic corpora, via tests/tools/libzs_corpus.so.

* stream i % 64 < 32 : Zipf text (5 000-word vocabulary, 1/(rank+1)), ratio ~3 at L6
* stream i % 64 >= 32: ``line-%08d\\n`` records, ratio ~6 at L6
Compression is host zlib L6 / memLevel 8 / default strategy (byte-identical to
the reference's shipped deflate).  Test and bench infrastructure only.
"""
import ctypes
import os
import subprocess

import numpy as np

TOOLS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools")
SO = os.path.join(TOOLS, "libzs_corpus.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            subprocess.run(["make", "-s", "-C", TOOLS], check=True)
        L = ctypes.CDLL(SO)
        L.zs_corpus_stream.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.zs_corpus_zipf.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
        L.zs_corpus_lines.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
        L.zs_corpus_bound.restype = ctypes.c_size_t
        L.zs_corpus_bound.argtypes = [ctypes.c_size_t]
        L.zs_corpus_deflate.restype = ctypes.c_size_t
        L.zs_corpus_deflate.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_int, ctypes.c_int]
        L.zs_corpus_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_size_t)]
        _lib = L
    return _lib


def stream(i, nbytes):
    buf = np.empty(nbytes, dtype=np.uint8)
    lib().zs_corpus_stream(buf.ctypes.data, nbytes, i)
    return buf.tobytes()


def batch(first, count, nbytes, level=6, wbits=-15, nthreads=8, compress=True):
    """Returns (raw: list[np.ndarray], comp: list[np.ndarray] or None)."""
    L = lib()
    raw = [np.empty(nbytes, dtype=np.uint8) for _ in range(count)]
    rp = (ctypes.c_void_p * count)(*[r.ctypes.data for r in raw])
    comp = None
    cp = None
    cl = (ctypes.c_size_t * count)()
    if compress:
        bound = L.zs_corpus_bound(nbytes)
        comp = [np.empty(bound, dtype=np.uint8) for _ in range(count)]
        cp = (ctypes.c_void_p * count)(*[c.ctypes.data for c in comp])
    L.zs_corpus_batch(first, count, nbytes, level, wbits, nthreads, rp, cp, cl)
    if compress:
        comp = [comp[k][:cl[k]] for k in range(count)]
    return raw, comp


def zipf_text(nbytes, i=0):
    return stream(i % 32, nbytes)


def lines_text(nbytes, i=32):
    return stream(32 + i % 32, nbytes)


def c5_stream(k, nbytes):
    """configs[4] stream k: Zipf text (seed 5000 + k) when
    k % 4 < 2, else line text starting at record k << 20; raw deflate (-15)
    when k is even, gzip (31) when odd.  Returns (raw ndarray, window_bits)."""
    buf = np.empty(nbytes, dtype=np.uint8)
    if k % 4 < 2:
        lib().zs_corpus_zipf(buf.ctypes.data, nbytes, 5000 + k)
    else:
        lib().zs_corpus_lines(buf.ctypes.data, nbytes, k << 20)
    return buf, (-15 if k % 2 == 0 else 31)
