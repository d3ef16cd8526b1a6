"""The CPU stage model of the GPU's zlib-identical deflate (tests/tools/dz_model.c)
against host zlib 1.2.11, byte for byte: hash chains -> per-position longest
match under zlib's chain budgets -> deflate_slow's lazy parse -> 16383-symbol
blocks flushed as trees.c does.  Pins the decomposition the HIP kernels of
deflate_zlib.hip implement."""
import ctypes
import os
import random
import subprocess
import zlib

import corpus

TOOLS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools")


def _lib():
    so = os.path.join(TOOLS, "libdz_model.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", TOOLS], check=True)
    L = ctypes.CDLL(so)
    L.dz_model_deflate.restype = ctypes.c_size_t
    L.dz_model_deflate.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_size_t]
    return L


def model(data, level, wbits=15):
    cap = 2 * len(data) + 1024
    buf = ctypes.create_string_buffer(cap)
    n = _lib().dz_model_deflate(data, len(data), level, wbits, buf, cap)
    return buf.raw[:n]


def zlib_raw(data, level, wbits=15):
    c = zlib.compressobj(level, zlib.DEFLATED, -wbits, 8, zlib.Z_DEFAULT_STRATEGY)
    return c.compress(data) + c.flush()


def test_model_small_and_edges():
    """deflate_fast (1..3, serial) and deflate_slow (4..9, stage model)."""
    rng = random.Random(1)
    cases = [b"", b"a", b"ab", b"abc", b"abcabcabc", b"hello hello hello world", bytes(100000),
             bytes(rng.getrandbits(8) for _ in range(70000))]
    for extra in (-1, 0, 1):  # all-literal input ending on a block boundary
        cases.append(bytes(rng.getrandbits(8) for _ in range(16383 + extra)))
    for d in cases:
        for lv in range(1, 10):
            assert model(d, lv) == zlib_raw(d, lv), (len(d), lv)


def test_model_corpora_and_windows():
    rng = random.Random(2)
    zipf = corpus.stream(0, 1 << 20)
    lines = corpus.stream(33, 1 << 20)
    mixed = bytes(rng.getrandbits(8) for _ in range(40000)) + corpus.stream(2, 300000)
    for d in (zipf, lines, mixed):
        for lv in (1, 3, 4, 6, 7):
            assert model(d, lv) == zlib_raw(d, lv)
    for wb in (9, 12, 14):
        assert model(mixed, 6, wb) == zlib_raw(mixed, 6, wb)
        assert model(mixed, 2, wb) == zlib_raw(mixed, 2, wb)
