"""GPU deflate (LZ77 match-find + Huffman emission)
through the C-ABI.

Bar, levels 1..9 (deflate_fast 1..3, deflate_slow 4..9; level 6 is
Z_DEFAULT_COMPRESSION): the GPU writes zlib's bytes -- the exact stream host
zlib 1.2.11 writes for deflateInit2(level, Z_DEFLATED, window_bits, 8,
Z_DEFAULT_STRATEGY) + deflate(Z_FINISH), which SURVEY.md §8c pins as
byte-identical to the reference's shipped deflate.  Every stream also
inflates back through the CPU oracle and host zlib.

Level 0 (deflate_stored): zlib's bytes too, with or without ZS_F_DEFLATE_FAST.

ZS_F_DEFLATE_FAST (the throughput path, any level): every GPU stream is
valid deflate that the oracle and host zlib inflate to the input, with
Z_STREAM_END, the whole stream consumed, the wrapper bytes and check value as
zlib writes them; its size is bounded against zlib at the same level.
"""
import ctypes
import random
import zlib

import numpy as np
import pytest

import corpus
import libz_ref
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zs():
    import zstreams
    zstreams.lib()
    return zstreams


def expected_check(data, wbits):
    if wbits > 15:
        return zlib.crc32(data)
    if wbits > 0:
        return zlib.adler32(data)
    return 1  # raw: strm->adler keeps adler32(0) (deflateResetKeep)


def zlib_bytes(data, wbits, level):
    """Host zlib's bytes for one deflate(Z_FINISH) with room for the whole output
    (the batch API's call).  Level 0 needs exactly that call: deflate_stored
    sizes its blocks by the output space each deflate() call offers (Python's
    compressobj grows its buffer call by call, giving other block lengths);
    levels 1..9 write the same bytes under any output schedule."""
    if level == 0:
        d = libz_ref.Deflater(0, wbits)
        r, used, out = d.call(data, len(data) + 5 * (len(data) // 65535 + 1) + 64, 4)
        d.end()
        assert r == 1 and used == len(data), (r, used, len(data))
        return out
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, 8, zlib.Z_DEFAULT_STRATEGY)
    return c.compress(data) + c.flush()


def check_stream(data, wbits, level, comp, info, fast=False):
    assert info["ret"] == 1, info
    if level == 0 or (1 <= level <= 9 and not fast):
        ref = zlib_bytes(data, wbits, level)
        assert comp == ref, ("not zlib's bytes", len(data), wbits, level, len(comp), len(ref))
    assert info["total_in"] == len(data) and info["total_out"] == len(comp), info
    assert info["adler"] == expected_check(data, wbits), info
    # zlib turns deflate windowBits 8 into 9 and writes CINFO 1, which an
    # inflateInit2(8) rejects ("invalid window size"): inflate those with 9
    iw = 9 if wbits == 8 else wbits
    out, oi = O.oneshot(comp, iw, max(len(data), 1) + 1024)
    assert oi["ret"] == 1 and oi["total_in"] == len(comp) and out == data, (len(data), wbits, level, oi)
    assert zlib.decompress(comp, iw) == data
    # wrapper header as host zlib writes it for the same parameters
    if wbits > 0:
        c = zlib.compressobj(level, zlib.DEFLATED, wbits)
        ref = c.compress(b"") + c.flush(zlib.Z_SYNC_FLUSH)
        hl = 10 if wbits > 15 else 2
        assert comp[:hl] == ref[:hl], (comp[:hl], ref[:hl])


def _patterns(rng):
    text = corpus.stream(1, 300000)
    lines = corpus.stream(33, 300000)
    rnd = bytes(rng.getrandbits(8) for _ in range(70000))
    return {
        "text": text, "lines": lines, "random": rnd, "zeros": bytes(200000),
        "abc": b"abc" * 70000, "mixed": text[:50000] + rnd[:30000] + bytes(40000) + lines[:50000],
    }


SIZES = [0, 1, 2, 3, 4, 5, 17, 258, 259, 4095, 32768, 65535, 65536, 65537, 131079, 200000]


def test_deflate_small_all_wrappers_levels(zs):
    rng = random.Random(3)
    pats = _patterns(rng)
    cases = []
    for name, p in pats.items():
        for n in SIZES:
            if n > len(p):
                continue
            for wb in (-15, 15, 31):
                for lv in (0, 1, 6, 9):
                    cases.append((p[:n], wb, lv))
    rng.shuffle(cases)
    got = zs.deflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    for (data, wb, lv), (comp, info) in zip(cases, got):
        check_stream(data, wb, lv, comp, info)


def test_deflate_window_bits_and_levels(zs):
    data = corpus.stream(5, 150000)
    cases = [(data, wb, lv) for wb in (-9, -12, 9, 8, 13, 25, 28) for lv in (-1, 2, 3, 4, 5, 7, 8)]
    got = zs.deflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    for (d, wb, lv), (comp, info) in zip(cases, got):
        check_stream(d, wb, 6 if lv == -1 else lv, comp, info)


def test_deflate_invalid_parameters(zs):
    data = b"hello hello hello"
    bad = [(-8, 6), (24, 6), (7, 6), (16, 6), (32, 6), (-17, 6), (15, 10), (15, -2)]
    got = zs.deflate_batch([data] * len(bad), [b[0] for b in bad], [b[1] for b in bad], [64] * len(bad))
    for b, (comp, info) in zip(bad, got):
        assert info["ret"] == -2 and comp == b"", (b, info)


def test_deflate_small_out_cap(zs):
    data = corpus.stream(7, 100000)
    full, _ = zs.deflate_batch([data], 31, 6)[0]
    part, info = zs.deflate_batch([data], 31, 6, [1000])[0]
    assert info["ret"] == 0 and info["total_out"] == 1000 and part == full[:1000]


def test_deflate_zlib_bytes_levels_1_to_9(zs):
    """Every deflate_fast (1..3) and deflate_slow (4..9) level, every wrapper,
    the corpora and edge sizes: byte-identical to host zlib (long matches,
    stored blocks, block ends at 16383 symbols, the empty final block, windows
    below 32 KiB; zero runs and short periods, where deflate_fast's skipped
    insertions shape every later chain)."""
    rng = random.Random(11)
    pats = _patterns(rng)
    cases = []
    for name, p in pats.items():
        for n in (0, 1, 3, 300, 16383, 16384, 65536, 70000, 200000):
            if n <= len(p):
                for lv in range(1, 10):
                    cases.append((p[:n], rng.choice((-15, 15, 31)), lv))
    # all-literal stretches whose symbol count ends exactly on a block boundary
    for extra in (-2, -1, 0, 1, 2):
        rnd = bytes(rng.getrandbits(8) for _ in range(2 * 16383 + extra))
        cases.append((rnd, -15, 6))
        cases.append((rnd, 15, 1))
    for wb in (-9, -10, -13, 9, 12, 25, 29):
        cases.append((pats["text"][:150000], wb, 6))
        cases.append((pats["lines"][:150000], wb, 2))
    got = zs.deflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    bad = [(i, len(d), wb, lv) for i, ((d, wb, lv), (comp, info)) in enumerate(zip(cases, got))
           if comp != zlib_bytes(d, wb, lv) or info["ret"] != 1]
    assert not bad, bad[:8]


@pytest.mark.parametrize("mode", ["demand", "none", "all"])
def test_deflate_slow_search_modes_are_zlibs(zs, monkeypatch, mode):
    """deflate_slow (levels 4..9) under each search kernel, forced on inputs of
    every size (ZS_ZD_MATCH): "demand" = zs_zd_msearch_kernel (walks of the
    parse from every 16th position, searches only where a walk asks; large
    jobs take it by default), "none" = no search kernel (every longest_match
    runs on demand in the parse from global memory: zd_search_g, the path a
    parse takes where the walks did not search), "all" = zs_zd_match_kernel
    (every position, both budgets).  Byte-identical to host zlib: the
    patterns and sizes around the 16 Ki search items and their 512-position
    extension, every level 4..9 (each chain budget, good / lazy / nice), the
    three wrappers, windowBits below 15 (a shorter MAX_DIST)."""
    monkeypatch.setenv("ZS_ZD_MATCH", mode)
    rng = random.Random(23)
    pats = _patterns(rng)
    # (every search of "none" is one thread's serial chain walk in global
    # memory: short inputs, the short-budget levels)
    sizes = (1, 300, 4000, 16384 + 513) if mode == "none" else \
        (1, 300, 16383, 16384 + 511, 16384 + 513, 3 * 16384 + 5, 200000)
    levels = (4, 5, 6) if mode == "none" else range(4, 10)
    cases = []
    for name, p in pats.items():
        for n in sizes:
            if n <= len(p):
                for lv in levels:
                    cases.append((p[:n], rng.choice((-15, 15, 31)), lv))
    for wb in (-9, -12, 13):
        cases.append((pats["text"][:20000 if mode == "none" else 100000], wb, 6))
        cases.append((pats["lines"][:20000 if mode == "none" else 100000], wb, 4 if mode == "none" else 9))
    got = zs.deflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    bad = [(i, len(d), wb, lv) for i, ((d, wb, lv), (comp, info)) in enumerate(zip(cases, got))
           if comp != zlib_bytes(d, wb, lv) or info["ret"] != 1]
    assert not bad, bad[:8]


def test_deflate_level0_is_zlibs(zs):
    """Level 0: zlib's deflate_stored blocks of 65535 bytes from the stream start,
    across the 64 KiB segment grid (the final block starting one segment early
    at 2 x 65535), every wrapper, with and without ZS_F_DEFLATE_FAST."""
    rng = random.Random(12)
    data = bytes(rng.getrandbits(8) for _ in range(5 * 65536 + 11))
    sizes = [0, 1, 65534, 65535, 65536, 65537, 2 * 65535, 2 * 65535 + 1, 2 * 65536, 3 * 65535 + 7,
             4 * 65536 - 3, 5 * 65535, 5 * 65536 + 11]
    cases = [(data[:n], wb) for n in sizes for wb in (-15, 15, 31)]
    for fast in (False, True):
        got = zs.deflate_batch([c[0] for c in cases], [c[1] for c in cases], 0, fast=fast)
        for (d, wb), (comp, info) in zip(cases, got):
            assert comp == zlib_bytes(d, wb, 0), (len(d), wb, fast, len(comp))
            check_stream(d, wb, 0, comp, info)


def test_deflate_zlib_bytes_large_c3_shape(zs):
    """configs[2] shape at 16 MiB per stream: gzip L6, one Zipf-text and one
    line-text stream, byte-identical to host zlib (window slides, thousands of
    blocks), and inflated back by the GPU."""
    datas = [corpus.stream(0, 16 << 20), corpus.stream(32, 16 << 20)]
    got = zs.deflate_batch(datas, 31, 6)
    for d, (comp, info) in zip(datas, got):
        assert info["ret"] == 1 and info["adler"] == zlib.crc32(d)
        assert comp == zlib_bytes(d, 31, 6)
    back = zs.inflate_batch([g[0] for g in got], 31, [len(d) for d in datas])
    for d, (out, info) in zip(datas, back):
        assert info["ret"] == 1 and out == d


def test_deflate_large_corpus_ratio_and_gpu_roundtrip(zs):
    """C3 shape at reduced size, fast mode (ZS_F_DEFLATE_FAST): gzip L6 GPU
    compress -> oracle + GPU inflate, size within 25% of zlib L6."""
    raws, _ = corpus.batch(0, 4, 8 << 20, compress=False)
    raws += corpus.batch(32, 2, 8 << 20, compress=False)[0]
    datas = [r.tobytes() for r in raws]
    got = zs.deflate_batch(datas, 31, 6, fast=True)
    comps = [g[0] for g in got]
    for d, (comp, info) in zip(datas, got):
        assert info["ret"] == 1 and info["adler"] == zlib.crc32(d)
        out, oi = O.oneshot(comp, 31, len(d) + 1024)
        assert oi["ret"] == 1 and out == d
        zl = len(zlib.compress(d, 6))
        # quality bar: within 25% of zlib L6 on these corpora
        assert len(comp) <= 1.25 * zl, (len(comp), zl)
    back = zs.inflate_batch(comps, 31, [len(d) for d in datas])
    for d, (out, info) in zip(datas, back):
        assert info["ret"] == 1 and info["adler"] == zlib.crc32(d) and out == d


def test_deflate_deterministic(zs):
    data = corpus.stream(9, 1 << 20)
    for fast in (False, True):
        a = zs.deflate_batch([data] * 3, -15, 6, fast=fast)
        assert a[0][0] == a[1][0] == a[2][0]


def test_deflate_fast_mode_all_levels(zs):
    """ZS_F_DEFLATE_FAST at every level: valid streams (property bar)."""
    rng = random.Random(5)
    pats = _patterns(rng)
    cases = [(p[:n], wb, lv) for p in pats.values() for n in (0, 5, 65537, 200000) if n <= len(p)
             for wb in (-15, 31) for lv in (1, 3, 4, 6, 9)]
    got = zs.deflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases], fast=True)
    for (d, wb, lv), (comp, info) in zip(cases, got):
        check_stream(d, wb, lv, comp, info, fast=True)


def test_compression_stream_js_schedule(zs):
    """CompressionStreamZlib (handle ABI, JS write schedule) == batch output,
    and the stream round-trips through DecompressionStreamZlib."""
    data = corpus.stream(40, 300000)
    for fmt, wb in (("deflate-raw", -15), ("deflate", 15), ("gzip", 31)):
        for level in (-1, 1, 9):
            ref, _ = zs.deflate_batch([data], wb, level)[0]
            for w in (4096, 65536):
                got = zs.compress(data, fmt, level, w)
                assert got == ref, (fmt, level, w)
            assert zs.decompress(ref, fmt, 4096) == data
    # empty input: flush alone gives a complete stream
    assert zlib.decompress(zs.compress(b"", "gzip"), 31) == b""
    # the reference's round-trip test shape: 24 000 random bytes, 4096-B writes
    rnd = bytes(random.Random(1).getrandbits(8) for _ in range(24000))
    assert zs.decompress(zs.compress(rnd, "deflate", -1, 4096), "deflate", 4096) == rnd


def test_zlib_abi_deflate_loop(zs):
    """deflateInit2_ / deflate / deflateEnd / deflateBound over the library's
    zlib ABI with a small output buffer (Z_FINISH, served in pieces)."""
    import libz_ref
    Z = libz_ref.ZStream
    L = ctypes.CDLL(zs.LIB_PATH)
    L.deflateInit2_.argtypes = [ctypes.POINTER(Z), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.deflate.argtypes = [ctypes.POINTER(Z), ctypes.c_int]
    L.deflateEnd.argtypes = [ctypes.POINTER(Z)]
    L.deflateBound.argtypes = [ctypes.POINTER(Z), ctypes.c_ulong]
    L.deflateBound.restype = ctypes.c_ulong
    sz = ctypes.sizeof(Z)
    s = Z()
    assert L.deflateInit2_(ctypes.byref(s), 6, 8, 15, 8, 0, b"2.0", sz) == -6  # Z_VERSION_ERROR
    for bad in ((6, 9, 15, 8, 0), (6, 8, -8, 8, 0), (6, 8, 15, 0, 0), (6, 8, 15, 8, 5), (10, 8, 15, 8, 0)):
        assert L.deflateInit2_(ctypes.byref(s), *bad, b"1.2.11", sz) == -2, bad
    data = corpus.stream(12, 500000)
    for wb in (-15, 15, 31):
        ref, _ = zs.deflate_batch([data], wb, 6)[0]
        s = Z()
        assert L.deflateInit2_(ctypes.byref(s), 6, 8, wb, 8, 0, b"1.2.11", sz) == 0
        assert L.deflateBound(ctypes.byref(s), len(data)) >= len(ref)
        ib = ctypes.create_string_buffer(data, len(data))
        ob = ctypes.create_string_buffer(7000)
        s.next_in = ctypes.cast(ib, ctypes.c_void_p)
        s.avail_in = len(data)
        out = bytearray()
        ret = 0
        while ret == 0:
            s.next_out = ctypes.cast(ob, ctypes.c_void_p)
            s.avail_out = len(ob)
            ret = L.deflate(ctypes.byref(s), 4)
            out += ob.raw[:len(ob) - s.avail_out]
        assert ret == 1 and bytes(out) == ref
        assert s.total_in == len(data) and s.total_out == len(ref) and s.adler == expected_check(data, wb)
        assert L.deflateEnd(ctypes.byref(s)) == 0


def test_deflate_device_pointers(zs):
    import torch
    data = corpus.stream(20, 3 << 20)
    ref, _ = zs.deflate_batch([data], -15, 6)[0]
    src = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    cap = zs.deflate_bound(len(data), -15)
    dst = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    info = zs.deflate_batch_device([src.data_ptr()], [len(data)], [dst.data_ptr()], [cap], -15, 6)[0]
    assert info["ret"] == 1 and dst[:info["total_out"]].cpu().numpy().tobytes() == ref


class _GpuDeflate:
    """deflateInit2_ / deflate / deflateEnd through the library's zlib ABI."""

    def __init__(self, zs, level, wb):
        import libz_ref
        self.Z = libz_ref.ZStream
        L = self.L = ctypes.CDLL(zs.LIB_PATH)
        L.deflateInit2_.argtypes = [ctypes.POINTER(self.Z), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.deflate.argtypes = [ctypes.POINTER(self.Z), ctypes.c_int]
        L.deflateEnd.argtypes = [ctypes.POINTER(self.Z)]
        self.s = self.Z()
        assert L.deflateInit2_(ctypes.byref(self.s), level, 8, wb, 8, 0, b"1.2.11", ctypes.sizeof(self.Z)) == 0
        self.ob = ctypes.create_string_buffer(5000)

    def call(self, data, flush):
        """One deflate() with `data`, then the same flush again while the output
        buffer comes back full (zlib's calling convention); returns (bytes, last ret)."""
        ib = ctypes.create_string_buffer(data, max(len(data), 1))
        s = self.s
        s.next_in = ctypes.cast(ib, ctypes.c_void_p)
        s.avail_in = len(data)
        out = bytearray()
        while True:
            s.next_out = ctypes.cast(self.ob, ctypes.c_void_p)
            s.avail_out = len(self.ob)
            ret = self.L.deflate(ctypes.byref(s), flush)
            out += self.ob.raw[:len(self.ob) - s.avail_out]
            if ret != 0 or s.avail_out != 0:
                return bytes(out), ret

    def call1(self, data, out_len, flush):
        """Exactly one deflate() call: (ret, consumed, produced bytes)."""
        ib = ctypes.create_string_buffer(data, max(len(data), 1))
        ob = ctypes.create_string_buffer(max(out_len, 1))
        s = self.s
        s.next_in = ctypes.cast(ib, ctypes.c_void_p) if data else None
        s.avail_in = len(data)
        s.next_out = ctypes.cast(ob, ctypes.c_void_p)
        s.avail_out = out_len
        ret = self.L.deflate(ctypes.byref(s), flush)
        return ret, len(data) - s.avail_in, ob.raw[:out_len - s.avail_out]

    def end(self):
        return self.L.deflateEnd(ctypes.byref(self.s))


def test_deflate_flush_points(zs):
    """Z_SYNC_FLUSH / Z_FULL_FLUSH / Z_PARTIAL_FLUSH / Z_BLOCK mid-stream: after
    every flush the output so far decodes (host zlib, streaming) to exactly the
    input so far; the finished stream decodes to the input with its trailer
    checked (the oracle and host zlib).  zlib.h: deflate() flush semantics."""
    rng = random.Random(7)
    data = corpus.stream(14, 1500000)
    for wb in (-15, 15, 31):
        for level in (1, 6, 9):
            g = _GpuDeflate(zs, level, wb)
            d = zlib.decompressobj(wb)
            out, got, off = bytearray(), bytearray(), 0
            while off < len(data):
                n = rng.choice([1, 100, 5000, 70000, 300000])
                chunk = data[off:off + n]
                off += len(chunk)
                fl = rng.choice([0, 0, 2, 3, 1, 5])  # NO_FLUSH, SYNC, FULL, PARTIAL, BLOCK
                o, ret = g.call(chunk, fl)
                assert ret == 0, (wb, level, fl, ret)
                out += o
                got += d.decompress(o)
                if fl:
                    assert bytes(got) == data[:off], (wb, level, fl, off, len(got))
            o, ret = g.call(b"", 4)
            assert ret == 1
            out += o
            assert g.s.adler == expected_check(data, wb) and g.s.total_in == len(data) and g.s.total_out == len(out)
            assert g.end() == 0
            eo, ei = O.oneshot(bytes(out), wb, len(data) + 64)
            assert ei["ret"] == 1 and eo == data and ei["total_in"] == len(out), (wb, level, ei)
            assert zlib.decompress(bytes(out), wb) == data


def test_deflate_sync_flush_is_zlibs(zs):
    """NO_FLUSH ... Z_SYNC_FLUSH, then Z_FINISH: zlib's exact bytes (levels 4..9:
    the sync flush ends the last block with BFINAL = 0 and no empty block, then
    the empty stored block; deflate.c deflate_slow / deflate()); a repeated
    flush with no input makes no progress (Z_BUF_ERROR)."""
    data = corpus.stream(15, 700000)
    for wb in (-15, 15, 31):
        for level in (1, 6, 9):
            c = zlib.compressobj(level, zlib.DEFLATED, wb, 8, zlib.Z_DEFAULT_STRATEGY)
            ref_sync = c.compress(data) + c.flush(zlib.Z_SYNC_FLUSH)
            ref_end = c.flush(zlib.Z_FINISH)
            g = _GpuDeflate(zs, level, wb)
            o1, r1 = g.call(data, 2)
            assert r1 == 0 and o1 == ref_sync, (wb, level, len(o1), len(ref_sync))
            o2, r2 = g.call(b"", 2)
            assert r2 == -5 and o2 == b""  # Z_BUF_ERROR
            o3, r3 = g.call(b"", 4)
            assert r3 == 1 and o3 == ref_end, (wb, level, o3.hex(), ref_end.hex())
            assert g.end() == 0


def test_deflate_stream_buffer_bound_fast_levels(zs, monkeypatch):
    """Level 0 in a stream (the throughput encoder's stored blocks): past
    ZS_DSTREAM_MAX_KB of gathered input a stream sends its blocks without
    waiting for a flush (a non-final block end, no injected flush marker), and
    still decodes to the input."""
    monkeypatch.setenv("ZS_DSTREAM_MAX_KB", "256")
    data = corpus.stream(16, 2 << 20)
    for wb in (-15, 31):
        g = _GpuDeflate(zs, 0, wb)
        out, early = bytearray(), 0
        for off in range(0, len(data), 65536):
            o, ret = g.call(data[off:off + 65536], 0)
            assert ret == 0
            out += o
            early += len(o)
        o, ret = g.call(b"", 4)
        assert ret == 1
        out += o
        assert early > 0 and g.end() == 0
        assert zlib.decompress(bytes(out), wb) == data


def _stream_data(rng, n):
    """Text, line text, random bytes and zero runs, mixed."""
    parts, k = [], 0
    while sum(len(p) for p in parts) < n:
        kind = rng.random()
        m = rng.choice([3000, 40000, 200000])
        if kind < 0.4:
            parts.append(corpus.stream(rng.randrange(64), m))
        elif kind < 0.6:
            parts.append(bytes(rng.getrandbits(8) for _ in range(min(m, 20000))))
        elif kind < 0.8:
            parts.append(bytes(m))
        else:
            parts.append(corpus.stream(32 + k % 32, m))
        k += 1
    return b"".join(parts)[:n]


def _compare_calls(zs, level, wb, calls, out_len):
    """Drive the library's deflate() and host zlib's with the same calls;
    every call's (ret, consumed, produced bytes) must be equal."""
    import libz_ref
    g = _GpuDeflate(zs, level, wb)
    h = libz_ref.Deflater(level, wb)
    assert h.rc == 0
    total = bytearray()
    for i, (chunk, fl) in enumerate(calls):
        a = g.call1(chunk, out_len, fl)
        b = h.call(chunk, out_len, fl)
        assert a == b, (level, wb, i, fl, len(chunk), a[:2], b[:2], len(a[2]), len(b[2]))
        # strm->adler after every call: zlib's read_buf checks each byte it reads
        assert g.s.adler == h.s.adler & 0xffffffff, (level, wb, i, g.s.adler, h.s.adler)
        total += a[2]
    assert g.s.adler == h.s.adler & 0xffffffff
    assert g.end() == h.end()
    return bytes(total)


@pytest.mark.parametrize("level", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_deflate_stream_calls_are_zlibs(zs, level):
    """zlib's deflate() call by call (reference: src/wasm/deflate_stream_wasm.c:51-55
    runs one deflate per process call): random input sizes and every flush value
    -- Z_NO_FLUSH (blocks sent as zlib completes them, nothing injected),
    Z_PARTIAL_FLUSH, Z_SYNC_FLUSH, Z_FULL_FLUSH, Z_BLOCK (the window carried
    across all but Z_FULL_FLUSH, bits continuing across unaligned ends) -- then
    Z_FINISH and its drain: each call's ret, consumed and produced bytes equal
    host zlib's, for raw, zlib and gzip streams."""
    rng = random.Random(100 + level)
    for wb in (-15, 15, 31):
        # deflate_fast (1..3) is serial per stream on the GPU: a smaller stream
        data = _stream_data(rng, 1_500_000 if level >= 4 else 400_000)
        calls, off = [], 0
        while off < len(data):
            n = rng.choice([1, 700, 5000, 33000, 70000, 250000])
            fl = rng.choice([0, 0, 0, 0, 1, 2, 3, 5])
            calls.append((data[off:off + n], fl))
            off += n
        calls.append((b"", rng.choice([0, 2])))  # nothing to do: Z_BUF_ERROR
        calls += [(b"", 4)] * 3
        out = _compare_calls(zs, level, wb, calls, 1 << 21)
        assert zlib.decompress(out, wb) == data


@pytest.mark.parametrize("mode", ["demand", "none"])
def test_deflate_stream_calls_search_modes_are_zlibs(zs, monkeypatch, mode):
    """The stream segments' searches under the demand-driven kernel and the
    on-demand global search (ZS_ZD_MATCH; by default segments take the
    all-positions kernel): a segment's parse starts at its entry (a loop top
    past the carried window, in deflate_slow's state there), where the
    walks start too.  Every call's ret, consumed and produced bytes equal host
    zlib's, levels 4 and 6, every flush value, raw and gzip."""
    monkeypatch.setenv("ZS_ZD_MATCH", mode)
    rng = random.Random(300 + (mode == "none"))
    for level, wb in ((4, -15), (6, 31)):
        data = _stream_data(rng, 600_000 if mode == "demand" else 120_000)
        calls, off = [], 0
        while off < len(data):
            n = rng.choice([1, 700, 5000, 33000, 70000])
            fl = rng.choice([0, 0, 0, 1, 2, 3, 5])
            calls.append((data[off:off + n], fl))
            off += n
        calls += [(b"", 4)] * 2
        out = _compare_calls(zs, level, wb, calls, 1 << 21)
        assert zlib.decompress(out, wb) == data


def test_deflate_stream_long_no_flush_is_zlibs(zs):
    """A 64 MiB stream fed in 1 MiB Z_NO_FLUSH calls, then Z_FINISH drained in
    64 KiB pieces: every call equals host zlib's (blocks sent as they complete,
    never a flush the caller did not ask for)."""
    data = corpus.stream(3, 32 << 20) + corpus.stream(40, 32 << 20)
    calls = [(data[o:o + (1 << 20)], 0) for o in range(0, len(data), 1 << 20)]
    calls += [(b"", 4)] * 400
    for level, wb in ((6, 31), (9, -15)):
        out = _compare_calls(zs, level, wb, calls, 1 << 22)
        assert zlib.decompress(out, wb) == data


def test_deflate_small_buffer_flush_loops_are_zlibs(zs):
    """zlib's calling convention with little output space: each segment's
    deflate(flush) is repeated with the unconsumed input while it returns with
    avail_out == 0.  The concatenated output equals host zlib's driven the same
    way -- including the repeated flush markers zlib writes when a flush call
    runs out of space right at its marker (zlib.h, deflate())."""
    import libz_ref
    rng = random.Random(77)
    data = _stream_data(rng, 900_000)
    for level, wb in ((6, -15), (9, 31), (4, 15), (1, -15), (3, 31)):
        segs, off = [], 0
        while off < len(data):
            n = rng.choice([5000, 40000, 120000])
            segs.append((data[off:off + n], rng.choice([0, 1, 2, 3, 5])))
            off += n
        segs.append((b"", 4))
        outs = []
        for drv in ("gpu", "zlib"):
            d = _GpuDeflate(zs, level, wb) if drv == "gpu" else libz_ref.Deflater(level, wb)
            call = d.call1 if drv == "gpu" else d.call
            out = bytearray()
            for chunk, fl in segs:
                rest = chunk
                k = 0
                while True:
                    space = (5, 7, 3000)[min(k, 2)] if fl else 3000
                    ret, cons, prod = call(rest, space, fl)
                    out += prod
                    rest = rest[cons:]
                    k += 1
                    if ret == 1 or ret < 0 or (len(prod) < space and not rest):
                        break
            assert d.end() == 0
            outs.append(bytes(out))
        assert outs[0] == outs[1], (level, wb, len(outs[0]), len(outs[1]))
        assert zlib.decompress(outs[0], wb) == data


def test_compression_stream_js_schedule_calls_are_zlibs(zs):
    """The reference's CompressionStreamZlib schedule (zlib-streams.js:64-156: 64 KiB
    writes, <= 32 KiB per deflate_process, 64 KiB out, Z_FINISH drain) through the
    handle ABI: every call's packed return and last_consumed equal what host
    zlib's deflate returns for the same call."""
    import libz_ref
    L = zs.lib()
    data = corpus.stream(41, 1_200_000) + bytes(100000) + corpus.stream(5, 300000)
    for fmt, wb, init in (("deflate-raw", -15, L.deflate_init_raw), ("gzip", 31, L.deflate_init_gzip),
                          ("deflate", 15, L.deflate_init)):
        for level in (1, 4, 6, 9):
            h = L.deflate_new()
            assert init(h, level) == 0
            ref = libz_ref.Deflater(level, wb)
            ob = ctypes.create_string_buffer(65536)
            got, exp = bytearray(), bytearray()
            for w in range(0, len(data), 65536):
                chunk = data[w:w + 65536]
                off = 0
                while off < len(chunk):
                    piece = chunk[off:off + 32768]
                    ib = ctypes.create_string_buffer(piece, len(piece))
                    r = L.deflate_process(h, ctypes.addressof(ib), len(piece), ctypes.addressof(ob), 65536, 0)
                    rr, cons, prod = ref.call(piece, 65536, 0)
                    assert (r >> 24, r & 0xffffff, L.deflate_last_consumed(h)) == (rr & 0xff, len(prod), cons), (fmt, level, w)
                    got += ob.raw[:r & 0xffffff]
                    exp += prod
                    if cons == 0:
                        break
                    off += cons
            while True:
                r = L.deflate_process(h, 0, 0, ctypes.addressof(ob), 65536, 4)
                rr, cons, prod = ref.call(b"", 65536, 4)
                assert (r >> 24, r & 0xffffff) == (rr & 0xff, len(prod)), (fmt, level)
                got += ob.raw[:r & 0xffffff]
                exp += prod
                if (r >> 24) == 1 or (r & 0xffffff) == 0:
                    break
            assert got == exp and zlib.decompress(bytes(got), wb) == data
            assert L.deflate_end(h) == ref.end() == 0


def test_deflate_init_rejects_unimplemented_parameters(zs):
    """memLevel != 8 and strategies other than Z_DEFAULT_STRATEGY would change
    zlib's bytes: deflateInit2_ refuses them (Z_STREAM_ERROR) instead of
    silently writing default-parameter bytes; an unfinished stream ends with
    Z_DATA_ERROR as zlib's deflateEnd says."""
    import libz_ref
    Z = libz_ref.ZStream
    L = ctypes.CDLL(zs.LIB_PATH)
    L.deflateInit2_.argtypes = [ctypes.POINTER(Z), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.deflateEnd.argtypes = [ctypes.POINTER(Z)]
    for mem, strat in ((9, 0), (1, 0), (8, 1), (8, 2), (8, 3), (8, 4)):
        s = Z()
        assert L.deflateInit2_(ctypes.byref(s), 6, 8, 15, mem, strat, b"1.2.11", ctypes.sizeof(Z)) == -2, (mem, strat)
    g = _GpuDeflate(zs, 6, 31)
    g.call1(b"abc" * 1000, 1 << 16, 0)
    assert g.end() == -3  # Z_DATA_ERROR: stream freed before Z_FINISH


def test_deflate_fixup_in_order_pass(zs, monkeypatch):
    """ZS_ZD_ROUNDS=0 skips the parallel cross-region fix-up rounds, so every
    job's regions are settled by the in-order pass (zs_zd_fix_seq_kernel):
    zlib's bytes at every deflate_slow level (4..9) on text, periodic runs (whose
    parse offsets never line up across 64 KiB regions), zeros and mixed inputs,
    under the demand-driven search the final build runs."""
    monkeypatch.setenv("ZS_ZD_ROUNDS", "0")
    rng = random.Random(21)
    pats = _patterns(rng)
    per = bytes(rng.getrandbits(8) for _ in range(1000)) * 1200  # period 1000, 1.2 MB
    datas = (pats["text"], pats["mixed"], bytes(1 << 20), per, b"ab" * 400000)
    cases = [(d, wb, lv) for d in datas for wb, lv in ((-15, 4), (31, 5), (15, 6), (-15, 7), (31, 8), (15, 9))]
    got = zs.deflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    bad = [(i, len(d), wb, lv) for i, ((d, wb, lv), (comp, info)) in enumerate(zip(cases, got))
           if comp != zlib_bytes(d, wb, lv) or info["ret"] != 1]
    assert not bad, bad


def test_deflate_long_zero_run_is_zlibs(zs):
    """300 MiB of zeros (> 4 096 regions of 64 KiB: the cascade a bounded number
    of parallel fix-up rounds cannot settle) and a 300 MiB period-777 run, at
    level 4 raw and level 9 gzip: zlib's bytes (deflate.c deflate_slow; trees.c
    block flushes), with the demand-driven search of the final build."""
    zeros = bytes(300 << 20)
    unit = bytes(random.Random(5).getrandbits(8) for _ in range(777))
    per = (unit * ((300 << 20) // 777 + 1))[:300 << 20]
    for data in (zeros, per):
        for wb, lv in ((-15, 4), (31, 9)):
            (comp, info), = zs.deflate_batch([data], wb, lv)
            ref = zlib_bytes(data, wb, lv)
            assert info["ret"] == 1 and comp == ref, (len(data), wb, lv, len(comp), len(ref))


# ---------------------------------------------------------------------------
# level 0 (deflate_stored) through the stream surfaces, call by call, and the
# reference's own stream drivers with their output-buffer schedules
# ---------------------------------------------------------------------------
class _GpuHandle:
    """One reference handle (deflate_* or inflate_* of the handle ABI): call() is
    one *_process with the packed return unpacked, like wasm_stream_common.c."""

    def __init__(self, zs, compress, wb, level=-1):
        L = self.L = zs.lib()
        p = "deflate_" if compress else "inflate_"
        init = {-15: "init_raw", 15: "init", 31: "init_gzip"}[wb]
        self.proc, self.cons, self.endf = (getattr(L, p + "process"), getattr(L, p + "last_consumed"),
                                           getattr(L, p + "end"))
        self.h = getattr(L, p + "new")()
        assert (getattr(L, p + init)(self.h, level) if compress else getattr(L, p + init)(self.h)) == 0

    def call(self, data, out_len, flush):
        ib = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
        ob = ctypes.create_string_buffer(max(out_len, 1))
        r = self.proc(self.h, ctypes.addressof(ib) if data else 0, len(data), ctypes.addressof(ob), out_len, flush)
        r &= 0xffffffff
        code = (r >> 24) & 0xff
        return (code - 256 if code & 0x80 else code), self.cons(self.h), ob.raw[:r & 0xffffff]

    def end(self):
        return self.endf(self.h)


class _HostDeflateHandle:
    """Host zlib behind the reference's glue (deflate_stream_wasm.c:51-55)."""

    def __init__(self, wb, level=-1):
        import libz_ref
        self.d = libz_ref.Deflater(6 if level < 0 else level, wb)

    def call(self, data, out_len, flush):
        r, cons, prod = self.d.call(data, out_len, flush)
        return (r & 0xff) - 256 if (r & 0xff) & 0x80 else r & 0xff, cons, prod

    def end(self):
        return self.d.end()


def _js_compress(h, data, out_buffer, write=65536):
    """CompressionStreamZlib (zlib-streams.js:64-141) over one handle: writes of
    `write` bytes, <= 32 KiB per process(flush 0) with an out_buffer-byte output
    buffer, advance by last_consumed, stop a write on 0; flush() calls
    process(Z_FINISH) until code 1 or nothing produced.  Returns the trace of
    (code, consumed, produced bytes) per call."""
    tr = []
    for w in range(0, len(data), write):
        chunk = data[w:w + write]
        off = 0
        while off < len(chunk):
            r = h.call(chunk[off:off + 32768], out_buffer, 0)
            tr.append(r)
            if r[1] == 0:
                break
            off += r[1]
    while True:
        r = h.call(b"", out_buffer, 4)
        tr.append(r)
        if r[0] == 1 or not r[2]:
            break
    return tr


def test_deflate_level0_stream_calls_are_zlibs(zs):
    """Level 0 through deflate() call by call: zlib's deflate_stored sizes its
    blocks from each call's output space and flush and from its window (direct
    blocks of >= min_block, the window and pending-buffer path for small calls,
    slides, Z_FULL_FLUSH restarts); random input sizes, output spaces from 7
    bytes to 2 MiB, every flush value, raw / zlib / gzip: every call's (ret,
    consumed, produced bytes) and strm->adler equal host zlib's."""
    import libz_ref
    rng = random.Random(500)
    for wb in (-15, 15, 31):
        data = _stream_data(rng, 700_000)
        g = _GpuDeflate(zs, 0, wb)
        h = libz_ref.Deflater(0, wb)
        off, k, out = 0, 0, bytearray()
        while True:
            fin = off >= len(data)
            n = 0 if fin else rng.choice([1, 100, 700, 5000, 33000, 70000, 250000])
            chunk = data[off:off + n]
            fl = 4 if fin else rng.choice([0, 0, 0, 1, 2, 3, 5])
            rest = chunk
            while True:
                space = rng.choice([7, 100, 1024, 4096, 40000, 65536, 1 << 21])
                a = g.call1(rest, space, fl)
                b = h.call(rest, space, fl)
                assert a == b, (wb, k, fl, len(rest), space, a[:2], b[:2], len(a[2]), len(b[2]))
                assert g.s.adler == h.s.adler & 0xffffffff, (wb, k)
                k += 1
                out += a[2]
                rest = rest[a[1]:]
                if a[0] != 0 or (not rest and len(a[2]) < space and fl != 4):
                    break
                assert k < 200000
            off += n
            if fin:
                assert a[0] == 1, a[:2]
                break
        assert g.end() == h.end()
        assert zlib.decompress(bytes(out), wb) == data


@pytest.mark.parametrize("out_buffer", [1024, 4096, 65536])
def test_compression_stream_level0_js_schedule_is_zlibs(zs, out_buffer):
    """CompressionStreamZlib(fmt, {level: 0, outBuffer}) (zlib-streams.js:16-17,
    64-141): the level reaches deflateInit2 (deflate_stream_wasm.c:22-49), so every
    deflate_process returns what host zlib's deflate_stored returns for the same
    call, for outBuffer 1 / 4 / 64 KiB and every wrapper."""
    data = corpus.stream(41, 300_000) + bytes(70000) + bytes(random.Random(3).getrandbits(8) for _ in range(50000))
    for wb in (-15, 15, 31):
        a = _js_compress(_GpuHandle(zs, True, wb, 0), data, out_buffer)
        b = _js_compress(_HostDeflateHandle(wb, 0), data, out_buffer)
        assert [t[:2] + (len(t[2]),) for t in a] == [t[:2] + (len(t[2]),) for t in b], (wb, out_buffer)
        assert a == b
        # (with a small outBuffer the wrapper's write loop stops on a call that only
        # drains pending output -- consumed 0, zlib-streams.js:96-99 -- and the rest
        # of that write never reaches deflate, in the reference as here)
        if out_buffer == 65536:
            assert zlib.decompress(b"".join(t[2] for t in a), wb) == data


def _roundtrip_inputs():
    """The reference's round-trip inputs (test/ref-data/roundtrip_inputs), input3
    as the Makefile rewrites it before the runs (Makefile:276: deflateRawSync of
    24000 'x' bytes, node's zlib at its default level)."""
    import os
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref-data", "roundtrip_inputs")
    ins = [open(os.path.join(d, n), "rb").read() for n in ("roundtrip_input.txt", "roundtrip_input1.txt",
                                                             "roundtrip_input3.bin")]
    c = zlib.compressobj(-1, zlib.DEFLATED, -15)
    ins.append(c.compress(b"x" * 24000) + c.flush())
    return ins


def _ref_roundtrip_driver(dfl, inf, data):
    """test_round_trip_stream.js:64-140 over a deflate and an inflate handle: deflate
    <= 32 KiB per call (Z_FINISH once the input is used) into a rolling 64 KiB
    output window (space = 65536 - position), every produced chunk fed at once to
    inflate (its own rolling window, Z_FINISH on the deflater's last chunk), then
    the inflater drained.  Returns the call trace and the inflated bytes."""
    W = 65536
    tr, out = [], bytearray()
    off, cpos, dpos = 0, 0, 0
    ddone = idone = False
    while not (ddone and idone):
        if not ddone:
            avail = len(data) - off
            fl = 4 if avail == 0 else 0
            code, cons, prod = dfl.call(data[off:off + min(avail, 32768)], W - cpos, fl)
            tr.append(("d", code, cons, prod))
            comp = prod
            while comp and not idone:
                ifl = 4 if (code == 1 and len(data) - off - cons == 0) else 0
                c2, cons2, p2 = inf.call(comp, W - dpos, ifl)
                tr.append(("i", c2, cons2, p2))
                assert c2 >= 0, tr[-1][:3]
                out += p2
                comp = comp[cons2:]
                dpos = 0 if len(p2) == W - dpos else dpos + len(p2)
                if c2 == 1:
                    idone = True
                    break
                if cons2 == 0:
                    break
            off += cons
            cpos = 0 if len(prod) == W - cpos else cpos + len(prod)
            if code == 1:
                ddone = True
        if ddone and not idone:
            c2, cons2, p2 = inf.call(b"", W - dpos, 4)
            tr.append(("i", c2, cons2, p2))
            out += p2
            dpos = 0 if len(p2) == W - dpos else dpos + len(p2)
            if c2 == 1 or (cons2 == 0 and not p2):
                idone = c2 == 1
                if not idone:
                    break
    return tr, bytes(out)


class _OracleInflateHandle:
    def __init__(self, wb):
        self.s = O.Stream(wb)

    def call(self, data, out_len, flush):
        r = self.s.call(data, out_len, flush)
        return r["ret"], r["consumed"], r["out"]


@pytest.mark.parametrize("level", [-1, 0, 1, 6, 9])
def test_reference_roundtrip_inputs_through_streams(zs, level):
    """The reference's round-trip runner (test_round_trip_stream.js) on its committed
    inputs and the Makefile's deflateRaw(24000 x 'x'), zlib wrapper: GPU deflate
    handle -> GPU inflate handle with the runner's rolling output windows; every
    call equals host zlib deflate -> oracle inflate driven the same way, and the
    output is the input.  Plus CompressionStreamZlib -> DecompressionStreamZlib
    (zlib-streams.js) at outBuffer 1 KiB on each input, bytes equal to host zlib's."""
    for data in _roundtrip_inputs():
        a_tr, a_out = _ref_roundtrip_driver(_GpuHandle(zs, True, 15, level), _GpuHandle(zs, False, 15), data)
        b_tr, b_out = _ref_roundtrip_driver(_HostDeflateHandle(15, level), _OracleInflateHandle(15), data)
        assert a_tr == b_tr and a_out == b_out == data, (len(data), level)
        for wb in (-15, 31):
            a = _js_compress(_GpuHandle(zs, True, wb, level), data, 1024)
            b = _js_compress(_HostDeflateHandle(wb, level), data, 1024)
            assert a == b, (len(data), level, wb)
            comp = b"".join(t[2] for t in a)
            assert zs.decompress(comp, {-15: "deflate-raw", 31: "gzip"}[wb], 1024) == data


@pytest.mark.parametrize("out_buffer", [1024, 4096])
def test_compression_stream_small_out_buffer_calls_are_zlibs(zs, out_buffer):
    """CompressionStreamZlib with outBuffer 1 / 4 KiB (zlib-streams.js:17, passed to
    every deflate_process, :83 / :122): blocks larger than the output space leave
    zlib's pending output for later calls, a call that only drains it consumes
    nothing (and the wrapper's write loop stops on 0), Z_FINISH drains in
    outBuffer pieces; every call's (code, consumed, produced bytes) equals host
    zlib's, levels 1 / 4 / 6 / 9, raw / zlib / gzip."""
    data = corpus.stream(42, 500_000) + bytes(random.Random(4).getrandbits(8) for _ in range(60000))
    for level in (1, 4, 6, 9):
        for wb in (-15, 15, 31):
            a = _js_compress(_GpuHandle(zs, True, wb, level), data, out_buffer)
            b = _js_compress(_HostDeflateHandle(wb, level), data, out_buffer)
            assert [t[:2] + (len(t[2]),) for t in a] == [t[:2] + (len(t[2]),) for t in b], (level, wb, out_buffer)
            assert a == b


@pytest.mark.parametrize("level", [1, 3, 4, 6, 9])
def test_deflate_output_full_consumed_is_zlibs(zs, level):
    """zlib's pull-on-demand: deflate() returns right after the block flush that
    fills avail_out, having read only what fill_window had read by then
    (deflate.c deflate_slow / deflate_fast, FLUSH_BLOCK, fill_window).  Calls
    with large inputs (100 KB .. 1.2 MB) and small output spaces (1 .. 40 KB),
    the caller passing the unconsumed rest again (zlib's calling convention),
    every flush value, raw / zlib / gzip; plus a header that does not fit (out
    1 byte): every call's (ret, consumed, produced bytes) and strm->adler equal
    host zlib's."""
    import libz_ref
    rng = random.Random(700 + level)
    for wb in (-15, 15, 31):
        data = _stream_data(rng, 2_500_000 if level >= 4 else 900_000)
        g = _GpuDeflate(zs, level, wb)
        h = libz_ref.Deflater(level, wb)
        off, k, out = 0, 0, bytearray()
        first = True
        while True:
            fin = off >= len(data)
            n = 0 if fin else rng.choice([100_000, 300_000, 1_200_000])
            chunk = data[off:off + n]
            fl = 4 if fin else rng.choice([0, 0, 0, 2, 1, 5, 3])
            rest = chunk
            while True:
                space = 1 if first else rng.choice([1000, 5000, 17000, 40000])
                first = False
                a = g.call1(rest, space, fl)
                b = h.call(rest, space, fl)
                assert a == b, (wb, k, fl, len(rest), space, a[:2], b[:2], len(a[2]), len(b[2]))
                assert g.s.adler == h.s.adler & 0xffffffff, (wb, k)
                k += 1
                out += a[2]
                rest = rest[a[1]:]
                if a[0] != 0 or (not rest and len(a[2]) < space and fl != 4):
                    break
                assert k < 100000
            off += n
            if fin:
                assert a[0] == 1, a[:2]
                break
        assert g.end() == h.end()
        assert zlib.decompress(bytes(out), wb) == data


@pytest.mark.parametrize("level", [1, 2, 3])
def test_deflate_fast_flush_then_tiny_calls_are_zlibs(zs, level):
    """deflate_fast after a flush leaves its last MIN_MATCH - 1 positions to the
    next fill_window (deflate.c s->insert), which inserts them only while
    lookahead + insert >= MIN_MATCH: a sync / partial / full flush, then 1- and
    2-byte calls (Z_NO_FLUSH and flushing), then more input, several times over;
    every call's (ret, consumed, produced bytes) and strm->adler equal host
    zlib's, raw / zlib / gzip."""
    rng = random.Random(900 + level)
    text = corpus.stream(33, 400_000)
    for wb in (-15, 15, 31):
        calls, off = [], 0
        while off < len(text):
            n = rng.choice([3000, 20000, 70000])
            calls.append((text[off:off + n], rng.choice([2, 1, 3])))
            off += n
            for _ in range(rng.randint(1, 3)):
                m = rng.choice([1, 2])
                calls.append((text[off:off + m], rng.choice([0, 0, 2, 1])))
                off += m
        calls += [(b"", 4)] * 2
        out = _compare_calls(zs, level, wb, calls, 1 << 20)
        assert zlib.decompress(out, wb) == text
