"""GPU parity: libzstreams_mi355x (HIP, gfx950) vs the CPU oracle, through the C-ABI.

Bar: bit-exact output and identical (ret, msg, total_in, total_out, adler) for
every job -- the fields of one zlib inflate(Z_FINISH) call.
"""
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys
import zlib

import pytest

import corpus
import oracle_lib as O
from golden.make_manifest import fixture, mutate

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
MAN = json.load(open(os.path.join(HERE, "golden", "manifest.json")))


@pytest.fixture(scope="module")
def zs():
    import zstreams
    zstreams.lib()
    return zstreams


def run_and_compare(zs, cases, parse=None):
    """cases: list of (data, wbits, cap).  One GPU batch; every job vs the oracle."""
    streams = [c[0] for c in cases]
    wbs = [c[1] for c in cases]
    caps = [c[2] for c in cases]
    got = zs.inflate_batch(streams, wbs, caps, parse=parse)
    bad = []
    for i, (c, (out, info)) in enumerate(zip(cases, got)):
        eo, ei = O.oneshot(c[0], c[1], c[2])
        if out != eo or info != ei:
            bad.append((i, c[1], c[2], len(c[0]), info, ei, len(out), len(eo)))
    assert not bad, f"{len(bad)}/{len(cases)} mismatches, first: {bad[:4]}"


def test_fixtures_deflate64(zs):
    names = sorted(MAN["fixtures"])
    got = zs.inflate_batch([fixture(n) for n in names], -16, [1 << 22] * len(names))
    for n, (out, info) in zip(names, got):
        m = MAN["fixtures"][n]
        assert info["ret"] == 1 and info["total_in"] == m["total_in"], (n, info)
        assert hashlib.sha256(out).hexdigest() == m["sha256"], n


def test_crafted_and_known_errors(zs):
    cases = [(bytes.fromhex(c["hex"]), c["wbits"], 1 << 16) for c in MAN["crafted"]]
    for e in MAN["fixture_errors"]:
        how = tuple(e["mutate"]) if e["mutate"] else None
        cases.append((mutate(fixture(e["fixture"]), how), e["wbits"], 1 << 22))
    run_and_compare(zs, cases)
    got = zs.inflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    for c, (out, info) in zip(MAN["crafted"], got):
        for k, v in c["expect"].items():
            assert (hashlib.sha256(out).hexdigest() if k == "sha256" else info[k]) == v, (c["name"], k)


def _random_streams(rng, n):
    cases = []
    for _ in range(n):
        kind = rng.random()
        size = rng.choice([0, 1, 100, 3000, 40000, 200000])
        if kind < 0.5:
            raw = corpus.stream(rng.randrange(64), size)
        elif kind < 0.7:
            raw = bytes(rng.getrandbits(8) for _ in range(min(size, 5000)))
        else:
            raw = bytes([rng.randrange(4)]) * size
        wb = rng.choice([-15, 15, 31, -9, 9 + 16, 47 - 32 + 32])
        if wb == 47:
            wb_enc = rng.choice([15, 31])
        else:
            wb_enc = wb
        c = zlib.compressobj(rng.choice([0, 1, 6, 9]), zlib.DEFLATED, wb_enc, rng.choice([1, 8, 9]),
                             rng.choice([0, 0, 1, 2, 3, 4]))
        comp = c.compress(raw) + c.flush()
        cases.append((comp, wb, len(raw) + 64))
    return cases


def test_valid_streams_all_wrappers(zs):
    run_and_compare(zs, _random_streams(random.Random(1), 300))


def test_corrupt_truncated_and_small_buffers(zs):
    rng = random.Random(2)
    base = _random_streams(rng, 400)
    cases = []
    for comp, wb, cap in base:
        b = bytearray(comp)
        r = rng.random()
        if r < 0.45 and b:
            for _ in range(rng.randint(1, 4)):
                i = rng.randrange(len(b))
                b[i] ^= 1 << rng.randrange(8)
        elif r < 0.7 and b:
            b = b[:rng.randrange(len(b))]
        elif r < 0.85:
            cap = rng.randint(0, cap)
        else:
            b += bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 10)))
        cases.append((bytes(b), wb if rng.random() < 0.9 else rng.choice([-15, 15, 31, 47, -16]), cap))
    run_and_compare(zs, cases)


def test_large_streams_roundtrip(zs):
    raws, comps = corpus.batch(30, 4, 6 << 20, level=6, wbits=-15, nthreads=4)
    got = zs.inflate_batch([c.tobytes() for c in comps], -15, [6 << 20] * 4)
    for r, c, (out, info) in zip(raws, comps, got):
        assert info["ret"] == 1 and info["total_in"] == len(c) and info["total_out"] == len(r)
        assert out == r.tobytes()


def test_gzip_zlib_checks_large(zs):
    raw = corpus.stream(3, 3 << 20)
    gz = zlib.compressobj(6, zlib.DEFLATED, 31)
    g = gz.compress(raw) + gz.flush()
    z = zlib.compress(raw, 6)
    got = zs.inflate_batch([g, z], [31, 15], [len(raw)] * 2)
    assert got[0][0] == raw and got[0][1]["ret"] == 1 and got[0][1]["adler"] == zlib.crc32(raw)
    assert got[1][0] == raw and got[1][1]["ret"] == 1 and got[1][1]["adler"] == zlib.adler32(raw)


def test_stream_api_js_schedule(zs):
    """DecompressionStreamZlib (handle ABI) output == oracle output under the
    reference's JS write schedule."""
    for name in ("100k_lines", "zeros_100k", "10k_lines"):
        data = fixture(name)
        for w in (1000, 4096, 65536):
            tr, out = zs.js_schedule(data, "deflate64-raw", w)
            etr, eo = O.js_schedule(data, w, -16)
            assert (tr, out) == (etr, eo), (name, w)
            if " -" not in etr:  # no negative code: the mirror's TransformStream completes
                assert zs.decompress(data, "deflate64-raw", w) == eo, (name, w)
    raw = corpus.stream(40, 300000)
    for fmt, wb in (("deflate-raw", -15), ("deflate", 15), ("gzip", 31)):
        c = zlib.compressobj(6, zlib.DEFLATED, wb)
        comp = c.compress(raw) + c.flush()
        assert zs.decompress(comp, fmt, 4096) == raw, fmt


def test_zlib_abi_payload_decompress_loop(zs):
    """test/payload_decompress.c:148-178 loop over the library's zlib ABI."""
    import libz_ref
    L = ctypes.CDLL(zs.LIB_PATH)
    L.inflateInit2_.argtypes = [ctypes.POINTER(libz_ref.ZStream), ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.inflate.argtypes = [ctypes.POINTER(libz_ref.ZStream), ctypes.c_int]
    L.inflateEnd.argtypes = [ctypes.POINTER(libz_ref.ZStream)]
    for name in ("10k_lines", "100k_lines"):
        data = fixture(name)
        s = libz_ref.ZStream()
        ib = ctypes.create_string_buffer(data, len(data))
        win = ctypes.create_string_buffer(65536)
        assert L.inflateInit2_(ctypes.byref(s), -16, b"1.2.11", ctypes.sizeof(libz_ref.ZStream)) == 0
        s.next_in = ctypes.cast(ib, ctypes.c_void_p)
        s.avail_in = len(data)
        s.next_out = ctypes.cast(win, ctypes.c_void_p)
        s.avail_out = 65536
        out = bytearray()
        ret = 0
        while ret == 0:
            before = s.avail_out
            ret = L.inflate(ctypes.byref(s), 4 if s.avail_in == 0 else 0)
            out += win.raw[:before - s.avail_out]
            if ret == 0:
                assert s.avail_out == 0
                s.next_out = ctypes.cast(win, ctypes.c_void_p)
                s.avail_out = 65536
        assert ret == 1 and L.inflateEnd(ctypes.byref(s)) == 0
        assert hashlib.sha256(bytes(out)).hexdigest() == MAN["fixtures"][name]["sha256"]


# ---------------------------------------------------------------------------
# speculative chunked path (streams >= 4 chunks of compressed data)
# ---------------------------------------------------------------------------
def _big_cases(rng, n, lo=1 << 20, hi=6 << 20):
    cases = []
    for i in range(n):
        size = rng.randint(lo, hi)
        raw = corpus.stream(rng.randrange(64), size)
        wb = rng.choice([-15, -15, 15, 31])
        c = zlib.compressobj(rng.choice([1, 6, 6, 9]), zlib.DEFLATED, wb, 8, rng.choice([0, 0, 0, 1]))
        cases.append((raw, c.compress(raw) + c.flush(), wb))
    return cases


@pytest.mark.parametrize("parse", ["lane", "wave", "split"])
def test_chunked_path_exact_and_taken(zs, parse):
    """Every parse mode of the block-parallel path (a lane per decode unit, a
    wave per unit, the split parse) takes every stream and gives the same exact
    results."""
    cases = _big_cases(random.Random(5), 8)
    got = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], [len(c[0]) for c in cases], parse=parse)
    st = zs.last_stats()
    assert st["chunked_jobs"] == len(cases), st
    for (raw, comp, wb), (out, info) in zip(cases, got):
        assert info["ret"] == 1 and info["total_in"] == len(comp) and out == raw, (wb, info)
    # text streams at the default strategy must not need the serial fallback
    assert st["fallback_jobs"] == 0, st


@pytest.mark.parametrize("parse", ["lane", "wave", "split"])
def test_chunked_path_errors_match_oracle(zs, parse):
    rng = random.Random(6)
    base = _big_cases(rng, 6, 600 << 10, 2 << 20)
    cases = []
    for raw, comp, wb in base:
        b = bytearray(comp)
        r = rng.random()
        if r < 0.4:
            i = rng.randrange(len(b) // 2, len(b))
            b[i] ^= 1 << rng.randrange(8)
        elif r < 0.7:
            b = b[:rng.randrange(len(b) // 2, len(b))]
        cap = len(raw) if rng.random() < 0.7 else rng.randint(len(raw) // 2, len(raw))
        cases.append((bytes(b), wb, cap))
    run_and_compare(zs, cases, parse)


@pytest.mark.parametrize("parse", [None, "split"])
def test_chunked_random_and_stored(zs, parse):
    """Random bytes and text at levels 0 / 1 / 6: stored first blocks are split
    parse leftovers (zs_unitw_list_kernel), the rest walks and splits."""
    rng = random.Random(7)
    raw = bytes(rng.getrandbits(8) for _ in range(1 << 20)) + corpus.stream(5, 1 << 20)
    comps = []
    for lvl in (0, 1, 6):
        c = zlib.compressobj(lvl, zlib.DEFLATED, -15)
        comps.append(c.compress(raw) + c.flush())
    got = zs.inflate_batch(comps, -15, [len(raw)] * 3, parse=parse)
    for (out, info), comp in zip(got, comps):
        assert info["ret"] == 1 and info["total_in"] == len(comp) and out == raw


def test_chunked_no_capacity_guess(zs):
    """Blocks far more compressible than their stream (random bytes, then line
    text): unit storage is never sized from the stream's ratio (token pages,
    exact entry placement), so the chain holds on the first and only pass."""
    import numpy as np
    rng = np.random.default_rng(11)
    raw = rng.integers(0, 256, 4 << 20, dtype=np.uint8).tobytes() + corpus.stream(41, 4 << 20)
    streams = []
    for wb in (-15, 31):
        c = zlib.compressobj(6, zlib.DEFLATED, wb)
        streams.append(c.compress(raw) + c.flush())
    got = zs.inflate_batch(streams, [-15, 31], [len(raw)] * 2)
    st = zs.last_stats()
    for (out, info), comp in zip(got, streams):
        assert info["ret"] == 1 and info["total_in"] == len(comp) and out == raw
    assert st["chunked_jobs"] == 2 and st["fallback_jobs"] == 0, st


def test_chunked_overprovisioned_out_cap(zs):
    """A caller that over-provisions out_cap (64x the output) still takes the
    chunked path with no fallback: nothing on it depends on out_cap / in_len."""
    raw = corpus.stream(7, 6 << 20)
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = c.compress(raw) + c.flush()
    got = zs.inflate_batch([comp], -15, [64 * len(raw)])
    st = zs.last_stats()
    assert got[0][0] == raw and got[0][1]["ret"] == 1 and got[0][1]["total_in"] == len(comp)
    assert st["chunked_jobs"] == 1 and st["fallback_jobs"] == 0, st


@pytest.mark.parametrize("parse", [None, "split"])
def test_chunked_fixed_strategy_16mib(zs, parse):
    """A 16 MiB Z_FIXED stream (fixed-Huffman blocks only, no header to search
    for): zs_find_fixed_kernel records the block starts, the stream splits into
    many units, and output + zlib fields match the oracle."""
    raw = corpus.stream(12, 8 << 20) + corpus.stream(44, 8 << 20)
    for wb in (-15, 31):
        c = zlib.compressobj(6, zlib.DEFLATED, wb, 8, zlib.Z_FIXED)
        comp = c.compress(raw) + c.flush()
        got = zs.inflate_batch([comp], wb, [len(raw)], parse=parse)
        st = zs.last_stats()
        eo, ei = O.oneshot(comp, wb, len(raw))
        assert got[0][0] == eo == raw and got[0][1] == ei, (got[0][1], ei)
        assert st["chunked_jobs"] == 1 and st["fallback_jobs"] == 0, st
        assert st["units"] >= 64, st  # ~16 K-symbol fixed blocks found, not one serial lane


def test_chunked_high_ratio(zs):
    """A ratio > 100 stream (long repeats with sparse changes, a few KiB of
    input per 4 MiB block) takes the chunked path with no fallback."""
    import numpy as np
    rng = np.random.default_rng(3)
    unit = rng.integers(0, 256, 1500, dtype=np.uint8)
    reps = np.tile(unit, (24 << 20) // 1500 + 1)[:24 << 20].copy()
    idx = rng.integers(0, len(reps), len(reps) // 4000)
    reps[idx] = rng.integers(0, 256, len(idx), dtype=np.uint8)
    raw = reps.tobytes()
    c = zlib.compressobj(9, zlib.DEFLATED, -15)
    comp = c.compress(raw) + c.flush()
    assert len(raw) / len(comp) > 100
    got = zs.inflate_batch([comp], -15, [len(raw)])
    st = zs.last_stats()
    eo, ei = O.oneshot(comp, -15, len(raw))
    assert got[0][0] == eo == raw and got[0][1] == ei
    assert st["chunked_jobs"] == 1 and st["fallback_jobs"] == 0 and st["units"] > 1, st


@pytest.mark.parametrize("parse", ["lane", "wave", "split"])
def test_chunked_token_pool_pages(zs, parse):
    """Streams with several symbols per compressed byte (Huffman-only and RLE
    over a 3-letter alphabet: 1-2 bit literal codes) outgrow the primary token
    regions (1 token per compressed byte + slack), so every unit's tokens spill
    into pool pages -- the lane parse's flush (16-byte stores of full token
    quads) and its page path, under both parse modes; output and zlib fields
    match the oracle, nothing falls back."""
    import numpy as np
    rng = np.random.default_rng(11)
    raw = rng.choice(np.frombuffer(b"abc", np.uint8), 12 << 20, p=[0.6, 0.3, 0.1]).tobytes()
    for strategy, wb in ((zlib.Z_HUFFMAN_ONLY, -15), (zlib.Z_RLE, 31)):
        c = zlib.compressobj(6, zlib.DEFLATED, wb, 8, strategy)
        comp = c.compress(raw) + c.flush()
        assert len(raw) / len(comp) > 4
        got = zs.inflate_batch([comp, comp], wb, [len(raw)] * 2, parse=parse)
        st = zs.last_stats()
        eo, ei = O.oneshot(comp, wb, len(raw))
        for out, info in got:
            assert out == eo == raw and info == ei, (info, ei)
        assert st["chunked_jobs"] == 2 and st["fallback_jobs"] == 0 and st["units"] > 2, st


def test_c2_full_size_vs_oracle(zs):
    """configs[1] at full size: one Zipf and one line-text 64 MiB raw stream
    (host zlib L6), output and (ret, msg, total_in, total_out) vs the oracle."""
    raws, comps = corpus.batch(0, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
    r2, c2 = corpus.batch(32, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
    raws += r2
    comps += c2
    got = zs.inflate_batch([c.tobytes() for c in comps], -15, [64 << 20] * 2)
    st = zs.last_stats()
    for r, c, (out, info) in zip(raws, comps, got):
        eo, ei = O.oneshot(c.tobytes(), -15, 64 << 20)
        assert info == ei and info["ret"] == 1 and info["total_out"] == 64 << 20
        assert out == eo and out == r.tobytes()
    assert st["chunked_jobs"] == 2 and st["fallback_jobs"] == 0, st


def test_c5_shape_vs_oracle(zs):
    """configs[4] shape: 256 x 4 MiB, raw (-15) / gzip (31) alternating, Zipf /
    line text alternating in pairs (corpus.c5_stream), host zlib L6; every job's
    output and zlib fields vs the oracle, all on the chunked path."""
    from concurrent.futures import ThreadPoolExecutor
    n = 256

    def make(k):
        raw, wb = corpus.c5_stream(k, 4 << 20)
        c = zlib.compressobj(6, zlib.DEFLATED, wb, 8)
        return raw.tobytes(), c.compress(raw.tobytes()) + c.flush(), wb

    with ThreadPoolExecutor(16) as ex:
        cases = list(ex.map(make, range(n)))
    got = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], [4 << 20] * n)
    st = zs.last_stats()
    bad = []
    for k, ((raw, comp, wb), (out, info)) in enumerate(zip(cases, got)):
        eo, ei = O.oneshot(comp, wb, 4 << 20)
        if out != eo or info != ei or out != raw:
            bad.append((k, wb, info, ei))
    assert not bad, bad[:4]
    assert st["chunked_jobs"] == n and st["fallback_jobs"] == 0, st


def _too_far_after_start():
    """Raw deflate whose SECOND block (a decode unit of its own) copies from a
    preset dictionary, i.e. reaches before the stream start while the output is
    still shorter than the window: inflate without the dictionary must report
    "invalid distance too far back" where zlib does (detected at the window
    link / emit on the block-parallel path, then decoded exactly)."""
    rng = random.Random(12)
    dictionary = bytes(rng.getrandbits(8) for _ in range(32768))
    co = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY, dictionary)
    head = bytes(rng.getrandbits(8) for _ in range(3000))
    tail = corpus.stream(3, 900 << 10)
    out = co.compress(head) + co.flush(zlib.Z_SYNC_FLUSH)
    out += co.compress(dictionary[5000:9000] + tail) + co.flush()
    return out, len(head) + 4000 + len(tail)


@pytest.mark.parametrize("copies", [1, 6])
def test_chunked_too_far_back_across_units(zs, copies):
    """A too-far distance in a later unit, with one stream per batch (windows by
    the parallel-prefix link) and six (the per-stream serial link)."""
    comp, n = _too_far_after_start()
    got = zs.inflate_batch([comp] * copies, -15, [n] * copies)
    st = zs.last_stats()
    eo, ei = O.oneshot(comp, -15, n)
    assert ei["ret"] == -3 and ei["msg"] == "invalid distance too far back", ei
    for out, info in got:
        assert info == ei and out == eo, (info, ei)
    assert st["chunked_jobs"] == copies and st["fallback_jobs"] == copies, st


# ---------------------------------------------------------------------------
# the headline's own kernel path at headline scale: lane-per-unit parse (the
# mode a batch of > ZS_WAVE_SEGS search segments takes) with the multi-group
# dealing of lane_decode.hip (units past 64 x the resident waves), and the
# per-stream serial window link (zs_link_kernel) on the C2 pair
# ---------------------------------------------------------------------------
def _c5_cases(n, nthreads=16):
    from concurrent.futures import ThreadPoolExecutor

    def make(k):
        raw, wb = corpus.c5_stream(k, 4 << 20)
        c = zlib.compressobj(6, zlib.DEFLATED, wb, 8)
        return raw, c.compress(raw) + c.flush(), wb

    with ThreadPoolExecutor(nthreads) as ex:
        return list(ex.map(make, range(n)))


def _compare_all_with_oracle(cases, got, cap, nthreads=16):
    """Every job's output and (ret, msg, total_in, total_out, adler) vs the
    oracle, the oracle's output vs the generator; oracle calls run on threads
    (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    def check(k):
        raw, comp, wb = cases[k]
        out, info = got[k]
        eo, ei = O.oneshot(comp, wb, cap)
        ok = out == eo and info == ei and len(eo) == len(raw) and eo == raw.tobytes()
        return None if ok else (k, wb, info, ei)

    with ThreadPoolExecutor(nthreads) as ex:
        bad = [b for b in ex.map(check, range(len(cases))) if b]
    assert not bad, f"{len(bad)} mismatches, first: {bad[:4]}"


def test_c5_lane_parse_multigroup_vs_oracle(zs):
    """configs[4] shape at a scale where the lane parse deals its sorted units
    over more than one group of resident waves: 1 280 x 4 MiB streams (raw / gzip
    alternating, Zipf / line text), lane mode forced, every job vs the oracle."""
    n = 1280
    cases = _c5_cases(n)
    got = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], [4 << 20] * n, parse="lane")
    st = zs.last_stats()
    assert st["parse"] == "lane" and st["link"] == "serial", st
    assert st["lane_resident_waves"] > 0 and st["units_std"] > 64 * st["lane_resident_waves"], st
    assert st["chunked_jobs"] == n and st["fallback_jobs"] == 0, st
    _compare_all_with_oracle(cases, got, 4 << 20)


def test_c2_pair_lane_parse_serial_link_vs_oracle(zs):
    """configs[1] streams at full size (one Zipf, one line text, 64 MiB each)
    through the lane parse and the serial per-stream link -- the kernels the C2
    headline runs -- vs the oracle."""
    raws, comps = corpus.batch(0, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
    r2, c2 = corpus.batch(32, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
    cases = [(r, c.tobytes(), -15) for r, c in zip(raws + r2, comps + c2)]
    got = zs.inflate_batch([c[1] for c in cases], -15, [64 << 20] * 2, parse="lane", link="serial")
    st = zs.last_stats()
    assert st["parse"] == "lane" and st["link"] == "serial", st
    assert st["chunked_jobs"] == 2 and st["fallback_jobs"] == 0, st
    _compare_all_with_oracle(cases, got, 64 << 20, nthreads=2)


def test_segmented_link_vs_oracle(zs):
    """The segmented link (zs_linkseg_kernel: a group of 5..64 streams cuts each
    chain into segments linked at once as u16 window maps, joined per stream,
    resolved by the emit) on 24 C5-shape streams of 2 MiB -- 8 segments of ~3
    members each -- every result field vs the oracle; the same batch through
    the per-stream serial link for contrast."""
    cases = []
    for k in range(24):
        raw, wb = corpus.c5_stream(k, 2 << 20)
        c = zlib.compressobj(6, zlib.DEFLATED, wb, 8)
        cases.append((raw, c.compress(raw) + c.flush(), wb))
    caps = [2 << 20] * len(cases)
    got = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], caps)
    st = zs.last_stats()
    assert st["link"] == "segmented" and st["chunked_jobs"] == 24 and st["fallback_jobs"] == 0, st
    _compare_all_with_oracle(cases, got, 2 << 20)
    got2 = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], caps, link="serial")
    assert zs.last_stats()["link"] == "serial"
    assert [g[0] for g in got2] == [g[0] for g in got] and [g[1] for g in got2] == [g[1] for g in got]



def test_c5_rank_share_world8_vs_oracle(zs):
    """configs[4] split over 8 ranks: the last rank's share of the 4 096 x 4 MiB
    mixed raw / gzip streams (shard.bench_shard, the partition bench.py's ranks
    derive), decoded on this GPU in the parse / link modes a 512-stream batch
    takes by default, every job vs the oracle."""
    import shard
    from concurrent.futures import ThreadPoolExecutor

    ids = shard.bench_shard(4096, 7, 8, shard.c5_kind)
    assert len(ids) == 512

    def make(k):
        raw, wb = corpus.c5_stream(k, 4 << 20)
        c = zlib.compressobj(6, zlib.DEFLATED, wb, 8)
        return raw, c.compress(raw) + c.flush(), wb

    with ThreadPoolExecutor(16) as ex:
        cases = list(ex.map(make, ids))
    got = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], [4 << 20] * len(cases))
    st = zs.last_stats()
    assert st["chunked_jobs"] == len(cases) and st["fallback_jobs"] == 0, st
    _compare_all_with_oracle(cases, got, 4 << 20)


# ---------------------------------------------------------------------------
# the segmented window link at the configurations the final build runs it
# (zs_capi.cpp link_segments: S = min(8, 512 / streams) segments per chain,
# round 6; 256 / streams before)
# ---------------------------------------------------------------------------
def test_c2_headline_batch_segmented_link_vs_oracle(zs):
    """configs[1] exactly as the headline bench runs it: 64 x 64 MiB raw-deflate
    streams (Zipf text 0..31, line text 32..63, host zlib L6) in ONE batch with
    default flags -- one group (ZS_GROUPS unset), split parse (round 5),
    segmented link with 8 segments per chain of ~720 members (round 6) -- every
    job's output and (ret, msg, total_in, total_out, adler) vs the oracle and
    the generator."""
    raws, comps = corpus.batch(0, 64, 64 << 20, level=6, wbits=-15, nthreads=16)
    cases = [(r, c.tobytes(), -15) for r, c in zip(raws, comps)]
    del comps
    got = zs.inflate_batch([c[1] for c in cases], -15, [64 << 20] * 64)
    st = zs.last_stats()
    assert st["parse"] == "split" and st["link"] == "segmented" and st["link_segments"] == 8, st
    assert st["groups"] == 1, st
    assert st["chunked_jobs"] == 64 and st["fallback_jobs"] == 0, st
    assert st["units_std"] >= 64 * 400, st  # chains of >= 400 members on average
    _compare_all_with_oracle(cases, got, 64 << 20)


def test_c2_strong_split_share_world8_vs_oracle(zs):
    """The share one rank of 8 decodes when the 64 x 64 MiB C2 batch is split
    across 8 GPUs (shard.bench_shard, bench.py --scaling strong / --sim-world 8):
    8 streams -> wave-per-unit parse and the segmented link with 8 segments per
    chain; every job vs the oracle."""
    import shard
    ids = shard.bench_shard(64, 7, 8, shard.c2_kind)
    assert len(ids) == 8
    cases = []
    for i in ids:
        r, c = corpus.batch(i, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
        cases.append((r[0], c[0].tobytes(), -15))
    got = zs.inflate_batch([c[1] for c in cases], -15, [64 << 20] * len(cases))
    st = zs.last_stats()
    assert st["parse"] == "wave" and st["link"] == "segmented" and st["link_segments"] == 8, st
    assert st["chunked_jobs"] == 8 and st["fallback_jobs"] == 0, st
    _compare_all_with_oracle(cases, got, 64 << 20, nthreads=8)


@pytest.mark.parametrize("parse", ["lane", "wave", "split"])
def test_c2_pair_forced_link_segments_vs_oracle(zs, parse):
    """ZS_F_LINKSEG(n), n = 2 / 4 / 8, on the C2 pair (one Zipf, one line-text
    64 MiB stream: chains of ~900 / ~500 members) under both parse modes: the
    segmented link at every segment count gives the oracle's results; and on
    short chains (2 MiB streams, fewer members than segments in some chains)
    with n = 8."""
    raws, comps = corpus.batch(0, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
    r2, c2 = corpus.batch(32, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
    cases = [(r, c.tobytes(), -15) for r, c in zip(raws + r2, comps + c2)]
    ref = None
    for n in (2, 4, 8):
        got = zs.inflate_batch([c[1] for c in cases], -15, [64 << 20] * 2, parse=parse, link=("segmented", n))
        st = zs.last_stats()
        assert st["parse"] == parse and st["link"] == "segmented" and st["link_segments"] == n, st
        assert st["chunked_jobs"] == 2 and st["fallback_jobs"] == 0, st
        if ref is None:
            _compare_all_with_oracle(cases, got, 64 << 20, nthreads=2)
            ref = got
        else:
            assert [g[1] for g in got] == [g[1] for g in ref]
            assert all(a[0] == b[0] for a, b in zip(got, ref))
    small = []
    for k in range(6):
        raw, wb = corpus.c5_stream(k, (k + 1) << 18)
        c = zlib.compressobj(6, zlib.DEFLATED, wb, 8)
        small.append((raw, c.compress(raw.tobytes()) + c.flush(), wb))
    cap = 6 << 18
    got = zs.inflate_batch([c[1] for c in small], [c[2] for c in small], [cap] * len(small), parse=parse,
                           link=("segmented", 8))
    st = zs.last_stats()
    assert st["link"] == "segmented" and st["link_segments"] == 8, st
    _compare_all_with_oracle(small, got, cap)


# ---------------------------------------------------------------------------
# the split parse (round 5): boundary walk + sub-unit decode + leftovers
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["zipf", "lines"])
def test_split_parse_forced_text_vs_oracle(zs, kind):
    """The split parse forced on 8 x 8 MiB streams of one text kind (Zipf words,
    or the periodic line text that defeated round 1's self-synchronising split):
    the walk's checkpoints are exact symbol boundaries, so every job equals the
    oracle whatever the text; the lane parse gives the same bytes."""
    base = 0 if kind == "zipf" else 32
    raws, comps = corpus.batch(base, 8, 8 << 20, level=6, wbits=-15, nthreads=8)
    cases = [(r, c.tobytes(), -15) for r, c in zip(raws, comps)]
    got = zs.inflate_batch([c[1] for c in cases], -15, [8 << 20] * 8, parse="split")
    st = zs.last_stats()
    assert st["parse"] == "split" and st["chunked_jobs"] == 8 and st["fallback_jobs"] == 0, st
    _compare_all_with_oracle(cases, got, 8 << 20, nthreads=8)
    lane = zs.inflate_batch([c[1] for c in cases], -15, [8 << 20] * 8, parse="lane")
    assert [g[1] for g in lane] == [g[1] for g in got] and all(a[0] == b[0] for a, b in zip(lane, got))


def test_split_parse_small_blocks_continue(zs):
    """Blocks of ~1-3 KiB (a sync flush every few KiB): a 32 KiB search segment
    holds more block starts than the finder records, so units run past their
    first block -- the split decodes the first block, the leftover kernel
    resumes at its end (WK_CONT) -- and more units end with a false start
    inside; every result field vs the oracle, for raw / zlib / gzip."""
    rng = random.Random(21)
    cases = []
    for k, wb in enumerate((-15, 15, 31, -15)):
        raw = corpus.stream(k + 3, 3 << 20)
        c = zlib.compressobj(6, zlib.DEFLATED, wb)
        parts, i = [], 0
        while i < len(raw):
            n = rng.randint(1 << 10, 6 << 10)
            parts.append(c.compress(raw[i:i + n]))
            parts.append(c.flush(zlib.Z_SYNC_FLUSH if rng.random() < 0.7 else zlib.Z_FULL_FLUSH))
            i += n
        parts.append(c.flush())
        cases.append((raw, b"".join(parts), wb))
    got = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], [3 << 20] * len(cases), parse="split")
    st = zs.last_stats()
    assert st["parse"] == "split" and st["chunked_jobs"] == len(cases) and st["fallback_jobs"] == 0, st
    for (raw, comp, wb), (out, info) in zip(cases, got):
        eo, ei = O.oneshot(comp, wb, 3 << 20)
        assert out == eo == raw and info == ei, (wb, info, ei)


def test_split_parse_first_unit_too_far(zs):
    """A raw stream written against a preset dictionary, inflated without it:
    its first block reaches before the stream start.  The split parse defers the
    too-far check of the stream's first unit to its wave scan of sub-unit
    outputs; the stream goes to the exact decoder, which reports zlib's
    "invalid distance too far back" -- every field vs the oracle; a clean
    stream in the same batch still decodes on the chunked path."""
    zdict = corpus.stream(9, 32 << 10)
    raw = zdict * 8 + corpus.stream(10, 2 << 20)
    c = zlib.compressobj(6, zlib.DEFLATED, -15, 8, 0, zdict)
    bad = c.compress(raw) + c.flush()
    c2 = zlib.compressobj(6, zlib.DEFLATED, -15)
    good = c2.compress(raw) + c2.flush()
    cap = len(raw)
    got = zs.inflate_batch([bad, good], -15, [cap, cap], parse="split")
    for comp, (out, info) in zip((bad, good), got):
        eo, ei = O.oneshot(comp, -15, cap)
        assert out == eo and info == ei, (info, ei)
    assert got[0][1]["ret"] == -3 and got[1][0] == raw


@pytest.mark.parametrize("parse", ["split", "lane"])
def test_all_literals_on_one_long_length(zs, parse):
    """a dynamic code with all 256 literals, end of block and
    length 257 on 10-bit codes (tests/crafted.py), 0xFF a frequent literal.
    The walk's canonical tail must count 256 literals of one length (a u8 count
    read literal 0xFF as the end of block: truncated output, silent for raw
    deflate); the split decode also checks the code at the walked end of block.
    Every field vs the oracle and host zlib, raw / zlib / gzip wrappers."""
    import crafted
    raw, comp = crafted.long_literal_stream(2 << 20, seed=7)
    zwrap = bytes([0x78, 0x01]) + comp + zlib.adler32(raw).to_bytes(4, "big")
    gwrap = (bytes([0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3]) + comp + zlib.crc32(raw).to_bytes(4, "little")
             + (len(raw) & 0xffffffff).to_bytes(4, "little"))
    cases = [(raw, comp, -15), (raw, zwrap, 15), (raw, gwrap, 31), (raw, comp, -15)]
    got = zs.inflate_batch([c[1] for c in cases], [c[2] for c in cases], [len(raw)] * len(cases), parse=parse)
    st = zs.last_stats()
    assert st["parse"] == parse and st["chunked_jobs"] == len(cases) and st["fallback_jobs"] == 0, st
    for (r, c, wb), (out, info) in zip(cases, got):
        eo, ei = O.oneshot(c, wb, len(r))
        assert out == eo == r and info == ei and info["ret"] == 1, (wb, info, ei)


def test_split_leftovers_from_start():
    """Round 6: a split unit that fails its own check (WK_LEFT) is decoded again
    from its start by the leftover kernel, header included (the split parse's
    unit headers write no zlib-layout tables).  ZS_SPLIT_LEFT=1 fails every
    split unit on purpose; Zipf and line text plus a truncated stream, vs the
    oracle (tests/split_left_check.py, in a child process: the knob is read
    once per process)."""
    env = dict(os.environ, ZS_SPLIT_LEFT="1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "split_left_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
