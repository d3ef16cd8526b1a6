"""GPU deflate64 encoder: window_bits -16 in the batch
deflate.  The reference has no deflate64 compressor (its fixtures come from
7-Zip, create_deflate64.cpp:40-46); the bar is the reference's deflate64
inflate -- the oracle at windowBits -16 -- giving back the input, with the
deflate64-only codes exercised: distances beyond 32 KiB (codes 30/31) and
code 285 runs longer than 258 (3 + 16 extra bits), which no committed fixture
uses.
"""
import random

import pytest

import corpus
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zs():
    import zstreams
    zstreams.lib()
    return zstreams


def _inflate64(comp, n):
    out, info = O.oneshot(comp, -16, n + 1024)
    return out, info


def test_deflate64_roundtrip_through_the_oracle(zs):
    rng = random.Random(64)
    text = corpus.stream(2, 700000)
    r40 = bytes(rng.getrandbits(8) for _ in range(40000))
    cases = [b"", b"a", text, text[:65536], bytes(1 << 20), b"abc" * 100000, r40 * 5,
             text[:100000] + bytes(300000) + text[:100000], bytes(rng.getrandbits(8) for _ in range(90000))]
    for level in (0, 1, 6, 9):
        got = zs.deflate_batch(cases, -16, level)
        for data, (comp, info) in zip(cases, got):
            assert info["ret"] == 1 and info["total_in"] == len(data) and info["total_out"] == len(comp), info
            out, oi = _inflate64(comp, len(data))
            assert oi["ret"] == 1 and oi["total_in"] == len(comp) and out == data, (level, len(data), oi)
    # and the GPU's own deflate64 inflate (serial wave decoder) agrees
    comps = [c for c, _ in zs.deflate_batch(cases, -16, 6)]
    back = zs.inflate_batch(comps, -16, [len(d) + 64 for d in cases])
    assert [o for o, _ in back] == cases


def test_deflate64_uses_code_285_runs(zs):
    """1 MiB of zeros: 258-byte matches need ~4 000 tokens; merged code-285
    runs need about one per 64 KiB block."""
    data = bytes(1 << 20)
    (c64, _), (c15, _) = zs.deflate_batch([data, data], [-16, -15], 6)
    assert len(c64) < 400 < len(c15), (len(c64), len(c15))
    out, oi = _inflate64(c64, len(data))
    assert oi["ret"] == 1 and out == data
    # code 285 means "258, no extra bits" to a standard inflate: it desynchronises
    out15, oi15 = O.oneshot(c64, -15, len(data) + 1024)
    assert out15 != data


def test_deflate64_reaches_64k_back(zs):
    """A 40 KiB random block repeated: only a deflate64 window (distance codes
    30/31) finds the repeats."""
    rng = random.Random(1)
    r = bytes(rng.getrandbits(8) for _ in range(40000))
    data = r * 6
    (c64, _), (c15, _) = zs.deflate_batch([data, data], [-16, -15], 6)
    assert len(c64) < 0.4 * len(c15), (len(c64), len(c15))
    out, oi = _inflate64(c64, len(data))
    assert oi["ret"] == 1 and out == data


@pytest.mark.parametrize("parse", ["lane", "wave", "split"])
def test_deflate64_chunked_block_parallel(zs, parse):
    """Large deflate64 streams take the block-parallel path (64 KiB history
    windows, 32 distance codes, code-285 copies split into tokens) with no
    serial fallback, and match the oracle at windowBits -16 (the reference's
    inflate9 semantics, src/inflate.c:1037-1193, inftrees.c:73-87)."""
    import numpy as np
    rng = np.random.default_rng(9)
    blk = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
    datas = [corpus.stream(3, 24 << 20),
             corpus.stream(35, 12 << 20) + bytes(3 << 20) + blk * 40 + corpus.stream(4, 2 << 20)]
    comps = [c for c, _ in zs.deflate_batch(datas, -16, 6)]
    got = zs.inflate_batch(comps, -16, [len(d) for d in datas], parse=parse)
    st = zs.last_stats()
    for d, c, (out, info) in zip(datas, comps, got):
        eo, ei = O.oneshot(c, -16, len(d))
        assert info == ei and info["ret"] == 1 and out == eo == d, (info, ei)
    assert st["chunked_jobs"] == 2 and st["fallback_jobs"] == 0 and st["units"] > 100, st
