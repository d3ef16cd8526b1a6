"""Long streams in pieces (zs_capi.cpp run_pieces).

A stream past one launch's limits (512 MiB compressed, 4 GiB out) decodes as a
sequence of pieces: each resumes at the block boundary where the previous one
stopped, with the output so far as its history, and the checks and the result
cover the whole stream.  ZS_PIECE_KB splits small streams the same way, so the
oracle checks every result field -- (ret, msg, total_in, total_out, adler) of
one zlib inflate(Z_FINISH) call, src/inflate.c:1275 -- at sizes it runs in
seconds, errors included; one test decodes a real > 512 MiB gzip stream.
"""
import random
import zlib

import pytest

import corpus
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def zs():
    import zstreams
    zstreams.lib()
    return zstreams


@pytest.fixture
def pieces(monkeypatch):
    monkeypatch.setenv("ZS_PIECE_KB", "192")


def _zlib(data, wbits, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, 8, strategy)
    return c.compress(data) + c.flush()


def _compare(zs, cases):
    got = zs.inflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    st = zs.last_stats()
    bad = []
    for i, (c, (out, info)) in enumerate(zip(cases, got)):
        eo, ei = O.oneshot(c[0], c[1], c[2])
        if out != eo or info != ei:
            bad.append((i, c[1], c[2], len(c[0]), info, ei, len(out), len(eo)))
    assert not bad, f"{len(bad)}/{len(cases)} mismatches, first: {bad[:3]}"
    return st


def test_pieces_match_oracle(zs, pieces):
    cases = []
    for k, wb in enumerate((-15, 15, 31)):
        for text in (corpus.zipf_text(3 << 20, k), corpus.lines_text(3 << 20, 40 + k)):
            cases.append((_zlib(text, wb), wb, len(text) + 100))
    # fixed-Huffman blocks (the fixed-block finder), and a small output cap (Z_BUF_ERROR)
    text = corpus.zipf_text(2 << 20, 7)
    cases.append((_zlib(text, -15, 6, zlib.Z_FIXED), -15, len(text)))
    cases.append((_zlib(text, 31), 31, len(text) // 2 + 12345))
    st = _compare(zs, cases)
    # every stream is longer than a piece: each is several chunked launches
    assert st["chunked_jobs"] > 2 * len(cases), st


def test_pieces_errors_match_oracle(zs, pieces):
    rng = random.Random(11)
    text = corpus.zipf_text(3 << 20, 3)
    cases = []
    for wb in (-15, 31, 15):
        comp = _zlib(text, wb)
        for frac in (0.35, 0.6, 0.9):
            cut = int(len(comp) * frac)
            cases.append((comp[:cut], wb, len(text) + 64))  # truncated inside a later piece
            b = bytearray(comp)
            for _ in range(3):
                b[cut + rng.randrange(64)] ^= 1 << rng.randrange(8)
            cases.append((bytes(b), wb, len(text) + 64))  # corrupt inside a later piece
        if wb != -15:
            b = bytearray(comp)
            b[-6] ^= 0x40  # the trailer: data check over the output of every piece
            cases.append((bytes(b), wb, len(text) + 64))
    _compare(zs, cases)


def test_pieces_deflate64(zs, pieces):
    text = corpus.lines_text(3 << 20, 50)
    (comp, info), = zs.deflate_batch([text], -16, 6)
    assert info["ret"] == 1
    got = zs.inflate_batch([comp, comp[: len(comp) * 2 // 3]], -16, [len(text) + 64] * 2)
    assert got[0][0] == text and got[0][1]["ret"] == 1 and got[0][1]["total_in"] == len(comp)
    eo, ei = O.oneshot(comp[: len(comp) * 2 // 3], -16, len(text) + 64)
    assert got[1][0] == eo and got[1][1] == ei


def test_stream_over_512_mib(zs):
    """One gzip stream of > 2^29 compressed bytes, past one launch's limits:
    decoded in pieces (no ZS_PIECE_KB), checked against its input on the device."""
    torch = pytest.importorskip("torch")
    n = 1300 << 20
    g = torch.Generator(device="cuda").manual_seed(5)
    data = torch.randint(0, 16, (n,), dtype=torch.uint8, device="cuda", generator=g)
    cap = zs.deflate_bound(n, 31)
    comp = torch.empty(cap, dtype=torch.uint8, device="cuda")
    (di,) = zs.deflate_batch_device([data.data_ptr()], [n], [comp.data_ptr()], [cap], 31, level=1)
    clen = di["total_out"]
    assert di["ret"] == 1 and clen > (1 << 29), di
    out = torch.empty(n + 256, dtype=torch.uint8, device="cuda")
    (r,) = zs.inflate_batch_device([comp.data_ptr()], [clen], [out.data_ptr()], [n + 256], 31)
    st = zs.last_stats()
    assert r["ret"] == 1 and r["total_in"] == clen and r["total_out"] == n, r
    assert torch.equal(out[:n], data)
    assert st["chunked_jobs"] >= 3 and st["fallback_jobs"] == 0, st
