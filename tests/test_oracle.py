"""CPU: the oracle reproduces every reference golden value, and agrees with host
zlib (independent implementation of the same inflate) on fuzzed streams."""
import hashlib
import json
import os
import random
import zlib

import pytest

import oracle_lib as O
import libz_ref as LZ
from golden.make_manifest import fixture, mutate

HERE = os.path.dirname(os.path.abspath(__file__))
MAN = json.load(open(os.path.join(HERE, "golden", "manifest.json")))


@pytest.mark.parametrize("name", sorted(MAN["fixtures"]))
def test_fixture_hash(name):
    m = MAN["fixtures"][name]
    out, info = O.oneshot(fixture(name), m["wbits"])
    assert info["ret"] == 1 and len(out) == m["len"] and info["total_in"] == m["total_in"]
    assert hashlib.sha256(out).hexdigest() == m["sha256"]


@pytest.mark.parametrize("case", MAN["crafted"], ids=lambda c: c["name"])
def test_crafted(case):
    out, info = O.oneshot(bytes.fromhex(case["hex"]), case["wbits"])
    for k, v in case["expect"].items():
        assert (hashlib.sha256(out).hexdigest() if k == "sha256" else info[k]) == v, k


@pytest.mark.parametrize("case", MAN["fixture_errors"], ids=lambda c: f'{c["fixture"]}{c["wbits"]}')
def test_fixture_errors(case):
    how = tuple(case["mutate"]) if case["mutate"] else None
    _, info = O.oneshot(mutate(fixture(case["fixture"]), how), case["wbits"])
    for k, v in case["expect"].items():
        assert info[k] == v, k


@pytest.mark.parametrize("case", MAN["traces"], ids=lambda c: f'{c["fixture"]}{c["wbits"]}w{c["write"]}')
def test_boundary_trace(case):
    tr, out = O.js_schedule(fixture(case["fixture"]), case["write"], case["wbits"])
    assert tr.count("\n") == case["calls"]
    assert hashlib.sha256(tr.encode()).hexdigest()[:16] == case["sha256_16"]


def _fuzz_case(rng):
    words = [bytes(rng.choice(b"abcdefghij") for _ in range(rng.randint(2, 8))) for _ in range(50)]
    if rng.random() < 0.8:
        raw = b" ".join(rng.choice(words) for _ in range(rng.randint(0, 3000)))
    else:
        raw = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 2000)))
    wb = rng.choice([-15, 15, 31])
    c = zlib.compressobj(rng.choice([0, 1, 6, 9]), zlib.DEFLATED, wb, 8, rng.choice([0, 0, 0, 1, 2, 3, 4]))
    comp = bytearray(c.compress(raw) + c.flush())
    mode = rng.random()
    if mode < 0.5 and comp:
        for _ in range(rng.randint(1, 3)):
            i = rng.randrange(len(comp))
            comp[i] ^= 1 << rng.randrange(8)
    elif mode < 0.65 and comp:
        comp = comp[:rng.randrange(len(comp))]
    cap = rng.choice([None, None, rng.randint(0, len(raw) + 10)])
    dwb = wb if rng.random() < 0.9 else rng.choice([-15, 15, 31, 47, -8, 9])
    return bytes(comp), dwb, cap


def test_oracle_vs_host_zlib_fuzz():
    rng = random.Random(20261015)
    for _ in range(600):
        comp, dwb, cap = _fuzz_case(rng)
        o1, i1 = O.oneshot(comp, dwb, cap)
        o2, i2 = LZ.oneshot(comp, dwb, cap)
        assert (o1, i1) == (o2, i2), (dwb, cap, i1, i2)


def test_checks_match_zlib():
    rng = random.Random(3)
    for n in (0, 1, 5551, 5552, 5553, 70000):
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert O.lib().zo_crc32(0, b, n) == zlib.crc32(b)
        assert O.lib().zo_adler32(1, b, n) == zlib.adler32(b)


def test_crafted_all_literals_on_one_long_length():
    """tests/crafted.py's 10-bit-literal dynamic blocks (the GPU test
    test_all_literals_on_one_long_length): the oracle and host zlib agree."""
    import crafted
    raw, comp = crafted.long_literal_stream(200 << 10, seed=3, block_syms=3000)
    assert zlib.decompress(comp, -15) == raw
    out, info = O.oneshot(comp, -15, len(raw))
    assert out == raw and info["ret"] == 1 and info["total_in"] == len(comp)
