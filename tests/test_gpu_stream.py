"""GPU parity of the streaming surfaces, call by call (SURVEY.md §8b Tier 2).

Every call of the handle ABI (src/wasm/wasm_stream_common.c:37-63) and of the
zlib ABI (inflate(strm, flush), src/inflate.c:597) must return what the
reference's zlib state machine returns for the same call: consumed, produced,
the bytes, ret, msg, total_in/total_out and adler.  The oracle
(oracle/zo_inflate.c, pinned by tests/test_oracle.py) is the checker; the
reference's own call schedule is pinned by the Appendix C trace hashes.
"""
import ctypes
import hashlib
import json
import os
import random
import struct
import zlib

import pytest

import corpus
import libz_ref
import oracle_lib as O
from golden.make_manifest import fixture

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
MAN = json.load(open(os.path.join(HERE, "golden", "manifest.json")))
FMT = {-15: "deflate-raw", 15: "deflate", 31: "gzip", -16: "deflate64-raw"}


@pytest.fixture(scope="module")
def zs():
    import zstreams
    zstreams.lib()
    return zstreams


def _comp(data, wbits, level=6, mem=8, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, mem, strategy)
    return c.compress(data) + c.flush()


@pytest.mark.parametrize("case", MAN["traces"], ids=lambda c: f'{c["fixture"]}{c["wbits"]}w{c["write"]}')
def test_appendix_c_traces(zs, case):
    """The reference's JS schedule on the GPU reproduces the per-call traces
    captured from the reference."""
    tr, out = zs.js_schedule(fixture(case["fixture"]), FMT[case["wbits"]], case["write"])
    assert tr.count("\n") == case["calls"]
    assert hashlib.sha256(tr.encode()).hexdigest()[:16] == case["sha256_16"], tr
    etr, eout = O.js_schedule(fixture(case["fixture"]), case["write"], case["wbits"])
    assert tr == etr and out == eout


def _schedule_cases():
    rng = random.Random(7)
    text = corpus.stream(3, 400000)
    lines = corpus.stream(40, 300000)
    rnd = bytes(rng.getrandbits(8) for _ in range(150000))
    cases = []
    for name in ("100k_lines", "zeros_100k", "payload_64k", "rand_block_gap"):
        cases.append((fixture(name), -16))
    cases.append((fixture("10k_lines"), -15))
    for wb in (-15, 15, 31):
        cases.append((_comp(text, wb), wb))
        cases.append((_comp(lines, wb, 9), wb))
        cases.append((_comp(rnd, wb, 6), wb))          # stored blocks
        cases.append((_comp(text[:60000], wb, 0), wb))  # level 0
        cases.append((_comp(text[:20000], wb, 1, strategy=zlib.Z_FIXED), wb))
        cases.append((_comp(text[:90000], wb, 6, strategy=zlib.Z_HUFFMAN_ONLY), wb))
        cases.append((_comp(b"", wb), wb))
    # corrupt / truncated
    g = _comp(text[:100000], 31)
    cases.append((g[:len(g) - 3], 31))
    b = bytearray(g)
    b[len(b) - 6] ^= 0x55  # CRC mismatch
    cases.append((bytes(b), 31))
    z = _comp(lines[:100000], 15)
    b = bytearray(z)
    b[len(b) // 2] ^= 0x10
    cases.append((bytes(b), 15))
    return cases


@pytest.mark.parametrize("write", [1000, 4096, 65536])
def test_js_schedule_traces_match_oracle(zs, write):
    """Per-call (n, produced, code, consumed) traces and output, GPU vs oracle."""
    bad = []
    for i, (data, wb) in enumerate(_schedule_cases()):
        tr, out = zs.js_schedule(data, FMT[wb], write)
        etr, eout = O.js_schedule(data, write, wb)
        if tr != etr or out != eout:
            bad.append((i, wb, len(data), tr[:300], etr[:300]))
    assert not bad, bad[:3]


@pytest.mark.parametrize("persist", [True, False], ids=["persistent", "batched"])
def test_concurrent_handles_match_oracle(zs, persist):
    """Many handles driven at once from their own threads -- on the persistent
    worker (a workgroup per handle, each call returned on its own) or batched
    into shared launches: every per-call trace and output still equals the
    oracle's for that stream alone."""
    from concurrent.futures import ThreadPoolExecutor
    cases = _schedule_cases() * 2
    writes = [4096 if i % 2 else 65536 for i in range(len(cases))]
    prev = zs.stream_persist(persist)
    try:
        before = zs.stream_stats()
        with ThreadPoolExecutor(16) as ex:
            got = list(ex.map(lambda a: zs.js_schedule(a[0][0], FMT[a[0][1]], a[1]), zip(cases, writes)))
        after = zs.stream_stats()
    finally:
        zs.stream_persist(prev)
    bad = []
    for i, ((data, wb), w, (tr, out)) in enumerate(zip(cases, writes, got)):
        etr, eout = O.js_schedule(data, w, wb)
        if tr != etr or out != eout:
            bad.append((i, wb, w, tr[:200], etr[:200]))
    assert not bad, bad[:3]
    calls = after["calls"] - before["calls"]
    launches = after["launches"] - before["launches"]
    if persist:  # the wrapper headers take the batch path, every later call the worker
        assert after["pk_calls"] - before["pk_calls"] > calls
    else:
        assert after["pk_calls"] == before["pk_calls"]
        assert 0 < launches < calls  # some calls shared a launch


def _gzip_header_all_fields(body_raw):
    """gzip member with FEXTRA, FNAME, FCOMMENT and FHCRC set."""
    hdr = bytearray(b"\x1f\x8b\x08\x1e") + struct.pack("<I", 12345) + b"\x00\x03"
    hdr += struct.pack("<H", 7) + b"extra!!" + b"name.txt\x00" + b"a comment\x00"
    hdr += struct.pack("<H", zlib.crc32(bytes(hdr)) & 0xffff)
    return bytes(hdr)


def _random_call_cases():
    rng = random.Random(11)
    text = corpus.stream(5, 200000)
    cases = []
    for wb in (-15, 15, 31, 47):
        cases.append((_comp(text, wb if wb != 47 else 31), wb))
    raw = text[:80000]
    gz = _gzip_header_all_fields(raw) + _comp(raw, -15) + struct.pack("<II", zlib.crc32(raw), len(raw))
    cases.append((gz, 31))
    cases.append((gz, 47))
    cases.append((fixture("100k_lines")[:60000], -16))
    cases.append((fixture("payload_65k"), -16))
    cases.append((bytes.fromhex("4b1c451f0000"), -16))  # len-285
    cases.append((_comp(bytes(rng.getrandbits(8) for _ in range(70000)), -15, 1), -15))
    cases.append((_comp(text[:50000], -15, 0), -15))
    # distances beyond a small window: legal in one call, too far once split
    cases.append((_comp(text[:60000], -15), -9))
    cases.append((_comp(text[:60000], -9), -9))
    # zlib FDICT header -> Z_NEED_DICT
    zd = zlib.compressobj(6, zlib.DEFLATED, 15, 8, zlib.Z_DEFAULT_STRATEGY, b"dictionary words")
    cases.append((zd.compress(text[:5000]) + zd.flush(), 15))
    # corruptions in headers / data / trailers
    for k in range(6):
        b = bytearray(_comp(text[:30000], 31))
        b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        cases.append((bytes(b), 31))
    return cases


class _GpuZ:
    """The library's zlib ABI (inflateInit2_ / inflate / inflateEnd)."""

    def __init__(self, L, wbits):
        self.L = L
        self.s = libz_ref.ZStream()
        self.rc = L.inflateInit2_(ctypes.byref(self.s), wbits, b"1.2.11", ctypes.sizeof(libz_ref.ZStream))

    def call(self, data, out_len, flush):
        ib = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
        ob = ctypes.create_string_buffer(max(out_len, 1))
        self.s.next_in = ctypes.addressof(ib) if data else None
        self.s.avail_in = len(data)
        self.s.next_out = ctypes.addressof(ob)
        self.s.avail_out = out_len
        r = self.L.inflate(ctypes.byref(self.s), flush)
        prod = out_len - self.s.avail_out
        return {"ret": r, "consumed": len(data) - self.s.avail_in, "produced": prod, "out": ob.raw[:prod],
                "msg": self.s.msg.decode() if self.s.msg else None, "total_in": self.s.total_in,
                "total_out": self.s.total_out, "adler": self.s.adler & 0xffffffff}

    def end(self):
        return self.L.inflateEnd(ctypes.byref(self.s))


def test_zlib_abi_random_call_schedules(zs):
    """Random avail_in / avail_out / flush per call (0 and 1 included), every
    call's result vs the oracle's zlib-style inflate."""
    L = ctypes.CDLL(zs.LIB_PATH)
    L.inflateInit2_.argtypes = [ctypes.POINTER(libz_ref.ZStream), ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.inflate.argtypes = [ctypes.POINTER(libz_ref.ZStream), ctypes.c_int]
    L.inflateEnd.argtypes = [ctypes.POINTER(libz_ref.ZStream)]
    rng = random.Random(2024)
    ins = [0, 1, 2, 3, 5, 9, 64, 700, 4096, 32768, 200000]
    outs = [0, 1, 2, 7, 258, 1000, 4096, 65536, 65536, 1 << 20]
    ncalls = 0
    for ci, (data, wb) in enumerate(_random_call_cases()):
        g, o = _GpuZ(L, wb), O.Stream(wb)
        assert g.rc == o.rc == 0
        off, idle = 0, 0
        for k in range(400):
            n = min(rng.choice(ins), len(data) - off)
            m = rng.choice(outs)
            fl = 4 if rng.random() < 0.2 else 0
            rg, ro = g.call(data[off:off + n], m, fl), o.call(data[off:off + n], m, fl)
            ncalls += 1
            assert rg == ro, (ci, wb, k, off, n, m, fl, {x: (rg[x], ro[x]) for x in rg if rg[x] != ro[x] and x != "out"})
            off += ro["consumed"]
            if ro["ret"] in (1, 2, -3):
                break
            idle = idle + 1 if ro["consumed"] == 0 and ro["produced"] == 0 else 0
            if idle > 6 and off >= len(data):
                break
        g.end()
        o.end()
    assert ncalls > 500


def test_zlib_abi_one_shot_fast_path(zs):
    """A fresh stream offered whole (>= 1 MiB) goes through the batch pipeline;
    the call's results still equal zlib's single inflate() call."""
    L = ctypes.CDLL(zs.LIB_PATH)
    L.inflateInit2_.argtypes = [ctypes.POINTER(libz_ref.ZStream), ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.inflate.argtypes = [ctypes.POINTER(libz_ref.ZStream), ctypes.c_int]
    L.inflateEnd.argtypes = [ctypes.POINTER(libz_ref.ZStream)]
    raw = corpus.stream(9, 6 << 20)
    for wb in (-15, 15, 31, -16):  # -16: deflate64 (inflate9_process), block-parallel too
        data = _comp(raw, wb) if wb != -16 else zs.deflate_batch([raw], -16, 6)[0][0]
        for out_len, fl in ((len(raw) + 10, 4), (len(raw), 0), (len(raw) // 2, 0), (len(raw) // 2, 4)):
            g, o = _GpuZ(L, wb), O.Stream(wb)
            rg, ro = g.call(data, out_len, fl), o.call(data, out_len, fl)
            assert rg == ro, (wb, out_len, fl)
            if ro["ret"] == 0:  # continue from a FULL stop through the resumable path
                rg, ro = g.call(data[ro["consumed"]:], 1 << 23, 4), o.call(data[ro["consumed"]:], 1 << 23, 4)
                assert rg == ro
            g.end()
            o.end()


def test_handle_output_space_small_large_small(zs):
    """One inflate handle whose calls offer small, then > 4 MiB, then small output
    space: the large call's output goes back through a pinned staging buffer
    that grows (reallocates) past the mapped one, and the next small call must
    use the new buffer's device view (a stale view would write freed memory).
    Every call's (produced, ret, last_consumed) and bytes equal the oracle's."""
    raw = corpus.stream(9, 12 << 20)
    comp = _comp(raw, -15)
    L = zs.lib()
    h = L.inflate_new()
    assert L.inflate_init_raw(h) == 0
    ref = O.Stream(-15)
    ib = ctypes.create_string_buffer(comp, len(comp))
    off, got, exp = 0, bytearray(), bytearray()
    plan = [(4096, 65536), (4096, 65536), (600 << 10, 8 << 20), (4096, 65536), (4096, 65536),
            (900 << 10, 6 << 20), (2048, 1000), (65536, 65536)]
    k = 0
    while True:
        n_in, n_out = plan[k % len(plan)]
        k += 1
        n_in = min(n_in, len(comp) - off)
        ob = ctypes.create_string_buffer(max(n_out, 1))
        r = L.inflate_process(h, ctypes.addressof(ib) + off, n_in, ctypes.addressof(ob), n_out, 0)
        prod, code, cons = r & 0xffffff, ((r >> 24) & 0xff), L.inflate_last_consumed(h)
        code = code - 256 if code & 0x80 else code
        e = ref.call(comp[off:off + n_in], n_out, 0)
        assert (prod, code, cons) == (len(e["out"]), e["ret"], e["consumed"]), (k, n_in, n_out, e["ret"])
        got += ob.raw[:prod]
        exp += e["out"]
        off += cons
        if code != 0:
            break
    assert code == 1 and bytes(got) == bytes(exp) == raw
    assert L.inflate_end(h) == 0


def test_persistent_worker_relaunch_and_reset(zs):
    """The persistent worker leaves after ZS_PK_IDLE_US (2 ms) without posts and
    the next call relaunches it: calls spaced 20 ms apart each find the launch
    gone.  inflateReset between two streams on the same handle (its device state
    set up again by the next call, on the worker's workgroup) and a gzip stream
    (header call on the batch path, the rest on the worker) keep every call
    equal to the oracle's."""
    import time
    L = zs.lib()
    prev = zs.stream_persist(True)
    try:
        raw = corpus.stream(33, 600000)
        for wb in (-15, 31):
            comp = _comp(raw, wb)
            h = L.inflate_new()
            assert (L.inflate_init_raw if wb < 0 else L.inflate_init_gzip)(h) == 0
            for rep in range(2):  # the second pass after a reset (init again on the same handle)
                if rep:
                    assert (L.inflate_init_raw if wb < 0 else L.inflate_init_gzip)(h) == 0
                ref = O.Stream(wb)
                st0 = zs.stream_stats()
                ib = ctypes.create_string_buffer(comp, len(comp))
                off, got, k, naps = 0, bytearray(), 0, 0
                while True:
                    if k % 3 == 2:
                        time.sleep(0.02)
                        naps += 1
                    k += 1
                    n_in = min(32768, len(comp) - off)
                    ob = ctypes.create_string_buffer(65536)
                    r = L.inflate_process(h, ctypes.addressof(ib) + off, n_in, ctypes.addressof(ob), 65536, 0)
                    prod, code, cons = r & 0xffffff, ((r >> 24) & 0xff), L.inflate_last_consumed(h)
                    code = code - 256 if code & 0x80 else code
                    e = ref.call(comp[off:off + n_in], 65536, 0)
                    assert (prod, code, cons) == (len(e["out"]), e["ret"], e["consumed"]), (wb, rep, k)
                    assert ob.raw[:prod] == e["out"]
                    got += ob.raw[:prod]
                    off += cons
                    if code != 0:
                        break
                assert code == 1 and bytes(got) == raw
                st1 = zs.stream_stats()
                assert st1["pk_calls"] - st0["pk_calls"] >= k - 1
                assert st1["pk_launches"] - st0["pk_launches"] >= naps
            assert L.inflate_end(h) == 0
    finally:
        zs.stream_persist(prev)


def test_more_handles_than_worker_mailboxes(zs):
    """80 handles at once on 80 threads -- more than the persistent worker's 64
    mailboxes (ZS_PK_WGS), plus deflate64 handles, which it never takes: the
    handles that get a mailbox run on the worker, the rest on batch launches,
    concurrently.  Every trace and output equals the oracle's."""
    from concurrent.futures import ThreadPoolExecutor
    rng = random.Random(21)
    cases = []
    for k in range(72):
        data = corpus.stream(40 + k % 8, 120000 + 997 * k)
        wb = (-15, 15, 31)[k % 3]
        cases.append((_comp(data, wb, 1 + k % 9), wb))
    for name in ("100k_lines", "zeros_100k", "payload_64k", "rand_block_gap"):
        cases += [(fixture(name), -16)] * 2
    rng.shuffle(cases)
    prev = zs.stream_persist(True)
    try:
        before = zs.stream_stats()
        with ThreadPoolExecutor(len(cases)) as ex:
            got = list(ex.map(lambda c: zs.js_schedule(c[0], FMT[c[1]], 32768), cases))
        after = zs.stream_stats()
    finally:
        zs.stream_persist(prev)
    bad = []
    for i, ((data, wb), (tr, out)) in enumerate(zip(cases, got)):
        etr, eout = O.js_schedule(data, 32768, wb)
        if tr != etr or out != eout:
            bad.append((i, wb, tr[:200], etr[:200]))
    assert not bad, bad[:3]
    assert after["pk_calls"] > before["pk_calls"]  # the worker took calls
    assert after["calls"] > before["calls"]        # and so did batch launches (headers, deflate64, extra handles)


def test_persistent_worker_idle_exit_does_not_strand_a_handle(zs):
    """one handle makes large calls (2 MiB in, ~8 MiB out: ~30 ms on
    its workgroup) while another pauses longer than the worker's idle time
    (ZS_PK_IDLE_US, 2 ms) between small calls.  During a large call nobody
    posts, so the small handle's workgroup leaves idle; its next call must not
    wait for the launch's whole life (ZS_PK_LIFE_MS, 250 ms) behind the large
    handle's busy workgroup: leaving idle closes the launch, the busy
    workgroup leaves after its call, and the waiter relaunches.  Both streams
    decode exactly; no small call waits 120 ms."""
    import threading
    import time
    L = zs.lib()
    prev = zs.stream_persist(True)
    big_raw = corpus.stream(34, 24 << 20)
    big = _comp(big_raw, -15)
    small_raw = corpus.stream(35, 1 << 20)
    small = _comp(small_raw, -15)
    res, lat = {}, []

    def run(comp, n_in, n_out, nap, key):
        h = L.inflate_new()
        assert L.inflate_init_raw(h) == 0
        ib = ctypes.create_string_buffer(comp, len(comp))
        off, got = 0, bytearray()
        while True:
            if nap:
                time.sleep(nap)
            n = min(n_in, len(comp) - off)
            ob = ctypes.create_string_buffer(n_out)
            t0 = time.perf_counter()
            r = L.inflate_process(h, ctypes.addressof(ib) + off, n, ctypes.addressof(ob), n_out, 0)
            if nap:
                lat.append(time.perf_counter() - t0)
            prod, code = r & 0xffffff, (r >> 24) & 0xff
            got += ob.raw[:prod]
            off += L.inflate_last_consumed(h)
            if code != 0:
                break
        res[key] = (code, bytes(got))
        assert L.inflate_end(h) == 0

    try:
        tb = threading.Thread(target=run, args=(big, 2 << 20, 8 << 20, 0, "big"))
        tb.start()
        time.sleep(0.05)
        run(small, 32768, 65536, 0.003, "small")
        tb.join()
    finally:
        zs.stream_persist(prev)
    assert res["big"] == (1, big_raw) and res["small"] == (1, small_raw)
    assert max(lat) < 0.12, sorted(lat)[-5:]


_LIFE_CHILD = r"""
import json, sys, time, zlib
import torch  # noqa: F401  (the library binds torch's HIP runtime, as in conftest)
import corpus, zstreams
raw = corpus.stream(36, 12 << 20)
c = zlib.compressobj(6, zlib.DEFLATED, -15)
comp = c.compress(raw) + c.flush()
zstreams.stream_persist(True)
s0 = zstreams.stream_stats()
t = time.perf_counter()
tr, out = zstreams.js_schedule(comp, "deflate-raw", 65536)
el = time.perf_counter() - t
s1 = zstreams.stream_stats()
print(json.dumps({"ok": out == raw, "trace": tr, "comp_len": len(comp), "seconds": el,
                  "pk_launches": s1["pk_launches"] - s0["pk_launches"], "pk_calls": s1["pk_calls"] - s0["pk_calls"]}))
"""


def test_persistent_worker_life_expiry_relaunch(zs):
    """VERDICT r4 item 4 (the 3.4-3.6 k aggregate runs held a relaunch of the
    worker in their timed region): the launch leaves once ZS_PK_LIFE_MS old
    and the calls posted meanwhile wait for the relaunch; waiters now look for
    it every 50 us once the launch is past its life.  In a child process with
    a 10 ms life, one handle decodes 12 MiB of line text on the JS schedule
    through many life expiries: every relaunch happens, the trace and output
    equal the oracle's, and the run is not slower than ~1 ms per relaunch over
    the same decode with the default life."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([here, os.path.join(os.path.dirname(here), "zlib-streams_amd"),
                                         env.get("PYTHONPATH", "")])

    def child(life_ms):
        e = dict(env, ZS_PK_LIFE_MS=str(life_ms))
        r = subprocess.run([sys.executable, "-c", _LIFE_CHILD], env=e, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    short, base = child(10), child(250)
    raw = corpus.stream(36, 12 << 20)
    comp = _comp(raw, -15)
    etr, eout = O.js_schedule(comp, 65536, -15)
    assert eout == raw
    for d in (short, base):
        assert d["ok"] and d["comp_len"] == len(comp) and d.pop("trace") == etr
    assert short["pk_launches"] >= 4, short
    # wall-clock bound with a margin for host scheduling: the bug it
    # guards against stranded posted calls for ~1 ms (tens under a tracer) per relaunch
    assert short["seconds"] < base["seconds"] + 0.005 * short["pk_launches"] + 0.25, (short, base)


def test_persistent_worker_small_call_after_large_does_not_oversleep(zs):
    """the waiter sleeps most of the handle's last call on
    the worker before polling, scaled down by this call's input (never up), so
    a 1 KiB call right after a 512 KiB one (up to 4 MiB out, milliseconds on the
    worker) does not sleep for milliseconds.  One handle alternates 512 KiB and
    1 KiB calls over 24 MiB of line text: the output equals the input and no
    small call takes 5 ms (the median under 1 ms)."""
    import time
    L = zs.lib()
    prev = zs.stream_persist(True)
    raw = corpus.stream(37, 24 << 20)
    comp = _comp(raw, -15)
    lat = []
    try:
        h = L.inflate_new()
        assert L.inflate_init_raw(h) == 0
        ib = ctypes.create_string_buffer(comp, len(comp))
        ob = ctypes.create_string_buffer(4 << 20)  # (calls within the 4 MiB staging stay on the worker)
        off, got, k = 0, bytearray(), 0
        while True:
            n = min((512 << 10) if k % 2 == 0 else 1024, len(comp) - off)
            t0 = time.perf_counter()
            r = L.inflate_process(h, ctypes.addressof(ib) + off, n, ctypes.addressof(ob), len(ob), 0)
            dt = time.perf_counter() - t0
            if k % 2 == 1:
                lat.append(dt)
            k += 1
            prod, code = r & 0xffffff, (r >> 24) & 0xff
            got += ob.raw[:prod]
            off += L.inflate_last_consumed(h)
            if code != 0:
                break
        assert L.inflate_end(h) == 0
    finally:
        zs.stream_persist(prev)
    assert code == 1 and bytes(got) == raw
    lat.sort()
    # the oversleep this guards against is >= 1.25 ms on EVERY small call (5/8
    # of the 512 KiB call's worker time, capped at 2 ms): the median tells;
    # single outliers are host scheduling (margin on the maximum)
    assert len(lat) >= 5 and lat[-1] < 0.05 and lat[len(lat) // 2] < 0.001, lat
