"""GPU zlib-identical deflate vs host zlib on a few inputs (debug driver)."""
import os, sys, zlib, random, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "zlib-streams_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import corpus, zstreams
rng = random.Random(3)
cases = [b"", b"a", b"abc", b"hello hello hello world", bytes(100000), bytes(rng.getrandbits(8) for _ in range(70000)),
         corpus.stream(0, 1 << 20), corpus.stream(33, 1 << 20),
         bytes(rng.getrandbits(8) for _ in range(40000)) + corpus.stream(2, 300000)]
bad = 0
for lv in (6, 4, 9):
    for wb in (-15, 15, 31):
        t = time.time()
        got = zstreams.deflate_batch(cases, wb, lv)
        for i, (d, (c, info)) in enumerate(zip(cases, got)):
            co = zlib.compressobj(lv, zlib.DEFLATED, wb, 8, 0)
            ref = co.compress(d) + co.flush()
            if c != ref:
                bad += 1
                k = next((j for j in range(min(len(c), len(ref))) if c[j] != ref[j]), min(len(c), len(ref)))
                print("MISMATCH level", lv, "wbits", wb, "case", i, "len", len(d), "sizes", len(c), len(ref), "first diff", k, info, flush=True)
        print("level", lv, "wbits", wb, "done", round(time.time() - t, 2), flush=True)
print("bad", bad)
