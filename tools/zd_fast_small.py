"""deflate_fast (levels 1..3) smoke: growing inputs, wall time per call, bytes
vs host zlib (for a first look on the box before the full tests)."""
import os, sys, time, zlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus, zstreams
for name, sid in (("zipf", 0), ("lines", 33)):
    for n in (1000, 65536, 1 << 20, 4 << 20):
        d = corpus.stream(sid, n)
        for lv in (1, 3):
            t0 = time.perf_counter()
            (comp, info), = zstreams.deflate_batch([d], -15, lv)
            dt = time.perf_counter() - t0
            c = zlib.compressobj(lv, zlib.DEFLATED, -15, 8, 0)
            ref = c.compress(d) + c.flush()
            print(f"{name} n={n} L{lv}: {dt*1e3:.1f} ms {n/dt/2**20:.2f} MiB/s ret={info['ret']} same={comp == ref} "
                  f"len={len(comp)} zlib={len(ref)}", flush=True)
