"""Deflate stream surface (CompressionStreamZlib: handle ABI deflate_process,
the reference's JS schedule: 64 KiB writes, <= 32 KiB per call, 64 KiB out,
Z_FINISH drain) on one handle: wall-clock MiB/s of input, bytes checked against
host zlib driven the same way, host zlib's rate beside it."""
import os, sys, time, zlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus, zstreams
n = (int(sys.argv[1]) if len(sys.argv) > 1 else 16) << 20
import numpy as np
kinds = os.environ.get("KINDS", "zipf,lines").split(",")
for name, sid in (("zipf", 0), ("lines", 33), ("random", -1)):
    if name not in kinds:
        continue
    d = corpus.stream(sid, n) if sid >= 0 else np.random.default_rng(7).integers(0, 256, n, dtype=np.uint8).tobytes()
    for lv in [int(x) for x in os.environ.get("LEVELS", "6,1").split(",")]:
        zstreams.compress(d[:1 << 20], "deflate-raw", lv, 65536)  # warm
        t0 = time.perf_counter()
        got = zstreams.compress(d, "deflate-raw", lv, 65536)
        dt = time.perf_counter() - t0
        c = zlib.compressobj(lv, zlib.DEFLATED, -15, 8, 0)
        t1 = time.perf_counter()
        ref = b"".join(c.compress(d[o:o + 32768]) for o in range(0, len(d), 32768)) + c.flush()
        dz = time.perf_counter() - t1
        print(f"{name} L{lv}: GPU stream {n / dt / 2**20:.1f} MiB/s, host zlib {n / dz / 2**20:.1f} MiB/s, "
              f"same={got == ref}", flush=True)
