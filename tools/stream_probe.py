"""One handle through the reference JS schedule (bench.py stream leg, one-handle
part): per-call time, and with the profiling build (ZS_LIB=...prof.so) the
stream kernel's in-kernel counters (zs_kprof.h KP_W_*)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import bench  # noqa: E402
import corpus  # noqa: E402
import zstreams  # noqa: E402

L = zstreams.lib()
mib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
sid = int(sys.argv[2]) if len(sys.argv) > 2 else 32
if len(sys.argv) > 3 and sys.argv[3] == "random":  # the perf harness's data: stored blocks
    import zlib
    raw = np.random.default_rng(sid).integers(0, 256, mib << 20, dtype=np.uint8)
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = np.frombuffer(co.compress(raw.tobytes()) + co.flush(), dtype=np.uint8)
else:
    r, c = corpus.batch(sid, 1, mib << 20, level=6, wbits=-15, nthreads=1)
    raw, comp = r[0], c[0]
out = np.empty((mib << 20) + 65536, dtype=np.uint8)
names = ["waves", "cyc_total", "windows", "empty", "syms", "bytes", "batches", "jumps", "cyc_decode", "cyc_chain",
         "cyc_expand", "serial", "cyc_window", "cyc_compose", "cyc_walk", "cyc_pre", "cyc_post", "cyc_tables", "steps", "redos"]
for rep in range(2):
    zstreams.kprof_read(reset=True)
    s0 = zstreams.stream_stats()
    h = L.inflate_new()
    L.inflate_init_raw(h)
    t0 = time.perf_counter()
    got, code, calls = bench._js_schedule_loop(L, h, comp, out, 65536)
    dt = time.perf_counter() - t0
    L.inflate_end(h)
    ok = got == len(raw) and np.array_equal(out[:len(raw)], raw)
    k = zstreams.kprof_read(reset=True)
    s1 = zstreams.stream_stats()
    n = max(1, s1["pk_calls"] - s0["pk_calls"])
    print(f"rep {rep}: {len(raw) / dt / 2**20:.1f} MiB/s, {calls} calls, {dt * 1e6 / calls:.1f} us/call, ok={ok}; "
          f"worker {s1['pk_calls'] - s0['pk_calls']} calls, {(s1['pk_busy_ns'] - s0['pk_busy_ns']) / n / 1e3:.1f} us busy, "
          f"{(s1['pk_wait_ns'] - s0['pk_wait_ns']) / n / 1e3:.1f} us wait per call", flush=True)
    if len(k) >= 96:
        w = dict(zip(names, k[64:64 + len(names)]))
        print("  kprof:", w, flush=True)
        if w["waves"]:
            print(f"  per call: cyc_total {w['cyc_total'] / w['waves']:.0f}, window cyc {w['cyc_window'] / w['waves']:.0f} "
                  f"({w['windows'] / w['waves']:.1f} windows, {w['empty'] / w['waves']:.1f} empty), serial steps "
                  f"{w['serial'] / w['waves']:.0f}; per window: decode {w['cyc_decode'] / max(1, w['windows']):.0f} chain "
                  f"{w['cyc_chain'] / max(1, w['windows']):.0f} expand {w['cyc_expand'] / max(1, w['windows']):.0f} cyc, "
                  f"{w['syms'] / max(1, w['windows'] - w['empty']):.0f} syms, {w['jumps'] / max(1, w['windows']):.1f} jump rounds",
                  flush=True)
            nw = max(1, w["windows"])
            print(f"  per window: compose {w['cyc_compose'] / nw:.0f} compose+walk {w['cyc_walk'] / nw:.0f} pre {w['cyc_pre'] / nw:.0f} "
                  f"post {w['cyc_post'] / nw:.0f}; per call: tables {w['cyc_tables'] / w['waves']:.0f}; wave-0 walk steps "
                  f"{w['steps'] / nw:.1f}, redos {w['redos'] / nw:.2f} per window", flush=True)
