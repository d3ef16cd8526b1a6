"""The bench's aggregate stream leg alone (N handles on native threads, the
reference JS call schedule, tools/js_driver.c), for rocprofv3 runs:
    python3 tools/stream_agg_probe.py [handles] [MiB per handle]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus  # noqa: E402
import zstreams  # noqa: E402

nh = int(sys.argv[1]) if len(sys.argv) > 1 else 64
each = (int(sys.argv[2]) if len(sys.argv) > 2 else 4) << 20
rs, cs = corpus.batch(32, nh, each, level=6, wbits=-15, nthreads=16)
outs = [np.empty(each + 65536, dtype=np.uint8) for _ in range(nh)]
J = ctypes.CDLL(os.path.join(ROOT, "tools", "libzs_jsdrive.so"))
P, S = ctypes.POINTER, ctypes.c_size_t
J.zs_js_drive.restype = ctypes.c_double
J.zs_js_drive.argtypes = [ctypes.c_char_p, P(ctypes.c_void_p), P(S), P(ctypes.c_void_p), P(S), ctypes.c_int, S,
                          P(ctypes.c_uint64), P(ctypes.c_int), P(ctypes.c_uint64)]
cp = (ctypes.c_void_p * nh)(*[c.ctypes.data for c in cs])
cl = (S * nh)(*[len(c) for c in cs])
op = (ctypes.c_void_p * nh)(*[o.ctypes.data for o in outs])
oc = (S * nh)(*[len(o) for o in outs])
zstreams.lib()
names = ["waves", "cyc_total", "windows", "empty", "syms", "bytes", "batches", "jumps", "cyc_decode", "cyc_chain",
         "cyc_expand", "serial", "cyc_window", "cyc_compose", "cyc_walk", "cyc_pre", "cyc_post", "cyc_tables", "steps", "redos"]
for rep in range(2):
    zstreams.kprof_read(reset=True)
    prod, codes, ncalls = (ctypes.c_uint64 * nh)(), (ctypes.c_int * nh)(), ctypes.c_uint64(0)
    st0 = zstreams.stream_stats()
    tm = J.zs_js_drive(zstreams.LIB_PATH.encode(), cp, cl, op, oc, nh, 65536, prod, codes, ctypes.byref(ncalls))
    st1 = zstreams.stream_stats()
    ok = all(prod[k] == each and codes[k] == 1 and np.array_equal(outs[k][:each], rs[k]) for k in range(nh))
    la = st1["launches"] - st0["launches"]
    print(f"rep {rep}: {nh * each / tm / 2**20:.1f} MiB/s, {ncalls.value} calls, {la} launches "
          f"({ncalls.value / max(1, la):.1f} calls/launch), {tm * 1e3:.1f} ms, ok={ok}", flush=True)
    st = zstreams.stream_stats()
    print(f"  launch us avg {(st['launch_ns'] - st0['launch_ns']) / 1e3 / max(1, la):.1f}, kernel us avg "
          f"{(st['kernel_ns'] - st0['kernel_ns']) / 1e3 / max(1, la):.1f}", flush=True)
    k = zstreams.kprof_read(reset=True)
    if len(k) >= 96:
        w = dict(zip(names, k[64:64 + len(names)]))
        if w["waves"]:
            print(f"  kprof per call: cyc_total {w['cyc_total'] / w['waves']:.0f}, {w['windows'] / w['waves']:.1f} windows, "
                  f"window cyc {w['cyc_window'] / max(1, w['windows']):.0f} (decode {w['cyc_decode'] / max(1, w['windows']):.0f} "
                  f"chain {w['cyc_chain'] / max(1, w['windows']):.0f} expand {w['cyc_expand'] / max(1, w['windows']):.0f}), "
                  f"tables {w['cyc_tables'] / w['waves']:.0f}, syms/window {w['syms'] / max(1, w['windows']):.0f}", flush=True)
