"""Stage split of ONE large stream on the block-parallel path: a 64 MiB GPU-encoded
deflate64 stream and a 64 MiB host-zlib raw deflate stream (C2 text)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import corpus, zstreams
nb = 64 << 20
dev = torch.device("cuda", 0)
raw = corpus.stream(40, nb // 2) + corpus.stream(7, nb // 2)
d64c = zstreams.deflate_batch([raw], -16, 6)[0][0]
r2, c2 = corpus.batch(40, 1, nb, level=6, wbits=-15, nthreads=1)
for name, comp, wb, ref in (("deflate64 GPU-encoded", d64c, -16, raw), ("raw deflate zlib L6", c2[0].tobytes(), -15, r2[0].tobytes())):
    d_in = torch.from_numpy(np.frombuffer(comp, dtype=np.uint8).copy()).to(dev)
    d_out = torch.empty(nb, dtype=torch.uint8, device=dev)
    f = lambda: zstreams.inflate_batch_device([d_in.data_ptr()], [len(comp)], [d_out.data_ptr()], [nb], wb)[0]
    r = f(); torch.cuda.synchronize()
    ok = r["ret"] == 1 and bytes(d_out.cpu().numpy()) == ref
    zstreams.profile(True)
    t0 = time.perf_counter()
    for _ in range(5): f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    k_ms, b_ms, k_n = zstreams.profile_read()
    st = zstreams.profile_stages()
    zstreams.profile(False)
    print(f"{name}: {nb / dt / 2**20:.0f} MiB/s {dt*1e3:.2f} ms ok={ok} {zstreams.last_stats()} "
          f"{ {k: round(v / k_n, 2) for k, v in st.items()} }", flush=True)
