"""One stream past one launch's limits (> 2^29 compressed bytes): C2 text,
GPU-encoded (zlib-identical L6, raw; and deflate64), decoded in pieces
(zs_capi.cpp run_pieces).  Prints MiB/s of output and checks the bytes."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import corpus, zstreams
dev = torch.device("cuda", 0)
nb = int(os.environ.get("LONG_MIB", "2560")) << 20
part = 64 << 20
src = torch.empty(nb, dtype=torch.uint8, device=dev)
for k in range(nb // part):  # C2-like text: Zipf / line streams, 64 MiB each
    s = corpus.stream(40 + k % 64, part)
    src[k * part:(k + 1) * part].copy_(torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy()))
torch.cuda.synchronize()
for name, wb, lvl in (("raw deflate, zlib-identical L6", -15, 6), ("deflate64 L6", -16, 6)):
    cap = zstreams.deflate_bound(nb, wb)
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    (di,) = zstreams.deflate_batch_device([src.data_ptr()], [nb], [comp.data_ptr()], [cap], wb, level=lvl)
    clen = di["total_out"]
    out = torch.empty(nb + 256, dtype=torch.uint8, device=dev)
    f = lambda: zstreams.inflate_batch_device([comp.data_ptr()], [clen], [out.data_ptr()], [nb + 256], wb)[0]
    r = f()
    torch.cuda.synchronize()
    ok = r["ret"] == 1 and r["total_in"] == clen and r["total_out"] == nb and bool(torch.equal(out[:nb], src))
    st = zstreams.last_stats()
    t0 = time.perf_counter()
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print(f"{name}: {nb >> 20} MiB out, {clen / 2**20:.0f} MiB compressed (> 512 MiB: {clen > 1 << 29}): "
          f"{nb / dt / 2**20:.0f} MiB/s, {dt * 1e3:.1f} ms, ok={ok}, {st}", flush=True)
    del comp, out
