"""GPU zlib-identical deflate probe: N x 64 MiB C2 streams (half Zipf, half
line text) resident in HBM, gzip level L, zlib-bytes mode; prints the stage
split and checks the bytes against host zlib.  Run under rocprofv3 for the
per-kernel split."""
import argparse, os, sys, time, zlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
ap = argparse.ArgumentParser()
ap.add_argument("--streams", type=int, default=16)
ap.add_argument("--mib", type=int, default=64)
ap.add_argument("--level", type=int, default=6)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
import numpy as np, torch
import corpus, zstreams
nb = a.mib << 20
ids = [i * 64 // a.streams if i < a.streams // 2 else 32 + (i - a.streams // 2) for i in range(a.streams)]
raws = []
comps = []
for i in ids:
    r, c = corpus.batch(i, 1, nb, level=a.level, wbits=-15, nthreads=1)
    raws.append(r[0]); comps.append(c[0])
dev = torch.device("cuda", 0)
d_in = torch.from_numpy(np.concatenate(raws)).to(dev)
bound = zstreams.deflate_bound(nb, 31)
slot = (bound + 4095) & ~4095
d_out = torch.empty(a.streams * slot, dtype=torch.uint8, device=dev)
ip = [d_in.data_ptr() + k * nb for k in range(a.streams)]
op = [d_out.data_ptr() + k * slot for k in range(a.streams)]
res = zstreams.deflate_batch_device(ip, [nb] * a.streams, op, [bound] * a.streams, 31, a.level)
torch.cuda.synchronize()
zstreams.profile(True)
t0 = time.perf_counter()
for _ in range(a.reps):
    res = zstreams.deflate_batch_device(ip, [nb] * a.streams, op, [bound] * a.streams, 31, a.level)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.reps
k_ms, stages, k_n = zstreams.profile_deflate()
zstreams.profile(False)
h = d_out.cpu().numpy()
ok = all(r["total_out"] == len(comps[k]) + 18 and np.array_equal(h[k * slot + 10:k * slot + r["total_out"] - 8], comps[k])
         for k, r in enumerate(res))
print(f"zlib-bytes deflate L{a.level}: {a.streams}x{a.mib} MiB  {a.streams * nb / dt / 2**20:.1f} MiB/s  "
      f"{dt * 1e3:.1f} ms/batch  identical={ok}  stages_ms={ {k: round(v / max(k_n, 1), 2) for k, v in stages.items()} }",
      flush=True)
