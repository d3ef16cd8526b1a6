"""Unit size distribution of the block-parallel path on C2 streams: tokens per
unit, blocks per verified unit (from its span), the longest units.  Runs one
batch of a few 64 MiB streams with ZS_DEBUG_CHUNKS=2 (per-unit dump on
stderr, captured through a pipe)."""
import os, sys, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import corpus, zstreams
    ids = [0, 1, 32, 33]
    comps = []
    for i in ids:
        _, c = corpus.batch(i, 1, 64 << 20, level=6, wbits=-15, nthreads=1)
        comps.append(c[0].tobytes())
    got = zstreams.inflate_batch(comps, -15, [(64 << 20) + 64] * len(comps))
    print("ok", all(g[1]["ret"] == 1 for g in got), zstreams.last_stats(), flush=True)
    sys.exit(0)
env = dict(os.environ, ZS_DEBUG_CHUNKS="2")
r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True)
print(r.stdout.strip())
units = []
for line in r.stderr.splitlines():
    if line.startswith("  unit "):
        f = line.split()
        d = {f[k]: f[k + 1] for k in range(0, len(f) - 1, 2)}
        units.append({k: int(v) for k, v in d.items() if v.lstrip("-").isdigit()})
chain = [u for u in units if u.get("chain") == 1]
print("units", len(units), "in chain", len(chain))
if chain:
    nt = sorted(u["ntok"] for u in chain)
    n = len(nt)
    print("tokens per chain unit: mean %.0f p50 %d p90 %d p99 %d max %d" % (sum(nt) / n, nt[n // 2], nt[int(n * .9)], nt[int(n * .99)], nt[-1]))
    big = sorted(chain, key=lambda u: -u["ntok"])[:12]
    for u in big:
        print("  ord %d start %d stop %d end %d span_bits %d ntok %d n_out %d" % (
            u["ord"], u["start"], u["stop"], u["end"], u["end"] - u["start"], u["ntok"], u["n_out"]))
    # how far past its stop did each unit run (bits), a sign of a missed start
    over = sorted((u["end"] - u["stop"]) for u in chain if u["stop"] != 0xffffffff and u["stop"] != 4294967295)
    if over:
        m = len(over)
        print("end - stop bits: p50 %d p90 %d p99 %d max %d" % (over[m // 2], over[int(m * .9)], over[int(m * .99)], over[-1]))
