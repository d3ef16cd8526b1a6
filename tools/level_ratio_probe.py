"""Per-level compression ratio of the GPU deflate against host zlib (round-2 verdict item 9).

Two C2-corpus streams (one Zipf text, one line text; 16 MiB each), raw deflate (-15), levels
0..9: GPU default mode (zlib's bytes at levels 4..9), GPU fast mode (ZS_F_DEFLATE_FAST), and
host zlib (memLevel 8, Z_DEFAULT_STRATEGY).  Every GPU output is inflated by host zlib and
compared with the input.  Prints one JSON object.

usage (GPU box): python3 tools/level_ratio_probe.py [--mib 16]
"""
import argparse, json, os, sys, time, zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=16)
    a = ap.parse_args()
    import corpus
    import zstreams
    raws, _ = corpus.batch(31, 2, a.mib << 20, 6, -15, 2, False)  # ids 31 (Zipf), 32 (lines)
    raws = [bytes(r) for r in raws]
    total = sum(len(r) for r in raws)
    rows = []
    for lv in range(10):
        row = {"level": lv}
        for mode, fast in (("gpu", False), ("gpu_fast", True)):
            t = time.time()
            out = zstreams.deflate_batch(raws, -15, lv, fast=fast)
            dt = time.time() - t
            size = 0
            for r, (c, info) in zip(raws, out):
                if info["ret"] != 1 or zlib.decompress(c, -15) != r:
                    raise SystemExit(f"level {lv} {mode}: bad round trip {info}")
                size += len(c)
            row[mode + "_ratio"] = round(total / size, 4)
            row[mode + "_bytes"] = size
        zsize = 0
        zbytes = []
        for r in raws:
            co = zlib.compressobj(lv, zlib.DEFLATED, -15, 8)
            z = co.compress(r) + co.flush()
            zbytes.append(z)
            zsize += len(z)
        row["zlib_ratio"] = round(total / zsize, 4)
        row["zlib_bytes"] = zsize
        out = zstreams.deflate_batch(raws, -15, lv)
        row["gpu_bytes_identical_to_zlib"] = all(c == z for (c, _), z in zip(out, zbytes))
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps({"input": f"2 x {a.mib} MiB (C2 corpus ids 31 Zipf, 32 lines), raw deflate -15", "levels": rows}))


if __name__ == "__main__":
    main()
