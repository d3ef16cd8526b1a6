"""Timing probe of the serial wave decoder (deflate64 and resumable calls).

usage (GPU box): python tools/serial_probe.py
Prints per-case milliseconds and MiB/s of output; every output is checked
against the committed fixture hashes.
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "zlib-streams_amd")]
import torch  # noqa: E402,F401  (HIP runtime first, as in tests/conftest.py)
import zstreams  # noqa: E402
from golden.make_manifest import fixture  # noqa: E402

MAN = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))


def timed(fn, reps=3):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        r = fn()
    return (time.perf_counter() - t) / reps * 1e3, r


def device_batch(streams, cap):
    """Device-resident batch: returns (results, pipeline ms from HIP events)."""
    offs, o = [], 0
    for c in streams:
        offs.append(o)
        o += (len(c) + 255) & ~255
    buf = bytearray(o + 256)
    for c, of in zip(streams, offs):
        buf[of:of + len(c)] = c
    d_in = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    d_out = torch.empty(len(streams) * cap, dtype=torch.uint8, device="cuda")
    args = ([d_in.data_ptr() + of for of in offs], [len(c) for c in streams],
            [d_out.data_ptr() + k * cap for k in range(len(streams))], [cap] * len(streams), -16)
    zstreams.inflate_batch_device(*args)
    zstreams.profile(True)
    res = zstreams.inflate_batch_device(*args)
    ms, bms, n = zstreams.profile_read()
    zstreams.profile(False)
    return res, bms / max(n, 1), d_out


def main():
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    zstreams.set_stream(stream.cuda_stream)
    names = list(MAN["fixtures"])
    suite = [fixture(n) for n in names]
    outb = sum(MAN["fixtures"][n]["len"] for n in names)
    cap = 4 << 20
    for reps in (1, 64, 256):
        res, ms, d_out = device_batch(suite * reps, cap)
        host = d_out[:len(names) * cap].cpu().numpy().tobytes()
        for i, n in enumerate(names):
            o = host[i * cap:i * cap + res[i]["total_out"]]
            assert hashlib.sha256(o).hexdigest() == MAN["fixtures"][n]["sha256"], n
        print(f"d64 suite x{reps}: {len(names) * reps} streams {ms:.2f} ms (batch, HIP events) "
              f"{outb * reps / ms / 1e3 / 1.048576:.1f} MiB/s", flush=True)
    for n in ("100k_lines", "10k_lines"):
        res, ms, _ = device_batch([fixture(n)], cap)
        print(f"d64 {n} alone: {ms:.2f} ms {MAN['fixtures'][n]['len'] / ms / 1e3 / 1.048576:.1f} MiB/s", flush=True)
    for w in (4096, 32768):
        ms, (tr, out) = timed(lambda: zstreams.js_schedule(fixture("100k_lines"), "deflate64-raw", w), 2)
        print(f"stream ABI 100k_lines W={w}: {tr.count(chr(10))} calls {ms:.1f} ms "
              f"{len(out) / ms / 1e3 / 1.048576:.1f} MiB/s", flush=True)


if __name__ == "__main__":
    main()
