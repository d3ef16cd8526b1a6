"""In-kernel counters of the serial wave decoder (profiling build).

usage (GPU box): ZS_LIB=$PWD/zlib-streams_amd/libzstreams_mi355x_prof.so python3 tools/serial_kprof.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "zlib-streams_amd")]
import torch  # noqa: E402,F401
import zstreams  # noqa: E402
from golden.make_manifest import fixture  # noqa: E402

NAMES = ["waves", "cyc_total", "windows", "empty", "syms", "bytes", "batches", "jumps", "cyc_decode", "cyc_chain",
         "cyc_expand", "serial_syms", "cyc_window"]


def main():
    for name in ("100k_lines", "10k_lines", "payload_64k"):
        zstreams.kprof_read(reset=True)
        zstreams.inflate_batch([fixture(name)], -16, [4 << 20])
        c = zstreams.kprof_read(reset=True)
        if len(c) < 80:
            sys.exit("no counters: ZS_LIB must point at libzstreams_mi355x_prof.so")
        d = {NAMES[i]: c[64 + i] for i in range(len(NAMES))}
        w = max(d["windows"] - d["empty"], 1)
        d.update({"syms_per_window": d["syms"] / w, "bytes_per_window": d["bytes"] / w,
                  "decode_cyc_per_window": d["cyc_decode"] / max(d["windows"], 1),
                  "chain_cyc_per_window": d["cyc_chain"] / max(d["windows"], 1),
                  "expand_cyc_per_batch": d["cyc_expand"] / max(d["batches"], 1),
                  "jumps_per_batch": d["jumps"] / max(d["batches"], 1),
                  "window_frac": d["cyc_window"] / max(d["cyc_total"], 1)})
        print(name, json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items()}), flush=True)


if __name__ == "__main__":
    main()
