"""Source hash of libzstreams_mi355x.so.

SHA-256 over the library's sources (every csrc/*.hip, *.h, *.cpp, the
Makefile, exports.map and the public header, each as name NUL content, in
sorted name order) and the `hipcc --version` text.  The Makefile stamps it into
the library (zs_source_hash(), zs_version()); tools/pmc_traffic.py records it
beside the PMC traffic so bench.py can tie the traffic figure to the sources a
library was built from, not to one binary (hipcc output is not bit-reproducible).
Run from anywhere: prints the hash.
"""
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def files():
    names = sorted(set(glob.glob("*.hip", root_dir=HERE) + glob.glob("*.h", root_dir=HERE) +
                       glob.glob("*.cpp", root_dir=HERE)))
    return names + ["Makefile", "exports.map", os.path.join("..", "..", "include", "zstreams_mi355x.h")]


def source_hash(hipcc=os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")):
    h = hashlib.sha256()
    for name in files():
        h.update(name.encode() + b"\0")
        with open(os.path.join(HERE, name), "rb") as f:
            h.update(f.read())
    try:
        ver = subprocess.run([hipcc, "--version"], capture_output=True, timeout=60).stdout
    except (OSError, subprocess.SubprocessError):
        ver = b"hipcc unavailable"
    h.update(ver)
    return h.hexdigest()


if __name__ == "__main__":
    sys.stdout.write(source_hash() + "\n")
