import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "zlib-streams_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

# torch first: libzstreams_mi355x.so then binds torch's HIP runtime (same
# soname) instead of loading a second one that torch cannot initialise after
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
