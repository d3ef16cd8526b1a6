"""Debug: random 4 MiB + line text 4 MiB through the chunked path with ZS_DEBUG_CHUNKS=2."""
import os, sys, zlib
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "zlib-streams_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import corpus, zstreams
rng = np.random.default_rng(11)
raw = rng.integers(0, 256, 4 << 20, dtype=np.uint8).tobytes() + corpus.stream(41, 4 << 20)
c = zlib.compressobj(6, zlib.DEFLATED, -15)
comp = c.compress(raw) + c.flush()
got = zstreams.inflate_batch([comp], -15, [len(raw)])
print("result", got[0][1], got[0][0] == raw, zstreams.last_stats(), file=sys.stderr)
