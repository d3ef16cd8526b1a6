"""Debug: deflate64 chunked (two streams) with ZS_DEBUG_CHUNKS=2; select with argv[1]."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "zlib-streams_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import corpus, zstreams
rng = np.random.default_rng(9)
blk = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
which = int(os.environ.get("CASE", "1"))
d = [corpus.stream(3, 24 << 20), corpus.stream(35, 12 << 20) + bytes(3 << 20) + blk * 40 + corpus.stream(4, 2 << 20)][which]
c = zstreams.deflate_batch([d], -16, 6)[0][0]
got = zstreams.inflate_batch([c], -16, [len(d)])
print("result", got[0][1], got[0][0] == d, zstreams.last_stats(), file=sys.stderr)
