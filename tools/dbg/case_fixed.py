"""Debug: 16 MiB Z_FIXED stream through the chunked path with ZS_DEBUG_CHUNKS=2."""
import os, sys, zlib
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "zlib-streams_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import corpus, zstreams
raw = corpus.stream(12, 8 << 20) + corpus.stream(44, 8 << 20)
c = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_FIXED)
comp = c.compress(raw) + c.flush()
got = zstreams.inflate_batch([comp], -15, [len(raw)])
print("result", got[0][1], got[0][0] == raw, zstreams.last_stats(), file=sys.stderr)
