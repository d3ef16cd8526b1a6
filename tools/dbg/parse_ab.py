"""Unit records (ZS_DEBUG_CHUNKS=2 dump) for one small chunked batch; run once
per ZS_PARSE mode and diff the outputs."""
import os, sys, zlib
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "zlib-streams_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import corpus, zstreams
raw = corpus.stream(3, 1 << 20)
c = zlib.compressobj(6, zlib.DEFLATED, -15); comp = c.compress(raw) + c.flush()
(out, info), = zstreams.inflate_batch([comp], -15, [len(raw)])
print(os.environ.get("ZS_PARSE"), info, out == raw, zstreams.last_stats(), flush=True)
