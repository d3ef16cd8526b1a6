import os, sys, zlib
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "zlib-streams_amd"))
import zstreams
for data in (b"", b"x"):
    for wb in (-15, 15, 31):
        for lv in (6, 1):
            c, info = zstreams.deflate_batch([data], wb, lv)[0]
            co = zlib.compressobj(lv, zlib.DEFLATED, wb, 8, 0)
            ref = co.compress(data) + co.flush()
            print(repr(data), wb, lv, c.hex(), ref.hex(), c == ref, info)
    print("handle:", zstreams.compress(data, "gzip").hex())
