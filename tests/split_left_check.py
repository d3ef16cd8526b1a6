"""Run by test_gpu_inflate.py::test_split_leftovers_from_start with ZS_SPLIT_LEFT=1
(read once per process, hence a child process): every unit the split parse walks
is sent to the leftover kernel as a failed split, which must decode it again
from the unit's start -- its header included, since the split parse's unit
headers keep no zlib-layout tables (round 6).  Exit 0 when every job matches
the oracle."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "zlib-streams_amd"))

import corpus  # noqa: E402
import oracle_lib as O  # noqa: E402
import zstreams  # noqa: E402


def main():
    raws, comps = corpus.batch(30, 4, 4 << 20, level=6, wbits=-15, nthreads=4)  # Zipf 30, 31, line text 32, 33
    cases = [(c.tobytes(), -15, 4 << 20) for c in comps]
    cases.append((cases[2][0][: len(cases[2][0]) // 2], -15, 4 << 20))  # truncated mid-stream
    got = zstreams.inflate_batch([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases], parse="split")
    st = zstreams.last_stats()
    bad = 0
    for k, (c, (out, info)) in enumerate(zip(cases, got)):
        eo, ei = O.oneshot(c[0], c[1], c[2])
        if out != eo or info != ei:
            bad += 1
            print("mismatch", k, info, ei, len(out), len(eo))
    bad += sum(bytes(got[k][0]) != bytes(raws[k]) for k in range(4))  # the generator's bytes too
    print("stats", st, "bad", bad)
    return 1 if bad or st["parse"] != "split" else 0


if __name__ == "__main__":
    sys.exit(main())
