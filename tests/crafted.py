"""Hand-built raw-deflate streams with chosen dynamic Huffman codes (test
infrastructure only).

``long_literal_stream`` writes dynamic blocks (RFC 1951 §3.2.7, the layout
src/inflate.c:905-1033 reads) whose literal/length code puts ALL 256 literals,
end-of-block and length symbol 257 on 10-bit codes; lengths 258..266 take
2..9 bits so the code is complete.  Literal 0xFF then has the last 10-bit
literal code in canonical order, the case where a literal count capped at 255
would read it as the first length symbol of that length (end of block).
"""
import random


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def bits(self, v, n):  # LSB first
        self.acc |= (v & ((1 << n) - 1)) << self.n
        self.n += n
        while self.n >= 8:
            self.out.append(self.acc & 0xFF)
            self.acc >>= 8
            self.n -= 8

    def huff(self, code, n):  # Huffman codes go MSB first
        r = 0
        for _ in range(n):
            r = (r << 1) | (code & 1)
            code >>= 1
        self.bits(r, n)

    def finish(self):
        if self.n:
            self.out.append(self.acc & 0xFF)
        self.acc = self.n = 0
        return bytes(self.out)


def canonical(lens):
    """RFC 1951 §3.2.2 canonical codes: list of (code, len) per symbol."""
    mx = max(lens)
    count = [0] * (mx + 1)
    for L in lens:
        if L:
            count[L] += 1
    code, nxt = 0, [0] * (mx + 2)
    for L in range(1, mx + 1):
        code = (code + count[L - 1]) << 1 if L > 1 else 0
        nxt[L] = code
    out = []
    for L in lens:
        if L:
            out.append((nxt[L], L))
            nxt[L] += 1
        else:
            out.append((0, 0))
    return out


CLORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]

# literal/length code lengths: 0..257 at 10 bits, 258..266 at 2,2,3,..,9 bits
LIT_LENS = [10] * 258 + [2, 2, 3, 4, 5, 6, 7, 8, 9] + [0] * 19
# distance code lengths: codes 0, 1 at 4 bits, 2..29 at 5 bits (complete)
DIST_LENS = [4, 4] + [5] * 28
assert sum(2.0 ** -L for L in LIT_LENS if L) == 1.0 and sum(2.0 ** -L for L in DIST_LENS) == 1.0


def _header(bw, final):
    bw.bits(final, 1)
    bw.bits(2, 2)
    bw.bits(len(LIT_LENS) - 257, 5)
    bw.bits(len(DIST_LENS) - 1, 5)
    bw.bits(19 - 4, 4)
    # code-length code: symbols 0..15 at 4 bits each (complete), 16..18 unused
    cl_lens = [4] * 16 + [0, 0, 0]
    for s in CLORDER:
        bw.bits(cl_lens[s], 3)
    clc = canonical(cl_lens)
    for L in LIT_LENS + DIST_LENS:
        bw.huff(*clc[L])


def long_literal_stream(nbytes, seed=0, block_syms=12000, ff_share=0.25):
    """Returns (raw, compressed raw deflate).  Literals are random bytes, a
    share of them 0xFF; about one symbol in four is a match (length symbols
    257..266, distances within the output so far)."""
    rng = random.Random(seed)
    lc = canonical(LIT_LENS)
    dc = canonical(DIST_LENS)
    bw = BitWriter()
    raw = bytearray()
    while len(raw) < nbytes:
        final = 1 if len(raw) + block_syms * 3 >= nbytes else 0
        _header(bw, final)
        nsym = 0
        while nsym < block_syms and (not final or len(raw) < nbytes):
            if len(raw) >= 4 and rng.random() < 0.25:
                ls = rng.randint(257, 266)
                lx = rng.randint(0, (1 << LEXT[ls - 257]) - 1)
                L = LBASE[ls - 257] + lx
                maxd = min(len(raw), 32768)
                dsym = rng.randint(0, 29)
                while DBASE[dsym] > maxd:
                    dsym -= 1
                dext = DEXT[dsym]
                dhi = min(DBASE[dsym] + (1 << dext) - 1, maxd)
                d = rng.randint(DBASE[dsym], dhi)
                bw.huff(*lc[ls])
                bw.bits(lx, LEXT[ls - 257])
                bw.huff(*dc[dsym])
                bw.bits(d - DBASE[dsym], dext)
                for _ in range(L):
                    raw.append(raw[-d])
            else:
                b = 0xFF if rng.random() < ff_share else rng.randint(0, 255)
                bw.huff(*lc[b])
                raw.append(b)
            nsym += 1
        bw.huff(*lc[256])
        if final:
            break
    return bytes(raw), bw.finish()
