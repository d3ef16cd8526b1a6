"""ctypes binding to the host zlib (libz.so.1, 1.2.11) inflate.

TEST INFRASTRUCTURE ONLY.  Host zlib is the upstream of the reference's vendored
zlib (src/zlib submodule, absent in the reference checkout); for windowBits
-15/15/31 its inflate is the same algorithm as the reference's src/inflate.c
(the deflate64 patch only changes the -16 path), so it is an independent pin
for the oracle's standard modes, including error codes, messages and byte
accounting.  Deflate output of host zlib is byte-identical to the reference's
shipped deflate.
"""
import ctypes
import ctypes.util


class ZStream(ctypes.Structure):
    _fields_ = [("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_uint),
                ("total_in", ctypes.c_ulong), ("next_out", ctypes.c_void_p),
                ("avail_out", ctypes.c_uint), ("total_out", ctypes.c_ulong),
                ("msg", ctypes.c_char_p), ("state", ctypes.c_void_p),
                ("zalloc", ctypes.c_void_p), ("zfree", ctypes.c_void_p),
                ("opaque", ctypes.c_void_p), ("data_type", ctypes.c_int),
                ("adler", ctypes.c_ulong), ("reserved", ctypes.c_ulong)]


_z = None


def libz():
    global _z
    if _z is None:
        _z = ctypes.CDLL(ctypes.util.find_library("z") or "libz.so.1")
        _z.zlibVersion.restype = ctypes.c_char_p
        _z.inflateInit2_.argtypes = [ctypes.POINTER(ZStream), ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        _z.inflate.argtypes = [ctypes.POINTER(ZStream), ctypes.c_int]
        _z.inflateEnd.argtypes = [ctypes.POINTER(ZStream)]
    return _z


def oneshot(data, wbits, cap=None):
    z = libz()
    if cap is None:
        cap = max(1 << 16, len(data) * 1100 + 1024)
    s = ZStream()
    ib = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    ob = ctypes.create_string_buffer(max(cap, 1))
    r = z.inflateInit2_(ctypes.byref(s), wbits, z.zlibVersion(), ctypes.sizeof(ZStream))
    if r != 0:
        return b"", {"ret": r, "msg": None, "total_in": 0, "total_out": 0, "adler": 0}
    s.next_in = ctypes.cast(ib, ctypes.c_void_p) if len(data) else None
    s.avail_in = len(data)
    s.next_out = ctypes.cast(ob, ctypes.c_void_p)
    s.avail_out = cap
    r = z.inflate(ctypes.byref(s), 4)
    info = {"ret": r, "msg": s.msg.decode() if s.msg else None, "total_in": s.total_in,
            "total_out": s.total_out, "adler": s.adler & 0xffffffff}
    z.inflateEnd(ctypes.byref(s))
    return ob.raw[:info["total_out"]], info


class Deflater:
    """Host zlib deflate driven call by call: deflateInit2_(level, 8, wbits, 8, 0),
    then deflate(strm, flush) with a given input and output space -- zlib's own
    per-call (ret, consumed, produced) for the reference's deflate (SURVEY §8c
    pins host zlib's bytes to the shipped deflate)."""

    def __init__(self, level, wbits):
        z = self.z = libz()
        z.deflateInit2_.argtypes = [ctypes.POINTER(ZStream), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        z.deflate.argtypes = [ctypes.POINTER(ZStream), ctypes.c_int]
        z.deflateEnd.argtypes = [ctypes.POINTER(ZStream)]
        self.s = ZStream()
        self.rc = z.deflateInit2_(ctypes.byref(self.s), level, 8, wbits, 8, 0, z.zlibVersion(), ctypes.sizeof(ZStream))

    def call(self, data, out_len, flush):
        ib = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
        ob = ctypes.create_string_buffer(max(out_len, 1))
        s = self.s
        s.next_in = ctypes.cast(ib, ctypes.c_void_p) if data else None
        s.avail_in = len(data)
        s.next_out = ctypes.cast(ob, ctypes.c_void_p)
        s.avail_out = out_len
        r = self.z.deflate(ctypes.byref(s), flush)
        prod = out_len - s.avail_out
        return r, len(data) - s.avail_in, ob.raw[:prod]

    def end(self):
        return self.z.deflateEnd(ctypes.byref(self.s))
