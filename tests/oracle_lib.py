"""ctypes binding to the CPU oracle (oracle/libzo_inflate.so).

TEST INFRASTRUCTURE ONLY: the oracle is the parity checker, never the product.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "libzo_inflate.so")


class ZoResult(ctypes.Structure):
    _fields_ = [("ret", ctypes.c_int), ("data_type", ctypes.c_int), ("msg", ctypes.c_char_p),
                ("total_in", ctypes.c_uint64), ("total_out", ctypes.c_uint64),
                ("adler", ctypes.c_uint32)]


class ZoStream(ctypes.Structure):
    _fields_ = [("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_uint32),
                ("total_in", ctypes.c_uint64), ("next_out", ctypes.c_void_p),
                ("avail_out", ctypes.c_uint32), ("total_out", ctypes.c_uint64),
                ("msg", ctypes.c_char_p), ("adler", ctypes.c_uint32),
                ("data_type", ctypes.c_int), ("st", ctypes.c_void_p)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        L.zo_oneshot.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                 ctypes.c_int, ctypes.POINTER(ZoResult)]
        L.zo_js_schedule.restype = ctypes.c_size_t
        L.zo_js_schedule.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.zo_crc32.restype = ctypes.c_uint32
        L.zo_crc32.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.zo_adler32.restype = ctypes.c_uint32
        L.zo_adler32.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
        L.zo_inflate_init2.argtypes = [ctypes.POINTER(ZoStream), ctypes.c_int]
        L.zo_inflate.argtypes = [ctypes.POINTER(ZoStream), ctypes.c_int]
        L.zo_inflate_end.argtypes = [ctypes.POINTER(ZoStream)]
        _lib = L
    return _lib


def oneshot(data, wbits, cap=None):
    """One inflate(Z_FINISH) over the whole input; returns (out_bytes, dict)."""
    if cap is None:
        cap = max(1 << 16, len(data) * 1100 + 1024)
    out = ctypes.create_string_buffer(max(cap, 1))
    res = ZoResult()
    lib().zo_oneshot(bytes(data), len(data), out, cap, wbits, ctypes.byref(res))
    info = {"ret": res.ret, "msg": res.msg.decode() if res.msg else None,
            "total_in": res.total_in, "total_out": res.total_out, "adler": res.adler}
    return out.raw[:res.total_out], info


def js_schedule(data, w, wbits, out_cap=1 << 26):
    tr = ctypes.create_string_buffer(1 << 20)
    out = ctypes.create_string_buffer(out_cap)
    ol = ctypes.c_size_t(0)
    n = lib().zo_js_schedule(bytes(data), len(data), w, wbits, tr, len(tr), out, out_cap, ctypes.byref(ol))
    return tr.raw[:n].decode(), out.raw[:ol.value]


class Stream:
    """Call-by-call driver of the oracle's zlib-style inflate (zo_inflate):
    the reference's per-call contract (consumed, produced, ret, msg, adler)."""

    def __init__(self, wbits):
        self.z = ZoStream()
        self.rc = lib().zo_inflate_init2(ctypes.byref(self.z), wbits)

    def call(self, data, out_len, flush):
        ib = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
        ob = ctypes.create_string_buffer(max(out_len, 1))
        self.z.next_in = ctypes.addressof(ib) if data else None
        self.z.avail_in = len(data)
        self.z.next_out = ctypes.addressof(ob)
        self.z.avail_out = out_len
        r = lib().zo_inflate(ctypes.byref(self.z), flush)
        prod = out_len - self.z.avail_out
        return {"ret": r, "consumed": len(data) - self.z.avail_in, "produced": prod, "out": ob.raw[:prod],
                "msg": self.z.msg.decode() if self.z.msg else None, "total_in": self.z.total_in,
                "total_out": self.z.total_out, "adler": self.z.adler}

    def end(self):
        lib().zo_inflate_end(ctypes.byref(self.z))
