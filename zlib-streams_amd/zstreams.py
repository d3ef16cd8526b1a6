"""Host-side mirror of the reference's Compression Streams surface over the
MI355X inflate core (libzstreams_mi355x.so, C-ABI, loaded with ctypes).

Reference interface mirrored here:
  * src/wasm/api/zlib-streams.js:15-157  ``_make`` / ``DecompressionStreamZlib``:
    formats "deflate", "deflate-raw", "gzip", "deflate64-raw"; 32 KiB input
    slices, 64 KiB output buffer, stop a write when a call consumes 0 bytes,
    ``Z_FINISH`` drain in ``flush()``; a negative code raises (transform 89-95,
    flush 125-130).
  * ``CompressionStreamZlib`` (zlib-streams.js:159-163, same ``_make`` with
    isCompress): formats "deflate", "deflate-raw", "gzip"; ``options.level``
    (default -1); process codes are not checked while compressing (:89, :123).
  * the handle ABI of src/wasm/*_stream_wasm.c (``inflate_new``,
    ``deflate_new`` ...).

Plus the batch entries ``inflate_batch`` / ``deflate_batch`` (many whole
streams per GPU launch).

There is no CPU path: if the shared library or a HIP device is missing, every
call raises ``ZStreamsError``.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ZS_LIB selects another build of the same library (e.g. the profiling build)
LIB_PATH = os.environ.get("ZS_LIB") or os.path.join(HERE, "libzstreams_mi355x.so")

Z_OK, Z_STREAM_END, Z_NEED_DICT = 0, 1, 2
Z_STREAM_ERROR, Z_DATA_ERROR, Z_MEM_ERROR, Z_BUF_ERROR = -2, -3, -4, -5
Z_NO_FLUSH, Z_FINISH = 0, 4
ZS_F_DEVICE = 1
ZS_F_CRC32 = 2  # raw / copy jobs: CRC-32 of the output in "adler" (ZIP entries)
ZS_F_DEFLATE_FAST = 4  # deflate levels 1..9: the throughput path instead of zlib's bytes
ZS_JOB_INFLATE, ZS_JOB_COPY = 0, 1

# windowBits per format, as the reference's init functions choose them
# (src/wasm/inflate_stream_wasm.c:22-45, inflate9_stream_wasm.c:15-20)
FORMAT_WBITS = {"deflate": 15, "deflate-raw": -15, "gzip": 31, "deflate64-raw": -16}
# deflateInit2 windowBits per compression format (src/wasm/deflate_stream_wasm.c:22-49)
DEFLATE_FORMAT_WBITS = {"deflate": 15, "deflate-raw": -15, "gzip": 31}

# exported symbols and their ctypes signatures (include/zstreams_mi355x.h)
_U = ctypes.c_size_t  # uintptr_t
_SIGS = {
    "inflate_new": (_U, []), "inflate_init": (ctypes.c_int, [_U]),
    "inflate_init_raw": (ctypes.c_int, [_U]), "inflate_init_gzip": (ctypes.c_int, [_U]),
    "inflate_process": (ctypes.c_int, [_U, _U, ctypes.c_uint, _U, ctypes.c_uint, ctypes.c_int]),
    "inflate_end": (ctypes.c_int, [_U]), "inflate_last_consumed": (ctypes.c_uint, [_U]),
    "inflate9_new": (_U, []), "inflate9_init": (ctypes.c_int, [_U]),
    "inflate9_init_raw": (ctypes.c_int, [_U]),
    "inflate9_process": (ctypes.c_int, [_U, _U, ctypes.c_uint, _U, ctypes.c_uint, ctypes.c_int]),
    "inflate9_end": (ctypes.c_int, [_U]), "inflate9_last_consumed": (ctypes.c_uint, [_U]),
    "deflate_new": (_U, []), "deflate_init": (ctypes.c_int, [_U, ctypes.c_int]),
    "deflate_init_raw": (ctypes.c_int, [_U, ctypes.c_int]), "deflate_init_gzip": (ctypes.c_int, [_U, ctypes.c_int]),
    "deflate_process": (ctypes.c_int, [_U, _U, ctypes.c_uint, _U, ctypes.c_uint, ctypes.c_int]),
    "deflate_end": (ctypes.c_int, [_U]), "deflate_last_consumed": (ctypes.c_uint, [_U]),
    "zs_deflate_bound": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_int32]),
    "zs_profile_deflate": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_uint32]),
    "zs_set_stream": (ctypes.c_int, [ctypes.c_void_p]),
    "zs_profile": (ctypes.c_int, [ctypes.c_int]),
    "zs_profile_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_uint64)]),
    "zs_profile_stages": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_uint32]),
    "zs_kprof_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_int]),
    "zs_last_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32)]),
    "zs_last_stats_ex": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]),
    "zs_stream_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    "zs_stream_stats_ex": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    "zs_stream_persist": (ctypes.c_int, [ctypes.c_int]),
    "zs_synchronize": (ctypes.c_int, []),
    "zs_version": (ctypes.c_char_p, []), "zs_source_hash": (ctypes.c_char_p, []), "zs_last_error": (ctypes.c_char_p, []),
}


class ZStreamsError(RuntimeError):
    pass


class ZsJob(ctypes.Structure):
    _fields_ = [("in_", ctypes.c_void_p), ("in_len", ctypes.c_uint64), ("out", ctypes.c_void_p),
                ("out_cap", ctypes.c_uint64), ("window_bits", ctypes.c_int32), ("mode", ctypes.c_int32)]


class ZipEntry(ctypes.Structure):
    _fields_ = [("local_off", ctypes.c_uint64), ("data_off", ctypes.c_uint64), ("comp_size", ctypes.c_uint64),
                ("uncomp_size", ctypes.c_uint64), ("name_off", ctypes.c_uint64), ("name_len", ctypes.c_uint32),
                ("crc32", ctypes.c_uint32), ("method", ctypes.c_uint16), ("flags", ctypes.c_uint16),
                ("reserved", ctypes.c_uint32)]


class ZsDJob(ctypes.Structure):
    _fields_ = [("in_", ctypes.c_void_p), ("in_len", ctypes.c_uint64), ("out", ctypes.c_void_p),
                ("out_cap", ctypes.c_uint64), ("window_bits", ctypes.c_int32), ("level", ctypes.c_int32)]


class ZsResult(ctypes.Structure):
    _fields_ = [("ret", ctypes.c_int32), ("reserved", ctypes.c_int32), ("total_in", ctypes.c_uint64),
                ("total_out", ctypes.c_uint64), ("adler", ctypes.c_uint32), ("reserved2", ctypes.c_uint32),
                ("msg", ctypes.c_char_p)]

    def as_dict(self):
        return {"ret": self.ret, "msg": self.msg.decode() if self.msg else None,
                "total_in": self.total_in, "total_out": self.total_out, "adler": self.adler}


_lib = None


def lib():
    """Load the shared library (fails loudly: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ZStreamsError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C zlib-streams_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        L.zs_zip_scan.restype = ctypes.c_int
        L.zs_zip_scan.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ZipEntry), ctypes.c_uint32,
                                  ctypes.POINTER(ctypes.c_uint32)]
        L.zs_inflate_batch.restype = ctypes.c_int
        L.zs_inflate_batch.argtypes = [ctypes.POINTER(ZsJob), ctypes.c_uint32, ctypes.POINTER(ZsResult), ctypes.c_uint32]
        L.zs_deflate_batch.restype = ctypes.c_int
        L.zs_deflate_batch.argtypes = [ctypes.POINTER(ZsDJob), ctypes.c_uint32, ctypes.POINTER(ZsResult), ctypes.c_uint32]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise ZStreamsError(f"libzstreams_mi355x error {rc}: {lib().zs_last_error().decode()}")


PARSE_FLAGS = {None: 0, "lane": 8, "wave": 16, "split": 4096}  # ZS_F_PARSE_LANE / _WAVE / _SPLIT
LINK_FLAGS = {None: 0, "serial": 32}  # ZS_F_LINK_SERIAL


def _link_flags(link):
    """link: None (auto), "serial", or ("segmented", n): ZS_F_LINKSEG(n)."""
    if isinstance(link, tuple):
        assert link[0] == "segmented" and 1 <= link[1] <= 8, link
        return link[1] << 8
    return LINK_FLAGS[link]


def inflate_batch(streams, window_bits=-15, out_caps=None, parse=None, link=None):
    """Inflate many whole streams on the GPU (host buffers).

    Each stream behaves like inflateInit2(window_bits) + one inflate(Z_FINISH)
    into an out_cap-byte buffer.  Returns [(bytes, result_dict)].  parse =
    "lane" / "wave" forces the block-parallel path's parse mode, link = "serial"
    its per-stream window link, link = ("segmented", n) the segmented link
    with n segments per chain (same results).
    """
    n = len(streams)
    if out_caps is None:
        out_caps = [max(1 << 16, 8 * len(s) + 4096) for s in streams]
    wbs = window_bits if isinstance(window_bits, (list, tuple)) else [window_bits] * n
    jobs = (ZsJob * max(n, 1))()
    res = (ZsResult * max(n, 1))()
    inbufs, outbufs = [], []
    for i, s in enumerate(streams):
        ib = ctypes.create_string_buffer(bytes(s), max(len(s), 1))
        ob = ctypes.create_string_buffer(max(out_caps[i], 1))
        inbufs.append(ib)
        outbufs.append(ob)
        jobs[i].in_ = ctypes.cast(ib, ctypes.c_void_p).value if len(s) else None
        jobs[i].in_len = len(s)
        jobs[i].out = ctypes.cast(ob, ctypes.c_void_p).value
        jobs[i].out_cap = out_caps[i]
        jobs[i].window_bits = wbs[i]
    _check(lib().zs_inflate_batch(jobs, n, res, PARSE_FLAGS[parse] | _link_flags(link)))
    return [(outbufs[i].raw[:res[i].total_out], res[i].as_dict()) for i in range(n)]


def zip_scan(data):
    """Entries of a ZIP archive (zs_zip_scan: central directory incl. ZIP64, else
    local headers as src/generator/create_deflate64.cpp:51-93 reads them).
    Returns a list of dicts (name, method, offsets, sizes, crc32)."""
    data = bytes(data)
    n = ctypes.c_uint32()
    rc = lib().zs_zip_scan(data, len(data), None, 0, ctypes.byref(n))
    if rc != 0:
        raise ZStreamsError(f"zs_zip_scan: malformed archive ({rc})")
    arr = (ZipEntry * max(n.value, 1))()
    _check(lib().zs_zip_scan(data, len(data), arr, n.value, ctypes.byref(n)))
    out = []
    for e in arr[:n.value]:
        out.append({"name": data[e.name_off:e.name_off + e.name_len].decode("utf-8", "replace"),
                    "method": e.method, "flags": e.flags, "local_off": e.local_off, "data_off": e.data_off,
                    "comp_size": e.comp_size, "uncomp_size": e.uncomp_size, "crc32": e.crc32})
    return out


ZIP_METHOD_WBITS = {8: -15, 9: -16}


def unzip(data):
    """Extract every entry of a ZIP archive on the GPU: deflate (8) and deflate64
    (9) payloads in ONE batch inflate, stored (0) entries as copy jobs, each
    output's CRC-32 computed on the GPU and checked against the entry.
    Returns {name: bytes}; raises ZStreamsError on any bad entry."""
    data = bytes(data)
    ents = zip_scan(data)
    for e in ents:
        if e["method"] not in (0, 8, 9):
            raise ZStreamsError(f"{e['name']}: unsupported method {e['method']}")
    n = len(ents)
    jobs = (ZsJob * max(n, 1))()
    res = (ZsResult * max(n, 1))()
    ib = ctypes.create_string_buffer(data, max(len(data), 1))
    base = ctypes.addressof(ib)
    outs = []
    for i, e in enumerate(ents):
        ob = ctypes.create_string_buffer(max(e["uncomp_size"], 1))
        outs.append(ob)
        jobs[i].in_ = base + e["data_off"]
        jobs[i].in_len = e["comp_size"]
        jobs[i].out = ctypes.addressof(ob)
        jobs[i].out_cap = e["uncomp_size"]
        jobs[i].window_bits = ZIP_METHOD_WBITS.get(e["method"], -15)
        jobs[i].mode = ZS_JOB_COPY if e["method"] == 0 else ZS_JOB_INFLATE
    if n:
        _check(lib().zs_inflate_batch(jobs, n, res, ZS_F_CRC32))
    got = {}
    for i, e in enumerate(ents):
        r = res[i]
        if r.ret != Z_STREAM_END or r.total_out != e["uncomp_size"]:
            raise ZStreamsError(f"{e['name']}: inflate ret {r.ret} "
                                f"({r.msg.decode() if r.msg else 'size mismatch'}), {r.total_out} of {e['uncomp_size']} bytes")
        if r.adler != e["crc32"]:
            raise ZStreamsError(f"{e['name']}: CRC-32 {r.adler:08x} != {e['crc32']:08x}")
        got[e["name"]] = outs[i].raw[:r.total_out]
    return got


def gunzip_members(data, out_hint=None):
    """Every member of a multi-member gzip file, each decoded on the GPU (the
    reference stops after the first member's trailer).  Returns the list of
    member outputs; a member that fails raises ZStreamsError."""
    data = bytes(data)
    outs, off = [], 0
    while off < len(data):
        if data[off:off + 2] != b"\x1f\x8b":
            break  # trailing non-gzip bytes are ignored, as gzip -d does with zeros
        cap = out_hint or max(1 << 16, 4 * (len(data) - off))
        while True:
            (o, r), = inflate_batch([data[off:]], 31, [cap])
            if r["ret"] == Z_BUF_ERROR and r["total_out"] == cap and cap < (1 << 32) - 1:
                cap = min(cap * 4, (1 << 32) - 1)
                continue
            break
        if r["ret"] != Z_STREAM_END:
            raise ZStreamsError(f"gzip member at {off}: ret {r['ret']} {r['msg']}")
        outs.append(o)
        off += r["total_in"]
    return outs


def inflate_batch_device(in_ptrs, in_lens, out_ptrs, out_caps, window_bits):
    """Inflate streams already resident in HBM (device pointers, outputs 16 B aligned)."""
    n = len(in_ptrs)
    jobs = (ZsJob * n)()
    res = (ZsResult * n)()
    for i in range(n):
        jobs[i].in_ = in_ptrs[i]
        jobs[i].in_len = in_lens[i]
        jobs[i].out = out_ptrs[i]
        jobs[i].out_cap = out_caps[i]
        jobs[i].window_bits = window_bits[i] if isinstance(window_bits, (list, tuple)) else window_bits
    _check(lib().zs_inflate_batch(jobs, n, res, ZS_F_DEVICE))
    return [res[i].as_dict() for i in range(n)]


def deflate_bound(n, window_bits=-15):
    """Output capacity that always holds one GPU-deflated stream of n bytes."""
    return int(lib().zs_deflate_bound(n, window_bits))


def deflate_batch(streams, window_bits=-15, level=-1, out_caps=None, fast=False):
    """Deflate many whole buffers on the GPU (host buffers).

    Each job behaves like deflateInit2(level, Z_DEFLATED, window_bits, 8,
    Z_DEFAULT_STRATEGY) + one deflate(Z_FINISH).  Every level writes zlib's bytes
    (unless fast=True: ZS_F_DEFLATE_FAST, the throughput path with its own block
    structure).  Returns [(bytes, result_dict)].
    """
    n = len(streams)
    wbs = window_bits if isinstance(window_bits, (list, tuple)) else [window_bits] * n
    lvs = level if isinstance(level, (list, tuple)) else [level] * n
    if out_caps is None:
        out_caps = [deflate_bound(len(s), wbs[i]) if -16 <= wbs[i] <= 31 else 64 for i, s in enumerate(streams)]
    jobs = (ZsDJob * max(n, 1))()
    res = (ZsResult * max(n, 1))()
    inbufs, outbufs = [], []
    for i, s in enumerate(streams):
        ib = ctypes.create_string_buffer(bytes(s), max(len(s), 1))
        ob = ctypes.create_string_buffer(max(out_caps[i], 1))
        inbufs.append(ib)
        outbufs.append(ob)
        jobs[i].in_ = ctypes.cast(ib, ctypes.c_void_p).value if len(s) else None
        jobs[i].in_len = len(s)
        jobs[i].out = ctypes.cast(ob, ctypes.c_void_p).value
        jobs[i].out_cap = out_caps[i]
        jobs[i].window_bits = wbs[i]
        jobs[i].level = lvs[i]
    _check(lib().zs_deflate_batch(jobs, n, res, ZS_F_DEFLATE_FAST if fast else 0))
    return [(outbufs[i].raw[:res[i].total_out], res[i].as_dict()) for i in range(n)]


def deflate_batch_device(in_ptrs, in_lens, out_ptrs, out_caps, window_bits, level=-1, fast=False):
    """Deflate buffers already resident in HBM (device pointers)."""
    n = len(in_ptrs)
    jobs = (ZsDJob * n)()
    res = (ZsResult * n)()
    for i in range(n):
        jobs[i].in_ = in_ptrs[i]
        jobs[i].in_len = in_lens[i]
        jobs[i].out = out_ptrs[i]
        jobs[i].out_cap = out_caps[i]
        jobs[i].window_bits = window_bits[i] if isinstance(window_bits, (list, tuple)) else window_bits
        jobs[i].level = level[i] if isinstance(level, (list, tuple)) else level
    _check(lib().zs_deflate_batch(jobs, n, res, ZS_F_DEVICE | (ZS_F_DEFLATE_FAST if fast else 0)))
    return [res[i].as_dict() for i in range(n)]


DEFLATE_STAGES = ("match", "parse", "blocks", "stitch")
DEFLATE_STAGE_KERNELS = {"match": "zs_dz_match_kernel", "parse": "zs_dz_parse_kernel",
                         "blocks": "zs_dz_block_kernel + zs_dz_check_kernel",
                         "stitch": "zs_dz_offsets_kernel + zs_dz_stitch_kernel + zs_dz_trailer_kernel"}
ZDEFLATE_STAGE_KERNELS = {"match": "zs_zd_prev_kernel + zs_zd_msearch_kernel (ZS_ZD_MATCH=all: zs_zd_match_kernel)",
                          "parse": "zs_zd_parse_kernel + zs_zd_fix_kernel rounds",
                          "blocks": "zs_zd_count/blocks/blist/tree/layout/emit kernels",
                          "stitch": "zs_dz_trailer_kernel"}


def profile_deflate():
    """Accumulated deflate timing since profile(True): (pipeline ms, {stage: ms}, batches)."""
    a = (ctypes.c_double * 6)()
    k = lib().zs_profile_deflate(a, 6)
    if k < 0:
        _check(k)
    return a[0], {DEFLATE_STAGES[i]: a[1 + i] for i in range(4)}, int(a[5])


def profile(enable):
    """Time the decode kernels with HIP events on the launch stream."""
    _check(lib().zs_profile(1 if enable else 0))


def profile_read():
    """(inflate-pipeline ms, whole-batch ms, batches) accumulated since profile(True).

    The pipeline is every kernel between the header parse and the finalize
    (find, parse, expand, link, emit, serial decode)."""
    ms = ctypes.c_double()
    bms = ctypes.c_double()
    n = ctypes.c_uint64()
    _check(lib().zs_profile_read(ctypes.byref(ms), ctypes.byref(bms), ctypes.byref(n)))
    return ms.value, bms.value, n.value


PROFILE_STAGES = ("header", "find", "parse", "expand", "link", "emit", "serial_decode", "finalize")
STAGE_KERNELS = {"header": "zs_header_kernel",
                 "find": "zs_find_kernel + zs_findval_kernel + zs_findsel_kernel + zs_find_fixed_kernel + zs_plan_kernel",
                 "parse": "zs_unit_header_kernel + (split parse) zs_walk_kernel + zs_split_kernel + zs_unitw_list_kernel"
                          " | zs_lane_kernel | zs_unitw_kernel, + zs_chain_kernel",
                 "expand": "zs_expand2_kernel (deflate64: zs_expand_kernel)",
                 "link": "zs_linkseg_kernel + zs_linkseg_join_kernel + zs_link_kernel (or the serial / prefix link)",
                 "emit": "zs_emit_kernel",
                 "serial_decode": "zs_decode_kernel", "finalize": "zs_check_kernel + zs_finalize_kernel"}


def profile_stages():
    """Accumulated ms per pipeline stage since profile(True), keyed by PROFILE_STAGES."""
    a = (ctypes.c_double * len(PROFILE_STAGES))()
    k = lib().zs_profile_stages(a, len(PROFILE_STAGES))
    if k < 0:
        _check(k)
    return {PROFILE_STAGES[i]: a[i] for i in range(k)}


def kprof_read(reset=True):
    """In-kernel counters of the profiling build (ZS_LIB=.../libzstreams_mi355x_prof.so);
    an empty list with the product library."""
    a = (ctypes.c_uint64 * 96)()
    k = lib().zs_kprof_read(a, 96, 1 if reset else 0)
    if k < 0:
        raise ZStreamsError("zs_kprof_read failed")
    return list(a[:k])


def last_stats():
    """Last batch: jobs on the chunked path, decode units planned for them, chunked
    jobs whose chain did not verify (decoded by the serial decoder instead), and
    jobs routed to the serial decoder directly."""
    a = (ctypes.c_uint32 * 12)()
    k = lib().zs_last_stats_ex(a, 12)
    if k < 0:
        _check(k)
    mode = {0: "lane", 1: "wave", 2: "split"}
    return {"chunked_jobs": a[0], "units": a[1], "fallback_jobs": a[2], "serial_jobs": a[3],
            "parse": mode.get(a[4]), "link": None if a[4] > 2 else ("serial" if a[5] == 0 else
                                                                    "segmented" if a[5] & 0x80000000 else "prefix"),
            "parse_d64": mode.get(a[6]), "link_d64": None if a[6] > 2 else ("serial" if a[7] == 0 else "prefix"),
            "link_segments": (a[5] & 0x7fffffff) if a[4] <= 2 and a[5] & 0x80000000 else None,
            "lane_resident_waves": a[8], "units_std": a[9], "units_d64": a[10],
            "groups": a[11] if k >= 12 else None}  # raw/zlib/gzip groups run at once on two streams (round 6)


def stream_stats():
    """Stream-call batching since load: launch sequences and the calls they ran."""
    a = (ctypes.c_uint64 * 10)()
    _check(lib().zs_stream_stats_ex(a))
    return {"launches": a[0], "calls": a[1], "launch_ns": a[2], "gather_ns": a[3], "kernel_ns": a[4],
            "pk_launches": a[5], "pk_calls": a[6], "pk_busy_ns": a[7], "pk_wait_ns": a[8], "pk_idle_ns": a[9]}


def stream_persist(on=None):
    """Persistent stream worker on / off (None: only read); returns the previous setting."""
    return bool(lib().zs_stream_persist(-1 if on is None else int(bool(on))))


def set_stream(hip_stream_handle):
    _check(lib().zs_set_stream(hip_stream_handle))


class _Handle:
    """The reference's handle ABI for one (de)compression stream."""

    def __init__(self, fmt, compress=False, level=-1):
        if fmt not in (DEFLATE_FORMAT_WBITS if compress else FORMAT_WBITS):
            raise ValueError(f"unsupported format {fmt!r}")
        L = lib()
        p = "deflate_" if compress else "inflate9_" if fmt == "deflate64-raw" else "inflate_"
        self._process = getattr(L, p + "process")
        self._last = getattr(L, p + "last_consumed")
        self._end = getattr(L, p + "end")
        self.h = getattr(L, p + "new")()
        if not self.h:
            raise MemoryError("stream allocation failed")
        init = {"deflate": "init", "deflate-raw": "init_raw", "gzip": "init_gzip",
                "deflate64-raw": "init_raw"}[fmt]
        args = (self.h, level) if compress else (self.h,)
        r = getattr(L, p + init)(*args)
        if r != 0:
            raise ZStreamsError("init failed:" + str(r))

    def process(self, data, out_buf, flush):
        ib = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
        r = self._process(self.h, ctypes.addressof(ib) if data else 0, len(data),
                          ctypes.addressof(out_buf), len(out_buf), flush)
        r &= 0xffffffff
        produced = r & 0x00ffffff
        code = (r >> 24) & 0xff
        return produced, (code - 256 if code & 0x80 else code), self._last(self.h)

    def end(self):
        if self.h:
            r = self._end(self.h)
            self.h = 0
            return r
        return 0


class DecompressionStreamZlib:
    """Mirror of the reference's ``DecompressionStreamZlib`` TransformStream
    (src/wasm/api/zlib-streams.js:15-157): feed chunks with ``transform``,
    finish with ``flush``; both return the list of enqueued output chunks."""

    def __init__(self, fmt="deflate", options=None):
        options = options or {}
        self.out_size = options.get("outBuffer", 64 * 1024)
        self._h = _Handle(fmt)
        self._out = ctypes.create_string_buffer(self.out_size)

    def transform(self, chunk):
        out = []
        off = 0
        try:
            while off < len(chunk):
                n = min(len(chunk) - off, 32 * 1024)
                produced, code, consumed = self._h.process(chunk[off:off + n], self._out, Z_NO_FLUSH)
                if produced:
                    out.append(self._out.raw[:produced])
                if code < 0:
                    raise ZStreamsError("process error:" + str(code))
                if consumed == 0:
                    break
                off += consumed
        except Exception:
            self._h.end()
            raise
        return out

    def flush(self):
        out = []
        try:
            while True:
                produced, code, _ = self._h.process(b"", self._out, Z_FINISH)
                if code < 0:
                    raise ZStreamsError("process error:" + str(code))
                if produced:
                    out.append(self._out.raw[:produced])
                if code == 1 or produced == 0:
                    break
        finally:
            r = self._h.end()
            if r != 0:
                raise ZStreamsError("end error:" + str(r))
        return out


class CompressionStreamZlib:
    """Mirror of the reference's ``CompressionStreamZlib``
    (src/wasm/api/zlib-streams.js:159-163 over ``_make(true, ...)``).  As in the
    reference, process codes are not checked while compressing (:89, :123)."""

    def __init__(self, fmt="deflate", options=None):
        options = options or {}
        level = options.get("level", -1)
        self.out_size = options.get("outBuffer", 64 * 1024)
        self._h = _Handle(fmt, compress=True, level=level if isinstance(level, int) else -1)
        self._out = ctypes.create_string_buffer(self.out_size)

    def transform(self, chunk):
        out = []
        off = 0
        try:
            while off < len(chunk):
                n = min(len(chunk) - off, 32 * 1024)
                produced, _, consumed = self._h.process(chunk[off:off + n], self._out, Z_NO_FLUSH)
                if produced:
                    out.append(self._out.raw[:produced])
                if consumed == 0:
                    break
                off += consumed
        except Exception:
            self._h.end()
            raise
        return out

    def flush(self):
        out = []
        try:
            while True:
                produced, code, _ = self._h.process(b"", self._out, Z_FINISH)
                if produced:
                    out.append(self._out.raw[:produced])
                if code == 1 or produced == 0:
                    break
        finally:
            r = self._h.end()
            if r != 0:
                raise ZStreamsError("end error:" + str(r))
        return out


def compress(data, fmt="deflate-raw", level=-1, write_size=65536):
    """Pipe ``data`` through a CompressionStreamZlib in ``write_size`` writes."""
    cs = CompressionStreamZlib(fmt, {"level": level})
    parts = []
    for i in range(0, len(data), write_size):
        parts += cs.transform(data[i:i + write_size])
    parts += cs.flush()
    return b"".join(parts)


def js_schedule(data, fmt="deflate-raw", write_size=4096):
    """The reference's DecompressionStreamZlib call schedule
    (src/wasm/api/zlib-streams.js:64-136) over the handle ABI, recording every
    process() call as "T n produced code consumed" / "F 0 produced code 0"
    lines.  Returns (trace, output); stops at the first
    negative code where the reference would throw."""
    h = _Handle(fmt)
    ob = ctypes.create_string_buffer(65536)
    lines, out = [], []
    failed = False
    try:
        for w in range(0, len(data), write_size):
            chunk = data[w:w + write_size]
            off = 0
            while off < len(chunk):
                n = min(len(chunk) - off, 32 * 1024)
                produced, code, consumed = h.process(chunk[off:off + n], ob, Z_NO_FLUSH)
                out.append(ob.raw[:produced])
                lines.append(f"T {n} {produced} {code} {consumed}\n")
                if code < 0:
                    failed = True
                    break
                if consumed == 0:
                    break
                off += consumed
            if failed:
                break
        while not failed:
            produced, code, _ = h.process(b"", ob, Z_FINISH)
            out.append(ob.raw[:produced])
            lines.append(f"F 0 {produced} {code} 0\n")
            if code < 0 or code == 1 or produced == 0:
                break
    finally:
        h.end()
    return "".join(lines), b"".join(out)


def decompress(data, fmt="deflate-raw", write_size=4096):
    """Pipe ``data`` through a DecompressionStreamZlib in ``write_size`` writes."""
    ds = DecompressionStreamZlib(fmt)
    parts = []
    for i in range(0, len(data), write_size):
        parts += ds.transform(data[i:i + write_size])
    parts += ds.flush()
    return b"".join(parts)
