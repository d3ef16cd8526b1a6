"""ZIP containers: zs_zip_scan (host parse, CPU-only
tests) and unzip / multi-member gzip through the GPU batch (gpu tests).

The reference reads the raw payload of the first local header of a 7-Zip
deflate64 archive (src/generator/create_deflate64.cpp:51-93); zs_zip_scan
generalises it to every entry (central directory incl. ZIP64, else the local
headers).  Archives here are built with Python's zipfile (methods 0 / 8) and by
hand for method 9 (deflate64: zipfile cannot write it), wrapping the
reference's own deflate64 fixtures.
"""
import gzip
import io
import random
import struct
import zipfile
import zlib

import pytest

import oracle_lib as O
from golden.make_manifest import fixture


@pytest.fixture(scope="module")
def zs():
    import zstreams
    zstreams.lib()
    return zstreams


def _payloads():
    rng = random.Random(5)
    text = b"".join(b"row %06d value %d\n" % (i, rng.randrange(1000)) for i in range(20000))
    return {"text.txt": text, "random.bin": bytes(rng.getrandbits(8) for _ in range(30000)), "empty": b"",
            "dir/small.txt": b"hello zip\n"}


def _zipfile(method, zip64=False):
    bio = io.BytesIO()
    with zipfile.ZipFile(bio, "w", compression=method) as z:
        for name, data in _payloads().items():
            if zip64:
                with z.open(name, "w", force_zip64=True) as f:
                    f.write(data)
            else:
                z.writestr(name, data)
    return bio.getvalue()


def _d64_zip(names, central=True):
    """Method-9 entries around the reference's deflate64 fixtures (local headers,
    then a central directory + end record unless central=False)."""
    local, cd = bytearray(), bytearray()
    expect = {}
    for name in names:
        comp = fixture(name)
        out, info = O.oneshot(comp, -16)
        assert info["ret"] == 1
        crc = zlib.crc32(out)
        fn = (name + ".txt").encode()
        off = len(local)
        local += struct.pack("<IHHHHHIIIHH", 0x04034b50, 21, 0, 9, 0, 0, crc, len(comp), len(out), len(fn), 0)
        local += fn + comp
        cd += struct.pack("<IHHHHHHIIIHHHHHII", 0x02014b50, 21, 21, 0, 9, 0, 0, crc, len(comp), len(out),
                          len(fn), 0, 0, 0, 0, 0, off) + fn
        expect[fn.decode()] = out
    if not central:
        return bytes(local), expect
    eocd = struct.pack("<IHHHHIIH", 0x06054b50, 0, 0, len(names), len(names), len(cd), len(local), 0)
    return bytes(local + cd + eocd), expect


@pytest.mark.parametrize("method,zip64", [(zipfile.ZIP_STORED, False), (zipfile.ZIP_DEFLATED, False),
                                          (zipfile.ZIP_DEFLATED, True)])
def test_scan_matches_zipfile(zs, method, zip64):
    data = _zipfile(method, zip64)
    ents = zs.zip_scan(data)
    infos = zipfile.ZipFile(io.BytesIO(data)).infolist()
    assert [e["name"] for e in ents] == [i.filename for i in infos]
    for e, i in zip(ents, infos):
        assert (e["method"], e["comp_size"], e["uncomp_size"], e["crc32"], e["local_off"]) == \
            (i.compress_type, i.compress_size, i.file_size, i.CRC, i.header_offset)
        assert e["data_off"] + e["comp_size"] <= len(data)


def test_scan_deflate64_central_and_local_only(zs):
    names = ["10k_lines", "payload_64k", "zeros_100k"]
    for central in (True, False):
        data, expect = _d64_zip(names, central)
        ents = zs.zip_scan(data)
        assert [e["name"] for e in ents] == list(expect)
        assert all(e["method"] == 9 for e in ents)
        assert [e["uncomp_size"] for e in ents] == [len(v) for v in expect.values()]
        # the payload is exactly the fixture (create_deflate64.cpp:51-93 extraction)
        for e, n in zip(ents, names):
            assert data[e["data_off"]:e["data_off"] + e["comp_size"]] == fixture(n)


def test_scan_rejects_garbage(zs):
    with pytest.raises(zs.ZStreamsError):
        zs.zip_scan(b"not a zip archive at all" * 10)
    data = bytearray(_zipfile(zipfile.ZIP_DEFLATED))
    cd = data.rfind(b"PK\x01\x02")
    data[cd + 42:cd + 46] = struct.pack("<I", 7)  # local header offset pointing nowhere
    with pytest.raises(zs.ZStreamsError):
        zs.zip_scan(bytes(data))


@pytest.mark.gpu
def test_unzip_gpu(zs):
    for method, z64 in ((zipfile.ZIP_STORED, False), (zipfile.ZIP_DEFLATED, False), (zipfile.ZIP_DEFLATED, True)):
        data = _zipfile(method, z64)
        got = zs.unzip(data)
        assert got == _payloads(), (method, z64)
    data, expect = _d64_zip(["100k_lines", "10k_lines", "payload_63k", "payload_65k", "rand_block_gap", "zeros_100k"])
    assert zs.unzip(data) == expect
    # a wrong CRC-32 in the central directory is caught (computed on the GPU)
    bad = bytearray(data)
    cd = bad.find(b"PK\x01\x02")
    bad[cd + 16] ^= 1
    with pytest.raises(zs.ZStreamsError, match="CRC-32"):
        zs.unzip(bytes(bad))


@pytest.mark.gpu
def test_gunzip_members_gpu(zs):
    parts = [b"first member\n" * 1000, b"", bytes(range(256)) * 300, b"x" * 70000]
    data = b"".join(gzip.compress(p, 6) for p in parts)
    assert zs.gunzip_members(data) == parts
    assert zs.gunzip_members(data + b"\0\0\0\0") == parts
