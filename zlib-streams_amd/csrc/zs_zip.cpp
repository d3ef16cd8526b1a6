// zs_zip.cpp -- ZIP container scan for the batch inflate.
//
// Realistic deflate64 inputs come out of ZIP files: the reference's generator
// takes the raw payload of the first local header of a 7-Zip "-mm=Deflate64"
// archive (src/generator/create_deflate64.cpp:51-93: signature search, method
// at +8, compressed size at +18, name / extra lengths at +26 / +28, payload
// after them).  zs_zip_scan() generalises that to every entry: the central
// directory when the archive has one (ZIP64 included), otherwise a walk over
// the local headers exactly as the reference reads the first one.  Entries
// then go to zs_inflate_batch() as raw deflate (method 8, windowBits -15),
// raw deflate64 (method 9, windowBits -16) or copy jobs (method 0), with
// ZS_F_CRC32 so the GPU checks each output against the entry's CRC-32.
// Parsing only: no byte of an entry is decoded on the host.
#include <cstring>

#include "../../include/zstreams_mi355x.h"

namespace {

uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

constexpr uint32_t SIG_LOCAL = 0x04034b50u, SIG_CENTRAL = 0x02014b50u, SIG_EOCD = 0x06054b50u;
constexpr uint32_t SIG_Z64_LOC = 0x07064b50u, SIG_Z64_EOCD = 0x06064b50u, SIG_DESC = 0x08074b50u;

// payload offset of the entry whose local header is at `off`
bool local_data(const uint8_t *zip, uint64_t len, uint64_t off, uint64_t *data_off) {
  if (off > len || len - off < 30 || rd32(zip + off) != SIG_LOCAL) return false;
  *data_off = off + 30 + rd16(zip + off + 26) + rd16(zip + off + 28);
  return *data_off <= len;
}

int scan_central(const uint8_t *zip, uint64_t len, uint64_t eocd, zs_zip_entry *out, uint32_t cap, uint32_t *n_out) {
  uint64_t count = rd16(zip + eocd + 10), cd_off = rd32(zip + eocd + 16);
  const bool z64 = count == 0xffffu || cd_off == 0xffffffffu;
  if (z64) {  // ZIP64 end of central directory locator, then record
    if (eocd < 20 || rd32(zip + eocd - 20) != SIG_Z64_LOC) return ZS_EFORMAT;
    const uint64_t rec = rd64(zip + eocd - 20 + 8);
    if (rec > len || len - rec < 56 || rd32(zip + rec) != SIG_Z64_EOCD) return ZS_EFORMAT;
    count = rd64(zip + rec + 32);
    cd_off = rd64(zip + rec + 48);
  }
  uint64_t p = cd_off;
  uint32_t n = 0;
  for (uint64_t k = 0; k < count; k++) {
    if (p > len || len - p < 46 || rd32(zip + p) != SIG_CENTRAL) return ZS_EFORMAT;
    const uint8_t *c = zip + p;
    zs_zip_entry e;
    std::memset(&e, 0, sizeof e);
    e.flags = rd16(c + 8);
    e.method = rd16(c + 10);
    e.crc32 = rd32(c + 16);
    e.comp_size = rd32(c + 20);
    e.uncomp_size = rd32(c + 24);
    const uint32_t nlen = rd16(c + 28), xlen = rd16(c + 30), clen = rd16(c + 32);
    e.local_off = rd32(c + 42);
    e.name_off = p + 46;
    e.name_len = nlen;
    if (len - p < 46ull + nlen + xlen + clen) return ZS_EFORMAT;
    // ZIP64 extended information (0x0001): the 0xffffffff fields, in order
    for (uint64_t x = p + 46 + nlen; x + 4 <= p + 46 + nlen + xlen;) {
      const uint32_t id = rd16(zip + x), sz = rd16(zip + x + 2);
      if (x + 4 + sz > p + 46 + nlen + xlen) break;
      if (id == 0x0001) {
        uint64_t q = x + 4;
        const uint64_t qe = q + sz;
        if (e.uncomp_size == 0xffffffffu && q + 8 <= qe) { e.uncomp_size = rd64(zip + q); q += 8; }
        if (e.comp_size == 0xffffffffu && q + 8 <= qe) { e.comp_size = rd64(zip + q); q += 8; }
        if (e.local_off == 0xffffffffu && q + 8 <= qe) { e.local_off = rd64(zip + q); q += 8; }
      }
      x += 4 + sz;
    }
    if (!local_data(zip, len, e.local_off, &e.data_off) || e.comp_size > len - e.data_off) return ZS_EFORMAT;
    if (n < cap) out[n] = e;
    n++;
    p += 46ull + nlen + xlen + clen;
  }
  *n_out = n;
  return 0;
}

// no central directory: consecutive local headers (create_deflate64.cpp:51-93)
int scan_local(const uint8_t *zip, uint64_t len, zs_zip_entry *out, uint32_t cap, uint32_t *n_out) {
  uint64_t p = 0;
  // the reference searches for the first signature
  while (p + 4 <= len && rd32(zip + p) != SIG_LOCAL) p++;
  uint32_t n = 0;
  while (p + 30 <= len && rd32(zip + p) == SIG_LOCAL) {
    const uint8_t *h = zip + p;
    zs_zip_entry e;
    std::memset(&e, 0, sizeof e);
    e.local_off = p;
    e.flags = rd16(h + 6);
    e.method = rd16(h + 8);
    e.crc32 = rd32(h + 14);
    e.comp_size = rd32(h + 18);
    e.uncomp_size = rd32(h + 22);
    e.name_off = p + 30;
    e.name_len = rd16(h + 26);
    if (!local_data(zip, len, p, &e.data_off) || e.comp_size > len - e.data_off) return ZS_EFORMAT;
    if ((e.flags & 8u) && e.comp_size == 0) return ZS_EFORMAT;  // sizes only in a data descriptor
    if (n < cap) out[n] = e;
    n++;
    p = e.data_off + e.comp_size;
    if (e.flags & 8u) p += (p + 4 <= len && rd32(zip + p) == SIG_DESC) ? 16 : 12;
  }
  if (n == 0) return ZS_EFORMAT;
  *n_out = n;
  return 0;
}

}  // namespace

extern "C" int zs_zip_scan(const void *zipv, uint64_t len, zs_zip_entry *out, uint32_t cap, uint32_t *n_out) {
  const uint8_t *zip = static_cast<const uint8_t *>(zipv);
  if (!zip || !n_out || (cap && !out)) return ZS_EINVAL;
  *n_out = 0;
  // end of central directory: last signature within the final 65 557 bytes
  if (len >= 22) {
    const uint64_t lo = len > 65557 ? len - 65557 : 0;
    for (uint64_t p = len - 22 + 1; p-- > lo;) {
      if (rd32(zip + p) == SIG_EOCD && p + 22 + rd16(zip + p + 20) <= len)
        return scan_central(zip, len, p, out, cap, n_out);
    }
  }
  return scan_local(zip, len, out, cap, n_out);
}
