// zs_device.h -- device helpers shared by the inflate kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define WAVE 64
#define TABLE_ENTRIES 1448   // ENOUGH (852 + 594), src/inftrees.h:52-55
// per unit slot: zlib-layout tables, their compact u16 copy, the LDS image
// (256 + 64 u16 roots, 64 B dist tail) and the split parse's walk tables
// (512 + 256 u8 entries, lane_decode.hip zs_walk_kernel)
#define TABLE_IMG_OFF (TABLE_ENTRIES + TABLE_ENTRIES / 2)
#define TABLE_WALK_OFF (TABLE_IMG_OFF + 176)
#define TABLE_LTAIL_OFF (TABLE_WALK_OFF + 192)  // the literal/length code's canonical tail (16 words, the walk)
#define TABLE_STRIDE (TABLE_LTAIL_OFF + 16)
#define FIXED_ZLIB_WORDS 544                              // fixed tables: 512 lit/len + 32 dist (zlib layout)
#define FIXED_WORDS (FIXED_ZLIB_WORDS + FIXED_ZLIB_WORDS / 2)  // + compact u16 copy
#define DIST_TABLE_OFF 852   // distance table follows the literal/length table

// ---------------------------------------------------------------------------
// constant tables (src/inftrees.c:59-87; op = 16+extra deflate, 128+extra d64,
// 64 invalid, 96 end of block)
// ---------------------------------------------------------------------------
static __constant__ uint16_t c_lbase[2][31] = {
    {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 0, 0},
    {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 3, 0, 0}};
static __constant__ uint8_t c_lop[2][31] = {
    {16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 18, 18, 18, 18, 19, 19, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21, 16, 73, 200},
    {128, 128, 128, 128, 128, 128, 128, 128, 129, 129, 129, 129, 130, 130, 130, 130, 131, 131, 131, 131, 132, 132, 132, 132,
     133, 133, 133, 133, 144, 73, 200}};
static __constant__ uint16_t c_dbase[2][32] = {
    {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193,
     12289, 16385, 24577, 0, 0},
    {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193,
     12289, 16385, 24577, 32769, 49153}};
static __constant__ uint8_t c_dop[2][32] = {
    {16, 16, 16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 21, 21, 22, 22, 23, 23, 24, 24, 25, 25, 26, 26, 27, 27, 28, 28, 29, 29, 64, 64},
    {128, 128, 128, 128, 129, 129, 130, 130, 131, 131, 132, 132, 133, 133, 134, 134, 135, 135, 136, 136, 137, 137, 138, 138,
     139, 139, 140, 140, 141, 141, 142, 142}};
static __constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum { T_CODES = 0, T_LENS = 1, T_DISTS = 2 };

__device__ __forceinline__ uint32_t mk_entry(uint32_t op, uint32_t bits, uint32_t val) {
  return op | (bits << 8) | (val << 16);
}
__device__ __forceinline__ uint32_t e_op(uint32_t e) { return e & 0xffu; }
__device__ __forceinline__ uint32_t e_bits(uint32_t e) { return (e >> 8) & 0xffu; }
__device__ __forceinline__ uint32_t e_val(uint32_t e) { return e >> 16; }

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (WAVE - 1); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ---------------------------------------------------------------------------
// Table builder: canonical Huffman -> zlib-layout 2-level table in LDS.
// Restates src/inftrees.c:33-321; the sort and the root fill run across lanes,
// the long-code sub-tables keep zlib's allocation order and sizing.
// Returns 0 ok, -1 bad code set, 1 table space exceeded.  `*root` is in/out.
// ---------------------------------------------------------------------------
#ifndef BUILD_TABLE_ATTR
// (round 6) inlined: as a call it cost zs_unit_header_kernel 102 VGPRs and
// scratch (occupancy 4); inlined 49 VGPRs, occupancy 7.  inflate_kernels.hip
// keeps the call (its stream decoders were slower with it inlined)
#define BUILD_TABLE_ATTR __attribute__((always_inline))
#endif
static __device__ BUILD_TABLE_ATTR int build_table(int type, const uint16_t *lens, uint32_t n, uint32_t *table, uint32_t *root_io,
                           uint16_t *sorted, uint32_t *scratch16, int d64) {
  const uint32_t lane = lane_id();
  const uint64_t lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint32_t cnt[16];
#pragma unroll
  for (int L = 0; L < 16; L++) cnt[L] = 0;
  for (uint32_t g = 0; g < n; g += WAVE) {
    uint32_t s = g + lane;
    uint32_t L = (s < n) ? lens[s] : 16u;
#pragma unroll
    for (int x = 0; x < 16; x++) cnt[x] += __popcll(__ballot(L == (uint32_t)x));
  }
  uint32_t maxlen = 0, minlen = 0;
#pragma unroll
  for (int x = 15; x >= 1; x--)
    if (maxlen == 0 && cnt[x]) maxlen = x;
  uint32_t root = *root_io;
  if (root > maxlen) root = maxlen;
  if (maxlen == 0) {
    if (d64) return -1;  // src/inftrees.c:131-132
    if (lane < 2) table[lane] = mk_entry(64, 1, 0);
    __builtin_amdgcn_wave_barrier();
    *root_io = 1;
    return 0;
  }
#pragma unroll
  for (int x = 1; x <= 15; x++)
    if (minlen == 0 && cnt[x]) minlen = x;
  if (root < minlen) root = minlen;
  int room = 1;
  bool over = false;
#pragma unroll
  for (int x = 1; x <= 15; x++) {
    room = (room << 1) - (int)cnt[x];
    over |= room < 0;
  }
  if (over) return -1;
  if (room > 0 && (type == T_CODES || maxlen != 1)) return -1;

  // canonical first codes and sorted offsets
  uint32_t start[16], first[16];
  start[0] = 0;
  start[1] = 0;
  first[0] = 0;
  first[1] = 0;
#pragma unroll
  for (int x = 1; x < 15; x++) {
    start[x + 1] = start[x] + cnt[x];
    first[x + 1] = (first[x] + cnt[x]) << 1;
  }
  // publish counts and starts for the serial sub-table pass
  if (lane < 16) {
    uint32_t c = 0, st = 0;
#pragma unroll
    for (int x = 0; x < 16; x++) {
      if ((uint32_t)x == lane) { c = cnt[x]; st = start[x]; }
    }
    scratch16[lane] = c;
    scratch16[16 + lane] = st;
  }
  // stable sort of symbols by length (ballot rank within each length)
  {
    uint32_t base[16];
#pragma unroll
    for (int x = 0; x < 16; x++) base[x] = start[x];
    for (uint32_t g = 0; g < n; g += WAVE) {
      uint32_t s = g + lane;
      uint32_t L = (s < n) ? lens[s] : 0u;
#pragma unroll
      for (int x = 1; x <= 15; x++) {
        uint64_t m = __ballot(L == (uint32_t)x);
        if (L == (uint32_t)x) sorted[base[x] + __popcll(m & lt_mask)] = (uint16_t)s;
        base[x] += __popcll(m);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();

  const uint32_t first_coded = (type == T_CODES) ? 20u : (type == T_LENS ? 257u : 0u);
  const uint32_t lim = (type == T_LENS) ? (d64 ? 851u : 852u) : (type == T_DISTS ? (d64 ? 593u : 592u) : 0xffffffffu);
  uint32_t used = 1u << root;
  if (used > lim) return 1;
  const uint32_t ncodes = start[15] + cnt[15];
  // number of codes of length <= root
  uint32_t nshort = 0;
#pragma unroll
  for (int x = 1; x <= 15; x++)
    if ((uint32_t)x <= root) nshort += cnt[x];

  auto sym_entry = [&](uint32_t s, uint32_t bits) -> uint32_t {
    if (s + 1u < first_coded) return mk_entry(0, bits, s);
    if (s >= first_coded) {
      uint32_t k = s - first_coded;
      if (type == T_LENS) return mk_entry(c_lop[d64][k], bits, c_lbase[d64][k]);
      return mk_entry(c_dop[d64][k], bits, c_dbase[d64][k]);
    }
    return mk_entry(96, bits, 0);
  };

  // root fill for short codes: lane-parallel over codes, replicated entries
  for (uint32_t g = 0; g < nshort; g += WAVE) {
    uint32_t i = g + lane;
    if (i < nshort) {
      uint32_t s = sorted[i];
      uint32_t L = lens[s];
      uint32_t st = scratch16[16 + L];
      uint32_t code = 0;
#pragma unroll
      for (int x = 1; x <= 15; x++)
        if ((uint32_t)x == L) code = first[x];
      code += i - st;
      uint32_t rev = __builtin_bitreverse32(code) >> (32 - L);
      uint32_t e = sym_entry(s, L);
      uint32_t reps = 1u << (root - L);
      for (uint32_t j = 0; j < reps; j++) table[rev + (j << L)] = e;
    }
  }
  // incomplete single 1-bit code: slot 1 is an invalid marker
  if (room > 0 && lane == 0) table[1] = mk_entry(64, 1, 0);

  // long codes, 64 at a time across the lanes.  In sorted order the codes of
  // one sub-table (same root bits `low`) are consecutive; a sub-table's size
  // depends only on the counts of its first code's length and longer ones
  // (src/inftrees.c:258-274, `count[len]` less the codes of that length
  // already placed), so every group start sizes its own sub-table and a scan
  // of the sizes gives zlib's allocation offsets (`next`).
  uint32_t c_low = 0xffffffffu, c_next = 0, c_size = 0, c_sum = 1u << root;
  const uint32_t rmask = (1u << root) - 1;
  for (uint32_t g0 = nshort; g0 < ncodes; g0 += WAVE) {
    const uint32_t i = g0 + lane;
    const bool act = i < ncodes;
    uint32_t s = 0, L = root + 1, rev = 0, low = 0xfffffffeu;
    if (act) {
      s = sorted[i];
      L = lens[s];
      const uint32_t st = scratch16[16 + L];
      uint32_t code = 0;
#pragma unroll
      for (int x = 1; x <= 15; x++)
        if ((uint32_t)x == L) code = first[x];
      code += i - st;
      rev = __builtin_bitreverse32(code) >> (32 - L);
      low = rev & rmask;
    }
    uint32_t prev_low = (uint32_t)__shfl_up((int)low, 1);
    if (lane == 0) prev_low = c_low;
    const bool start = act && low != prev_low;
    uint32_t curr = 0, size = 0;
    if (start) {
      const uint32_t st = scratch16[16 + L];
      curr = L - root;
      int left = 1 << curr;
      while (curr + root < maxlen) {
        const uint32_t x = curr + root;
        const uint32_t remain = scratch16[x] - ((x == L) ? (i - st) : 0u);
        left -= (int)remain;
        if (left <= 0) break;
        curr++;
        left <<= 1;
      }
      size = 1u << curr;
    }
    // inclusive sum of sizes and the latest group start at or before each lane
    uint32_t incl = size;
    int sl = start ? (int)lane : -1;
#pragma unroll
    for (uint32_t d = 1; d < WAVE; d <<= 1) {
      const uint32_t v = (uint32_t)__shfl_up((int)incl, d);
      const int m = __shfl_up(sl, d);
      if (lane >= d) {
        incl += v;
        sl = max(sl, m);
      }
    }
    const uint32_t gnext_own = c_sum + incl - size;
    const uint32_t gnext_sl = (uint32_t)__shfl((int)gnext_own, sl < 0 ? 0 : sl);
    const uint32_t gsize_sl = (uint32_t)__shfl((int)size, sl < 0 ? 0 : sl);
    const uint32_t gnext = sl < 0 ? c_next : gnext_sl;
    const uint32_t gsize = sl < 0 ? c_size : gsize_sl;
    const uint32_t total = uni((uint32_t)__shfl((int)incl, WAVE - 1));
    if (c_sum + total > lim) return 1;  // zlib stops at the first sub-table past the bound: same result
    if (start) table[low] = mk_entry(curr, root, gnext);
    if (act) {
      const uint32_t e = sym_entry(s, L - root);
      const uint32_t step = 1u << (L - root);
      const uint32_t reps = gsize >> (L - root);
      const uint32_t idx0 = gnext + (rev >> root);
      for (uint32_t j = 0; j < reps; j++) table[idx0 + j * step] = e;
    }
    const uint32_t last = min(ncodes - g0, (uint32_t)WAVE) - 1u;
    c_low = uni((uint32_t)__shfl((int)low, last));
    c_next = uni((uint32_t)__shfl((int)gnext, last));
    c_size = uni((uint32_t)__shfl((int)gsize, last));
    c_sum += total;
  }
  __builtin_amdgcn_wave_barrier();
  *root_io = root;
  return 0;
}


// masked 32-bit input word (bytes at or past end_byte read as zero)
static __device__ __forceinline__ uint32_t in_word(const uint32_t *w, uint32_t wi, uint32_t end_byte) {
  uint32_t b = wi * 4u;
  if (b + 4u <= end_byte) return w[wi];
  if (b >= end_byte) return 0u;
  uint32_t keep = end_byte - b;  // 1..3
  return w[wi] & ((1u << (8u * keep)) - 1u);
}
