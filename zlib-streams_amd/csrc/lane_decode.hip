// lane_decode.hip -- the speculative chunk decoder: parse pass + expand pass.
//
// Reference hot loop: src/inffast.c:100-287 (literal/length/distance decode +
// copy), with block headers from src/inflate.c:834-1033 and tables from
// src/inftrees.c:33-321.
//
// Parse pass (zs_lane_kernel, one 64-lane wave = 64 independent chunk decoders):
//   * LDS holds every lane's ROOT tables as compact 16-bit entries: a 9-bit
//     literal/length root (1 KiB per lane) and a 6-bit distance root (128 B),
//     ~80 KiB per wave.  A root entry for a code longer than the root carries
//     the offset and index width of its sub-table, which lives as compact
//     16-bit entries in the lane's global table area (one dependent load);
//     invalid codes re-run zlib's two-level lookup on the lane's zlib-layout
//     table to report exactly what inflate reports;
//   * length/distance base and extra-bit counts are computed arithmetically
//     from the code index (no table loads);
//   * every symbol becomes one u32 token (no history reads at all);
//   * block headers / stored blocks are processed cooperatively: the whole
//     wave works on one lane's header (bits staged in LDS, ballot-parallel
//     table build), then writes that lane's compact roots and sub-tables.
// Expand pass (zs_expand_kernel): see below.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zs_common.h"
#include "zs_device.h"
#include "zs_kprof.h"

#include <hipcub/device/device_radix_sort.hpp>
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#if KP_ON
__device__ unsigned long long g_kprof[KP_COUNT];
// wave-uniform value, added once per wave (v is evaluated by every lane, so
// that a kp_wave_sum inside it sees the whole wave)
#define KP_ADD(i, v)                                              \
  do {                                                            \
    const unsigned long long kp_v_ = (unsigned long long)(v);     \
    if (lane_id() == 0) atomicAdd(&g_kprof[i], kp_v_);            \
  } while (0)
#define KP_MAX(i, v)                                              \
  do {                                                            \
    const unsigned long long kp_v_ = (unsigned long long)(v);     \
    if (lane_id() == 0) atomicMax(&g_kprof[i], kp_v_);            \
  } while (0)
__device__ __forceinline__ uint32_t kp_wave_sum(uint32_t v) {
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint32_t kp_wave_max(uint32_t v) {
  for (int o = 32; o; o >>= 1) v = max(v, (uint32_t)__shfl_xor(v, o));
  return v;
}
#else
#define KP_ADD(i, v) ((void)0)
#define KP_MAX(i, v) ((void)0)
#endif

#define MARK_BASE 256u
#define HIST 32768u
#define STAGE_WORDS 256  // 1 KiB of staged header bits per cooperative step
#define LROOT_N 256      // 8-bit literal/length root (LDS)
#define DROOT_N 64       // 6-bit distance root
#define ZBUILD 852       // zlib build area (ENOUGH_LENS; the distance table reuses it)
#define RING 16          // input words per lane staged in LDS for a group of steps

// compact entry (u16): [1:0] kind, [5:2] code bits, [15:6] symbol.
// CK_SLOW: [5:2] = sub-table index bits (0 = invalid code), [15:6] = sub-table
// offset (zlib's link entry, src/inftrees.c:250-262); sub-table entries carry
// the TOTAL code length in [5:2] (root bits + sub bits <= 15).  In the 8-bit
// LDS literal/length root, [5:2] = 15 means "look up zlib's 9-bit root in the
// lane's global compact table" (the prefix covers 9-bit or longer codes).
enum { CK_SYM = 0, CK_LEN = 1, CK_EOB = 2, CK_SLOW = 3 };

__device__ __forceinline__ uint16_t compact_len_entry(uint32_t z, uint32_t add_bits = 0) {
  const uint32_t op = e_op(z), bits = e_bits(z) + add_bits, val = e_val(z);
  if (op == 0) return (uint16_t)(CK_SYM | (bits << 2) | (val << 6));
  if (op & 32) return (uint16_t)(CK_EOB | (bits << 2));  // 96 = end of block
  if (op & 64) return (uint16_t)CK_SLOW;                 // invalid code
  if ((op & 0xf0u) == 0) return (uint16_t)(CK_SLOW | (op << 2) | (val << 6));  // sub-table link
  // length base -> code index k (lbase of src/inftrees.c:59-61; deflate64's
  // code 285 is op 144, base 3 + 16 extra bits, src/inftrees.c:73-77)
  const uint32_t e = op & 15u;
  uint32_t k;
  if (val == 258 || op == 144) k = 28;
  else if (e == 0) k = val - 3;
  else k = 4 * (e + 1) + ((val - 3) >> e) - 4;
  return (uint16_t)(CK_LEN | (bits << 2) | (k << 6));
}
__device__ __forceinline__ uint16_t compact_dist_entry(uint32_t z, uint32_t add_bits = 0) {
  const uint32_t op = e_op(z), bits = e_bits(z) + add_bits, val = e_val(z);
  if (op & 64) return (uint16_t)CK_SLOW;
  if ((op & 0xf0u) == 0) return (uint16_t)(CK_SLOW | (op << 2) | (val << 6));
  const uint32_t e = op & 15u;
  const uint32_t d = (e == 0) ? val - 1 : 2 * (e + 1) + ((val - 1) >> e) - 2;
  return (uint16_t)(CK_SYM | (bits << 2) | (d << 6));
}

#define OP_ROOT9 15u

// Split parse walk tables (zs_walk_kernel): u8 entries indexed by the next
// WK_LBITS (literal/length) or WK_DBITS (distance) input bits.  An entry holds
// the bits the whole element takes -- code plus extra bits -- so the walk
// needs no symbol values at all: [4:0] bits, WK_HASD a length (a distance
// follows), WK_BIG deflate64's code 285 (16 extra bits: a length > 65535 is
// two tokens), WK_EXC anything the walk resolves off its fast path (end of
// block, an invalid code, a code longer than the table's index).  A distance
// entry WK_BAD (WK_EXC | WK_BIG) is an invalid code; a plain WK_EXC distance
// entry is a code longer than the index (the walk's canonical tail decodes it).
#define WK_LBITS 9u
#define WK_DBITS 8u
#define WK_HASD 0x20u
#define WK_EXC 0x40u
#define WK_BIG 0x80u
#define WK_BAD (WK_EXC | WK_BIG)
#define WK_EOBE (WK_EXC | WK_HASD)  // end-of-block entry: | its code bits
template <bool D64>
__device__ __forceinline__ uint32_t walk_len_entry(uint32_t ce) {  // from a compact literal/length entry
  const uint32_t kind = ce & 3u, bits = (ce >> 2) & 15u, sym = ce >> 6;
  if (kind == CK_SYM) return bits;
  if (kind == CK_EOB) return WK_EOBE | bits;  // end of block: its code bits (resolved without the tables)
  if (kind != CK_LEN) return WK_EXC;
  const uint32_t xb = sym < 8u ? 0u : (sym < 28u ? (sym >> 2) - 1u : (D64 ? 16u : 0u));
  return (bits + xb) | WK_HASD | ((D64 && sym >= 28u) ? WK_BIG : 0u);
}
__device__ __forceinline__ uint32_t walk_dist_entry(uint32_t ce) {  // from a compact distance entry
  if ((ce & 3u) != CK_SYM) return WK_EXC;
  const uint32_t bits = (ce >> 2) & 15u, dsym = (ce >> 6) & 31u;
  return bits + (dsym < 4u ? 0u : (dsym >> 1) - 1u);  // extra bits: src/inftrees.c:65-72
}
// walk entries from zlib-layout tables (root lbits / dbits) for index i
template <bool D64>
__device__ __forceinline__ uint32_t walk_len_z(const uint32_t *zt, uint32_t lbits, uint32_t i) {
  const uint32_t z = zt[i & ((1u << lbits) - 1u)];
  const uint32_t op = e_op(z);
  if (op != 0 && (op & 0xf0u) == 0) return WK_EXC;  // sub-table: longer than WK_LBITS (lbits = 9 here)
  return walk_len_entry<D64>(compact_len_entry(z));
}
__device__ __forceinline__ uint32_t walk_dist_z(const uint32_t *zt, uint32_t dbits, uint32_t i) {
  const uint32_t z = zt[i & ((1u << dbits) - 1u)];
  const uint32_t op = e_op(z);
  if (op & 64u) return WK_BAD;
  if ((op & 0xf0u) == 0) {  // sub-table: the index's bits past the root pick the entry if the code fits
    const uint32_t avail = WK_DBITS - dbits;
    const uint32_t z2 = zt[e_val(z) + ((i >> dbits) & ((1u << min(op, avail)) - 1u))];
    if (dbits + e_bits(z2) > WK_DBITS) return WK_EXC;  // longer than the index: the canonical tail
    if (e_op(z2) & 64u) return WK_BAD;
    return walk_dist_entry(compact_dist_entry(z2, dbits));
  }
  return walk_dist_entry(compact_dist_entry(z));
}

// LDS root entry for 8-bit prefix i from a zlib literal/length table with
// lbits-bit root (lbits <= 9)
__device__ __forceinline__ uint16_t lds_len_root(const uint32_t *zt, uint32_t lbits, uint32_t i) {
  if (lbits <= 8) return compact_len_entry(zt[i & ((1u << lbits) - 1u)]);
  const uint32_t z0 = zt[i], z1 = zt[i | 256u];
  const bool link = e_op(z0) != 0 && (e_op(z0) & 0xf0u) == 0;
  if (z0 == z1 && !link) return compact_len_entry(z0);  // code of <= 8 bits (or invalid both ways)
  return (uint16_t)(CK_SLOW | (OP_ROOT9 << 2));
}

typedef __attribute__((address_space(1))) const uint32_t gcu32;
typedef __attribute__((address_space(1))) uint32_t gu32;

// Raw buffer stores through a wave-uniform resource (round 6): a lane whose
// byte offset is BUF_SKIP (out of range) stores nothing -- no memory traffic --
// so a store every lane issues at every iteration (uniform control flow, hence
// exact vmcnt waits for the loads around it) can still be a conditional one.
// gfx9 raw buffer resource: word 3 = 0x00020000 (untyped, offsets in bytes);
// num_records bounds the offsets (< 4 GiB).
#define BUF_SKIP 0x80000000u
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}
typedef __attribute__((address_space(1))) const uint16_t gcu16;

// masked input word: bytes at or past end_byte read as zero; never reads a
// word that holds no input byte
__device__ __forceinline__ uint32_t in_word_g(gcu32 *w, uint32_t wi, uint32_t end_byte) {
  const uint32_t v = w[min(wi, (end_byte - 1u) >> 2)];
  const uint32_t b = wi * 4u;
  const uint32_t keep = b >= end_byte ? 0u : end_byte - b;
  return keep >= 4u ? v : __builtin_amdgcn_ubfe(v, 0, 8u * keep);
}

// Token storage (zs_common.h): token x of a unit lives in its primary
// region (x < tcap) or in pool page k of its page table, page k holding
// 2^k pool units of 2^ZS_TP_LOG tokens (geometric: 16 pages cover 4 Gi
// tokens).  Only the unit's writer calls tok_ensure (one lane at a time);
// each page is taken from the pool with one atomic.  Returns false when the
// pool is exhausted.
__device__ __forceinline__ uint32_t tok_page(uint32_t r, uint32_t *off) {  // r = x - tcap
  const uint32_t q = (r >> ZS_TP_LOG) + 1u;
  const uint32_t k = 31u - (uint32_t)__builtin_clz(q);
  *off = r - (((1u << k) - 1u) << ZS_TP_LOG);
  return k;
}
__device__ __forceinline__ bool tok_ensure(const ZsTokPool &pool, uint32_t unit, uint32_t tcap, uint32_t x_end) {
  if (x_end <= tcap) return true;
  uint32_t off;
  const uint32_t kl = tok_page(x_end - 1u - tcap, &off);
  if (kl >= ZS_TP_MAXPG) return false;
  uint32_t *pt = pool.ptab + (size_t)unit * ZS_TP_MAXPG;
  for (uint32_t k = 0; k <= kl; k++) {
    uint32_t pg = __hip_atomic_load(pt + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!pg) {
      pg = atomicAdd(pool.next, 1u << k) + 1u;
      if (pg - 1u + (1u << k) > pool.npages) return false;
      __hip_atomic_store(pt + k, pg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  return true;
}
// address of token x (pages already ensured); page ids are read from L2
__device__ __forceinline__ uint32_t *tok_addr(const ZsTokPool &pool, uint32_t *tokens, uint32_t unit, uint64_t prim,
                                              uint32_t tcap, uint32_t x) {
  if (x < tcap) return tokens + prim + x;
  uint32_t off;
  const uint32_t k = tok_page(x - tcap, &off);
  const uint32_t pg =
      __hip_atomic_load(pool.ptab + (size_t)unit * ZS_TP_MAXPG + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return tokens + pool.base + ((uint64_t)(pg - 1u) << ZS_TP_LOG) + off;
}

enum { LM_SYM = 0, LM_BLOCK = 1, LM_DONE = 2 };

struct KpPhase {
  uint64_t t[5];
};

struct LaneState {
  gcu32 *w;           // 4-byte aligned input base
  uint32_t end_byte, limit;
  uint32_t wi, nw, nkeep, nbits;  // nw: next input word (index wi); nkeep: its valid bytes (0..4)
  uint32_t rk;        // ring index of nw during a group
  uint32_t lastw;     // last word index holding input
  uint64_t hold;
  gu32 *tok;          // primary token region (parse pass); later tokens: pool pages
  uint32_t ntok, tcap;
  uint32_t unit;      // unit slot (page table row)
  uint32_t gk;        // tokens of the current group (in LDS)
#if KP_ON
  uint32_t kp_steps, kp_slow_l, kp_slow_d, kp_refills;
#endif
  uint4 dta, dtb;     // the lane's distance tail header (lim / offs), loaded at group start
  uint32_t pos, cap;  // entries the tokens expand to / entry capacity
  uint32_t capx;      // min(cap, pos + tcap - ntok) at block start: one check covers both
  gcu16 *cl, *cd;     // compact sub-tables (global) of the current block
  const uint32_t *zl, *zd;  // zlib-layout tables (global): invalid-code reporting
  uint32_t zlmask, zdmask;
  uint32_t lbits, dbits;    // root widths of the current block's zlib tables
  uint32_t stop, bit, whave;
  uint32_t sidx, send;      // unit slot whose start is `stop`; end of the job's unit slots
  int mode, code, last;
};

// prefetch word wi raw; the end-of-input mask is applied when it is used, so
// the load's latency hides behind the current symbol
__device__ __forceinline__ void lane_fetch(LaneState &s) {
  s.nw = s.w[min(s.wi, s.lastw)];
  const uint32_t b = s.wi * 4u;
  s.nkeep = b >= s.end_byte ? 0u : min(s.end_byte - b, 4u);
}
__device__ __forceinline__ uint32_t lane_take(const LaneState &s) {
  return s.nkeep >= 4u ? s.nw : __builtin_amdgcn_ubfe(s.nw, 0, 8u * s.nkeep);
}
__device__ __forceinline__ void lane_prime(LaneState &s, uint32_t bit) {
  s.lastw = (s.end_byte - 1u) >> 2;
  s.wi = bit >> 5;
  const uint32_t w0 = in_word_g(s.w, s.wi, s.end_byte);
  s.wi += 1;
  lane_fetch(s);
  s.hold = (uint64_t)w0 >> (bit & 31);
  s.nbits = 32 - (bit & 31);
}
// refill from the group's LDS ring (words are masked at fill time)
__device__ __forceinline__ void lane_refill(LaneState &s, const uint32_t *__restrict__ rp) {
  if (s.nbits < 32) {
#if KP_ON
    s.kp_refills++;
#endif
    s.hold |= (uint64_t)s.nw << s.nbits;
    s.nbits += 32;
    s.wi++;
    s.rk++;
    s.nw = rp[s.rk * WAVE];
  }
}
// input words wi .. wi + RING - 1 (masked) into registers
__device__ __forceinline__ void lane_load_ring(const LaneState &s, uint32_t (&v)[RING]) {
  if (s.wi + RING <= s.lastw) {  // all full words: 16-byte loads
    const uint32_t *src = (const uint32_t *)(s.w + s.wi);
#pragma unroll
    for (int q = 0; q < RING / 4; q++) {
      uint4 x;
      __builtin_memcpy(&x, src + 4 * q, 16);
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < RING; q++) v[q] = in_word_g(s.w, s.wi + q, s.end_byte);
  }
}
__device__ __forceinline__ void lane_store_ring(LaneState &s, uint32_t *__restrict__ rp, const uint32_t (&v)[RING]) {
#pragma unroll
  for (int q = 0; q < RING; q++) rp[q * WAVE] = v[q];
  s.nw = v[0];
  s.rk = 0;
}
// group start: ring[0..RING) = input words wi .. wi + RING - 1 (masked)
__device__ __forceinline__ void lane_fill_ring(LaneState &s, uint32_t *__restrict__ rp) {
  uint32_t v[RING];
  lane_load_ring(s, v);
  lane_store_ring(s, rp, v);
}
// bit position of the next unconsumed bit (wi = index of the prefetched word)
__device__ __forceinline__ uint32_t lane_pos(const LaneState &s) { return s.wi * 32u - s.nbits; }

// zlib's two-level lookup (src/inffast.c:125-135) on the zlib-layout table;
// used only to size an invalid code for the truncated-vs-invalid decision
__device__ __noinline__ uint32_t invalid_code_bits(const uint32_t *zt, uint32_t zmask, uint32_t hold) {
  uint32_t z = zt[hold & zmask];
  uint32_t used = e_bits(z);
  if (e_op(z) != 0 && (e_op(z) & 0xf0u) == 0) {
    z = zt[e_val(z) + ((hold >> used) & ((1u << e_op(z)) - 1u))];
    used += e_bits(z);
  }
  return used;
}

// one symbol; returns true when the lane left symbol mode.  Bits past the end
// of the input read as zero; truncation is decided once the symbol is
// complete (or, for an invalid code, from zlib's code length), which gives
// the same ZD_TRUNC / error split as checking before every bit pull.
// code longer than the 6-bit distance root: canonical decode from the lane's
// 64-byte tail (two LDS round trips); returns a compact entry (total length)
__device__ __forceinline__ uint32_t dist_tail(const uint32_t *__restrict__ dtl, uint32_t hold) {
  const uint4 a = *reinterpret_cast<const uint4 *>(dtl);
  const uint4 b = *reinterpret_cast<const uint4 *>(dtl + 4);
  const uint32_t rev = __builtin_bitreverse32(hold) >> 17;  // next 15 bits, first bit highest
  const uint32_t lw[5] = {a.x, a.y, a.z, a.w, b.x};
  uint32_t L = 7, fl = lw[0] & 0xffffu, of = (b.x >> 16) & 0xffu;  // lim[0], offs[0]
#pragma unroll
  for (int k = 1; k < 9; k++) {
    const uint32_t lim = (lw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
    // offs[k] lives at byte 18 + k: word 4 + (2 + k) / 4 of the 32 bytes read
    const uint32_t ob = 18 + k;
    const uint32_t ow = ob < 20 ? b.x : (ob < 24 ? b.y : b.z);
    const uint32_t ofk = (ow >> (8 * (ob & 3))) & 0xffu;
    const bool ge = rev >= lim;
    L += ge ? 1u : 0u;
    fl = ge ? lim : fl;
    of = ge ? ofk : of;
  }
  const uint32_t idx = of + ((rev - fl) >> (15u - L));
  const uint32_t sym = reinterpret_cast<const uint8_t *>(dtl)[27 + min(idx, 29u)];
  return CK_SYM | (L << 2) | (sym << 6);
}


// dist_tail with the 32-byte tail header already in registers (loaded at group
// start): the canonical search is VALU only and its one LDS read (the symbol)
// is issued next to the distance root's.  lane_step_fast computes it on every
// step, no branch: with 64 lanes some lane needs a long distance code on most
// wave-steps, and the branch paid two dependent LDS round trips (C2 parse
// 11.4 -> 10.8 ms).  Measured and dropped: the header unpacked at group start
// into lim << 8 | offs words, one select per length (11.7 ms: one serial
// select chain instead of three independent ones, at one wave per SIMD)
__device__ __forceinline__ uint32_t dist_tail_r(const uint4 a, const uint4 b, const uint32_t *__restrict__ dtl,
                                                uint32_t hold) {
  const uint32_t rev = __builtin_bitreverse32(hold) >> 17;
  const uint32_t lw[5] = {a.x, a.y, a.z, a.w, b.x};
  uint32_t L = 7, fl = lw[0] & 0xffffu, of = (b.x >> 16) & 0xffu;
#pragma unroll
  for (int k = 1; k < 9; k++) {
    const uint32_t lim = (lw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
    const uint32_t ob = 18 + k;
    const uint32_t ow = ob < 20 ? b.x : (ob < 24 ? b.y : b.z);
    const uint32_t ofk = (ow >> (8 * (ob & 3))) & 0xffu;
    const bool ge = rev >= lim;
    L += ge ? 1u : 0u;
    fl = ge ? lim : fl;
    of = ge ? ofk : of;
  }
  const uint32_t idx = of + ((rev - fl) >> (15u - L));
  const uint32_t sym = reinterpret_cast<const uint8_t *>(dtl)[27 + min(idx, 29u)];
  return CK_SYM | (L << 2) | (sym << 6);
}

#if KP_ON
#define KPT(i)                       \
  do {                               \
    const uint64_t now_ = KP_NOW();  \
    kp.t[i] += now_ - kp_last;       \
    kp_last = now_;                  \
  } while (0)
#else
#define KPT(i) ((void)0)
#endif

template <bool D64>
__device__ __forceinline__ bool lane_step(LaneState &s, const uint16_t *__restrict__ lt, const uint16_t *__restrict__ dt,
                                          uint32_t *__restrict__ tb, const uint32_t *__restrict__ dtl,
                                          const uint32_t *__restrict__ rp, KpPhase &kp) {
#if KP_ON
  uint64_t kp_last = KP_NOW();
#else
  (void)kp;
#endif
  lane_refill(s, rp);
  KPT(0);
  uint32_t e = lt[(uint32_t)s.hold & (LROOT_N - 1)];
#if KP_ON
  s.kp_steps++;
#endif
  if ((e & 3u) == CK_SLOW) {
#if KP_ON
    s.kp_slow_l++;
#endif
    const uint32_t op = (e >> 2) & 15u;
    uint32_t e2 = CK_SLOW;
    if (op == OP_ROOT9) {  // zlib's 9-bit root (compact, global), then its sub-table
      e2 = s.cl[(uint32_t)s.hold & 511u];
      const uint32_t op2 = (e2 >> 2) & 15u;
      if ((e2 & 3u) == CK_SLOW && op2) e2 = s.cl[(e2 >> 6) + (((uint32_t)s.hold >> 9) & ((1u << op2) - 1u))];
    } else if (op) {
      e2 = s.cl[(e >> 6) + (((uint32_t)s.hold >> s.lbits) & ((1u << op) - 1u))];
    }
    if ((e2 & 3u) == CK_SLOW) {
      const uint32_t used = invalid_code_bits(s.zl, s.zlmask, (uint32_t)s.hold);
      s.code = lane_pos(s) + used > s.limit ? ZD_TRUNC : (ZD_ERROR | (ZM_LITLEN_CODE << 8));
      s.mode = LM_DONE;
      return true;
    }
    e = e2;
  }
  KPT(1);
  const uint32_t used = (e >> 2) & 15u;
  s.hold >>= used;
  s.nbits -= used;
  const uint32_t kind = e & 3u, sym = e >> 6;
  uint32_t len = 1, dist = 0;
  if (kind == CK_LEN) {
    // length code sym (0..28): base/extra of src/inftrees.c:59-64, computed
    uint32_t xb = 0;
    if (sym < 8) {
      len = sym + 3;
    } else if (sym < 28) {
      xb = (sym >> 2) - 1;
      len = ((4u + (sym & 3u)) << xb) + 3u;
    } else if (D64) {  // deflate64 code 285: 3 + 16 extra bits
      xb = 16;
      len = 3;
    } else {
      len = 258;
    }
    len += (uint32_t)s.hold & ((1u << xb) - 1u);
    s.hold >>= xb;
    s.nbits -= xb;
    lane_refill(s, rp);
    uint32_t d = dt[(uint32_t)s.hold & (DROOT_N - 1)];
    if ((d & 3u) == CK_SLOW) {
#if KP_ON
      s.kp_slow_d++;
#endif
      const uint32_t op = (d >> 2) & 15u;
      uint32_t d2 = CK_SLOW;
      if (op) d2 = dist_tail(dtl, (uint32_t)s.hold);
      if ((d2 & 3u) == CK_SLOW) {
        const uint32_t dused = invalid_code_bits(s.zd, s.zdmask, (uint32_t)s.hold);
        s.code = lane_pos(s) + dused > s.limit ? ZD_TRUNC : (ZD_ERROR | (ZM_DIST_CODE << 8));
        s.mode = LM_DONE;
        return true;
      }
      d = d2;
    }
    const uint32_t dused = (d >> 2) & 15u, dsym = d >> 6;
    uint32_t dx = 0;
    if (dsym < 4) {
      dist = dsym + 1;
    } else {
      dx = (dsym >> 1) - 1;
      dist = ((2u + (dsym & 1u)) << dx) + 1u;
    }
    s.hold >>= dused;
    dist += (uint32_t)s.hold & ((1u << dx) - 1u);
    s.hold >>= dx;
    s.nbits -= dused + dx;
  }
  KPT(2);
  if (lane_pos(s) > s.limit) {
    s.code = ZD_TRUNC;
    s.mode = LM_DONE;
    return true;
  }
  KPT(3);
  if (kind == CK_EOB) {
    s.bit = lane_pos(s);
    s.mode = LM_BLOCK;
    return true;
  }
  if (s.pos + len > s.capx) {
    s.code = ZD_FULL;
    s.mode = LM_DONE;
    return true;
  }
  if (dist > s.pos + s.whave) {
    s.code = ZD_ERROR | (ZM_TOO_FAR << 8);
    s.mode = LM_DONE;
    return true;
  }
  if (D64 && len > 0xffffu) {  // a deflate64 copy longer than a token holds: two copies, same distance
    tb[s.gk * WAVE] = (0xffffu << 16) | (dist - 1u);
    s.gk++;
    s.ntok++;
    tb[s.gk * WAVE] = ((len - 0xffffu) << 16) | (dist - 1u);
  } else {
    tb[s.gk * WAVE] = kind == CK_SYM ? sym : ((len << 16) | (dist - 1u));
  }
  KPT(4);
  s.gk++;
  s.ntok++;
  s.pos += len;
  return false;
}

// refill without a branch: the ring word after nw is read every time (same word
// when no refill happens), the hold / counters advance by selects
__device__ __forceinline__ void lane_refill_bf(LaneState &s, const uint32_t *__restrict__ rp) {
  const uint32_t r = s.nbits < 32u;
  const uint64_t add = (uint64_t)s.nw << (s.nbits & 31u);
  s.hold |= r ? add : 0ull;
  s.nbits += r << 5;
  s.wi += r;
  s.rk += r;
  s.nw = rp[s.rk * WAVE];
}

// The common symbol, straight-line: literal / length from the LDS root (codes
// longer than the root via the lane's compact sub-tables in a wave-uniform side
// branch), length / distance bases by shifts and selects (no sym < 8 / sym < 28
// branches), refills by selects, distance from the LDS root (the canonical tail
// in a side branch), the exception test as one bitwise OR and the token stored
// unconditionally (a slot past gk is never read).  Anything lane_step would
// treat differently -- end of block, invalid codes, a full unit, a too-far
// distance, truncation, a deflate64 copy longer than a token -- restores the
// lane's reader and runs lane_step itself, so results are lane_step's by
// construction.  At one wave per SIMD the parse is issue-bound on this loop:
// the short-circuit form (branchy length bases, `||` exception chain,
// conditional refills) compiled to nested exec-mask branches; written this
// way C2's parse went 18.0 -> 15.0 ms.
template <bool D64>
__device__ __forceinline__ bool lane_step_fast(LaneState &s, const uint16_t *__restrict__ lt,
                                               const uint16_t *__restrict__ dt, uint32_t *__restrict__ tb,
                                               const uint32_t *__restrict__ dtl, const uint32_t *__restrict__ rp,
                                               KpPhase &kp) {
  const uint64_t h0 = s.hold;
  const uint32_t nb0 = s.nbits, wi0 = s.wi, rk0 = s.rk, nw0 = s.nw;
  lane_refill_bf(s, rp);
  uint32_t e = lt[(uint32_t)s.hold & (LROOT_N - 1)];
  uint32_t kind = e & 3u;
  if (__builtin_expect(__ballot(kind == CK_SLOW) != 0, 0)) {
#if KP_ON
    const uint64_t kq = KP_NOW();
    s.kp_slow_l++;  // every lane of a wave taking the side branch: sum / lane steps = its wave-step share
#endif
    if (kind == CK_SLOW) {
      const uint32_t op = (e >> 2) & 15u;
      uint32_t e2 = CK_SLOW;
      if (op == OP_ROOT9) {
        e2 = s.cl[(uint32_t)s.hold & 511u];
        const uint32_t op2 = (e2 >> 2) & 15u;
        if ((e2 & 3u) == CK_SLOW && op2) e2 = s.cl[(e2 >> 6) + (((uint32_t)s.hold >> 9) & ((1u << op2) - 1u))];
      } else if (op) {
        e2 = s.cl[(e >> 6) + (((uint32_t)s.hold >> s.lbits) & ((1u << op) - 1u))];
      }
      e = e2;
      kind = e & 3u;
    }
#if KP_ON
    kp.t[0] += KP_NOW() - kq;
#endif
  }
  const uint32_t used = (e >> 2) & 15u, sym = e >> 6;
  const uint32_t isl = kind == CK_LEN;
  // length code sym (0..28), src/inftrees.c:59-64: extra = max(sym/4 - 1, 0),
  // base = ((4 + sym%4) << extra) + 3, minus 4 for sym < 4; code 28 is 258
  // (deflate64 285: 3 + 16 extra bits)
  const uint32_t top = sym >= 28u;
  uint32_t xb = (uint32_t)max((int)(sym >> 2) - 1, 0);
  xb = top ? (D64 ? 16u : 0u) : xb;
  xb = isl ? xb : 0u;
  uint32_t lbase = ((4u + (sym & 3u)) << (xb & 15u)) + 3u - (sym < 4u ? 4u : 0u);
  lbase = top ? (D64 ? 3u : 258u) : lbase;
  s.hold >>= used;
  const uint32_t len = isl ? lbase + ((uint32_t)s.hold & ((1u << xb) - 1u)) : 1u;
  s.hold >>= xb;
  s.nbits -= used + xb;
  lane_refill_bf(s, rp);
  uint32_t d = dt[(uint32_t)s.hold & (DROOT_N - 1)];
  const uint32_t dtr = dist_tail_r(s.dta, s.dtb, dtl, (uint32_t)s.hold);
  const bool dslow = isl && (d & 3u) == CK_SLOW;
  d = dslow ? (((d >> 2) & 15u) ? dtr : (uint32_t)CK_SLOW) : d;
  // distance code dsym (0..31), src/inftrees.c:65-72: extra = max(dsym/2 - 1, 0),
  // base = ((2 + dsym%2) << extra) + 1, minus 2 for dsym < 2
  const uint32_t dused = (d >> 2) & 15u, dsym = (d >> 6) & 31u;
  const uint32_t dx = min((uint32_t)max((int)(dsym >> 1) - 1, 0), 14u);
  const uint32_t dist = ((2u + (dsym & 1u)) << dx) + 1u - (dsym < 2u ? 2u : 0u) +
                        ((uint32_t)(s.hold >> dused) & ((1u << dx) - 1u));
  const uint32_t dcons = isl ? dused + dx : 0u;
  s.hold >>= dcons;
  s.nbits -= dcons;
#if KP_ON
  s.kp_steps++;
#else
  (void)kp;
#endif
  const uint32_t exc = (uint32_t)(kind >= CK_EOB) | (isl & (uint32_t)((d & 3u) == CK_SLOW)) |
                       (uint32_t)(lane_pos(s) > s.limit) | (uint32_t)(s.pos + len > s.capx) |
                       (isl & (uint32_t)(dist > s.pos + s.whave)) | (uint32_t)(D64 && len > 0xffffu);
  tb[s.gk * WAVE] = isl ? ((len << 16) | (dist - 1u)) : sym;
  if (exc) {
    s.hold = h0;
    s.nbits = nb0;
    s.wi = wi0;
    s.rk = rk0;
    s.nw = nw0;
#if KP_ON
    s.kp_steps--;
#endif
    return lane_step<D64>(s, lt, dt, tb, dtl, rp, kp);
  }
  s.gk++;
  s.ntok++;
  s.pos += len;
  return false;
}

// Wave-uniform bit reader over the LDS-staged header bits.
struct StageBits {
  const uint32_t *st;
  uint32_t base;  // bit index of st[0] in the input
  __device__ __forceinline__ uint32_t peek(uint32_t bit, uint32_t n) const {
    const uint32_t r = bit - base;
    const uint64_t v = (uint64_t)st[r >> 5] | ((uint64_t)st[(r >> 5) + 1] << 32);
    return (uint32_t)(v >> (r & 31)) & ((n >= 32) ? 0xffffffffu : ((1u << n) - 1u));
  }
};

// Symbol steps run in groups of GROUP; each lane's tokens of a group wait in
// LDS (tokbuf, which shares space with the header build area: headers are
// only processed between groups) and leave in one flush, so the step loop
// itself issues no global stores (vmcnt is in-order: a store in the loop
// would make every input refill wait for it).
#define GROUP 16

struct BuildLDS {  // one wave's header-decode / table-build area
  uint32_t stage[STAGE_WORDS + 4];
  uint32_t tab[ZBUILD];
  uint16_t lens[320];
  uint16_t sorted[320];
  uint32_t scr[32];
};

// Distance codes longer than the 6-bit root decode canonically from 64 bytes
// per lane (src/inftrees.c assigns codes canonically: consecutive values in
// symbol order within a length, lengths in increasing order):
//   [0, 18)  u16 lim[k]: left-aligned 15-bit end of the length-(6+k) codes
//   [18, 27) u8 offs[k]: rank of the first length-(7+k) code among tail codes
//   [27, 57) u8 sym[]:   tail symbols (length >= 7) in canonical order
#define DTAIL_BYTES 64

// Input ring: at every group start each lane loads its next RING input words
// into ring[k][lane] (lane-interleaved: conflict-free whatever k each lane
// reads); the steps refill from it, one word prefetched ahead, so a refill
// never waits on global memory.  Like tokbuf it lives only during a group and
// shares space with the header build area.

struct LaneLDS {
  uint16_t lroot[WAVE][LROOT_N];
  uint16_t droot[WAVE][DROOT_N];
  uint32_t dtail[WAVE][DTAIL_BYTES / 4];
  union {
    BuildLDS b;
    struct {
      uint32_t tokbuf[GROUP][WAVE];
      uint32_t ring[RING][WAVE];
    } g;
  };
};

__device__ void stage_bits(BuildLDS &L, const uint32_t *w, uint32_t end_byte, uint32_t bit, StageBits &sb) {
  const uint32_t lane = lane_id();
  const uint32_t b16 = (bit >> 7) << 4;  // byte offset, multiple of 16
  const uint32_t wi = (b16 >> 2) + lane * 4;
#pragma unroll
  for (int k = 0; k < 4; k++) L.stage[lane * 4 + k] = in_word(w, wi + k, end_byte);
  if (lane < 4) L.stage[STAGE_WORDS + lane] = 0;
  __builtin_amdgcn_wave_barrier();
  sb.st = L.stage;
  sb.base = b16 * 8u;
}

__device__ __forceinline__ uintptr_t readlane_ptr(const void *p, uint32_t ln) {
  const uint64_t v = reinterpret_cast<uintptr_t>(p);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, ln);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), ln);
  return (uintptr_t)(((uint64_t)hi << 32) | lo);
}

// canonical tail of a distance code (lengths dl[0..n), n <= 32): limits of
// lengths 6..14 (u16 [0, 18)), the rank of each length 7..15's first code among
// the tail codes (u8 [18, 27)), the tail symbols in canonical order (u8 [27,
// 59)).  Wave-cooperative (round 6; one lane's serial loops over LDS were half
// of a unit header's time): counts by ballots, lane i places symbol i.
__device__ void build_dist_tail(const uint16_t *dl, uint32_t n, uint8_t *out) {
  const uint32_t lane = lane_id();
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const uint32_t len = lane < n ? (dl[lane] & 15u) : 0u;
  uint32_t count[16];
  count[0] = 0;
#pragma unroll
  for (int L = 1; L < 16; L++) count[L] = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(len == (uint32_t)L));
  uint32_t code = 0, first[16];
  first[0] = 0;
#pragma unroll
  for (int L = 1; L < 16; L++) {
    code = (code + count[L - 1]) << 1;
    first[L] = code;
  }
  uint32_t v = 0, off = 0, rank = 0;  // lane k < 9: limit k and rank k; lane i: its rank among the tail
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int L = 6 + k;
    if (lane == (uint32_t)k) {
      v = min((first[L] + count[L]) << (15 - L), 0xffffu);
      off = rank;
    }
    rank += count[7 + k];
  }
  if (lane < 9u) {
    reinterpret_cast<uint16_t *>(out)[lane] = (uint16_t)v;
    out[18 + lane] = (uint8_t)off;
  }
  uint32_t base = 0, mine = 64u;
#pragma unroll
  for (int L = 7; L < 16; L++) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(len == (uint32_t)L);
    if (len == (uint32_t)L) mine = base + (uint32_t)__builtin_popcountll(m & lt_mask);
    base += (uint32_t)__builtin_popcountll(m);
  }
  if (mine < 32u) out[27 + mine] = (uint8_t)lane;
}

// The literal/length code's canonical tail for the split parse's walk (codes
// longer than its 9-bit table), 16 words: 0-3 the left-justified 15-bit
// limits of lengths 9..15 (u16 each, lim[L] = (first[L] + count[L]) << (15 - L)),
// 4-5 the literal count of each length 10..15 (9 bits each, three per word:
// 0..256), 6-7 for
// each length 10..15 the index in the list below of its first symbol >= 256
// (u8), 8-15 that list: the symbols >= 256 (end of block, lengths) whose codes
// are longer than 9 bits, in canonical order, as sym - 256 (u8).  Canonical
// order puts a length's literals first, then its symbols >= 256 in order, so
// a long code's index within its length tells a literal from the list entry
// -- the walk resolves every code from registers and LDS, no global table.
// Wave-cooperative (every lane calls it): counts by ballots, 64 code lengths
// at a time; lanes 0..15 write the 16 words.
__device__ void build_lit_tail(const uint16_t *ll, uint32_t n, uint32_t *out) {
  const uint32_t lane = lane_id();
  uint32_t cnt = 0, nl = 0, nn = 0;  // lane L (1..15): codes of length L, literals, symbols >= 256 among them
  uint32_t lst = 0;                  // lane k (0..31): list byte k
  uint32_t base = 0;                 // running list position (uniform)
  for (uint32_t b = 0; b < n; b += WAVE) {
    const uint32_t i = b + lane;
    const uint32_t len = i < n ? (ll[i] & 15u) : 0u;
#pragma unroll
    for (uint32_t L = 1; L < 16; L++) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(len == L);
      const uint32_t c = (uint32_t)__builtin_popcountll(m);
      const uint32_t cl = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(len == L && i < 256u));
      cnt += lane == L ? c : 0u;
      nl += lane == L ? cl : 0u;
      nn += lane == L ? c - cl : 0u;
    }
  }
  // the list: symbols 256.. sit in the chunk at 256 (lane k: symbol 256 + k);
  // each lane's rank in canonical order, then list byte t = the lane ranked t
  {
    const uint32_t i = 256u + lane;
    const uint32_t len = i < n ? (ll[i] & 15u) : 0u;
    uint32_t rank = 64u;
#pragma unroll
    for (uint32_t L = 10; L < 16; L++) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(len == L);
      if (len == L) rank = base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
      base += (uint32_t)__builtin_popcountll(m);
    }
    for (uint32_t t = 0; t < min(base, 32u); t++) {
      const uint64_t hit = __builtin_amdgcn_ballot_w64(rank == t);
      lst = lane == t ? (uint32_t)__builtin_ctzll(hit) : lst;
    }
  }
  uint32_t code = 0, lim[16], nlit[16], nbase[16];
  lim[0] = nlit[0] = 0;
  uint32_t prev = 0, nb = 0;
#pragma unroll
  for (int L = 1; L < 16; L++) {
    const uint32_t cL = __builtin_amdgcn_readlane(cnt, L);
    nlit[L] = __builtin_amdgcn_readlane(nl, L);
    nbase[L] = nb;
    if (L >= 10) nb += __builtin_amdgcn_readlane(nn, L);
    code = (code + prev) << 1;
    lim[L] = min((code + cL) << (15 - L), 0xffffu);
    prev = cL;
  }
  // list bytes: lane k holds byte k; pack 4 per word
  const uint32_t b0 = __shfl(lst, (int)((lane & 7u) * 4u)), b1 = __shfl(lst, (int)((lane & 7u) * 4u + 1u));
  const uint32_t b2 = __shfl(lst, (int)((lane & 7u) * 4u + 2u)), b3 = __shfl(lst, (int)((lane & 7u) * 4u + 3u));
  const uint32_t lw = (b0 & 0xffu) | ((b1 & 0xffu) << 8) | ((b2 & 0xffu) << 16) | ((b3 & 0xffu) << 24);
  if (lane < 8u) out[8 + lane] = lw;
  if (lane == 0) {
    out[0] = lim[9] | (lim[10] << 16);
    out[1] = lim[11] | (lim[12] << 16);
    out[2] = lim[13] | (lim[14] << 16);
    out[3] = lim[15];
    // 9-bit counts: a complete code may put all 256 literals on one length
    out[4] = nlit[10] | (nlit[11] << 9) | (nlit[12] << 18);
    out[5] = nlit[13] | (nlit[14] << 9) | (nlit[15] << 18);
    out[6] = nbase[10] | (nbase[11] << 8) | (nbase[12] << 16) | (nbase[13] << 24);
    out[7] = nbase[14] | (nbase[15] << 8);
  }
}

// The code lengths of a dynamic header, 64 bit offsets at a time, all in
// parallel (round 6, for zs_unit_header_kernel): lane l decodes the
// code-length symbol at bit + l; the true symbols of the window are found by
// pointer doubling over "next offset" (symbol k at P_k = J^k(0)), their output
// positions by a prefix sum of their repeat counts, a repeat-previous (16) its
// value by a max-scan for the last explicit length.  Same B.lens and end bit as
// the serial loop in wave_dyn_header for every header zlib accepts; on any
// error it returns nonzero without telling which (the unit header then leaves
// the unit to the parse pass, which decodes the header again and reports it).
__device__ int wave_code_lengths_par(BuildLDS &B, const uint32_t *w, uint32_t end_byte, StageBits &sb, uint32_t &bit,
                                     uint32_t total, uint32_t cmask) {
  const uint32_t lane = lane_id();
  const uint32_t limit = end_byte * 8u;
  uint32_t have = 0, prevlen = 0;
  while (have < total) {
    if (bit - sb.base > (STAGE_WORDS - 2) * 32u - 128u) stage_bits(B, w, end_byte, bit, sb);
    const uint32_t xj = sb.peek(bit + lane, 14);
    const uint32_t ej = B.tab[xj & cmask];
    const uint32_t ebj = e_bits(ej), evj = e_val(ej);
    const uint32_t xbj = evj < 16 ? 0u : (evj == 16 ? 2u : (evj == 17 ? 3u : 7u));
    const uint32_t repj = evj < 16 ? 1u : ((evj == 18 ? 11u : 3u) + ((xj >> ebj) & ((1u << xbj) - 1u)));
    const uint32_t lenj = ebj + xbj;
    if (__builtin_amdgcn_ballot_w64(lenj == 0u)) return -1;  // (a complete code-length code has no 0-bit entry)
    // J^(2^b): the offset 2^b symbols on (64: past the window)
    uint32_t Jb[6];
    Jb[0] = min(lane + lenj, 64u);
#pragma unroll
    for (int b = 1; b < 6; b++) {
      const uint32_t pv = Jb[b - 1];
      const uint32_t g = (uint32_t)__shfl((int)pv, (int)(pv & 63u));
      Jb[b] = pv >= 64u ? 64u : g;
    }
    uint32_t P = 0;  // symbol k = lane starts at offset P (64: not in this window)
#pragma unroll
    for (int b = 0; b < 6; b++) {
      const uint32_t g = (uint32_t)__shfl((int)Jb[b], (int)(P & 63u));
      if ((lane >> b) & 1u) P = P >= 64u ? 64u : g;
    }
    const bool valid = P < 64u;
    const uint32_t src = P & 63u;
    const uint32_t ev = (uint32_t)__shfl((int)evj, (int)src), rep = (uint32_t)__shfl((int)repj, (int)src);
    const uint32_t ln = (uint32_t)__shfl((int)lenj, (int)src);
    // output positions: exclusive prefix sum of the repeat counts
    const uint32_t cnt = valid ? rep : 0u;
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)incl, o);
      if (lane >= (uint32_t)o) incl += t;
    }
    const uint32_t hk = have + incl - cnt;
    const bool act = valid && hk < total;
    const bool err = act && ((bit + P + ln > limit) || (ev == 16u && hk == 0u) || (hk + rep > total));
    if (__builtin_amdgcn_ballot_w64(err)) return -1;
    // values: 17 / 18 zeros, 16 the last explicit length before it
    const uint32_t vbase = ev < 16u ? ev : 0u;
    int lastx = (act && ev != 16u) ? (int)lane : -1;
    {  // exclusive max-scan of lastx
      int m = lastx;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(m, o);
        if (lane >= (uint32_t)o) m = max(m, t);
      }
      const int ex = __shfl_up(m, 1);
      lastx = lane ? ex : -1;
    }
    const uint32_t pvv = (uint32_t)__shfl((int)vbase, lastx < 0 ? 0 : lastx);
    const uint32_t val = ev == 16u ? (lastx < 0 ? prevlen : pvv) : vbase;
    if (act && rep == 1u) B.lens[hk] = (uint16_t)val;
    uint64_t m = __builtin_amdgcn_ballot_w64(act && rep > 1u);
    while (m) {
      const uint32_t j = (uint32_t)__builtin_ctzll(m);
      m &= m - 1ull;
      const uint32_t b0 = __builtin_amdgcn_readlane(hk, j), r = __builtin_amdgcn_readlane(rep, j);
      const uint32_t v = __builtin_amdgcn_readlane(val, j);
      for (uint32_t t = lane; t < r; t += WAVE) B.lens[b0 + t] = (uint16_t)v;
    }
    const uint64_t am = __builtin_amdgcn_ballot_w64(act);
    const uint32_t nk = (uint32_t)__builtin_popcountll(am);  // the active symbols are a prefix
    if (nk == 0u) return -1;
    const uint32_t last = nk - 1u;
    bit += __builtin_amdgcn_readlane(P, last) + __builtin_amdgcn_readlane(ln, last);
    have = __builtin_amdgcn_readlane(hk, last) + __builtin_amdgcn_readlane(rep, last);
    prevlen = __builtin_amdgcn_readlane(val, last);
    __builtin_amdgcn_wave_barrier();
  }
  return 0;
}

// Dynamic block header after the 3 block-type bits (src/inflate.c:905-1033):
// code-length code, code lengths, then the literal/length and distance tables
// (src/inftrees.c restated in build_table) into the unit's global table area
// (zlib layout + compact copy) and the compact root images lroot_out (256 u16)
// and droot_out (64 u16), which may be LDS or global.  Wave-cooperative: every
// lane calls it with the same arguments.  Returns 0, or ZD_* | msg << 8.
template <bool D64>
__device__ int wave_dyn_header(BuildLDS &B, const uint32_t *w, uint32_t end_byte, uint32_t &bit, uint32_t *tabg,
                               uint16_t *ctab, uint32_t &lbits, uint32_t &dbits, uint16_t *lroot_out,
                               uint16_t *droot_out, uint8_t *dtail_out, uint8_t *walk_out = nullptr,
                               uint32_t *ltail_out = nullptr, bool zl_out = true, bool par_lens = false,
                               uint64_t *kt = nullptr) {
  const uint32_t lane = lane_id();
  const uint32_t limit = end_byte * 8u;
#if KP_ON
  if (kt) kt[0] = KP_NOW();
#endif
  StageBits sb;
  stage_bits(B, w, end_byte, bit, sb);
  if (bit + 14 > limit) {
    return ZD_TRUNC;
  }
  const uint32_t h = sb.peek(bit, 14);
  const uint32_t nlen = (h & 31) + 257, ndist = ((h >> 5) & 31) + 1, ncode = ((h >> 10) & 15) + 4;
  bit += 14;
  if (nlen > 286 || ndist > (D64 ? 32u : 30u)) {
    return ZD_ERROR | (ZM_TOO_MANY << 8);
  }
  if (bit + 3 * ncode > limit) {
    return ZD_TRUNC;
  }
  if (lane < 19) B.lens[c_clorder[lane]] = lane < ncode ? (uint16_t)sb.peek(bit + 3 * lane, 3) : (uint16_t)0;
  bit += 3 * ncode;
  __builtin_amdgcn_wave_barrier();
  uint32_t cbits = 7;
  if (build_table(T_CODES, B.lens, 19, B.tab, &cbits, B.sorted, B.scr, 0)) {
    return ZD_ERROR | (ZM_CODE_LENGTHS << 8);
  }
  const uint32_t total = nlen + ndist;
  const uint32_t cmask = (1u << cbits) - 1u;
  if (par_lens) {
    if (wave_code_lengths_par(B, w, end_byte, sb, bit, total, cmask)) return ZD_ERROR | (ZM_REPEAT << 8);
  } else {
  // the code lengths, a 64-bit window at a time: every lane decodes the
  // code-length symbol starting at bit + lane, then the true symbols of the
  // window are followed from lane 0 with readlane (scalar), the checks and
  // writes in zlib's order (src/inflate.c:1000-1033)
  uint32_t have = 0;
  while (have < total) {
    if (bit - sb.base > (STAGE_WORDS - 2) * 32u - 128u) stage_bits(B, w, end_byte, bit, sb);
    const uint32_t xj = sb.peek(bit + lane, 14);
    const uint32_t ej = B.tab[xj & cmask];
    const uint32_t ebj = e_bits(ej), evj = e_val(ej);
    const uint32_t xbj = evj < 16 ? 0u : (evj == 16 ? 2u : (evj == 17 ? 3u : 7u));
    const uint32_t repj = evj < 16 ? 1u : ((evj == 18 ? 11u : 3u) + ((xj >> ebj) & ((1u << xbj) - 1u)));
    uint32_t o = 0;
    while (o < WAVE && have < total) {
      const uint32_t ev = __builtin_amdgcn_readlane(evj, o), eb = __builtin_amdgcn_readlane(ebj, o);
      const uint32_t xb = __builtin_amdgcn_readlane(xbj, o);
      if (ev < 16) {
        if (bit + o + eb > limit) {
          return ZD_TRUNC;
        }
        if (lane == 0) B.lens[have] = (uint16_t)ev;
        have++;
      } else {
        const uint32_t rep = __builtin_amdgcn_readlane(repj, o);
        if (bit + o + eb + xb > limit) {
          return ZD_TRUNC;
        }
        if (ev == 16 && have == 0) {
          return ZD_ERROR | (ZM_REPEAT << 8);
        }
        if (have + rep > total) {
          return ZD_ERROR | (ZM_REPEAT << 8);
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t fillv = ev == 16 ? uni(B.lens[have - 1]) : 0u;
        for (uint32_t k = lane; k < rep; k += WAVE) B.lens[have + k] = (uint16_t)fillv;
        __builtin_amdgcn_wave_barrier();
        have += rep;
      }
      o += eb + xb;
    }
    bit += o;
  }
  }
  __builtin_amdgcn_wave_barrier();
#if KP_ON
  if (kt) kt[1] = KP_NOW();
#endif
  if (uni(B.lens[256]) == 0) {
    return ZD_ERROR | (ZM_MISSING_EOB << 8);
  }
  // literal/length table: build in LDS, keep the full zlib table in global
  // (slow path), compact root into the lane's LDS slot
  lbits = 9;
  if (build_table(T_LENS, B.lens, nlen, B.tab, &lbits, B.sorted, B.scr, D64 ? 1 : 0)) {
    return ZD_ERROR | (ZM_LITLEN_SET << 8);
  }
  __builtin_amdgcn_wave_barrier();
  for (uint32_t i = lane; i < ZBUILD; i += WAVE) {
    if (zl_out) tabg[i] = B.tab[i];
    ctab[i] = compact_len_entry(B.tab[i], i < (1u << lbits) ? 0u : lbits);
  }
  for (uint32_t i = lane; i < LROOT_N; i += WAVE) lroot_out[i] = lds_len_root(B.tab, lbits, i);
  if (walk_out)
    for (uint32_t i = lane; i < (1u << WK_LBITS); i += WAVE) walk_out[i] = (uint8_t)walk_len_z<D64>(B.tab, lbits, i);
  if (ltail_out) build_lit_tail(B.lens, nlen, ltail_out);
  __builtin_amdgcn_wave_barrier();
#if KP_ON
  if (kt) kt[2] = KP_NOW();
#endif
  dbits = 6;
  if (build_table(T_DISTS, B.lens + nlen, ndist, B.tab, &dbits, B.sorted, B.scr, D64 ? 1 : 0)) {
    return ZD_ERROR | (ZM_DIST_SET << 8);
  }
  __builtin_amdgcn_wave_barrier();
  for (uint32_t i = lane; i < (D64 ? 594u : 592u); i += WAVE) {
    if (zl_out) tabg[DIST_TABLE_OFF + i] = B.tab[i];
    ctab[DIST_TABLE_OFF + i] = compact_dist_entry(B.tab[i], i < (1u << dbits) ? 0u : dbits);
  }
  droot_out[lane] = compact_dist_entry(B.tab[lane & ((1u << dbits) - 1u)]);
  if (walk_out)
    for (uint32_t i = lane; i < (1u << WK_DBITS); i += WAVE)
      walk_out[(1u << WK_LBITS) + i] = (uint8_t)walk_dist_z(B.tab, dbits, i);
  build_dist_tail(B.lens + nlen, ndist, dtail_out);
  __builtin_amdgcn_wave_barrier();
  return 0;
}

// Install compact roots for lane ln from zlib tables zl (root bits lb) and zd (db).
__device__ void install_roots(uint16_t *lroot, uint16_t *droot, const uint32_t *zl, uint32_t lb, const uint32_t *zd,
                              uint32_t db) {
  const uint32_t lane = lane_id();
  for (uint32_t i = lane; i < LROOT_N; i += WAVE) lroot[i] = lds_len_root(zl, lb, i);
  droot[lane] = compact_dist_entry(zd[lane & ((1u << db) - 1u)]);
  __builtin_amdgcn_wave_barrier();
}

// Cooperative block-boundary processing for lane `ln` (all lanes call it with
// the same ln): end/stop checks, stored blocks, fixed and dynamic headers
// (src/inflate.c:834-1033); installs the lane's tables.
template <bool D64>
__device__ void coop_block(LaneState &s, uint32_t ln, BuildLDS &LB, uint16_t *lroot_ln, uint16_t *droot_ln,
                           uint32_t *dtail_ln, uint32_t *lane_tab, const uint32_t *fixed,
                           uint32_t *tokens, const ZsTokPool &pool, const ZsChunkDev *units) {
  const uint32_t lane = lane_id();
  const uint32_t *w = reinterpret_cast<const uint32_t *>(readlane_ptr((const void *)(uintptr_t)s.w, ln));
  uint32_t *tok = reinterpret_cast<uint32_t *>(readlane_ptr((const void *)(uintptr_t)s.tok, ln));
  uint32_t *tabg = reinterpret_cast<uint32_t *>(readlane_ptr(lane_tab, ln));
  uint16_t *ctab = reinterpret_cast<uint16_t *>(tabg + TABLE_ENTRIES);  // compact copy (roots + sub-tables)
  const uint16_t *cl = ctab, *cd = ctab + DIST_TABLE_OFF;
  uint32_t ntok = __builtin_amdgcn_readlane(s.ntok, ln);
  const uint32_t tcap = __builtin_amdgcn_readlane(s.tcap, ln);
  const uint32_t end_byte = __builtin_amdgcn_readlane(s.end_byte, ln);
  const uint32_t limit = end_byte * 8u;
  uint32_t stop = __builtin_amdgcn_readlane(s.stop, ln);
  const uint32_t cap = __builtin_amdgcn_readlane(s.cap, ln);
  uint32_t bit = __builtin_amdgcn_readlane(s.bit, ln);
  uint32_t pos = __builtin_amdgcn_readlane(s.pos, ln);
  int last = __builtin_amdgcn_readlane(s.last, ln);
  int mode = LM_DONE, code = 0;
  const uint32_t *zl = fixed, *zd = fixed + 512;
  uint32_t lbits = 9, dbits = 5;
  for (;;) {
    if (last) {
      code = ZD_END;
      break;
    }
    if (bit >= stop) {
      // A unit stops only at a block boundary that is a recorded start (its
      // successor's).  A block end past `stop` means `stop` was not a
      // boundary of this decode (a false start, or one this decode ran
      // over): move the stop to the next recorded start at or past `bit`
      // and keep decoding, so false starts never break the chain.
      uint32_t si = __builtin_amdgcn_readlane(s.sidx, ln);
      const uint32_t se = __builtin_amdgcn_readlane(s.send, ln);
      while (si < se && units[si].start_bit < bit) si++;
      stop = si < se ? units[si].start_bit : ZS_NONE;
      if (lane == ln) {
        s.sidx = si;
        s.stop = stop;
      }
      if (bit == stop) {
        code = ZD_STOP;
        break;
      }
    }
    if (bit + 3 > limit) {
      code = ZD_TRUNC;
      break;
    }
    StageBits sb;
    stage_bits(LB, w, end_byte, bit, sb);
    const uint32_t hdr = sb.peek(bit, 3);
    last = hdr & 1;
    const uint32_t type = hdr >> 1;
    bit += 3;
    if (type == 0) {  // stored (src/inflate.c:870-904)
      bit = (bit + 7) & ~7u;
      if (bit + 32 > limit) {
        code = ZD_TRUNC;
        break;
      }
      stage_bits(LB, w, end_byte, bit, sb);
      const uint32_t v = sb.peek(bit, 32);
      if ((v & 0xffffu) != ((v >> 16) ^ 0xffffu)) {
        code = ZD_ERROR | (ZM_STORED_LEN << 8);
        break;
      }
      bit += 32;
      const uint32_t n = v & 0xffffu;
      if (bit / 8 + n > end_byte) {
        code = ZD_TRUNC;
        break;
      }
      if (pos + n > cap) {
        code = ZD_FULL;
        break;
      }
      {  // stored bytes become literal tokens (coalesced: 64 per store)
        const uint32_t b0 = bit / 8;
        if (ntok + n <= tcap) {
          for (uint32_t k = lane; k < n; k += WAVE) {
            const uint32_t b = b0 + k;
            tok[ntok + k] = (w[b >> 2] >> (8u * (b & 3u))) & 0xffu;
          }
        } else {  // past the primary region: pool pages (taken by lane 0, then visible to all)
          const uint32_t unit = __builtin_amdgcn_readlane(s.unit, ln);
          uint32_t okp = 1;
          if (lane == 0) okp = tok_ensure(pool, unit, tcap, ntok + n) ? 1u : 0u;
          okp = __builtin_amdgcn_readfirstlane(okp);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
          if (!okp) {
            code = ZD_FULL;
            break;
          }
          const uint32_t *prim = reinterpret_cast<const uint32_t *>(readlane_ptr((const void *)(uintptr_t)s.tok, ln));
          const uint64_t prim_off = (uint64_t)(prim - tokens);
          for (uint32_t k = lane; k < n; k += WAVE) {
            const uint32_t b = b0 + k;
            *tok_addr(pool, tokens, unit, prim_off, tcap, ntok + k) = (w[b >> 2] >> (8u * (b & 3u))) & 0xffu;
          }
        }
        ntok += n;
      }
      pos += n;
      bit += n * 8;
      continue;
    }
    if (type == 1) {  // fixed: global fixed tables (lit root 9, dist root 5)
      zl = fixed;
      zd = fixed + 512;
      cl = reinterpret_cast<const uint16_t *>(fixed + FIXED_ZLIB_WORDS);
      cd = cl + 512;
      lbits = 9;
      dbits = 5;
      install_roots(lroot_ln, droot_ln, zl, lbits, zd, dbits);
      mode = LM_SYM;
      break;
    }
    if (type == 3) {
      code = ZD_ERROR | (ZM_BLOCK_TYPE << 8);
      break;
    }
    {
      const int hc = wave_dyn_header<D64>(LB, w, end_byte, bit, tabg, ctab, lbits, dbits, lroot_ln, droot_ln,
                                     reinterpret_cast<uint8_t *>(dtail_ln));
      if (hc) {
        code = hc;
        break;
      }
    }
    zl = tabg;
    zd = tabg + DIST_TABLE_OFF;
    cl = ctab;
    cd = ctab + DIST_TABLE_OFF;
    mode = LM_SYM;
    break;
  }
  if (lane == ln) {
    s.pos = pos;
    s.ntok = ntok;
    s.last = last;
    s.bit = bit;
    s.mode = mode;
    if (mode == LM_SYM) {
      s.zl = zl;
      s.zd = zd;
      s.zlmask = (1u << lbits) - 1u;
      s.zdmask = (1u << dbits) - 1u;
      s.lbits = lbits;
      s.dbits = dbits;
      s.cl = (gcu16 *)cl;
      s.cd = (gcu16 *)cd;
      s.capx = cap;
      lane_prime(s, bit);
    } else {
      s.code = code;
    }
  }
}

// Parse pass: one lane per chunk, symbols -> tokens (no history reads at all).
template <bool D64>
__global__ void __launch_bounds__(64) zs_lane_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                      ZsChunkDev *__restrict__ chunks, uint32_t nchunks,
                                                      uint32_t *__restrict__ tokens, uint32_t *__restrict__ tables,
                                                      const uint32_t *__restrict__ fixed, const uint32_t *__restrict__ order,
                                                      ZsTokPool pool, uint32_t lane_map) {
  __shared__ LaneLDS L;
  const uint32_t lane = threadIdx.x;
  // units by decreasing span: a wave's lanes run similar lengths, the longest first
  // (lane_map: the sorted units dealt round-robin over groups of `lane_map` waves)
  const uint32_t ci = lane_map ? (blockIdx.x / lane_map) * lane_map * WAVE + lane * min(lane_map, gridDim.x - (blockIdx.x / lane_map) * lane_map) + blockIdx.x % lane_map
                               : blockIdx.x * WAVE + lane;
  const uint32_t c = ci < nchunks ? order[ci] : ci;
  LaneState s;
  s.mode = LM_DONE;
  s.code = ZD_SKIP;
  s.pos = 0;
  s.last = 0;
  s.bit = 0;
  s.stop = ZS_NONE;
  s.sidx = s.send = 0;
  s.w = nullptr;
  s.tok = nullptr;
  s.ntok = 0;
  s.tcap = 0;
  s.unit = 0;
  s.end_byte = 0;
  s.limit = 0;
  s.cap = 0;
  s.whave = 0;
  s.zl = fixed;
  s.zd = fixed + 512;
  s.zlmask = s.zdmask = 0;
  s.lbits = s.dbits = 0;
  s.capx = 0;
  s.wi = s.nw = s.nkeep = s.nbits = s.lastw = s.gk = s.rk = 0;
#if KP_ON
  const uint64_t kp_t0 = KP_NOW();
  uint64_t kp_coop = 0, kp_steps_c = 0, kp_flush = 0, kp_init = 0;
  uint32_t kp_groups = 0, kp_coopn = 0, kp_wsteps = 0;
  s.kp_steps = s.kp_slow_l = s.kp_slow_d = s.kp_refills = 0;
#endif
  s.hold = 0;
  uint32_t *lane_tab = tables + (size_t)min(c, nchunks - 1) * TABLE_STRIDE;
  s.cl = s.cd = (gcu16 *)(lane_tab + TABLE_ENTRIES);
  if (c < nchunks) {
    const ZsChunkDev ch = chunks[c];
    if (ch.start_bit != ZS_NONE && heads[ch.job].code == ZD_END) {
      const ZsJobDev jb = jobs[ch.job];
      const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
      const uint32_t mis = (uint32_t)(ip & 3u);
      s.w = (gcu32 *)(ip - mis);
      s.end_byte = mis + (uint32_t)jb.in_len;
      s.limit = s.end_byte * 8u;
      s.tok = (gu32 *)(tokens + ch.tok);
      s.tcap = ch.tcap;
      s.unit = c;
      s.cap = ch.cap;
      s.whave = ch.ord == 0 ? ((jb.flags & ZS_JF_CONT) ? min(jb.hist, D64 ? 65536u : HIST) : 0u)  // a later piece's unit 0: history
                            : (D64 ? 65536u : HIST);
      s.bit = ch.start_bit;
      s.stop = ch.stop_bit;
      s.sidx = c + 1;
      s.send = ch.first + ch.nunits;
      s.mode = LM_BLOCK;
      s.code = 0;
      if (ch.hdr_info & 1u) {  // first header prebuilt by zs_unit_header_kernel: straight to symbols
        const uint32_t lb = (ch.hdr_info >> 8) & 15u, db = (ch.hdr_info >> 12) & 15u;
        uint32_t *tabg = lane_tab;
        const uint16_t *ctab = reinterpret_cast<const uint16_t *>(tabg + TABLE_ENTRIES);
        const uint4 *img = reinterpret_cast<const uint4 *>(tabg + TABLE_ENTRIES + TABLE_ENTRIES / 2);
        uint4 *lr = reinterpret_cast<uint4 *>(L.lroot[lane]);
        uint4 *dr = reinterpret_cast<uint4 *>(L.droot[lane]);
#pragma unroll 4
        for (int k = 0; k < LROOT_N * 2 / 16; k++) lr[k] = img[k];
#pragma unroll
        for (int k = 0; k < DROOT_N * 2 / 16; k++) dr[k] = img[LROOT_N * 2 / 16 + k];
        uint4 *dt4 = reinterpret_cast<uint4 *>(L.dtail[lane]);
#pragma unroll
        for (int k = 0; k < DTAIL_BYTES / 16; k++) dt4[k] = img[(LROOT_N + DROOT_N) * 2 / 16 + k];
        s.mode = LM_SYM;
        s.last = (ch.hdr_info >> 1) & 1u;
        s.bit = ch.hdr_bit;
        s.zl = tabg;
        s.zd = tabg + DIST_TABLE_OFF;
        s.zlmask = (1u << lb) - 1u;
        s.zdmask = (1u << db) - 1u;
        s.lbits = lb;
        s.dbits = db;
        s.cl = (gcu16 *)ctab;
        s.cd = (gcu16 *)(ctab + DIST_TABLE_OFF);
        s.capx = s.cap;
        lane_prime(s, s.bit);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  const uint16_t *lt = L.lroot[lane];
  const uint16_t *dt = L.droot[lane];
  uint32_t *tb = &L.g.tokbuf[0][lane];
  uint32_t *rp = &L.g.ring[0][lane];
  const uint32_t *dtl = L.dtail[lane];
  KpPhase kph = {{0, 0, 0, 0, 0}};
  uint32_t pre[RING];
  uint32_t pre_wi = ~0u;  // input word the prefetched group words start at
#if KP_ON
  kp_init = KP_NOW() - kp_t0;
#endif
  for (;;) {
    uint64_t need = __ballot(s.mode == LM_BLOCK);
#if KP_ON
    const uint64_t kc0 = KP_NOW();
    kp_coopn += __builtin_popcountll(need);
#endif
    while (need) {
      const uint32_t ln = (uint32_t)__builtin_ctzll(need);
      need &= need - 1;
      coop_block<D64>(s, ln, L.b, L.lroot[ln], L.droot[ln], L.dtail[ln], lane_tab, fixed, tokens, pool, chunks);
    }
#if KP_ON
    const uint64_t kc1 = KP_NOW();
    kp_coop += kc1 - kc0;
    const uint32_t kp_st0 = s.kp_steps;
#endif
    if (__ballot(s.mode == LM_SYM) == 0) break;
    s.gk = 0;
    if (s.mode == LM_SYM) {
#if KP_ON
      const uint64_t kf = KP_NOW();
#endif
      if (s.wi == pre_wi) lane_store_ring(s, rp, pre);  // words loaded during the last flush
      else lane_fill_ring(s, rp);
      s.dta = *reinterpret_cast<const uint4 *>(dtl);
      s.dtb = *reinterpret_cast<const uint4 *>(dtl + 4);
#if KP_ON
      __builtin_amdgcn_s_waitcnt(0);
      kph.t[4] += KP_NOW() - kf;
#endif
      // a step reads at most 2 more ring words and stores 1 token (2 for a
      // deflate64 copy longer than 65535)
      while (s.gk + (D64 ? 2u : 1u) <= GROUP && s.rk + 2 < RING)
        if (lane_step_fast<D64>(s, lt, dt, tb, dtl, rp, kph)) break;
    }
    __builtin_amdgcn_wave_barrier();
#if KP_ON
    const uint64_t kc2 = KP_NOW();
    kp_steps_c += kc2 - kc1;
    kp_groups++;
    kp_wsteps += kp_wave_max(s.kp_steps - kp_st0);
#endif
    // the next group's input words, loaded while this group's tokens leave
    // (the loads precede the stores, so waiting for them never waits for a store)
    pre_wi = s.mode == LM_SYM ? s.wi : ~0u;
    if (s.mode == LM_SYM) lane_load_ring(s, pre);
    const uint32_t g0 = s.ntok - s.gk;
    // Every lane writes its own unit's region, so a store instruction of the
    // wave touches ~64 cache lines and the count of store instructions is what
    // costs: full token quads go as 16-byte stores, written transposed -- in
    // round r, lane (q = lane / 16, m = lane % 16) stores quad q of source lane
    // 16 r + m, so a source's four lanes write its 64 contiguous bytes together
    // -- and the last gk % 4 tokens singly.  C2 parse: 16 dword stores per
    // group 15.0 ms, 4 per-lane 16-byte stores + 3 singles 11.6 ms, transposed
    // 11.4 ms.  Measured and dropped: the input prefetch transposed the same way
    // (12.5 ms: its 4 loads were not the cost, the 20 extra lane shuffles were).
    {
      typedef uint32_t u32x4a4t __attribute__((ext_vector_type(4), aligned(4)));
      const uint32_t q = lane >> 4;
      const uint32_t nq = s.ntok <= s.tcap ? (s.gk >> 2) : 0u;
      const uintptr_t dst = (uintptr_t)(s.tok + g0);
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        const uint32_t src = 16u * r + (lane & 15u);
        const uint32_t nq_s = (uint32_t)__shfl((int)nq, (int)src);
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)dst, (int)src);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)dst >> 32), (int)src);
        if (q < nq_s) {
          u32x4a4t v;
          v.x = L.g.tokbuf[4 * q][src];
          v.y = L.g.tokbuf[4 * q + 1][src];
          v.z = L.g.tokbuf[4 * q + 2][src];
          v.w = L.g.tokbuf[4 * q + 3][src];
          *reinterpret_cast<__attribute__((address_space(1))) u32x4a4t *>(((uint64_t)hi << 32 | lo) + 16u * q) = v;
        }
      }
    }
    if (s.ntok <= s.tcap) {
      const uint32_t t0 = s.gk & ~3u;
#pragma unroll
      for (uint32_t j = 0; j < 3; j++)
        if (t0 + j < s.gk) s.tok[g0 + t0 + j] = L.g.tokbuf[t0 + j][lane];
    } else if (tok_ensure(pool, s.unit, s.tcap, s.ntok)) {  // past the primary region: pool pages
      const uint64_t prim_off = (uint64_t)((const uint32_t *)s.tok - tokens);
      for (uint32_t j = 0; j < s.gk; j++) *tok_addr(pool, tokens, s.unit, prim_off, s.tcap, g0 + j) = L.g.tokbuf[j][lane];
    } else {
      s.code = ZD_FULL;
      s.mode = LM_DONE;
    }
    __builtin_amdgcn_wave_barrier();  // tokbuf area is reused by the next header build
#if KP_ON
    kp_flush += KP_NOW() - kc2;
#endif
  }
#if KP_ON
  {
    const uint64_t tot = KP_NOW() - kp_t0;
    KP_ADD(KP_P_WAVES, 1);
    KP_ADD(KP_P_CYC_TOTAL, tot);
    KP_MAX(KP_P_CYC_MAX, tot);
    if (kp_groups) {
      KP_ADD(KP_P_BUSY, 1);
      KP_ADD(KP_P_CYC_BUSY, tot);
    }
    KP_ADD(KP_P_CYC_INIT, kp_init);
    KP_ADD(KP_P_CYC_COOP, kp_coop);
    KP_ADD(KP_P_CYC_STEPS, kp_steps_c);
    KP_ADD(KP_P_CYC_FLUSH, kp_flush);
    KP_ADD(KP_P_GROUPS, kp_groups);
    KP_ADD(KP_P_COOP, kp_coopn);
    KP_ADD(KP_P_WAVE_STEPS, kp_wsteps);
    const uint32_t ls = kp_wave_sum(s.kp_steps), sl = kp_wave_sum(s.kp_slow_l), sd = kp_wave_sum(s.kp_slow_d),
                   rf = kp_wave_sum(s.kp_refills);
    KP_ADD(KP_P_LANE_STEPS, ls);
    KP_ADD(KP_P_SLOW_LIT, sl);
    KP_ADD(KP_P_SLOW_DIST, sd);
    KP_ADD(KP_P_REFILLS, rf);
    for (int i = 0; i < 5; i++) KP_ADD(KP_S_REFILL1 + i, kph.t[i]);
  }
#endif
  if (c < nchunks) {
    ZsChunkDev *ch = &chunks[c];
    ch->code = s.code;
    ch->end_bit = (s.code == ZD_END || s.code == ZD_STOP) ? s.bit : 0u;
    ch->n_out = s.pos;
    ch->n_tok = s.ntok;
  }
}

// ---------------------------------------------------------------------------
// Parse pass, wave per unit (zs_unitw_kernel): for batches with few units
// (one large stream, a handful of files) a lane per unit leaves the GPU idle
// and every unit pays the lane decoder's serial latency.  Here a whole wave
// decodes ONE unit: each window, lane j decodes the complete symbol starting
// at bit P + j (zlib's two-level tables in LDS, shared by the wave), and a
// uniform walk from P follows the true symbol boundaries through the window,
// admitting symbols until the window ends or a symbol needs lane_step's
// exceptional handling (end of block, invalid code, truncation, a full unit,
// a too-far distance), which it applies exactly as lane_step decides it.
// Block headers, stored blocks and unit stops go through coop_block, so the
// unit's tokens, end bit, code, n_out and n_tok equal the lane decoder's.
// ---------------------------------------------------------------------------
#define UW_STG 128
#define UF_OFFS 8                    // fast window: symbol offsets per lane
#define UF_BITS (UF_OFFS * WAVE)     // ... bits per window
#define UF_JN (UF_BITS + WAVE)       // jump-table entries (offsets past the window loop on themselves)
#define UW_SETS 1  // symbol offsets per lane per window (2: measured 28% slower, the walk dominates)
struct UnitWLDS {
  BuildLDS b;
  uint16_t lroot[LROOT_N];  // coop_block's compact roots (not used by this decoder)
  uint16_t droot[DROOT_N];
  uint32_t dtail[DTAIL_BYTES / 4];
  uint32_t lt[ZBUILD];  // current block: zlib literal/length table
  uint32_t dt[594];     // ... and distance table
  uint32_t stg[UW_STG + 8];  // staged input words (one global load per ~3 fast windows)
  uint16_t jmp[2][UF_JN];    // fast window: pointer-doubling tables
};

enum { UW_SYM = 0, UW_EOB = 1, UW_INVL = 2, UW_INVD = 3 };

struct UwSym {
  uint32_t kind, endr, len, dist, tok, dend;  // endr / dend: bits past the window start
};

// Fast window: the stages of Inflater::fast_window (inflate_kernels.hip) in
// token mode.  A complete symbol at every offset P + lane + 64 i of a 512-bit
// window (8 per lane, each stage's LDS loads issued back to back), the chain
// from P by pointer doubling (lane m ends with the start of the m-th symbol),
// then the longest prefix of plain symbols: complete inside the input, fitting
// the unit, distance within written history, no end of block / invalid code
// (and, for deflate64, no copy longer than one token).  Lane k < n returns
// symbol k's (L, D) (L: 0x80000000 | literal, or length); *T the output
// bytes, *endrel the bits consumed.  Anything else is left to the exact step.
template <bool D64>
__device__ uint32_t uw_fast(UnitWLDS &L, uint32_t P, uint32_t sbase, uint32_t lmask, uint32_t dmask, uint32_t limit,
                            uint32_t pos, uint32_t capx, uint32_t whave, uint32_t *T, uint32_t *endrel, uint32_t *Lo,
                            uint32_t *Do, bool *stopped) {
  const uint32_t lane = lane_id();
  auto bits_at = [&](uint32_t q) -> uint64_t {
    const uint32_t w = (q >> 5) - sbase, sh = q & 31u;
    uint64_t h = (((uint64_t)L.stg[w + 1]) << 32 | L.stg[w]) >> sh;
    if (sh) h |= (uint64_t)L.stg[w + 2] << (64u - sh);
    return h;
  };
  auto perm = [](uint32_t from_lane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(from_lane << 2), (int)v);
  };
  uint32_t nbp0 = 0, nbp1 = 0;  // total bits per slot, 8 bits each (0 = not a plain symbol)
  uint32_t lv[UF_OFFS], dv[UF_OFFS];
  uint64_t hh[UF_OFFS];
  uint32_t ee[UF_OFFS], e2[UF_OFFS], used[UF_OFFS];
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) hh[i] = bits_at(P + lane + i * WAVE);
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) ee[i] = L.lt[(uint32_t)hh[i] & lmask];
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) {
    const uint32_t op = e_op(ee[i]);
    used[i] = e_bits(ee[i]);
    const bool sub = op != 0 && (op & 0xf0u) == 0;
    e2[i] = L.lt[sub ? e_val(ee[i]) + (((uint32_t)(hh[i] >> used[i])) & ((1u << op) - 1)) : 0u];
  }
  uint64_t hd[UF_OFFS];
  uint32_t sb[UF_OFFS], de[UF_OFFS];
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) {
    const uint32_t op0 = e_op(ee[i]);
    if (op0 != 0 && (op0 & 0xf0u) == 0) {
      used[i] += e_bits(e2[i]);
      ee[i] = e2[i];
    }
    const uint32_t op = e_op(ee[i]);
    const uint32_t xb = (op == 0 || (op & 96u)) ? 0u : op & (D64 ? 31u : 15u);
    lv[i] = op == 0 ? (0x80000000u | e_val(ee[i])) : e_val(ee[i]) + ((uint32_t)(hh[i] >> used[i]) & ((1u << xb) - 1u));
    sb[i] = used[i] + xb;
    hd[i] = hh[i] >> sb[i];
    de[i] = L.dt[(uint32_t)hd[i] & dmask];
  }
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) {
    const uint32_t dop0 = e_op(de[i]);
    const uint32_t du0 = e_bits(de[i]);
    const bool dsub = (dop0 & 0xf0u) == 0;
    e2[i] = L.dt[dsub ? e_val(de[i]) + (((uint32_t)(hd[i] >> du0)) & ((1u << dop0) - 1)) : 0u];
  }
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) {
    const uint32_t op = e_op(ee[i]);
    uint32_t d = de[i];
    uint32_t dused = e_bits(d);
    if ((e_op(d) & 0xf0u) == 0) {
      dused += e_bits(e2[i]);
      d = e2[i];
    }
    const uint32_t dop = e_op(d);
    const uint32_t dx = dop & 15u;
    uint32_t nb = 0;
    dv[i] = 0;
    if (op == 0) {
      nb = used[i];
    } else if ((op & 96u) == 0 && (dop & 64u) == 0 && !(D64 && lv[i] > 0xffffu)) {
      nb = sb[i] + dused + dx;
      dv[i] = e_val(d) + ((uint32_t)(hd[i] >> dused) & ((1u << dx) - 1u));
    }
    if (P + lane + i * WAVE + nb > limit) nb = 0;
    if (i < 4) nbp0 |= nb << (8u * i);
    else nbp1 |= nb << (8u * (i - 4u));
  }
  // the chain from P by pointer doubling
  uint16_t *ja = L.jmp[0], *jb = L.jmp[1];
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) {
    const uint32_t q = lane + i * WAVE;
    const uint32_t nb = ((i < 4 ? nbp0 : nbp1) >> (8u * (i & 3u))) & 0xffu;
    ja[q] = (uint16_t)(q + nb);
  }
  ja[UF_BITS + lane] = (uint16_t)(UF_BITS + lane);
  __builtin_amdgcn_wave_barrier();
  uint32_t sp = 0;
#pragma unroll
  for (uint32_t k = 0; k < 6; k++) {
    const uint32_t half = 1u << k;
    const uint32_t t = perm(lane >= half ? lane - half : 0u, sp);
    const uint32_t g = ja[t];
    if (lane >= half && lane < 2u * half) sp = g;
    if (k < 5) {
#pragma unroll
      for (uint32_t i = 0; i < UF_OFFS + 1; i++) {
        const uint32_t q = lane + i * WAVE;
        jb[q] = ja[ja[q]];
      }
      __builtin_amdgcn_wave_barrier();
      uint16_t *tmp = ja;
      ja = jb;
      jb = tmp;
    }
  }
  const uint32_t xs = sp < UF_BITS ? sp : 0u;
  const uint32_t px0 = perm(xs & 63u, nbp0), px1 = perm(xs & 63u, nbp1);
  const uint32_t nbs = (((xs >> 6) < 4u ? px0 : px1) >> (8u * ((xs >> 6) & 3u))) & 0xffu;
  const uint64_t badc = __ballot(!(sp < UF_BITS && nbs != 0));
  const uint32_t cnt = badc ? (uint32_t)__builtin_ctzll(badc) : WAVE;
  const uint32_t s63 = __builtin_amdgcn_readlane(sp, WAVE - 1);
  const uint32_t nb63 = __builtin_amdgcn_readlane(nbs, WAVE - 1);
  const uint32_t cur = cnt < WAVE ? 0u : s63 + nb63;
  __builtin_amdgcn_wave_barrier();  // the jump tables are rewritten by the next window
  // a symbol that is not plain stopped the chain inside the window (the exact
  // step takes it); otherwise the chain only left the window
  const bool inner_stop = cnt < WAVE && __builtin_amdgcn_readlane(sp, cnt) < UF_BITS;
  *stopped = true;
  if (cnt == 0) return 0;
  // symbol k -> lane k, then the admissible prefix (lane_step's FULL / too-far order)
  const uint32_t src = sp & 63u, sl = sp >> 6;
  uint32_t Ls = 0, Ds = 0;
#pragma unroll
  for (uint32_t i = 0; i < UF_OFFS; i++) {
    const uint32_t a = perm(src, lv[i]);
    const uint32_t b = perm(src, dv[i]);
    if (sl == i) {
      Ls = a;
      Ds = b;
    }
  }
  const bool act = lane < cnt;
  const bool lit = (Ls & 0x80000000u) != 0;
  const uint32_t olen = act ? (lit ? 1u : Ls) : 0u;
  uint32_t incl = olen;
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xf, 0xf, false);
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xf, 0xf, false);
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xf, 0xf, false);
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x118, 0xf, 0xf, false);
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x142, 0xa, 0xf, false);
  incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x143, 0xc, 0xf, false);
  const uint32_t ost = incl - olen;
  const bool ok = act && pos + incl <= capx && (lit || Ds <= pos + ost + whave);
  const uint64_t badm = __ballot(!ok);
  const uint32_t n = badm ? (uint32_t)__builtin_ctzll(badm) : WAVE;
  if (n == 0) return 0;
  *stopped = n < cnt || inner_stop;
  *T = __builtin_amdgcn_readlane(incl, n - 1);
  *endrel = n < WAVE ? __builtin_amdgcn_readlane(sp, n) : cur;
  *Lo = Ls;
  *Do = Ds;
  return n;
}

// field f of offset set j at lane ql, wave-uniform
__device__ __forceinline__ uint32_t uw_rl(const UwSym (&y)[UW_SETS], uint32_t UwSym::*f, uint32_t j, uint32_t ql) {
  uint32_t v = __builtin_amdgcn_readlane(y[0].*f, ql);
#pragma unroll
  for (int k = 1; k < UW_SETS; k++)
    if (j == (uint32_t)k) v = __builtin_amdgcn_readlane(y[k].*f, ql);
  return v;
}

// the complete symbol in `hold` (its first bit at window bit rel)
template <bool D64>
__device__ __forceinline__ UwSym uw_decode(const uint32_t *lt, const uint32_t *dt, uint32_t lmask, uint32_t dmask,
                                           uint64_t hold, uint32_t rel) {
  UwSym r;
  uint32_t e = lt[(uint32_t)hold & lmask];
  uint32_t used = e_bits(e), op = e_op(e);
  if (op != 0 && (op & 0xf0u) == 0) {
    e = lt[e_val(e) + (((uint32_t)(hold >> used)) & ((1u << op) - 1u))];
    used += e_bits(e);
    op = e_op(e);
  }
  r.kind = UW_SYM;
  r.endr = rel + used;
  r.len = 1;
  r.dist = 0;
  r.tok = e_val(e);
  r.dend = 0;
  if (op & 32) {  // end of block (zlib's op 96 carries the invalid bit too)
    r.kind = UW_EOB;
  } else if (op & 64) {
    r.kind = UW_INVL;
  } else if (op != 0) {  // length: base + extra, then the distance
    const uint32_t xb = op & (D64 ? 31u : 15u);
    const uint64_t h1 = hold >> used;
    r.len = e_val(e) + ((uint32_t)h1 & ((1u << xb) - 1u));
    const uint64_t h2 = h1 >> xb;
    uint32_t d = dt[(uint32_t)h2 & dmask];
    uint32_t dused = e_bits(d), dop = e_op(d);
    if ((dop & 0xf0u) == 0) {
      d = dt[e_val(d) + (((uint32_t)(h2 >> dused)) & ((1u << dop) - 1u))];
      dused += e_bits(d);
      dop = e_op(d);
    }
    r.dend = rel + used + xb + dused;
    if (dop & 64) {
      r.kind = UW_INVD;
    } else {
      const uint32_t dx = dop & 15u;
      r.dist = e_val(d) + ((uint32_t)(h2 >> dused) & ((1u << dx) - 1u));
      r.endr = r.dend + dx;
      r.tok = (r.len << 16) | (r.dist - 1u);
    }
  }
  return r;
}

__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Split parse state of a unit (zs_walk_kernel / zs_split_kernel, below)
enum { WK_NONE = 0, WK_SPLIT = 1, WK_CONT = 2, WK_LEFT = 3 };
struct ZsWalkDev {
  uint32_t status;   // WK_*
  uint32_t nsub;     // WK_SPLIT: sub-units (checkpoints + 1)
  uint32_t ntok;     // tokens of the first block (a deflate64 length > 65535 counts two)
  uint32_t eob_bit;  // where the first block's end-of-block code starts
  uint32_t end_bit;  // the bit after it
  uint32_t pos;      // WK_CONT: entries of the first block
  uint32_t sidx;     // WK_CONT: the first later unit slot starting at or past end_bit ...
  uint32_t stop;     // ... and its start bit (ZS_NONE: none)
};

// One unit with a whole wave (the body of zs_unitw_kernel).  wk (split
// parse leftovers): a WK_CONT unit resumes at its first block's end with the
// split's output counts, exactly where the lane decoder would be there.
template <bool D64>
__device__ void unitw_unit(UnitWLDS &L, uint32_t c, const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                           ZsChunkDev *__restrict__ chunks, uint32_t *__restrict__ tokens, uint32_t *__restrict__ tables,
                           const uint32_t *__restrict__ fixed, ZsTokPool pool, const ZsWalkDev *wk) {
  const uint32_t lane = threadIdx.x;
  const ZsChunkDev ch = chunks[c];
  if (ch.start_bit == ZS_NONE || heads[ch.job].code != ZD_END) {
    if (lane == 0) {
      chunks[c].code = ZD_SKIP;
      chunks[c].end_bit = 0;
      chunks[c].n_out = 0;
      chunks[c].n_tok = 0;
    }
    return;
  }
  const ZsJobDev jb = jobs[ch.job];
  LaneState s;
  const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
  const uint32_t mis = (uint32_t)(ip & 3u);
  s.w = (gcu32 *)(ip - mis);
  s.end_byte = mis + (uint32_t)jb.in_len;
  s.limit = s.end_byte * 8u;
  s.tok = (gu32 *)(tokens + ch.tok);
  s.tcap = ch.tcap;
  s.unit = c;
  s.cap = ch.cap;
  s.capx = ch.cap;
  s.whave = ch.ord == 0 ? ((jb.flags & ZS_JF_CONT) ? min(jb.hist, D64 ? 65536u : HIST) : 0u)  // a later piece's unit 0: history
                        : (D64 ? 65536u : HIST);
  s.bit = ch.start_bit;
  s.stop = ch.stop_bit;
  s.sidx = c + 1;
  s.send = ch.first + ch.nunits;
  s.mode = LM_BLOCK;
  s.code = 0;
  s.pos = 0;
  s.ntok = 0;
  s.last = 0;
  s.gk = s.rk = 0;
  s.wi = s.nw = s.nkeep = s.nbits = s.lastw = 0;
  s.hold = 0;
#if KP_ON
  s.kp_steps = s.kp_slow_l = s.kp_slow_d = s.kp_refills = 0;
#endif
  uint32_t *lane_tab = tables + (size_t)c * TABLE_STRIDE;
  s.zl = fixed;
  s.zd = fixed + 512;
  s.cl = s.cd = (gcu16 *)(lane_tab + TABLE_ENTRIES);
  s.zlmask = s.zdmask = 0;
  s.lbits = 9;
  s.dbits = 5;
  if (ch.hdr_info & 1u) {  // first header prebuilt by zs_unit_header_kernel
    s.mode = LM_SYM;
    s.last = (ch.hdr_info >> 1) & 1u;
    s.bit = ch.hdr_bit;
    s.zl = lane_tab;
    s.zd = lane_tab + DIST_TABLE_OFF;
    s.lbits = (ch.hdr_info >> 8) & 15u;
    s.dbits = (ch.hdr_info >> 12) & 15u;
  }
  if (wk && wk->status == WK_LEFT) {  // a failed split: from the unit's start, header included (round 6: the
    s.mode = LM_BLOCK;                 // split parse's unit headers leave no zlib-layout tables)
    s.bit = ch.start_bit;
    s.last = 0;
    s.zl = fixed;
    s.zd = fixed + 512;
    s.lbits = 9;
    s.dbits = 5;
  }
  if (wk && wk->status == WK_CONT) {  // the split decoded the first block: resume at its end
    s.mode = LM_BLOCK;
    s.bit = wk->end_bit;
    s.pos = wk->pos;
    s.ntok = wk->ntok;
    s.last = 0;
    s.sidx = wk->sidx;
    s.stop = wk->stop;
  }
  const uint64_t prim = ch.tok;
  for (;;) {
    if (s.mode == LM_BLOCK) {
      coop_block<D64>(s, 0, L.b, L.lroot, L.droot, L.dtail, lane_tab, fixed, tokens, pool, chunks);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the header's global tables, read below
      // coop_block left the outcome in lane 0: every lane takes it
      s.pos = uni32(s.pos);
      s.ntok = uni32(s.ntok);
      s.last = (int)uni32((uint32_t)s.last);
      s.bit = uni32(s.bit);
      s.mode = (int)uni32((uint32_t)s.mode);
      s.code = (int)uni32((uint32_t)s.code);
      s.sidx = uni32(s.sidx);
      s.stop = uni32(s.stop);
      s.lbits = uni32(s.lbits);
      s.dbits = uni32(s.dbits);
      s.zl = reinterpret_cast<const uint32_t *>(readlane_ptr(s.zl, 0));
      s.zd = reinterpret_cast<const uint32_t *>(readlane_ptr(s.zd, 0));
    }
    if (s.mode != LM_SYM) break;
    // the block's tables into LDS
    const bool fx = s.zl == fixed;
    const uint32_t nl = fx ? 512u : ZBUILD, nd = fx ? 32u : (D64 ? 594u : 592u);
    for (uint32_t i = lane; i < nl; i += WAVE) L.lt[i] = s.zl[i];
    for (uint32_t i = lane; i < nd; i += WAVE) L.dt[i] = s.zd[i];
    __syncthreads();
    const uint32_t lmask = (1u << s.lbits) - 1u, dmask = (1u << s.dbits) - 1u;
    uint32_t sbase = 0;
    bool staged = false, exact_next = false;
    for (;;) {
      const uint32_t P = s.bit;
      // a fast window reads words P/32 .. P/32 + 20 (a symbol ends <= 511 + 60
      // bits past P), the exact step P/32 .. P/32 + 5
      if (!staged || (P >> 5) + 22 > sbase + UW_STG + 8) {
        __syncthreads();
        sbase = P >> 5;
        L.stg[lane] = in_word_g(s.w, sbase + lane, s.end_byte);
        L.stg[WAVE + lane] = in_word_g(s.w, sbase + WAVE + lane, s.end_byte);
        if (lane < 8) L.stg[UW_STG + lane] = in_word_g(s.w, sbase + UW_STG + lane, s.end_byte);
        staged = true;
        __syncthreads();
      }
      if (!exact_next && P + UF_BITS + 64u <= uni32(s.limit)) {
        uint32_t T = 0, er = 0, Ls = 0, Ds = 0;
        bool stopped = true;
        const uint32_t n = uw_fast<D64>(L, P, sbase, lmask, dmask, uni32(s.limit), uni32(s.pos), uni32(s.capx),
                                        uni32(s.whave), &T, &er, &Ls, &Ds, &stopped);
        if (n) {
          const uint32_t ntok = uni32(s.ntok), tcap = uni32(s.tcap);
          uint32_t okp = 1;
          if (ntok + n > tcap) {
            if (lane == 0) okp = tok_ensure(pool, s.unit, tcap, ntok + n) ? 1u : 0u;
            okp = uni32(okp);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
          }
          if (!okp) {
            s.code = ZD_FULL;
            s.mode = LM_DONE;
            break;
          }
          if (lane < n)
            *tok_addr(pool, tokens, s.unit, prim, tcap, ntok + lane) =
                (Ls & 0x80000000u) ? (Ls & 0xffu) : ((Ls << 16) | (Ds - 1u));
          s.ntok = ntok + n;
          s.pos = uni32(s.pos) + T;
          s.bit = P + er;
          exact_next = stopped;  // the symbol that stopped the prefix needs the exact step
          continue;
        }
      }
      exact_next = false;
      // each lane decodes the complete symbol(s) starting at bit P + lane
      // (+ 64 j) (src/inffast.c:107-166 on zlib's tables)
      const uint32_t base = (P & 31u) + 32u * ((P >> 5) - sbase);
      UwSym y[UW_SETS];
#pragma unroll
      for (int j = 0; j < UW_SETS; j++) {
        const uint32_t rel = lane + 64u * (uint32_t)j;
        const uint32_t off = base + rel, k = off >> 5, sh = off & 31u;
        const uint64_t ab = (uint64_t)L.stg[k] | ((uint64_t)L.stg[k + 1] << 32);
        const uint64_t hold = sh ? ((ab >> sh) | ((uint64_t)L.stg[k + 2] << (64u - sh))) : ab;
        y[j] = uw_decode<D64>(L.lt, L.dt, lmask, dmask, hold, rel);
      }
      // walk the true boundaries through the window: every value is
      // wave-uniform (readlane), so the walk runs on the scalar unit
      uint64_t chosen[UW_SETS] = {}, dbl[UW_SETS] = {};
      uint32_t q = 0, pos = uni32(s.pos);
      const uint32_t limit = uni32(s.limit), capx = uni32(s.capx), whave = uni32(s.whave);
      bool exc = false;
      // symbols that need lane_step's exceptional handling, per offset
      uint64_t xm[UW_SETS];
      uint32_t pk[UW_SETS];
#pragma unroll
      for (int j = 0; j < UW_SETS; j++) {
        xm[j] = __ballot(y[j].kind != UW_SYM || P + y[j].endr > limit);
        pk[j] = y[j].endr | (y[j].len << 8);  // endr < 256, len <= 65538
      }
      while (q < UW_SETS * WAVE) {
        const uint32_t j = UW_SETS > 1 ? q >> 6 : 0u, ql = q & 63u;
        uint64_t xj = xm[0];
        uint32_t w, dq;
        if (UW_SETS > 1) {
#pragma unroll
          for (int k = 1; k < UW_SETS; k++)
            if (j == (uint32_t)k) xj = xm[k];
        }
        if ((xj >> ql) & 1u) {  // exactly as lane_step orders its checks
          const uint32_t kq = uw_rl(y, &UwSym::kind, j, ql);
          const uint32_t eq = uw_rl(y, &UwSym::endr, j, ql);
          if (kq == UW_INVL) {  // invalid literal/length code: truncated or invalid by zlib's code length
            s.code = P + eq > limit ? ZD_TRUNC : (ZD_ERROR | (ZM_LITLEN_CODE << 8));
            s.mode = LM_DONE;
          } else if (kq == UW_INVD) {
            const uint32_t de = uw_rl(y, &UwSym::dend, j, ql);
            s.code = P + de > limit ? ZD_TRUNC : (ZD_ERROR | (ZM_DIST_CODE << 8));
            s.mode = LM_DONE;
          } else if (P + eq > limit) {
            s.code = ZD_TRUNC;
            s.mode = LM_DONE;
          } else {  // end of block
            s.bit = P + eq;
            s.mode = LM_BLOCK;
          }
          exc = true;
          break;
        }
        {
          uint32_t pv = __builtin_amdgcn_readlane(pk[0], ql), dv = __builtin_amdgcn_readlane(y[0].dist, ql);
#pragma unroll
          for (int k = 1; k < UW_SETS; k++)
            if (j == (uint32_t)k) {
              pv = __builtin_amdgcn_readlane(pk[k], ql);
              dv = __builtin_amdgcn_readlane(y[k].dist, ql);
            }
          w = pv;
          dq = dv;
        }
        const uint32_t lq = w >> 8, eq = w & 0xffu;
        if (pos + lq > capx) {
          s.code = ZD_FULL;
          s.mode = LM_DONE;
          exc = true;
          break;
        }
        if (dq > pos + whave) {
          s.code = ZD_ERROR | (ZM_TOO_FAR << 8);
          s.mode = LM_DONE;
          exc = true;
          break;
        }
        chosen[j] |= 1ull << ql;
        if (D64 && lq > 0xffffu) dbl[j] |= 1ull << ql;  // two tokens, same distance
        pos = uni32(pos + lq);
        q = uni32(eq);
      }
      // the admitted symbols' tokens, in window order
      uint32_t nb[UW_SETS], nt = 0;
#pragma unroll
      for (int j = 0; j < UW_SETS; j++) {
        nb[j] = nt;
        nt += (uint32_t)__builtin_popcountll(chosen[j]) + (uint32_t)__builtin_popcountll(dbl[j]);
      }
      if (nt) {
        const uint32_t ntok = uni32(s.ntok), tcap = uni32(s.tcap);
        uint32_t okp = 1;
        if (ntok + nt > tcap) {
          if (lane == 0) okp = tok_ensure(pool, s.unit, tcap, ntok + nt) ? 1u : 0u;
          okp = uni32(okp);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        }
        if (!okp) {
          s.code = ZD_FULL;
          s.mode = LM_DONE;
          break;
        }
        const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
        for (int j = 0; j < UW_SETS; j++) {
          if ((chosen[j] >> lane) & 1u) {
            const uint32_t x = ntok + nb[j] + (uint32_t)__builtin_popcountll(chosen[j] & below) +
                               (uint32_t)__builtin_popcountll(dbl[j] & below);
            if (D64 && ((dbl[j] >> lane) & 1u)) {
              *tok_addr(pool, tokens, s.unit, prim, tcap, x) = (0xffffu << 16) | (y[j].dist - 1u);
              *tok_addr(pool, tokens, s.unit, prim, tcap, x + 1) = ((y[j].len - 0xffffu) << 16) | (y[j].dist - 1u);
            } else {
              *tok_addr(pool, tokens, s.unit, prim, tcap, x) = y[j].tok;
            }
          }
        }
        s.ntok = ntok + nt;
      }
      s.pos = pos;
      if (exc) break;
      s.bit = P + q;
    }
    if (s.mode != LM_BLOCK) break;
    __syncthreads();
  }
  if (lane == 0) {
    ZsChunkDev *o = &chunks[c];
    o->code = s.code;
    o->end_bit = (s.code == ZD_END || s.code == ZD_STOP) ? s.bit : 0u;
    o->n_out = s.pos;
    o->n_tok = s.ntok;
  }
}

template <bool D64>
__global__ void __launch_bounds__(64) zs_unitw_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                       ZsChunkDev *__restrict__ chunks, uint32_t nchunks,
                                                       uint32_t *__restrict__ tokens, uint32_t *__restrict__ tables,
                                                       const uint32_t *__restrict__ fixed, const uint32_t *__restrict__ order,
                                                       ZsTokPool pool) {
  __shared__ UnitWLDS L;
  const uint32_t c = order[blockIdx.x];  // units by decreasing span
  if (c >= nchunks) return;
  unitw_unit<D64>(L, c, jobs, heads, chunks, tokens, tables, fixed, pool, nullptr);
}

// The split parse's leftovers (list[0 .. *count)), a wave per unit over a
// fixed grid: units whose first block is stored or did not decode, the rest of
// units that run past their first block (WK_CONT), and any split that failed
// its own consistency check (WK_LEFT, decoded again from the start).
template <bool D64>
__global__ void __launch_bounds__(64) zs_unitw_list_kernel(const ZsJobDev *__restrict__ jobs,
                                                            const ZsHeadDev *__restrict__ heads,
                                                            ZsChunkDev *__restrict__ chunks, uint32_t *__restrict__ tokens,
                                                            uint32_t *__restrict__ tables, const uint32_t *__restrict__ fixed,
                                                            const uint32_t *__restrict__ list, const uint32_t *__restrict__ count,
                                                            ZsTokPool pool, const ZsWalkDev *__restrict__ walks) {
  __shared__ UnitWLDS L;
  const uint32_t n = *count;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t c = list[k];
    unitw_unit<D64>(L, c, jobs, heads, chunks, tokens, tables, fixed, pool, &walks[c]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Split parse (round 5): an EXACT intra-block split of every unit's first block.
//
// The lane parse (zs_lane_kernel) decodes one ~16 K-symbol block per lane at
// one wave per SIMD, so its time is one block's serial decode: ~16 K steps of
// ~1 260 cycles.  Here the serial part is only a boundary walk, and the token
// decode runs on many waves:
//   zs_walk_kernel   one lane per unit: the block's symbols are walked by their
//                    LENGTHS only (u8 tables: code + extra bits of a literal /
//                    length, then of a distance; no values, no tokens), and
//                    every WK_K0 tokens the walk records a checkpoint (bit,
//                    token index).  Nothing is speculative: the checkpoints are
//                    true symbol boundaries of the block.
//   zs_split_kernel  one wave per walked unit, lane j decoding sub-unit j
//                    (checkpoint j to checkpoint j + 1) into the unit's tokens
//                    with lane_step_fast's decoder, the block's one table image
//                    in LDS shared by the whole wave (~9 KiB per wave instead of
//                    the lane parse's 52 KiB): many waves per SIMD hide latency.
//                    The checks that need the output position (unit full,
//                    distance too far back) run after a wave scan of the
//                    sub-units' output counts; then the unit stops exactly as
//                    coop_block decides at the block's end.
//   zs_unitw_list_kernel  the leftovers, a wave per unit: units that run past
//                    their first block (resumed at its end), stored or
//                    undecodable first blocks.
// Results (tokens, n_out, n_tok, end bit, code for STOP / END units) equal the
// lane decoder's; units that end otherwise only need a code that is neither
// ZD_STOP nor ZD_END (the chain never uses them: zs_chain_kernel), and get the
// one the lane decoder would report for the first anomaly the walk meets.
// Reference: src/inffast.c:100-287 (the symbol loop), src/inflate.c:1037-1193.
// ---------------------------------------------------------------------------
#define WK_CP 64u    // checkpoint slots per unit slot: <= 64 sub-units, one wave
#ifndef WK_K0
#define WK_K0 256u   // tokens per sub-unit to start with (doubled, checkpoints halved, when WK_CP - 1 run out)
#endif
// index bits of the walk's LDS tables: the stored tables' (WK_LBITS / WK_DBITS)
// or one fewer, folded at load (an entry whose two halves differ becomes
// WK_EXC: the walk needs only an element's bit count, so two codes that share
// the shorter index and take the same bits stay on the fast path)
#ifndef WKL_BITS
#define WKL_BITS WK_LBITS
#endif
#ifndef WKD_BITS
#define WKD_BITS (WK_DBITS - 1u)  // 9 / 7 index bits
#endif
static_assert(WKL_BITS + 1u >= WK_LBITS && WKL_BITS <= WK_LBITS && WKD_BITS + 1u >= WK_DBITS && WKD_BITS <= WK_DBITS,
              "walk tables fold by one bit at most");
#ifndef WK_RES
#define WK_RES 2u  // measured: C2 walk 3.92 ms resolving every group, 3.81 every second
#endif
#ifndef WK_GSN
#define WK_GSN 10u  // measured (C2 parse): 9 steps 7.44 ms, 10 steps 7.34
#endif
// steps per group: <= 60 (48) bits each, so a group reads words p / 32 .. p / 32 + 16
// (!D64: 10 steps read at most word p / 32 + 16 too: (31 + 9 x 48) / 32 + 2)
#define WK_GS(d64) ((d64) ? 7u : WK_GSN)
static_assert(WK_GSN <= 10u, "a walk group reads at most 17 ring words");
#define WK_PF 16u   // words per prefetch: the ring is two such halves
#define WK_RW 32u   // input ring words per lane
#define WK_RS 35u   // a lane's ring row: WK_RW words, words 0 and 1 again (a 3-word read never wraps), odd stride
#ifndef WK_RIL
#define WK_RIL 1    // the lanes' ring rows interleaved (word k of lane L at [k][L]: every ring read conflict-free)
#endif
#define WK_WS (WK_RIL ? WAVE : 1u)  // u32 elements between consecutive words of a lane's ring
// a lane's ring row in a wave's ring of WAVE * WK_RS words
#define WK_ROW(ring, lane) ((ring) + (WK_RIL ? (lane) : (lane) * WK_RS))
#define WK_DT0 6u   // the distance tail's words from here on live in LDS (its symbols: bytes 27 ..)
#define WK_DTN 9u
// The tables are lane-interleaved (dword k of lane L at [k][L]): whatever
// entries the 64 lanes look up, lane L always hits bank L mod 32, so a wave's
// table read is conflict-free (own tables at a 512-byte stride put every
// lane's entry i on the same bank: 6 extra LDS cycles per read).  The ring is
// one row per lane at an odd stride, so that a half (16 consecutive words) is
// written with 8 two-word stores and the lanes' rows spread over the banks.
struct WalkLDS {
  uint32_t wl[(1u << WKL_BITS) / 4][WAVE];
  uint32_t wd[(1u << WKD_BITS) / 4][WAVE];
  uint32_t dtail[WK_DTN][WAVE];  // words WK_DT0 .. of the block's canonical distance tail (codes past WKD_BITS)
  uint32_t ring[WAVE * WK_RS];
};
// byte i of a lane's interleaved u8 table (base = &table[0][lane])
__device__ __forceinline__ uint32_t wk_byte(const uint32_t *base, uint32_t i) {
  return reinterpret_cast<const uint8_t *>(base)[((i >> 2) * WAVE) * 4u + (i & 3u)];
}
// the same from the table's LDS address as an integer (lane column included):
// the byte address in two independent ops and one combine
__device__ __forceinline__ uint32_t wk_byte_a(uint32_t base, uint32_t i, uint32_t nbits) {
  typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
  const uint32_t a = ((i & ((1u << nbits) - 4u)) << 6) | ((i & 3u) | base);
  return *(lds_cu8 *)(uintptr_t)a;
}
// n16 uint4 of a walk table into the lane's interleaved LDS table, folded by
// one index bit when fold (the entries of the upper half n16 uint4 further on)
__device__ __forceinline__ void walk_table_load(uint32_t *dst, const uint4 *src, uint32_t n16, bool fold) {
  for (uint32_t k = 0; k < n16; k++) {
    uint4 a = src[k];
    uint32_t aw[4] = {a.x, a.y, a.z, a.w};
    if (fold) {
      const uint4 b = src[k + n16];
      const uint32_t bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t d = aw[q] ^ bw[q];
        uint32_t r = aw[q];
#pragma unroll
        for (int y = 0; y < 4; y++)
          if ((d >> (8 * y)) & 0xffu) r = (r & ~(0xffu << (8 * y))) | (WK_EXC << (8 * y));
        aw[q] = r;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) dst[(4 * k + q) * WAVE] = aw[q];
  }
}
// dist_tail_r on a lane-interleaved tail (header in registers)
__device__ __forceinline__ uint32_t walk_tail(const uint4 a, const uint4 b, const uint32_t *dtl, uint32_t hold) {
  const uint32_t rev = __builtin_bitreverse32(hold) >> 17;
  const uint32_t lw[5] = {a.x, a.y, a.z, a.w, b.x};
  uint32_t L = 7, fl = lw[0] & 0xffffu, of = (b.x >> 16) & 0xffu;
#pragma unroll
  for (int k = 1; k < 9; k++) {
    const uint32_t lim = (lw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
    const uint32_t ob = 18 + k;
    const uint32_t ow = ob < 20 ? b.x : (ob < 24 ? b.y : b.z);
    const uint32_t ofk = (ow >> (8 * (ob & 3))) & 0xffu;
    const bool ge = rev >= lim;
    L += ge ? 1u : 0u;
    fl = ge ? lim : fl;
    of = ge ? ofk : of;
  }
  const uint32_t idx = of + ((rev - fl) >> (15u - L));
  const uint32_t sym = wk_byte(dtl, 27u - 4u * WK_DT0 + min(idx, 29u));  // dtl holds the tail from word WK_DT0
  return CK_SYM | (L << 2) | (sym << 6);
}

// a literal/length code past the walk's table from the canonical tail
// (build_lit_tail's 16 words, in registers): its walk
// entry (end of block: 0x100 | WK_EXC | code bits; invalid: WK_EXC)
// build_lit_tail's 16 words in registers: the header words as an array (only
// constant indices), the symbol list as named words (an array indexed by a
// select tree was turned into scratch memory)
struct WalkLitTail {
  uint32_t w[8];
  uint32_t n0, n1, n2, n3, n4, n5, n6, n7;
};
template <bool D64>
__device__ __forceinline__ uint32_t walk_lit_tail(const WalkLitTail &T, uint32_t bits) {
  const uint32_t(&lt)[8] = T.w;
  const uint32_t rev = __builtin_bitreverse32(bits) >> 17;  // the next 15 bits, first bit highest
  const uint32_t lim[7] = {lt[0] & 0xffffu, lt[0] >> 16, lt[1] & 0xffffu, lt[1] >> 16,
                           lt[2] & 0xffffu, lt[2] >> 16, lt[3] & 0xffffu};  // lengths 9 .. 15
  uint32_t L = 10, fl = lim[0], nl = lt[4] & 0x1ffu, nb = lt[6] & 0xffu;
#pragma unroll
  for (int k = 1; k < 6; k++) {
    const bool ge = rev >= lim[k];
    L += ge ? 1u : 0u;
    fl = ge ? lim[k] : fl;
    nl = ge ? ((lt[4 + k / 3] >> (9 * (k % 3))) & 0x1ffu) : nl;
    nb = ge ? ((lt[6 + (k >> 2)] >> (8 * (k & 3))) & 0xffu) : nb;
  }
  if (rev < lim[0] || rev >= lim[6]) return WK_EXC;  // not a long code of this table: invalid
  const uint32_t idx = (rev - fl) >> (15u - L);
  if (idx < nl) return L;  // a literal
  const uint32_t k = min(nb + idx - nl, 31u);
  // word k / 4 of the list by a tree of selects on k's bits (a select chain on
  // k / 4 == j became an indexed private array, i.e. scratch memory)
  const uint32_t a0 = (k & 4u) ? T.n1 : T.n0, a1 = (k & 4u) ? T.n3 : T.n2;
  const uint32_t a2 = (k & 4u) ? T.n5 : T.n4, a3 = (k & 4u) ? T.n7 : T.n6;
  const uint32_t b0 = (k & 8u) ? a1 : a0, b1 = (k & 8u) ? a3 : a2;
  const uint32_t w = (k & 16u) ? b1 : b0;
  const uint32_t sym = (w >> (8u * (k & 3u))) & 0xffu;  // symbol - 256
  if (sym == 0) return 0x100u | WK_EXC | L;  // end of block
  const uint32_t q = sym - 1u;  // length code 0..28 (src/inftrees.c:59-64; deflate64 285: 16 extra bits)
  const uint32_t xb = q < 8u ? 0u : (q < 28u ? (q >> 2) - 1u : (D64 ? 16u : 0u));
  return (L + xb) | WK_HASD | ((D64 && q >= 28u) ? WK_BIG : 0u);
}
// word wi as read raw, with the bytes at or past the input's end zeroed
__device__ __forceinline__ uint32_t walk_mask(uint32_t v, uint32_t wi, uint32_t end_byte) {
  const uint32_t b = wi * 4u;
  const uint32_t keep = b >= end_byte ? 0u : end_byte - b;
  return keep >= 4u ? v : __builtin_amdgcn_ubfe(v, 0, 8u * keep);
}
// WK_PF raw input words from word wi (a multiple of WK_PF): four 16-byte loads
// when they are all whole input words, else word loads clamped to the last
// word (masked when written).  Nothing uses the values here, so the loads stay
// in flight through a group.
__device__ __forceinline__ void walk_prefetch(const LaneState &s, uint32_t wi, uint32_t (&v)[WK_PF]) {
  if (wi + WK_PF <= (s.end_byte >> 2)) {
    const uint32_t *src = (const uint32_t *)(s.w + wi);
#pragma unroll
    for (int q = 0; q < WK_PF / 4; q++) {
      uint4 x;
      __builtin_memcpy(&x, src + 4 * q, 16);
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (uint32_t q = 0; q < WK_PF; q++) v[q] = s.w[min(wi + q, s.lastw)];
  }
}
// The walk's per-group prefetch, issued by every lane at every group (round
// 6): the same vector-memory operations every group let the compiler wait for
// exactly the previous group's prefetch (vmcnt counts in order; a refill issued
// by some lanes only made it wait vmcnt(0) -- for every outstanding prefetch
// and checkpoint store of the wave).  A lane that did not advance reloads the
// same words (L2 hits); lanes without input read a valid dummy address.  The
// clamped word loads near the input's end (once per stream) are waited for
// at once, so they leave nothing outstanding.
__device__ __forceinline__ void walk_prefetch_u(const gcu32 *base, uint32_t wi, uint32_t fastlim, uint32_t lastw,
                                                uint32_t (&v)[WK_PF]) {
  if (__builtin_expect(wi + WK_PF <= fastlim, 1)) {
    const uint32_t *src = (const uint32_t *)(base + wi);
#pragma unroll
    for (int q = 0; q < WK_PF / 4; q++) {
      uint4 x;
      __builtin_memcpy(&x, src + 4 * q, 16);
      v[4 * q] = x.x;
      v[4 * q + 1] = x.y;
      v[4 * q + 2] = x.z;
      v[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (uint32_t q = 0; q < WK_PF; q++) v[q] = base[min(wi + q, lastw)];
#pragma unroll
    for (uint32_t q = 0; q < WK_PF; q++) __asm__ volatile("" : "+v"(v[q]));  // waited for here
  }
}
// a prefetched half into the lane's ring row (the mirror words with half 0)
__device__ __forceinline__ void walk_put_half(uint32_t *rr, uint32_t wi, uint32_t (&v)[WK_PF], uint32_t end_byte) {
  if (wi + WK_PF > (end_byte >> 2)) {
#pragma unroll
    for (uint32_t q = 0; q < WK_PF; q++) v[q] = walk_mask(v[q], wi + q, end_byte);
  }
  uint32_t *h = rr + (wi & WK_PF) * WK_WS;
#pragma unroll
  for (uint32_t q = 0; q < WK_PF; q++) h[q * WK_WS] = v[q];
  if (!(wi & WK_PF)) {
    rr[WK_RW * WK_WS] = v[0];
    rr[(WK_RW + 1u) * WK_WS] = v[1];
  }
}

enum { WS_RUN = 0, WS_EOB = 1, WS_BAD = 2, WS_IDLE = 3 };

// keep checkpoints 1, 3, 5, ... (the walk's stride doubles; rare)
__device__ __forceinline__ void walk_halve(uint2 *cp) {
  for (uint32_t i = 0; i < (WK_CP - 1u) / 2u; i++) cp[i] = cp[2u * i + 1u];
}

template <bool D64>
__global__ void __launch_bounds__(64) zs_walk_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                      ZsChunkDev *__restrict__ chunks, uint32_t nchunks,
                                                      const uint32_t *__restrict__ tables, const uint32_t *__restrict__ order,
                                                      ZsTokPool pool, uint32_t lane_map, ZsWalkDev *__restrict__ walks,
                                                      uint2 *__restrict__ cps, uint32_t *__restrict__ lists,
                                                      uint32_t *__restrict__ counts) {
  __shared__ WalkLDS L;
  const uint32_t lane = threadIdx.x;
  const uint32_t ci = lane_map ? (blockIdx.x / lane_map) * lane_map * WAVE +
                                     lane * min(lane_map, gridDim.x - (blockIdx.x / lane_map) * lane_map) +
                                     blockIdx.x % lane_map
                               : blockIdx.x * WAVE + lane;
  const uint32_t c = ci < nchunks ? order[ci] : ZS_NONE;
  LaneState s;
  s.w = nullptr;
  s.end_byte = s.limit = 0;
  s.wi = s.nw = s.nkeep = s.nbits = s.lastw = s.rk = 0;
  s.hold = 0;
  uint32_t wst = WS_IDLE, code = 0, tcap = 0;
  uint32_t *wl = &L.wl[0][lane];
  uint32_t *wd = &L.wd[0][lane];
  uint32_t *dtl = &L.dtail[0][lane];
  uint32_t *rr = WK_ROW(L.ring, lane);
  s.dta = s.dtb = make_uint4(0, 0, 0, 0);
  WalkLitTail ltw;  // the literal/length code's canonical tail (registers)
#pragma unroll
  for (int k = 0; k < 8; k++) ltw.w[k] = 0;
  ltw.n0 = ltw.n1 = ltw.n2 = ltw.n3 = ltw.n4 = ltw.n5 = ltw.n6 = ltw.n7 = 0;
  if (c < nchunks) {
    const ZsChunkDev ch = chunks[c];
    if (ch.start_bit != ZS_NONE && heads[ch.job].code == ZD_END) {
      if (ch.hdr_info & 1u) {
        const ZsJobDev jb = jobs[ch.job];
        const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
        const uint32_t mis = (uint32_t)(ip & 3u);
        s.w = (gcu32 *)(ip - mis);
        s.end_byte = mis + (uint32_t)jb.in_len;
        s.limit = s.end_byte * 8u;
        tcap = ch.tcap;
        const uint32_t *tabg = tables + (size_t)c * TABLE_STRIDE;
        const uint4 *wt = reinterpret_cast<const uint4 *>(tabg + TABLE_WALK_OFF);
        walk_table_load(wl, wt, (1u << WKL_BITS) / 16u, WKL_BITS < WK_LBITS);
        walk_table_load(wd, wt + (1u << WK_LBITS) / 16u, (1u << WKD_BITS) / 16u, WKD_BITS < WK_DBITS);
        // the distance tail: its header in registers for the whole walk, its symbols in LDS
        const uint32_t *img = tabg + TABLE_IMG_OFF + (LROOT_N + DROOT_N) / 2;
        s.dta = make_uint4(img[0], img[1], img[2], img[3]);
        s.dtb = make_uint4(img[4], img[5], img[6], img[7]);
#pragma unroll
        for (int k = 0; k < 8; k++) ltw.w[k] = tabg[TABLE_LTAIL_OFF + k];
        const uint32_t *nlg = tabg + TABLE_LTAIL_OFF + 8;
        ltw.n0 = nlg[0];
        ltw.n1 = nlg[1];
        ltw.n2 = nlg[2];
        ltw.n3 = nlg[3];
        ltw.n4 = nlg[4];
        ltw.n5 = nlg[5];
        ltw.n6 = nlg[6];
        ltw.n7 = nlg[7];
#pragma unroll
        for (uint32_t k = 0; k < WK_DTN; k++) dtl[k * WAVE] = img[WK_DT0 + k];
        s.lastw = (s.end_byte - 1u) >> 2;
        wst = WS_RUN;
      } else {  // stored or undecodable first block: a leftover from the start
        walks[c].status = WK_NONE;
        const uint32_t k = atomicAdd(&counts[1], 1u);  // lists: [0, nchunks) splits, [nchunks, 2 nchunks) leftovers
        lists[nchunks + k] = c;
      }
    }
  }
  uint2 *cp = cps + (size_t)(c < nchunks ? c : nchunks) * WK_CP;  // (slot nchunks: idle lanes' dummy)
  // the per-group checkpoint store: the whole checkpoint array as one buffer
  const __amdgpu_buffer_rsrc_t cpr = buf_rsrc(cps, (nchunks + 1u) * WK_CP * 8u);
  const uint32_t cpo = (c < nchunks ? c : nchunks) * WK_CP * 8u;
  uint32_t ntok = 0, K = WK_K0, ncp = 0, ncut = WK_K0, eob = 0, endb = 0;
  // The bit reader is one absolute bit position per lane, p: each step reads
  // the three ring words holding bits [p, p + 64) (ring slot = word % WK_RW;
  // the ring holds words [filled - WK_RW, filled)), looks the literal/length
  // entry up at p and the distance entry at p + its bits, and advances p by
  // both elements' bits -- no bit buffer, no refills.  The ring is refilled a
  // half at a time from a prefetch that stays in flight for groups.
  uint32_t p = c < nchunks && wst == WS_RUN ? chunks[c].hdr_bit : 0u;
  uint32_t filled = (p >> 5) & ~(WK_PF - 1u), pre[WK_PF];
  bool live = wst == WS_RUN;
  if (live) {  // both halves now (words filled .. filled + 31), then the next prefetch
    walk_prefetch(s, filled, pre);
    uint32_t pre2[WK_PF];
    walk_prefetch(s, filled + WK_PF, pre2);
    walk_put_half(rr, filled, pre, s.end_byte);
    walk_put_half(rr, filled + WK_PF, pre2, s.end_byte);
    filled += WK_RW;
    walk_prefetch(s, filled, pre);
  }
  uint32_t xp = live ? 0u : 1u;  // an exception is pending: the lane stands at its symbol until the next group start
  uint32_t gi = 0;                // groups
  // the per-group prefetch's source: the lane's input while it walks, then a
  // fixed valid address (the tables) through the fast path
  const gcu32 *pbase = live ? s.w : (const gcu32 *)tables;
  uint32_t pflim = live ? (s.end_byte >> 2) : 0xffffffffu;
  if (!live) filled = 0;
  // the ring row's address, opaque to the compiler (so that a step's ring
  // address is one shift-and-mask and one add, not folded LDS offsets)
  typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
  uint32_t rra = (uint32_t)(uintptr_t)(lds_cu32 *)rr;
  uint32_t wla = (uint32_t)(uintptr_t)(lds_cu32 *)wl, wda = (uint32_t)(uintptr_t)(lds_cu32 *)wd;
  asm volatile("" : "+v"(rra), "+v"(wla), "+v"(wda));
  __builtin_amdgcn_wave_barrier();
#if KP_ON
  const uint64_t kp_t0 = KP_NOW();
  uint64_t kp_cyc_x = 0, kp_cyc_g = 0, kp_cyc_s = 0, kp_cyc_r = 0;
  uint32_t kp_wsteps = 0, kp_exc = 0, kp_slow_l = 0, kp_slow_d = 0;
#endif
  // The steps are straight-line: a lane whose symbol needs more than the
  // tables (a long code, the end of the block, an invalid code, deflate64's
  // symbol 285, or the input's end) stands still with xp set, and the group
  // start resolves it exactly (the unit's compact tables, the canonical
  // distance tail); a checkpoint is taken by selects and stored at the next
  // group start.  Lanes that are done step on harmlessly (LDS reads stay in
  // bounds; nothing they compute is kept).
  while (__builtin_amdgcn_ballot_w64(live)) {
#if KP_ON
    const uint64_t kg0 = KP_NOW();
#endif
#if KP_ON
    const uint64_t kr0 = KP_NOW();
#endif
    {  // a lane that has consumed its older half refills it from the prefetch
      const bool wr = live && filled - (p >> 5) <= WK_RW - WK_PF;
      if (wr) {
        walk_put_half(rr, filled, pre, s.end_byte);
        filled += WK_PF;
      }
      if (!live) {  // (a lane that has stopped reads the dummy from here on)
        pbase = (const gcu32 *)tables;
        pflim = 0xffffffffu;
        filled = 0;
      }
      walk_prefetch_u(pbase, filled, pflim, s.lastw, pre);
    }
#if KP_ON
    kp_cyc_r += KP_NOW() - kr0;
#endif
    // a checkpoint at the first group start past every K tokens (the lane
    // stands on a symbol boundary here; a pending symbol is not yet counted).
    // Every lane issues the store at every group, after the prefetch (one
    // store per group: see walk_prefetch_u); only a lane past the next K tokens
    // stores (round 6: a buffer store whose other lanes' offsets are out of
    // range -- storing the pending slot at every group was 0.6 GB of writes).
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(live && ntok >= ncut && ncp == WK_CP - 1u) != 0, 0)) {
      // out of slots (a 65th sub-unit): keep every second checkpoint, twice
      // the stride.  Round 6: this halved on storing the 63rd checkpoint, i.e.
      // every unit past 63 x 256 tokens -- zlib's 16 383-symbol blocks, nearly
      // every C2 unit -- ran as 32 sub-units of 512 tokens
      if (live && ntok >= ncut && ncp == WK_CP - 1u) {
        walk_halve(cp);
        ncp = (WK_CP - 1u) / 2u;
        K *= 2u;
        ncut = (ncp + 1u) * K;
      }
      __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): nothing of the rare path left outstanding
    }
    {  // the checkpoint, stored only by a lane that keeps it (others: out of range, dropped)
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      const bool keep = live && ntok >= ncut;
      const u32x2 v = {p, ntok};
      __builtin_amdgcn_raw_buffer_store_b64(v, cpr, keep ? (cpo + ncp * 8u) : BUF_SKIP, 0, 0);
      if (keep) {  // the next sub-unit starts here
        ncp++;
        ncut += K;
      }
    }
    // the pending symbols, exactly (every WK_RES groups: a pass costs about
    // a group's steps, a lane that waits loses half a group on average)
    gi++;
    if ((gi % WK_RES) == 0 && __builtin_amdgcn_ballot_w64(live && xp)) {
#if KP_ON
      const uint64_t kq = KP_NOW();
      kp_exc += lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)) ? 1u : 0u;
#endif
      const bool pend = live && xp;
      uint32_t x0 = 0, x1 = 0, x2 = 0, bits = 0, e2 = 0;
      if (pend) {
        const uint32_t *r = rr + ((p >> 5) & (WK_RW - 1u)) * WK_WS;
        x0 = r[0];
        x1 = r[WK_WS];
        x2 = r[2u * WK_WS];
        bits = __builtin_amdgcn_alignbit(x1, x0, p);
        e2 = wk_byte(wl, bits & ((1u << WKL_BITS) - 1u));
      }
      // past the table: the end of block from its own entry, every longer
      // code from the canonical tail (registers and LDS; no global table)
      if (pend && (e2 & WK_EXC)) {
#if KP_ON
        kp_slow_l++;
#endif
        e2 = ((e2 & WK_EOBE) == WK_EOBE) ? (0x100u | WK_EXC | (e2 & 31u)) : walk_lit_tail<D64>(ltw, bits);
      }
      if (pend) {
        if (e2 & WK_EXC) {
          if (e2 & 0x100u) {  // end of block
            eob = p;
            endb = p + (e2 & 31u);
            wst = endb > s.limit ? WS_BAD : WS_EOB;
            code = ZD_TRUNC;
          } else {  // invalid literal/length code
            wst = WS_BAD;
            code = p > s.limit ? ZD_TRUNC : (ZD_ERROR | (ZM_LITLEN_CODE << 8));
          }
          live = false;
        } else {
          const uint32_t n2 = e2 & 31u;
          const uint32_t q2 = (p & 31u) + n2;
          const uint32_t db2 = __builtin_amdgcn_alignbit(q2 < 32u ? x1 : x2, q2 < 32u ? x0 : x1, q2);
          uint32_t d2 = 0;
          if (e2 & WK_HASD) {
            d2 = wk_byte(wd, db2 & ((1u << WKD_BITS) - 1u));
            if (d2 == WK_EXC) {  // a distance code longer than the table's index: the canonical tail
#if KP_ON
              kp_slow_d++;
#endif
              const uint32_t de = walk_tail(s.dta, s.dtb, dtl, db2);
              const uint32_t dsym = (de >> 6) & 31u;
              d2 = (!D64 && dsym >= 30u) ? WK_BAD : walk_dist_entry(de);
            }
          }
          const uint32_t pn = p + n2 + (d2 & 31u);
          if (d2 & WK_EXC) {  // invalid distance code
            wst = WS_BAD;
            code = pn > s.limit ? ZD_TRUNC : (ZD_ERROR | (ZM_DIST_CODE << 8));
            live = false;
          } else if (pn > s.limit) {
            wst = WS_BAD;
            code = ZD_TRUNC;
            live = false;
          } else {
            p = pn;
            ntok += (D64 && (e2 & WK_BIG) && ((bits >> (n2 - 16u)) & 0xffffu) >= 65533u) ? 2u : 1u;  // deflate64 > 65535: two tokens
          }
        }
        xp = live ? 0u : 1u;  // a lane that is done stays where it stopped
      }
#if KP_ON
      kp_cyc_x += KP_NOW() - kq;
#endif
    }
#if KP_ON
    const uint64_t ks0 = KP_NOW();
    kp_cyc_g += ks0 - kg0;
    kp_wsteps += WK_GS(D64);
#endif
    // unrolled: the next step's ring read issues before this step's
    // bookkeeping (a rolled loop serialises them: 472 vs 326 cycles a step).
    // A step only looks its two entries up and advances p; which step (if
    // any) met an exception -- an entry past the tables, or the input's end
    // (p only grows, so the first step past it) -- is found once at the end
    // of the group from the positions each step started at, and the lane
    // stands there (the steps after it ran on garbage).
    {
      constexpr uint32_t GS = WK_GS(D64);
      uint32_t pk[GS + 1], xk[GS];
#pragma unroll
      for (uint32_t g = 0; g < GS; g++) {
        pk[g] = p;
        lds_cu32 *r = (lds_cu32 *)(uintptr_t)(rra + 4u * WK_WS * __builtin_amdgcn_ubfe(p, 5, 5));
        const uint32_t x0 = r[0], x1 = r[WK_WS], x2 = r[2u * WK_WS];
        const uint32_t lo = __builtin_amdgcn_alignbit(x1, x0, p);  // input bits [p, p + 32)
        const uint32_t hi = __builtin_amdgcn_alignbit(x2, x1, p);  // [p + 32, p + 64)
        const uint32_t e = wk_byte_a(wla, lo, WKL_BITS);
        const uint32_t n = e & 31u;  // <= 31: the distance code starts in lo:hi
        const uint32_t d = wk_byte_a(wda, __builtin_amdgcn_alignbit(hi, lo, n), WKD_BITS);
        const uint32_t dd = (e & WK_HASD) ? d : 0u;
        p += n + (dd & 31u);
        xk[g] = (e | dd) & (D64 ? (WK_EXC | WK_BIG) : WK_EXC);
      }
      pk[GS] = p;
      uint32_t k = GS;  // the first step with an exception (GS: none)
#pragma unroll
      for (int g = (int)GS - 1; g >= 0; g--) k = (xk[g] || pk[g + 1] > s.limit) ? (uint32_t)g : k;
      k = xp ? 0u : k;  // a lane that stood still (pending, or done) stays
      uint32_t pst = pk[0];
#pragma unroll
      for (uint32_t g = 1; g <= GS; g++) pst = k == g ? pk[g] : pst;
      p = pst;
      ntok += k;
      xp = (k < GS) ? 1u : 0u;
    }
#if KP_ON
    kp_cyc_s += KP_NOW() - ks0;
#endif
  }
#if KP_ON
  {  // walk counters in slots no other kernel of the split parse writes
    const uint64_t tot = KP_NOW() - kp_t0;
    KP_ADD(44, tot);
    KP_MAX(45, tot);
    KP_ADD(46, kp_wsteps);
    KP_ADD(47, kp_cyc_x);
    KP_ADD(38, kp_cyc_g);
    KP_ADD(39, kp_wave_sum(kp_exc));
    KP_ADD(KP_P_CYC_STEPS, kp_cyc_s);
    KP_ADD(KP_P_CYC_BUSY, kp_cyc_r);
    KP_ADD(KP_P_SLOW_LIT, kp_wave_sum(kp_slow_l));
    KP_ADD(KP_P_SLOW_DIST, kp_wave_sum(kp_slow_d));
  }
#endif
  if (wst == WS_EOB && !tok_ensure(pool, c, tcap, ntok)) {
    wst = WS_BAD;
    code = ZD_FULL;
  }
  if (wst == WS_EOB) {
    ZsWalkDev w;
    w.status = WK_SPLIT;
    w.nsub = ncp + 1u;
    w.ntok = ntok;
    w.eob_bit = eob;
    w.end_bit = endb;
    w.pos = 0;
    w.sidx = 0;
    w.stop = ZS_NONE;
    walks[c] = w;
    const uint32_t k = atomicAdd(&counts[0], 1u);
    lists[k] = c;
  } else if (wst == WS_BAD) {
    chunks[c].code = (int32_t)code;
    chunks[c].end_bit = 0;
    chunks[c].n_out = 0;
    chunks[c].n_tok = 0;
  }
}

// Wide tables of the split decode (one copy per wave, so LDS is cheap): u32
// entries that carry everything a symbol needs -- code bits, extra-bit count
// and the literal or the length / distance base -- so a step does no base
// arithmetic; a code longer than the index takes a wave-uniform side branch.
//   literal / length, 9-bit index: [3:0] code bits, [5:4] kind (SK_*),
//     [10:6] extra bits, [31:16] literal byte or length base
//   distance, 8-bit index: [3:0] code bits, [4] long code (canonical tail),
//     [5] invalid code, [10:6] extra bits, [31:16] distance base - 1 (the
//     token's field)
#define SPL_BITS 9u
#define SPD_BITS 8u
enum { SK_LIT = 0, SK_LEN = 1, SK_EOB = 2, SK_SLOW = 3 };
template <bool D64>
__device__ __forceinline__ uint32_t split_len_entry(uint32_t ce) {  // from a compact literal/length entry
  const uint32_t kind = ce & 3u, bits = (ce >> 2) & 15u, sym = ce >> 6;
  if (kind == CK_SYM) return bits | (SK_LIT << 4) | (sym << 16);
  if (kind == CK_EOB) return bits | (SK_EOB << 4);
  if (kind != CK_LEN) return SK_SLOW << 4;
  // length code sym (0..28), src/inftrees.c:59-64 (deflate64 285: 3 + 16 extra bits)
  uint32_t xb = sym < 8u ? 0u : (sym < 28u ? (sym >> 2) - 1u : (D64 ? 16u : 0u));
  uint32_t base = sym < 8u ? sym + 3u : (sym < 28u ? ((4u + (sym & 3u)) << xb) + 3u : (D64 ? 3u : 258u));
  return bits | (SK_LEN << 4) | (xb << 6) | (base << 16);
}
__device__ __forceinline__ uint32_t split_dist_entry(uint32_t ce, bool d64) {  // from a compact distance entry
  if ((ce & 3u) != CK_SYM) return 0x20u;
  const uint32_t bits = (ce >> 2) & 15u, dsym = (ce >> 6) & 31u;
  if (!d64 && dsym >= 30u) return 0x20u;
  const uint32_t dx = dsym < 4u ? 0u : (dsym >> 1) - 1u;
  const uint32_t base = dsym < 4u ? dsym + 1u : ((2u + (dsym & 1u)) << dx) + 1u;  // src/inftrees.c:65-72
  return bits | (dx << 6) | ((base - 1u) << 16);
}

// The split decode reads its input like the walk: an absolute bit position p
// per lane over a ring row of 32 words (two halves of 16, the older half
// refilled from a prefetch that stays in flight), three words giving the 64
// bits from p -- every field of a symbol (code, extra bits, distance code,
// distance extra bits: <= 48 bits, deflate64 60) is one funnel shift of them.
#ifndef SP_GSN
#define SP_GSN 8u
#endif
#ifndef SPLIT_ALIGN
#define SPLIT_ALIGN 1  // measured (C2 split): 3.22 ms with 10-step groups at any token offset, 3.02 aligned 8-step groups
#endif
#ifndef SPLIT_PAIR
#define SPLIT_PAIR 1  // token stores in 64-byte pairs of groups (round 6: C2 split writes 5.29 -> 3.99 GB,
                      // step time within noise; non-temporal stores instead: parse 7.0 -> 13.0 ms)
#endif
#ifndef SPLIT_NOSTORE
#define SPLIT_NOSTORE 0  // (diagnostic builds only: no token stores, wrong output)
#endif
#define SP_GS(d64) ((d64) ? 7u : SP_GSN)  // steps per group: <= 60 (48) bits each, words p / 32 .. p / 32 + 16
template <bool D64>
struct __attribute__((aligned(16))) SplitLDS {
  uint32_t lw[1u << SPL_BITS];
  uint32_t dw[1u << SPD_BITS];
  uint32_t dtail[DTAIL_BYTES / 4];
  uint32_t tokbuf[D64 ? 2u * SP_GS(true) : 1u][WAVE];  // deflate64: a group's tokens (two per step at most); else in registers
  uint32_t ring[WAVE * WK_RS];
};
struct SplitLane {
  uint32_t p, ntok, pos, need, bad, gk;
};

// one symbol of a walked sub-unit.  Every symbol before the sub-unit's end is
// a literal or a length (the walk met them), so anything else only marks the
// lane bad (bit 0x20 of t.bad: the unit is decoded again from its start).
template <bool D64, bool NEEDC>
__device__ __forceinline__ void split_step3(SplitLane &t, uint32_t rra, const uint32_t *__restrict__ lw,
                                            const uint32_t *__restrict__ dw, uint32_t *__restrict__ tb, uint32_t *tr,
                                            uint4 dta, uint4 dtb, const uint32_t *__restrict__ dtl, gcu16 *cl,
                                            uint32_t lbits) {
  typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
  lds_cu32 *r = (lds_cu32 *)(uintptr_t)(rra + ((t.p >> 5) & (WK_RW - 1u)) * (4u * WK_WS));
  const uint32_t x0 = r[0], x1 = r[WK_WS], x2 = r[2u * WK_WS];
  const uint32_t hl = __builtin_amdgcn_alignbit(x1, x0, t.p), hh = __builtin_amdgcn_alignbit(x2, x1, t.p);
  uint32_t e = lw[hl & ((1u << SPL_BITS) - 1u)];
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(((e >> 4) & 3u) == SK_SLOW) != 0, 0)) {
    if (((e >> 4) & 3u) == SK_SLOW) {  // longer than 9 bits: zlib's root and sub-table (compact, global)
      uint32_t e2 = cl[hl & ((1u << lbits) - 1u)];
      const uint32_t op2 = (e2 >> 2) & 15u;
      if ((e2 & 3u) == CK_SLOW && op2) e2 = cl[(e2 >> 6) + ((hl >> lbits) & ((1u << op2) - 1u))];
      e = split_len_entry<D64>(e2);
    }
  }
  const uint32_t cb = e & 15u, xb = (e >> 6) & 31u;
  const bool isl = (e & 0x10u) != 0;  // SK_LEN (SK_SLOW is resolved above; what stays invalid is marked bad below)
  const uint32_t len = (e >> 16) + __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(hh, hl, cb), 0, xb);  // literal: its byte
  const uint32_t k2 = cb + xb;  // <= 31
  const uint32_t c = __builtin_amdgcn_alignbit(hh, hl, k2);
  uint32_t d = dw[c & ((1u << SPD_BITS) - 1u)];
  if (__builtin_expect(__builtin_amdgcn_ballot_w64((d & e & 0x10u) != 0) != 0, 0)) {
    // a length's distance code longer than 8 bits: canonical decode from the tail
    if (d & e & 0x10u) d = split_dist_entry(dist_tail_r(dta, dtb, dtl, c), D64);
  }
  const uint32_t k3 = k2 + (d & 15u), dx = (d >> 6) & 31u;  // k3 <= 46, + dx <= 60
  const uint32_t dxv = (uint32_t)((((uint64_t)hh << 32) | hl) >> k3);
  const uint32_t dm1 = (d >> 16) + __builtin_amdgcn_ubfe(dxv, 0, dx);  // distance - 1
  t.p += isl ? k3 + dx : k2;
  t.bad |= e | (isl ? d : 0u);  // bit 0x20: end of block / unresolved code / invalid distance
  if (NEEDC) t.need = max(t.need, (isl && dm1 >= t.pos) ? dm1 + 1u - t.pos : 0u);
  if (!D64) {
    *tr = isl ? ((len << 16) | dm1) : len;  // a register of the group (the step index is a constant)
  } else if (__builtin_expect(__builtin_amdgcn_ballot_w64(isl && len > 0xffffu) != 0, 0)) {
    // a deflate64 copy longer than a token holds: two copies, same distance
    if (isl && len > 0xffffu) {
      tb[t.gk * WAVE] = (0xffffu << 16) | dm1;
      t.gk++;
      t.ntok++;
      tb[t.gk * WAVE] = ((len - 0xffffu) << 16) | dm1;
    } else {
      tb[t.gk * WAVE] = isl ? ((len << 16) | dm1) : len;
    }
  } else {
    tb[t.gk * WAVE] = isl ? ((len << 16) | dm1) : len;
  }
  t.gk++;
  t.ntok++;
  t.pos += isl ? len : 1u;
}

// a lane's sub-unit, group by group: refill, SP_GS steps (guarded only when
// some lane is within a group of its end), then the group's tokens leave in
// 16-byte transposed stores (zs_lane_kernel's flush)
template <bool D64, bool NEEDC>
__device__ __forceinline__ void split_sub3(SplitLDS<D64> &L, SplitLane &t, LaneState &s, uint32_t t1, uint32_t &filled,
                                           uint32_t (&pre)[WK_PF], uint32_t rra, uint4 dta, uint4 dtb,
                                           uint32_t *__restrict__ tokens, const ZsTokPool &pool, bool act
#if KP_ON
                                           , uint64_t &kp_grp, uint32_t &kp_ws
#endif
) {
  const uint32_t lane = threadIdx.x;
  uint32_t *tb = &L.tokbuf[0][lane];
  uint32_t *rr = WK_ROW(L.ring, lane);
  constexpr uint32_t GS = SP_GS(D64), TPS = D64 ? 2u : 1u;
  // !D64: a group's tokens are stored one group late, right after the next
  // refill's wait (vmcnt counts stores too: stored at the end of their own
  // group, they made that wait wait for them -- C2 split 3.2 ms, 2.3 without
  // stores at all)
  uint32_t tkp[GS], g0p = 0, gkp = 0;
#if SPLIT_PAIR
  // (round 6) a whole group starting a 64-byte half line (token regions are
  // line-aligned) waits in hold[] for the next one: the pair leaves as one
  // 64-byte run -- single 32-byte pieces cost 64-byte write-backs (C2 split:
  // 5.3 GB written for 3.0 GB of tokens)
  static_assert(D64 || SP_GS(false) == 8u, "pairs of 8-token groups");
  uint32_t hold[GS], holdp = 0;
  bool hv = false;
  auto store32 = [&](uint32_t at, const uint32_t (&v)[GS]) {
    typedef uint32_t u32x4a4t __attribute__((ext_vector_type(4), aligned(4)));
    gu32 *dst = s.tok + at;
#pragma unroll
    for (uint32_t q = 0; q < GS; q += 4u) {
      u32x4a4t x;
      x.x = v[q]; x.y = v[q + 1]; x.z = v[q + 2]; x.w = v[q + 3];
      *reinterpret_cast<__attribute__((address_space(1))) u32x4a4t *>(dst + q) = x;
    }
  };
  auto flush_hold = [&]() {
    if (hv) store32(holdp, hold);
    hv = false;
  };
#endif
  auto store_prev = [&]() {
#if KP_ON
    const uint64_t kf0 = KP_NOW();
#endif
#if SPLIT_PAIR
    if (!D64 && gkp && !SPLIT_NOSTORE) {
      const bool whole = gkp == GS && g0p + GS <= s.tcap;
      if (whole && hv && holdp + GS == g0p) {  // the pair: 64 bytes
        store32(holdp, hold);
        store32(g0p, tkp);
        hv = false;
        gkp = 0;
      } else {
        flush_hold();
        if (whole && (g0p & (2u * GS - 1u)) == 0u) {  // the first half of a pair: wait for the second
#pragma unroll
          for (uint32_t j = 0; j < GS; j++) hold[j] = tkp[j];
          holdp = g0p;
          hv = true;
          gkp = 0;
        }
      }
    }
#endif
    if (gkp && !SPLIT_NOSTORE) {
      if (gkp == GS && g0p + GS <= s.tcap) {  // 16-byte stores, then 8 / 4 bytes
        typedef uint32_t u32x4a4t __attribute__((ext_vector_type(4), aligned(4)));
        typedef uint32_t u32x2a4t __attribute__((ext_vector_type(2), aligned(4)));
        gu32 *dst = s.tok + g0p;
#pragma unroll
        for (uint32_t q = 0; q + 4u <= GS; q += 4u) {
          u32x4a4t v;
          v.x = tkp[q]; v.y = tkp[q + 1]; v.z = tkp[q + 2]; v.w = tkp[q + 3];
          *reinterpret_cast<__attribute__((address_space(1))) u32x4a4t *>(dst + q) = v;
        }
        if (GS % 4u >= 2u) {
          u32x2a4t v;
          v.x = tkp[GS & ~3u]; v.y = tkp[(GS & ~3u) + 1u];
          *reinterpret_cast<__attribute__((address_space(1))) u32x2a4t *>(dst + (GS & ~3u)) = v;
        }
        if (GS % 2u) dst[GS - 1u] = tkp[GS - 1u];
      } else {
        const uint64_t prim_off = (uint64_t)((const uint32_t *)s.tok - tokens);
#pragma unroll
        for (uint32_t j = 0; j < GS; j++)
          if (j < gkp) {
            if (g0p + j < s.tcap) s.tok[g0p + j] = tkp[j];
            else *tok_addr(pool, tokens, s.unit, prim_off, s.tcap, g0p + j) = tkp[j];
          }
      }
    }
    gkp = 0;
#if KP_ON
    kp_grp += KP_NOW() - kf0;
#endif
  };
  // SPLIT_ALIGN: a first group short enough that every later group's tokens
  // start on a GS-token (for GS = 8: 32-byte) boundary of the token region
  uint32_t first_n = (SPLIT_ALIGN && !D64 && act) ? ((GS - (t.ntok % GS)) % GS) : 0u;
  for (;;) {
    const bool run = act && t.ntok < t1 && !(t.bad & 0x20u) && t.pos <= s.capx;
    if (__builtin_amdgcn_ballot_w64(run) == 0) break;
#if KP_ON
    const uint64_t kg0 = KP_NOW();
#endif
    {  // a lane that has consumed its older half refills it from the prefetch
      const bool wr = run && filled - (t.p >> 5) <= WK_RW - WK_PF;
      if (__builtin_amdgcn_ballot_w64(wr)) {
        if (wr) {
          walk_put_half(rr, filled, pre, s.end_byte);
          filled += WK_PF;
          walk_prefetch(s, filled, pre);
        }
      }
    }
#if KP_ON
    kp_grp += KP_NOW() - kg0;
    kp_ws += lane == (uint32_t)__builtin_ctzll(__ballot(1)) ? GS : 0u;
#endif
    if (!D64) store_prev();
    t.gk = 0;
    const uint32_t g0 = t.ntok;
    uint32_t tk[GS];  // the group's tokens (!D64: registers; deflate64: tokbuf)
    if (__builtin_amdgcn_ballot_w64(run && (t1 - t.ntok < GS * TPS || first_n != 0)) == 0) {
      if (run) {
#pragma unroll
        for (uint32_t g = 0; g < GS; g++)
          split_step3<D64, NEEDC>(t, rra, L.lw, L.dw, tb, &tk[g], dta, dtb, L.dtail, s.cl, s.lbits);
      }
    } else {
      const uint32_t lim = first_n ? min(t1, t.ntok + first_n) : t1;
      if (run) {
#pragma unroll
        for (uint32_t g = 0; g < GS; g++)
          if (t.ntok < lim) split_step3<D64, NEEDC>(t, rra, L.lw, L.dw, tb, &tk[g], dta, dtb, L.dtail, s.cl, s.lbits);
      }
    }
    first_n = 0;
    if (t.ntok > t1) {  // an inconsistent decode: never write past the walked tokens
      t.bad |= 0x20u;
      t.gk -= min(t.gk, t.ntok - t1);
      t.ntok = t1;
    }
    if (!D64) {  // the group's tokens wait in registers: stored after the next group's refill
#pragma unroll
      for (uint32_t j = 0; j < GS; j++) tkp[j] = tk[j];
      g0p = g0;
      gkp = run ? t.gk : 0u;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
#if KP_ON
    const uint64_t kf0 = KP_NOW();
#endif
    {  // 16-byte transposed stores of full token quads
      typedef uint32_t u32x4a4t __attribute__((ext_vector_type(4), aligned(4)));
      const uint32_t q = lane >> 4;
      const uint32_t nq = (run && t.ntok <= s.tcap) ? (t.gk >> 2) : 0u;
      const uintptr_t dst = (uintptr_t)(s.tok + g0);
#pragma unroll
      for (uint32_t rq = 0; rq < (GS * TPS + 15u) / 16u; rq++) {
#pragma unroll
        for (uint32_t r = 0; r < 4; r++) {
          const uint32_t src = 16u * r + (lane & 15u);
          const uint32_t nq_s = (uint32_t)__shfl((int)nq, (int)src);
          const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)dst, (int)src);
          const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)dst >> 32), (int)src);
          const uint32_t qq = q + 4u * rq;
          if (qq < nq_s) {
            u32x4a4t v;
            v.x = L.tokbuf[4 * qq][src];
            v.y = L.tokbuf[4 * qq + 1][src];
            v.z = L.tokbuf[4 * qq + 2][src];
            v.w = L.tokbuf[4 * qq + 3][src];
            *reinterpret_cast<__attribute__((address_space(1))) u32x4a4t *>(((uint64_t)hi << 32 | lo) + 16u * qq) = v;
          }
        }
      }
    }
    if (run) {
      if (t.ntok <= s.tcap) {
        const uint32_t t0 = t.gk & ~3u;
#pragma unroll
        for (uint32_t j = 0; j < 3; j++)
          if (t0 + j < t.gk) s.tok[g0 + t0 + j] = L.tokbuf[t0 + j][lane];
      } else {  // past the primary region: pool pages (taken by the walk)
        const uint64_t prim_off = (uint64_t)((const uint32_t *)s.tok - tokens);
        for (uint32_t j = 0; j < t.gk; j++) *tok_addr(pool, tokens, s.unit, prim_off, s.tcap, g0 + j) = L.tokbuf[j][lane];
      }
    }
    __builtin_amdgcn_wave_barrier();  // tokbuf is rewritten by the next group
#if KP_ON
    kp_grp += KP_NOW() - kf0;
#endif
  }
  if (!D64) store_prev();  // the last group's tokens
#if SPLIT_PAIR
  if (!D64) flush_hold();
#endif
}

template <bool D64>
__global__ void __launch_bounds__(64) zs_split_kernel(const ZsJobDev *__restrict__ jobs, ZsChunkDev *__restrict__ chunks,
                                                       uint32_t nchunks, uint32_t *__restrict__ tokens,
                                                       const uint32_t *__restrict__ tables, ZsTokPool pool,
                                                       ZsWalkDev *__restrict__ walks, const uint2 *__restrict__ cps,
                                                       uint32_t *__restrict__ lists, uint32_t *__restrict__ counts,
                                                       int force_left) {
  __shared__ SplitLDS<D64> L;
  const uint32_t lane = threadIdx.x;
  const uint32_t nsplit = counts[0];
  constexpr uint32_t HMAX = D64 ? 65536u : HIST;
  typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
#if KP_ON
  const uint64_t kp_t0 = KP_NOW();
  uint64_t kp_grp = 0, kp_pro = 0, kp_sub = 0;
  uint32_t kp_units = 0, kp_ws = 0;
#endif
  // units are taken one at a time from a counter: waves that get the longest
  // units take fewer (a fixed deal left a tail of 5 vs 6 units).  (Round 6:
  // claiming the next unit when this one starts, so the atomic's round trip
  // overlaps the decode, measured no faster: parse 6.70 vs 6.67 ms)
  uint32_t kn = 0;
  if (lane == 0) kn = atomicAdd(&counts[2], 1u);
  kn = uni(kn);
  for (;;) {
    const uint32_t k = kn;
    if (k >= nsplit) break;
    uint32_t kx = 0;
    const uint32_t c = lists[k];
    const ZsWalkDev wk = walks[c];
#if KP_ON
    kp_units++;
    const uint64_t ku0 = KP_NOW();
#endif
    const ZsChunkDev ch = chunks[c];
    const ZsJobDev jb = jobs[ch.job];
    const uint32_t *tabg = tables + (size_t)c * TABLE_STRIDE;
    __builtin_amdgcn_wave_barrier();  // the previous unit is done with the tables
    {  // the wide tables from the unit's compact tables (zlib layout, roots lbits / dbits)
      const uint16_t *ccl = reinterpret_cast<const uint16_t *>(tabg + TABLE_ENTRIES), *ccd = ccl + DIST_TABLE_OFF;
      const uint32_t lb = (ch.hdr_info >> 8) & 15u, db = (ch.hdr_info >> 12) & 15u;
#pragma unroll
      for (uint32_t q = 0; q < (1u << SPL_BITS) / WAVE; q++) {
        const uint32_t i = q * WAVE + lane;
        const uint32_t ce = ccl[i & ((1u << lb) - 1u)];
        L.lw[i] = ((ce & 3u) == CK_SLOW) ? (SK_SLOW << 4) : split_len_entry<D64>(ce);
      }
#pragma unroll
      for (uint32_t q = 0; q < (1u << SPD_BITS) / WAVE; q++) {
        const uint32_t i = q * WAVE + lane;
        uint32_t ce = ccd[i & ((1u << db) - 1u)];
        uint32_t v;
        if ((ce & 3u) == CK_SLOW && ((ce >> 2) & 15u)) {  // sub-table: the index's bits past the root pick it if it fits
          const uint32_t op = (ce >> 2) & 15u, avail = SPD_BITS - db;
          ce = ccd[(ce >> 6) + ((i >> db) & ((1u << min(op, avail)) - 1u))];
          v = ((ce >> 2) & 15u) > SPD_BITS ? 0x10u : split_dist_entry(ce, D64);
        } else {
          v = split_dist_entry(ce, D64);
        }
        L.dw[i] = v;
      }
      if (lane < DTAIL_BYTES / 4) L.dtail[lane] = tabg[TABLE_IMG_OFF + (LROOT_N + DROOT_N) / 2 + lane];
    }
    const bool act = lane < wk.nsub;
    const uint2 *cpu = cps + (size_t)c * WK_CP;
    const uint2 a0 = cpu[lane ? lane - 1u : 0u];
    const uint2 a = lane == 0 ? make_uint2(ch.hdr_bit, 0u) : a0;
    const uint2 b = lane + 1u == wk.nsub ? make_uint2(wk.eob_bit, wk.ntok) : cpu[lane];
    LaneState s;
    const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
    const uint32_t mis = (uint32_t)(ip & 3u);
    s.w = (gcu32 *)(ip - mis);
    s.end_byte = mis + (uint32_t)jb.in_len;
    s.limit = s.end_byte * 8u;
    s.lastw = (s.end_byte - 1u) >> 2;
    s.tok = (gu32 *)(tokens + ch.tok);
    s.tcap = ch.tcap;
    s.unit = c;
    s.lbits = (ch.hdr_info >> 8) & 15u;
    s.cl = (gcu16 *)(tabg + TABLE_ENTRIES);
    s.capx = ch.cap;
    const uint32_t t1 = b.y, b1 = b.x;
    SplitLane t;
    t.p = a.x;
    t.ntok = a.y;
    t.pos = t.need = t.bad = t.gk = 0;
    uint32_t *rr = WK_ROW(L.ring, lane);
    uint32_t filled = (t.p >> 5) & ~(WK_PF - 1u), pre[WK_PF];
    if (act) {  // both halves now (words filled .. filled + 31), then the next prefetch
      walk_prefetch(s, filled, pre);
      uint32_t pre2[WK_PF];
      walk_prefetch(s, filled + WK_PF, pre2);
      walk_put_half(rr, filled, pre, s.end_byte);
      walk_put_half(rr, filled + WK_PF, pre2, s.end_byte);
      filled += WK_RW;
      walk_prefetch(s, filled, pre);
    }
    uint32_t rra = (uint32_t)(uintptr_t)(lds_cu32 *)rr;
    asm volatile("" : "+v"(rra));
    __builtin_amdgcn_wave_barrier();
    uint4 dta, dtb;
    {  // the distance tail header is the same for every lane: scalar registers
      const uint4 x = *reinterpret_cast<const uint4 *>(L.dtail), y = *reinterpret_cast<const uint4 *>(L.dtail + 4);
      dta = make_uint4(uni(x.x), uni(x.y), uni(x.z), uni(x.w));
      dtb = make_uint4(uni(y.x), uni(y.y), uni(y.z), uni(y.w));
    }
    const uint32_t whave = ch.ord == 0 ? ((jb.flags & ZS_JF_CONT) ? min(jb.hist, HMAX) : 0u) : HMAX;
#if KP_ON
    const uint64_t ku1 = KP_NOW();
    kp_pro += ku1 - ku0;
#endif
    if (whave < HMAX)  // only a stream's first unit can reach before its window
      split_sub3<D64, true>(L, t, s, t1, filled, pre, rra, dta, dtb, tokens, pool, act
#if KP_ON
                            , kp_grp, kp_ws
#endif
      );
    else
      split_sub3<D64, false>(L, t, s, t1, filled, pre, rra, dta, dtb, tokens, pool, act
#if KP_ON
                             , kp_grp, kp_ws
#endif
      );
#if KP_ON
    const uint64_t ku2 = KP_NOW();
    kp_sub += ku2 - ku1;
#endif
    const bool full = act && t.pos > s.capx;
    uint32_t bad = (t.bad & 0x20u) ? 1u : 0u;
    if (act && !full && (t.p != b1 || t.ntok != t1)) bad = 1;
    if (act && !full && !bad && lane + 1u == wk.nsub) {
      // the walk's end of block, checked: the code at eob_bit must decode to
      // end-of-block and take end_bit - eob_bit bits (src/inflate.c:1125-1129)
      const uint32_t *r = rr + ((b1 >> 5) & (WK_RW - 1u)) * WK_WS;
      const uint32_t hl = __builtin_amdgcn_alignbit(r[WK_WS], r[0], b1);
      uint32_t e = L.lw[hl & ((1u << SPL_BITS) - 1u)];
      if (((e >> 4) & 3u) == SK_SLOW) {
        uint32_t e2 = s.cl[hl & ((1u << s.lbits) - 1u)];
        const uint32_t op2 = (e2 >> 2) & 15u;
        if ((e2 & 3u) == CK_SLOW && op2) e2 = s.cl[(e2 >> 6) + ((hl >> s.lbits) & ((1u << op2) - 1u))];
        e = split_len_entry<D64>(e2);
      }
      if (((e >> 4) & 3u) != SK_EOB || b1 + (e & 15u) != wk.end_bit) bad = 1;
    }
    const bool anybad = __ballot(act && bad) != 0 || force_left, anyfull = __ballot(full) != 0;
    // output position of every sub-unit: a wave scan of their entry counts
    uint64_t incl = act ? t.pos : 0u;
#pragma unroll
    for (uint32_t o = 1; o < WAVE; o <<= 1) {
      const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)incl, o);
      const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(incl >> 32), o);
      if (lane >= o) incl += ((uint64_t)hi << 32) | lo;
    }
    const uint64_t P = incl - (act ? t.pos : 0u);
    const uint64_t total = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(incl >> 32), WAVE - 1) << 32) |
                           __builtin_amdgcn_readlane((uint32_t)incl, WAVE - 1);
    const bool far = whave < HMAX && __ballot(act && (uint64_t)t.need > P + whave) != 0;
    if (lane == 0) {
      ZsChunkDev *o = &chunks[c];
      if (anybad) {  // decode again from the start (never expected)
        walks[c].status = WK_LEFT;
        lists[nchunks + atomicAdd(&counts[1], 1u)] = c;
      } else if (far || anyfull || total > ch.cap) {  // the lane decoder stops inside the block
        o->code = far ? (ZD_ERROR | (ZM_TOO_FAR << 8)) : ZD_FULL;
        o->end_bit = 0;
        o->n_out = 0;
        o->n_tok = 0;
      } else {
        // the block's end, as coop_block meets it: the final block ends the
        // stream; else a recorded start at this bit ends the unit; else the
        // unit goes on (a block the finder did not record, or a false start)
        const uint32_t bit = wk.end_bit;
        int32_t code = -1;
        uint32_t si = c + 1u, stop = ZS_NONE;
        if ((ch.hdr_info >> 1) & 1u) {
          code = ZD_END;
        } else {
          const uint32_t se = ch.first + ch.nunits;
          while (si < se && chunks[si].start_bit < bit) si++;
          stop = si < se ? chunks[si].start_bit : ZS_NONE;
          if (stop == bit) code = ZD_STOP;
        }
        if (code >= 0) {
          o->code = code;
          o->end_bit = bit;
          o->n_out = (uint32_t)total;
          o->n_tok = wk.ntok;
        } else {
          ZsWalkDev w = wk;
          w.status = WK_CONT;
          w.pos = (uint32_t)total;
          w.sidx = si;
          w.stop = stop;
          walks[c] = w;
          lists[nchunks + atomicAdd(&counts[1], 1u)] = c;
        }
      }
    }
    if (lane == 0) kx = atomicAdd(&counts[2], 1u);
    kn = uni(kx);
  }
#if KP_ON
  // split counters in the lane parse's step-phase slots (no lane parse runs):
  // 40 units, 41 cycles, 42 wave-steps, 43 group fill + flush cycles
  KP_ADD(40, kp_units);
  KP_ADD(41, KP_NOW() - kp_t0);
  KP_ADD(42, kp_wave_sum(kp_ws));
  KP_ADD(43, kp_grp);
  KP_ADD(4, kp_pro);  // (lane-parse slots, unused by the split parse) unit prologue: tables, checkpoints, ring
  KP_ADD(5, kp_sub);  // the sub-unit decode (steps + group refills / stores)
#endif
}

// ---------------------------------------------------------------------------
// Expand pass: one 256-thread workgroup (4 waves) per chunk, tokens -> u16
// entries.  The last 32 Ki entries live in an LDS ring; every round the 256
// threads produce 256 consecutive entries in parallel: a max-scan over
// round-stamped token-start marks finds each entry's token, sources before the
// round come from the ring (markers 256 + w for positions before the chunk),
// sources inside the round are resolved by pointer jumping through LDS (only
// distances shorter than the round reach into it).  Three barriers per round:
//   B1 marks visible (and the previous round's ring writes),
//   B2 per-wave max-scan totals visible,
//   B3 every ring read of the round done + per-wave "unresolved" flags visible.
// Output leaves the ring in 4 KiB pieces (16 B per thread) after B1, when every
// entry before the round is in the ring.
// ---------------------------------------------------------------------------
#define EXP_T 256                 // threads = tokens per batch
#define EXP_W (EXP_T / WAVE)
#define EXP_E 4                   // consecutive entries per thread per round
#define EXP_N (EXP_T * EXP_E)     // entries per round
#define EXP_FLUSH 2048            // entries per flush piece (8 per thread)

__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {  // inclusive, wave64
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v) {  // inclusive, wave64, values >= 0
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}
__device__ __forceinline__ void exp_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

#define TV_LIT 0x80000000u  // s_tval: literal byte | TV_LIT, else match distance
#define JR 0x80000000u      // s_j: resolved value | JR, else index of the source in the round

// Deflate64 (D64): a 64 Ki-entry ring and 64 KiB of history, so markers
// 256 + w need 17 bits: the ring keeps the low 16 bits and a flag byte per 4
// entries the 17th (entries go to HBM as u32).
template <bool D64>
__global__ void __launch_bounds__(EXP_T) zs_expand_kernel(const ZsJobDev *__restrict__ jobs,
                                                           const ZsChunkDev *__restrict__ chunks,
                                                           uint16_t *__restrict__ scratch,
                                                           const uint32_t *__restrict__ tokens,
                                                           const uint32_t *__restrict__ order, ZsTokPool pool,
                                                           uint32_t *__restrict__ fallback) {
  constexpr uint32_t HN = D64 ? 65536u : HIST;
  __shared__ __attribute__((aligned(16))) uint16_t ring[HN];
  __shared__ uint8_t qflag[D64 ? HN / 4 : 4];  // bit k of qflag[i >> 2]: bit 16 of entry 4 (i >> 2) + k
  __shared__ __attribute__((aligned(16))) uint32_t s_mark[EXP_N];
  __shared__ uint32_t s_tval[EXP_T];
  __shared__ uint32_t s_red[EXP_W], s_flag[EXP_W];
  __shared__ __attribute__((aligned(16))) uint32_t s_j[2][EXP_N];
  __shared__ uint32_t s_jf[2][EXP_W];
  const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
  const uint32_t unit = order[blockIdx.x];
  const ZsChunkDev ch = chunks[unit];  // chain members by decreasing output (longest first)
  if (!ch.in_chain) return;
  gcu32 *tk = (gcu32 *)(tokens + ch.tok);
  const uint32_t ntok = ch.n_tok, tcap = ch.tcap;
  const uint32_t *ptab = pool.ptab + (size_t)unit * ZS_TP_MAXPG;
  auto tread = [&](uint32_t x) -> uint32_t {
    if (x < tcap) return tk[x];
    uint32_t off;
    const uint32_t k = tok_page(x - tcap, &off);
    return tokens[pool.base + ((uint64_t)(ptab[k] - 1u) << ZS_TP_LOG) + off];
  };
  uint16_t *out = scratch + ch.scratch;
  uint32_t *out32 = reinterpret_cast<uint32_t *>(scratch + ch.scratch);  // D64: u32 entries
  auto rget = [&](uint32_t i) -> uint32_t {  // ring entry i (masked index)
    if (!D64) return ring[i];
    return ring[i] | (((uint32_t)(qflag[i >> 2] >> (i & 3u)) & 1u) << 16);
  };
#if KP_ON
  const uint64_t kp_t0 = KP_NOW();
  uint64_t kp_jump = 0;
  uint32_t kp_rounds = 0, kp_jits = 0, kp_jrounds = 0, kp_batches = 0;
#endif
  // history before the chunk (every unit after the first, and the first of a
  // later piece of a long stream): markers 256 + w for position w - HN
  if (ch.ord != 0 || (jobs[ch.job].flags & ZS_JF_CONT)) {
    uint32_t *r32 = reinterpret_cast<uint32_t *>(ring);
    for (uint32_t i = tid; i < HN / 2; i += EXP_T) r32[i] = ((MARK_BASE + 2 * i) & 0xffffu) | ((MARK_BASE + 2 * i + 1) << 16);
    if (D64)
      for (uint32_t i = tid; i < HN / 4; i += EXP_T) qflag[i] = i >= (HN - MARK_BASE) / 4 ? 0xfu : 0u;
  }
  for (uint32_t i = tid; i < EXP_N; i += EXP_T) s_mark[i] = 0;
#if KP_ON
  const uint64_t kp_init = KP_NOW() - kp_t0;
#endif
  uint32_t pos = 0, flushed = 0, stamp = 0;
  uint32_t tnext = tid < ntok ? tread(tid) : 0u;
  for (uint32_t tb = 0; tb < ntok; tb += EXP_T) {
    const uint32_t t = tnext;
    if (tb + EXP_T + tid < ntok) tnext = tread(tb + EXP_T + tid);  // next batch, in flight during this one
    const bool valid = tb + tid < ntok;
    const uint32_t hi = t >> 16;
    const uint32_t len = valid ? (hi ? hi : 1u) : 0u;
    const uint32_t incl = wave_scan_add(len);
    if (lane == WAVE - 1) s_red[wv] = incl;
    exp_barrier();
    uint32_t before = 0, S = 0;
#pragma unroll
    for (uint32_t w = 0; w < EXP_W; w++) {
      const uint32_t x = s_red[w];
      before += w < wv ? x : 0u;
      S += x;
    }
    const uint32_t tstart = pos + before + incl - len;
    s_tval[tid] = hi ? (t & 0xffffu) + 1u : (TV_LIT | (t & 0xffu));
    uint32_t own_carry = 0;
    // rounds start 4-aligned (8-byte ring stores); entries below pos are the
    // previous batch's, already final in the ring, and stay inactive
    for (uint32_t R = pos & ~(uint32_t)(EXP_E - 1); R < pos + S; R += EXP_N) {
      const uint32_t lo = max(R, pos);  // entries below lo are final in the ring
      if ((++stamp & 0x7fffffu) == 0) {  // stamp wrap: drop stale marks
        for (uint32_t i = tid; i < EXP_N; i += EXP_T) s_mark[i] = 0;
        exp_barrier();
        stamp++;
      }
      const uint32_t st = stamp & 0x7fffffu;
      if (len && tstart >= R && tstart < R + EXP_N) s_mark[tstart - R] = (st << 9) | (tid + 1);
      exp_barrier();  // B1: marks, token values and the previous round's ring writes visible
      while (lo - flushed >= EXP_FLUSH) {
        const uint32_t ri = (flushed + tid * 8) & (HN - 1);
        if (D64) {
          uint32_t x[8];
#pragma unroll
          for (int k = 0; k < 8; k++) x[k] = rget(ri + k);
          *reinterpret_cast<uint4 *>(out32 + flushed + tid * 8) = make_uint4(x[0], x[1], x[2], x[3]);
          *reinterpret_cast<uint4 *>(out32 + flushed + tid * 8 + 4) = make_uint4(x[4], x[5], x[6], x[7]);
        } else {
          const uint4 v4 = *reinterpret_cast<const uint4 *>(&ring[ri]);
          *reinterpret_cast<uint4 *>(out + flushed + tid * 8) = v4;
        }
        flushed += EXP_FLUSH;
      }
      // owner token of each of this thread's entries: running max of marks
      const uint4 m4 = *reinterpret_cast<const uint4 *>(&s_mark[tid * EXP_E]);
      uint32_t mk[EXP_E] = {m4.x, m4.y, m4.z, m4.w};
      uint32_t run[EXP_E];
#pragma unroll
      for (int k = 0; k < EXP_E; k++) {
        const uint32_t x = (mk[k] >> 9) == st ? (mk[k] & 511u) : 0u;
        run[k] = k ? max(run[k - 1], x) : x;
      }
      const uint32_t winc = wave_scan_max(run[EXP_E - 1]);
      const uint32_t wexc = __shfl_up(winc, 1);
      if (lane == WAVE - 1) s_red[wv] = winc;
      exp_barrier();  // B2
      uint32_t base = max(own_carry, lane ? wexc : 0u), all = own_carry;
#pragma unroll
      for (uint32_t w = 0; w < EXP_W; w++) {
        const uint32_t x = s_red[w];
        base = w < wv ? max(base, x) : base;
        all = max(all, x);
      }
      own_carry = all;
      const uint32_t e0 = R + tid * EXP_E;
      uint32_t v[EXP_E], q[EXP_E];
      uint32_t unres = 0;
#pragma unroll
      for (int k = 0; k < EXP_E; k++) {
        const uint32_t e = e0 + k;
        const uint32_t own = max(base, run[k]);
        const uint32_t vj = s_tval[(own ? own : 1u) - 1u];
        v[k] = vj & 0xffffu;
        q[k] = 0;
        if (e >= lo && e < pos + S && !(vj & TV_LIT)) {
          const int p = (int)e - (int)vj;
          if (p < (int)lo) {
            v[k] = rget((uint32_t)p & (HN - 1));
          } else {
            q[k] = (uint32_t)(p - (int)R);
            unres |= 1u << k;
          }
        }
      }
      const bool wave_unres = __ballot(unres != 0) != 0;
      if (lane == 0) s_flag[wv] = wave_unres;
      exp_barrier();  // B3: every ring read of the round done, flags visible
      bool any = false;
#pragma unroll
      for (uint32_t w = 0; w < EXP_W; w++) any |= s_flag[w] != 0;
#if KP_ON
      kp_rounds++;
      const uint64_t kj0 = KP_NOW();
#endif
      if (any) {  // in-round sources: pointer jumping through LDS, one barrier per step
#if KP_ON
        kp_jrounds++;
#endif
        for (uint32_t it = 0;; it++) {
#if KP_ON
          kp_jits++;
#endif
          const uint32_t b = it & 1u;
          uint4 o;
          o.x = (unres & 1u) ? q[0] : (JR | v[0]);
          o.y = (unres & 2u) ? q[1] : (JR | v[1]);
          o.z = (unres & 4u) ? q[2] : (JR | v[2]);
          o.w = (unres & 8u) ? q[3] : (JR | v[3]);
          *reinterpret_cast<uint4 *>(&s_j[b][tid * EXP_E]) = o;
          const bool wu = __ballot(unres != 0) != 0;
          if (lane == 0) s_jf[b][wv] = wu;
          exp_barrier();
          bool more = false;
#pragma unroll
          for (uint32_t w = 0; w < EXP_W; w++) more |= s_jf[b][w] != 0;
          if (!more) break;
#pragma unroll
          for (int k = 0; k < EXP_E; k++) {
            if (unres & (1u << k)) {
              const uint32_t x = s_j[b][q[k]];
              if (x & JR) {
                v[k] = x & ~JR;
                unres &= ~(1u << k);
              } else {
                q[k] = x;
              }
            }
          }
        }
      }
#if KP_ON
      kp_jump += KP_NOW() - kj0;
#endif
      if (e0 >= lo && e0 + EXP_E <= pos + S) {
        uint2 w2;
        w2.x = (v[0] & 0xffffu) | (v[1] << 16);
        w2.y = (v[2] & 0xffffu) | (v[3] << 16);
        *reinterpret_cast<uint2 *>(&ring[e0 & (HN - 1)]) = w2;
        if (D64)
          qflag[(e0 & (HN - 1)) >> 2] =
              (uint8_t)(((v[0] >> 16) & 1u) | ((v[1] >> 15) & 2u) | ((v[2] >> 14) & 4u) | ((v[3] >> 13) & 8u));
      } else {
#pragma unroll
        for (int k = 0; k < EXP_E; k++)
          if (e0 + k >= lo && e0 + k < pos + S) {
            const uint32_t ri = (e0 + k) & (HN - 1);
            ring[ri] = (uint16_t)v[k];
            if (D64) qflag[ri >> 2] = (uint8_t)((qflag[ri >> 2] & ~(1u << (ri & 3u))) | (((v[k] >> 16) & 1u) << (ri & 3u)));
          }
      }
    }
    pos += S;
#if KP_ON
    kp_batches++;
#endif
  }
  exp_barrier();
  while (pos - flushed >= EXP_FLUSH) {
    const uint32_t ri = (flushed + tid * 8) & (HN - 1);
    if (D64) {
      uint32_t x[8];
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = rget(ri + k);
      *reinterpret_cast<uint4 *>(out32 + flushed + tid * 8) = make_uint4(x[0], x[1], x[2], x[3]);
      *reinterpret_cast<uint4 *>(out32 + flushed + tid * 8 + 4) = make_uint4(x[4], x[5], x[6], x[7]);
    } else {
      const uint4 v4 = *reinterpret_cast<const uint4 *>(&ring[ri]);
      *reinterpret_cast<uint4 *>(out + flushed + tid * 8) = v4;
    }
    flushed += EXP_FLUSH;
  }
  for (uint32_t k = tid; k < pos - flushed; k += EXP_T) {
    if (D64) out32[flushed + k] = rget((flushed + k) & (HN - 1));
    else out[flushed + k] = ring[(flushed + k) & (HN - 1)];
  }
  (void)fallback;
#if KP_ON
  if (wv == 0) {
    const uint64_t tot = KP_NOW() - kp_t0;
    KP_ADD(KP_E_BLOCKS, 1);
    KP_ADD(KP_E_CYC_TOTAL, tot);
    KP_MAX(KP_E_CYC_MAX, tot);
    KP_ADD(KP_E_CYC_INIT, kp_init);
    KP_ADD(KP_E_ROUNDS, kp_rounds);
    KP_ADD(KP_E_JUMP_ITERS, kp_jits);
    KP_ADD(KP_E_JUMP_ROUNDS, kp_jrounds);
    KP_ADD(KP_E_CYC_JUMP, kp_jump);
    KP_ADD(KP_E_BATCHES, kp_batches);
  }
#endif
}

// ---------------------------------------------------------------------------
// Expand, 32 KiB window (zs_expand2_kernel): rounds of 2048 entries, 8
// consecutive entries per thread, decoupled from the token batches (1024
// tokens, 4 per thread, loaded whenever the next round reaches past the last
// loaded token), so every round but the unit's last is full.
//  - Marks: each token writes key (start - R + 1) << 16 | payload at its start
//    entry (payload: the literal byte, or distance + 256); a running max over
//    the round (thread, wave DPP scan, per-wave totals) gives every entry its
//    token's payload directly -- the max-key mark, or the carry of the last
//    token started before the round (key 0).  Readers zero their marks.
//  - The ring holds HIST + 2048 entries, so a round's writes never land on a
//    slot any entry of the round may still read (its sources reach back at
//    most HIST): every entry is written in the same phase that computes it --
//    the literal, the ring value of a source before the round, or PTR | the
//    in-round index of its source.
//  - After one barrier, entries holding a pointer follow it through the ring
//    and write back what they found (a value, or the target's own pointer:
//    pointer jumping without barriers; every pointer points strictly back, so
//    each lane terminates on its own).
// Three barriers per round (+1 per token batch); ~15 VALU per entry.
// ---------------------------------------------------------------------------
#ifndef EX2_T
#define EX2_T 512  // measured (C2 expand): 256 x 8 entries 8.5 ms, 512 x 4 7.2, 1024 x 4 10.2, 1024 x 2 12.9
#endif
#define EX2_W (EX2_T / WAVE)
#ifndef EX2_E
#define EX2_E 4                 // consecutive entries per thread per round
#endif
#define EX2_N (EX2_T * EX2_E)   // entries per round
#define EX2_RS (HIST + EX2_N)   // ring slots
#ifndef EX2_TPT
#define EX2_TPT 2               // tokens per thread per batch
#endif
#define EX2_TB (EX2_T * EX2_TPT)
#define EX2_PTR (0x10000u - EX2_N)  // ring value >= PTR: pointer to in-round entry (value & (N - 1))
static_assert(EX2_RS % EX2_N == 0 && (EX2_E == 2 || EX2_E % 4 == 0) && MARK_BASE + HIST <= EX2_PTR, "expand2 layout");
// E entries (2E bytes) at u16 index i of a 16-byte-aligned LDS / global array
__device__ __forceinline__ void ex2_copy(uint16_t *dst, const uint16_t *src) {
#pragma unroll
  for (int c = 0; c < EX2_E / 8; c++) reinterpret_cast<uint4 *>(dst)[c] = reinterpret_cast<const uint4 *>(src)[c];
  if (EX2_E == 4) *reinterpret_cast<uint2 *>(dst) = *reinterpret_cast<const uint2 *>(src);
  if (EX2_E == 2) *reinterpret_cast<uint32_t *>(dst) = *reinterpret_cast<const uint32_t *>(src);
}

__global__ void __launch_bounds__(EX2_T) zs_expand2_kernel(const ZsJobDev *__restrict__ jobs,
                                                            const ZsChunkDev *__restrict__ chunks,
                                                            uint16_t *__restrict__ scratch,
                                                            const uint32_t *__restrict__ tokens,
                                                            const uint32_t *__restrict__ order, ZsTokPool pool) {
  __shared__ __attribute__((aligned(16))) uint16_t ring[EX2_RS];
  __shared__ __attribute__((aligned(16))) uint32_t s_mark[EX2_N];
  __shared__ uint32_t s_red[EX2_W];
  __shared__ uint32_t s_bs[2][EX2_W];
  const uint32_t tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
  const uint32_t unit = order[blockIdx.x];
  const ZsChunkDev ch = chunks[unit];
  if (!ch.in_chain) return;
  gcu32 *tk = (gcu32 *)(tokens + ch.tok);
  const uint32_t ntok = ch.n_tok, tcap = ch.tcap, total = ch.n_out;
  const uint32_t *ptab = pool.ptab + (size_t)unit * ZS_TP_MAXPG;
  // address of token x (x >= ntok: any valid word, its length is masked):
  // one load per token whatever the path, so the prefetch registers are not
  // copied (and waited for) where the paths merge
  auto taddr = [&](uint32_t x) -> gcu32 * {
    if (x >= ntok) return (gcu32 *)tokens;
    if (x < tcap) return tk + x;
    uint32_t off;
    const uint32_t k = tok_page(x - tcap, &off);
    return (gcu32 *)(tokens + pool.base + ((uint64_t)(ptab[k] - 1u) << ZS_TP_LOG) + off);
  };
  uint16_t *out = scratch + ch.scratch;
  // history before the unit: position p in [-HIST, 0) sits at slot p + RS
  if (ch.ord != 0 || (jobs[ch.job].flags & ZS_JF_CONT)) {
    uint32_t *r32 = reinterpret_cast<uint32_t *>(ring + EX2_N);
    for (uint32_t i = tid; i < HIST / 2; i += EX2_T) r32[i] = (MARK_BASE + 2 * i) | ((MARK_BASE + 2 * i + 1) << 16);
  }
  for (uint32_t i = tid; i < EX2_N; i += EX2_T) s_mark[i] = 0;
  // token batches: thread tid holds tokens tb + 4 tid + j (payload, start entry)
  uint32_t nxt[EX2_TPT], pay[EX2_TPT], ts[EX2_TPT];
  uint32_t tb = 0, bend = 0, par = 0;
#pragma unroll
  for (int j = 0; j < EX2_TPT; j++) {
    nxt[j] = *taddr(tid * EX2_TPT + j);
  }
#if KP_ON
  const uint64_t kp_t0 = KP_NOW();
  uint64_t kp_batch = 0, kp_pre = 0, kp_spin = 0;
  uint32_t kp_rounds = 0, kp_passes = 0, kp_srounds = 0, kp_batches = 0;
  uint32_t kp_pc = 0, kp_pf = 0, kp_pt = 0, kp_me = 0;  // wave pieces: all, with a marker, of those in the last HIST; markers
#endif
  auto load_batch = [&]() {
#if KP_ON
    const uint64_t kb0 = KP_NOW();
    kp_batches++;
#endif
    uint32_t lsum = 0, ex[EX2_TPT];
#pragma unroll
    for (int j = 0; j < EX2_TPT; j++) {
      const uint32_t t = nxt[j], hi = t >> 16;
      const uint32_t len = tb + tid * EX2_TPT + j < ntok ? (hi ? hi : 1u) : 0u;
      ex[j] = lsum;
      lsum += len;
      pay[j] = hi ? (t & 0xffffu) + 1u + MARK_BASE : (t & 0xffu);
      ts[j] = len ? 0u : 0xffffffffu;
    }
    const uint32_t incl = wave_scan_add(lsum);
    if (lane == WAVE - 1) s_bs[par][wv] = incl;
#pragma unroll
    for (int j = 0; j < EX2_TPT; j++) __asm__ volatile("" : "+v"(pay[j]));  // done with nxt before it reloads
    exp_barrier();
    // next batch, in flight while this one is used (issued after the barrier,
    // so that no wait for it lands before the next batch)
#pragma unroll
    for (int j = 0; j < EX2_TPT; j++) {
      nxt[j] = *taddr(tb + EX2_TB + tid * EX2_TPT + j);
    }
    uint32_t before = 0, S = 0;
#pragma unroll
    for (uint32_t w = 0; w < EX2_W; w++) {
      const uint32_t x = s_bs[par][w];
      before += w < wv ? x : 0u;
      S += x;
    }
    par ^= 1u;
    const uint32_t b0 = bend + before + incl - lsum;
#pragma unroll
    for (int j = 0; j < EX2_TPT; j++) ts[j] = ts[j] ? ts[j] : b0 + ex[j];
    bend += S;
    tb += EX2_TB;
#if KP_ON
    kp_batch += KP_NOW() - kb0;
#endif
  };
  uint32_t R = 0, Rs = 0, carry = 0, flushed = 0, Fs = 0;
  const uint32_t toff = tid * EX2_E;
#if KP_ON
  // (profiling) a flushed wave piece (256 entries): does any entry still hold a
  // history marker?  Round 6 measured 81% of C2's entries and 99.9% of its
  // pieces do -- an emit that patched only marked pieces could not pay
  auto kp_piece = [&](uint32_t fs, uint32_t fl) {
    uint32_t m = 0;
    for (int k = 0; k < EX2_E; k++) m += ring[fs + toff + k] >= MARK_BASE ? 1u : 0u;
    kp_pc++;
    kp_me += kp_wave_sum(m);
    const bool f = __ballot(m != 0) != 0;
    kp_pf += f ? 1u : 0u;
    kp_pt += f && fl + wv * WAVE * EX2_E + WAVE * EX2_E > total - min(total, (uint32_t)HIST) ? 1u : 0u;
  };
#endif
  auto place = [&]() {  // marks of the loaded batch's tokens that start in round R
#pragma unroll
    for (int j = 0; j < EX2_TPT; j++) {
      const uint32_t rel = ts[j] - R;
      if (rel < EX2_N) s_mark[rel] = ((rel + 1u) << 16) | pay[j];
    }
  };
  // one loop for batches and rounds: the prefetched tokens stay in one set of
  // registers (a second loop made the compiler copy them at its back edge,
  // waiting for the loads every round)
  for (;;) {
    if (bend < R + EX2_N && tb < ntok) {  // round R reaches past the loaded tokens
      load_batch();
      place();
      continue;
    }
    if (R >= total) break;
#if KP_ON
    const uint64_t kr0 = KP_NOW();
    kp_rounds++;
#endif
    exp_barrier();  // B1: marks visible; the previous round's entries final
    while (R - flushed >= EX2_N) {
#if KP_ON
      kp_piece(Fs, flushed);
#endif
      ex2_copy(out + flushed + toff, &ring[Fs + toff]);
      flushed += EX2_N;
      Fs = Fs + EX2_N == EX2_RS ? 0u : Fs + EX2_N;
    }
    uint32_t mk[EX2_E];
    {
      uint4 *mp = reinterpret_cast<uint4 *>(&s_mark[toff]);
#pragma unroll
      for (int c = 0; c < EX2_E / 4; c++) {
        const uint4 a = mp[c];
        mk[4 * c] = a.x, mk[4 * c + 1] = a.y, mk[4 * c + 2] = a.z, mk[4 * c + 3] = a.w;
      }
#pragma unroll
      for (int c = 0; c < EX2_E / 4; c++) mp[c] = make_uint4(0, 0, 0, 0);
      if (EX2_E == 2) {
        uint2 *m2 = reinterpret_cast<uint2 *>(&s_mark[toff]);
        const uint2 a = *m2;
        mk[0] = a.x, mk[1 % EX2_E] = a.y;
        *m2 = make_uint2(0, 0);
      }
    }
    uint32_t tmax = 0;
#pragma unroll
    for (int k = 0; k < EX2_E; k++) tmax = max(tmax, mk[k]);
    const uint32_t winc = wave_scan_max(tmax);
    const uint32_t wexc = __shfl_up(winc, 1);
    if (lane == WAVE - 1) s_red[wv] = winc;
    exp_barrier();  // B2
    uint32_t run = max(carry, lane ? wexc : 0u), all = carry;
#pragma unroll
    for (uint32_t w = 0; w < EX2_W; w++) {
      const uint32_t x = s_red[w];
      run = w < wv ? max(run, x) : run;
      all = max(all, x);
    }
    carry = all & 0xffffu;
    const uint32_t s0 = Rs + toff;
    uint32_t v[EX2_E], unres = 0;
#pragma unroll
    for (int k = 0; k < EX2_E; k++) {
      run = max(run, mk[k]);
      const uint32_t pl = run & 0xffffu;
      const uint32_t x = s0 + (uint32_t)k + MARK_BASE - pl;  // source slot (wrapped below)
      const uint32_t xs = min(x, x + EX2_RS);
      const uint32_t rv = ring[xs < EX2_RS ? xs : 0u];
      const bool lit = pl < MARK_BASE;
      const bool in = pl <= toff + (uint32_t)k + MARK_BASE;  // distance <= e - R: source inside the round
      v[k] = lit ? pl : (in ? EX2_PTR + xs - Rs : rv);
      unres |= (!lit && in) ? 1u << k : 0u;
    }
#pragma unroll
    for (int c = 0; c < EX2_E / 8; c++) {
      uint4 w4;
      w4.x = v[8 * c] | (v[8 * c + 1] << 16);
      w4.y = v[8 * c + 2] | (v[8 * c + 3] << 16);
      w4.z = v[8 * c + 4] | (v[8 * c + 5] << 16);
      w4.w = v[8 * c + 6] | (v[8 * c + 7] << 16);
      *reinterpret_cast<uint4 *>(&ring[s0 + 8 * c]) = w4;
    }
    if (EX2_E == 4)
      *reinterpret_cast<uint2 *>(&ring[s0]) = make_uint2(v[0] | (v[1] << 16), v[2 % EX2_E] | (v[3 % EX2_E] << 16));
    if (EX2_E == 2) *reinterpret_cast<uint32_t *>(&ring[s0]) = v[0] | (v[1 % EX2_E] << 16);
    exp_barrier();  // B3: every entry holds a value or a pointer
#if KP_ON
    const uint64_t kr1 = KP_NOW();
    kp_pre += kr1 - kr0;
    kp_srounds += __ballot(unres != 0) ? 1u : 0u;
#endif
    while (unres) {
#if KP_ON
      kp_passes++;
#endif
      // other lanes write the ring meanwhile: no load may be reused across passes
      __asm__ volatile("" ::: "memory");
#ifndef EX2_SPIN_SEQ
      uint32_t r[EX2_E];
#pragma unroll
      for (int k = 0; k < EX2_E; k++) r[k] = ring[Rs + ((unres >> k) & 1u ? (v[k] & (EX2_N - 1u)) : 0u)];
#pragma unroll
      for (int k = 0; k < EX2_E; k++) {
        if (unres & (1u << k)) {
          if (r[k] < EX2_PTR) unres &= ~(1u << k);
          v[k] = r[k];
          ring[s0 + k] = (uint16_t)r[k];
        }
      }
#else
#pragma unroll
      for (int k = 0; k < EX2_E; k++) {
        if (unres & (1u << k)) {
          const uint32_t r = ring[Rs + (v[k] & (EX2_N - 1u))];
          if (r < EX2_PTR) unres &= ~(1u << k);
          v[k] = r;
          ring[s0 + k] = (uint16_t)r;
        }
      }
#endif
    }
#if KP_ON
    kp_spin += KP_NOW() - kr1;
#endif
    R += EX2_N;
    Rs = Rs + EX2_N == EX2_RS ? 0u : Rs + EX2_N;
    place();
  }
  exp_barrier();
  while (total - flushed >= EX2_N) {
#if KP_ON
    kp_piece(Fs, flushed);
#endif
    ex2_copy(out + flushed + toff, &ring[Fs + toff]);
    flushed += EX2_N;
    Fs = Fs + EX2_N == EX2_RS ? 0u : Fs + EX2_N;
  }
  for (uint32_t k = tid; k < total - flushed; k += EX2_T) out[flushed + k] = ring[Fs + k];
#if KP_ON  // per wave: E_BLOCKS waves, JUMP_ITERS spin passes (max over lanes), JUMP_ROUNDS rounds with a spin,
           // CYC_INIT token-batch cycles, CYC_JUMP spin cycles, slot 25 B1..B3 cycles
  {
    const uint64_t tot = KP_NOW() - kp_t0;
    KP_ADD(KP_E_BLOCKS, 1);
    KP_ADD(KP_E_CYC_TOTAL, tot);
    KP_MAX(KP_E_CYC_MAX, tot);
    KP_ADD(KP_E_CYC_INIT, kp_batch);
    KP_ADD(KP_E_ROUNDS, kp_rounds);
    KP_ADD(KP_E_JUMP_ITERS, kp_wave_max(kp_passes));
    KP_ADD(KP_E_JUMP_ROUNDS, kp_srounds);
    KP_ADD(KP_E_CYC_JUMP, kp_spin);
    KP_ADD(KP_E_BATCHES, kp_batches);
    KP_ADD(KP_E_JUMP_ROUNDS + 1, kp_pre);
    KP_ADD(6, kp_pc);  // (lane-parse slots the split parse leaves unused)
    KP_ADD(7, kp_pf);
    KP_ADD(8, kp_pt);
    KP_ADD(12, kp_me);
  }
#endif
}

// First dynamic header of every unit after the stream's first (the finder
// only records BFINAL = 0, BTYPE = 2 starts whose header validated), one wave
// per unit across the whole GPU: tables go to the unit's global table area and
// the compact root image next to them; the parse pass then starts each lane
// directly in symbol mode.  A header that does not decode is left to the parse
// pass, which redoes it cooperatively and reports exactly.
//
// Round 5: the stream's first unit too (ord 0), and fixed-code first blocks
// (BTYPE 1: the fixed tables are copied into the unit's table area, so every
// consumer treats them as a prebuilt block), each with the split parse's walk
// tables (TABLE_WALK_OFF).
template <bool D64>
__global__ void __launch_bounds__(64) zs_unit_header_kernel(const ZsJobDev *__restrict__ jobs,
                                                             const ZsHeadDev *__restrict__ heads,
                                                             ZsChunkDev *__restrict__ units, uint32_t *__restrict__ tables,
                                                             const uint32_t *__restrict__ fixed, int zl_out) {
  __shared__ BuildLDS B;
#if KP_ON
  const uint64_t kt0 = KP_NOW();
  uint64_t kt[3] = {kt0, kt0, kt0};
#endif
  const uint32_t c = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const ZsChunkDev ch = units[c];
  if (ch.start_bit == ZS_NONE || heads[ch.job].code != ZD_END) return;
  const ZsJobDev jb = jobs[ch.job];
  const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
  const uint32_t mis = (uint32_t)(ip & 3u);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(ip - mis);
  const uint32_t end_byte = mis + (uint32_t)jb.in_len;
  StageBits sb;
  stage_bits(B, w, end_byte, ch.start_bit, sb);
  if (ch.start_bit + 3 > end_byte * 8u) return;
  const uint32_t hdr3 = sb.peek(ch.start_bit, 3);
  const uint32_t btype = hdr3 >> 1;
  if (btype != 2u && btype != 1u) return;  // stored / invalid: the parse pass decides
  uint32_t bit = ch.start_bit + 3;
  uint32_t *tabg = tables + (size_t)c * TABLE_STRIDE;
  uint16_t *ctab = reinterpret_cast<uint16_t *>(tabg + TABLE_ENTRIES);
  uint16_t *img = reinterpret_cast<uint16_t *>(tabg + TABLE_IMG_OFF);
  uint8_t *walk = reinterpret_cast<uint8_t *>(tabg + TABLE_WALK_OFF);
  uint32_t lbits = 9, dbits = 6;
  if (btype == 1u) {  // fixed codes (src/inflate.c:260-298): lit/len root 9, distance root 5
    const uint16_t *fc = reinterpret_cast<const uint16_t *>(fixed + FIXED_ZLIB_WORDS);
    for (uint32_t i = lane; i < 512u; i += WAVE) {
      tabg[i] = fixed[i];
      ctab[i] = fc[i];
      walk[i] = (uint8_t)walk_len_z<D64>(fixed, 9u, i);
    }
    if (lane < 32) {
      tabg[DIST_TABLE_OFF + lane] = fixed[512 + lane];
      ctab[DIST_TABLE_OFF + lane] = fc[512 + lane];
      B.lens[lane] = 5;
    }
    for (uint32_t i = lane; i < LROOT_N; i += WAVE) img[i] = lds_len_root(fixed, 9u, i);
    img[LROOT_N + lane] = compact_dist_entry(fixed[512 + (lane & 31u)]);
    for (uint32_t i = lane; i < (1u << WK_DBITS); i += WAVE) walk[(1u << WK_LBITS) + i] = (uint8_t)walk_dist_z(fixed + 512, 5u, i);
    __builtin_amdgcn_wave_barrier();
    build_dist_tail(B.lens, 32, reinterpret_cast<uint8_t *>(img + LROOT_N + DROOT_N));
    if (lane < 16) tabg[TABLE_LTAIL_OFF + lane] = lane < 4 ? 0x80008000u : 0u;  // no code past 9 bits
    lbits = 9;
    dbits = 5;
  } else if (wave_dyn_header<D64>(B, w, end_byte, bit, tabg, ctab, lbits, dbits, img, img + LROOT_N,
                                  reinterpret_cast<uint8_t *>(img + LROOT_N + DROOT_N), walk,
                                  tabg + TABLE_LTAIL_OFF, zl_out != 0, true
#if KP_ON
                                  , kt
#endif
                                  )) {
    return;
  }
  if (lane == 0) {
    units[c].hdr_bit = bit;
    units[c].hdr_info = 1u | ((hdr3 & 1u) << 1) | (lbits << 8) | (dbits << 12);
  }
#if KP_ON  // (lane-parse slots the split parse leaves unused) units, cycles: all, prologue, code lengths, lit/len tables, rest
  if (btype == 2u) {
    const uint64_t te = KP_NOW();
    KP_ADD(0, 1);
    KP_ADD(1, te - kt0);
    KP_ADD(2, kt[0] - kt0);
    KP_ADD(11, kt[1] - kt[0]);
    KP_ADD(13, kt[2] - kt[1]);
    KP_ADD(14, te - kt[2]);
  }
#endif
}

// compact copies of the fixed tables (after zs_fixed_tables_kernel's zlib layout)
__global__ void __launch_bounds__(64) zs_fixed_compact_kernel(uint32_t *__restrict__ fixed) {
  uint16_t *fc = reinterpret_cast<uint16_t *>(fixed + FIXED_ZLIB_WORDS);
  for (uint32_t i = threadIdx.x; i < 512; i += WAVE) fc[i] = compact_len_entry(fixed[i]);
  for (uint32_t i = threadIdx.x; i < 32; i += WAVE) fc[512 + i] = compact_dist_entry(fixed[512 + i]);
}
extern "C" void zs_launch_fixed_compact(uint32_t *fixed, hipStream_t st) {
  hipLaunchKernelGGL(zs_fixed_compact_kernel, dim3(1), dim3(64), 0, st, fixed);
}

// Schedule keys of every unit slot: the compressed span before the parse, the
// output entries before the expand (0 for inactive or failed slots).
__global__ void zs_unit_keys_kernel(const ZsJobDev *__restrict__ jobs, const ZsChunkDev *__restrict__ chunks, uint32_t n,
                                    int after_parse, uint32_t *__restrict__ keys, uint32_t *__restrict__ ids) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ZsChunkDev ch = chunks[i];
  uint32_t k = 0;
  if (ch.start_bit != ZS_NONE) {
    if (after_parse) {
      k = ch.in_chain ? ch.n_out : 0u;
    } else {
      const uint64_t end = ch.stop_bit != ZS_NONE ? ch.stop_bit : (uint64_t)jobs[ch.job].in_len * 8u + 32u;
      k = (uint32_t)min<uint64_t>(end > ch.start_bit ? end - ch.start_bit : 1u, 0xffffffffu);
      k = max(k, 1u);
    }
  }
  keys[i] = k;
  ids[i] = i;
}

namespace {
struct SortWs {  // grown on demand; the library serializes batches
  uint32_t *buf = nullptr;  // keys in/out, ids in/out
  void *tmp = nullptr;
  size_t cap = 0, tmp_bytes = 0;
};
SortWs g_sorts[2];  // one per concurrent chunked group (zs_launch_chunked ctx)
// order[0..n) = unit slots by decreasing key (stable)
int sort_units(int ctx, const ZsJobDev *d_jobs, const ZsChunkDev *d_chunks, uint32_t n, int after_parse, uint32_t **order,
               hipStream_t st) {
  SortWs &g_sort = g_sorts[ctx & 1];
  if (n > g_sort.cap) {
    if (g_sort.buf) (void)hipFree(g_sort.buf);
    if (g_sort.tmp) (void)hipFree(g_sort.tmp);
    g_sort.buf = nullptr;
    g_sort.tmp = nullptr;
    const size_t c = std::max<size_t>(n, 2 * g_sort.cap);
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                 (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)c, 0, 32, st);
    if (hipMalloc(&g_sort.buf, 4 * c * sizeof(uint32_t)) != hipSuccess || hipMalloc(&g_sort.tmp, tb) != hipSuccess)
      return -1;
    g_sort.cap = c;
    g_sort.tmp_bytes = tb;
  }
  uint32_t *kin = g_sort.buf, *kout = kin + g_sort.cap, *vin = kout + g_sort.cap, *vout = vin + g_sort.cap;
  hipLaunchKernelGGL(zs_unit_keys_kernel, dim3((n + 255) / 256), dim3(256), 0, st, d_jobs, d_chunks, n, after_parse, kin,
                     vin);
  size_t tb = g_sort.tmp_bytes;
  if (hipcub::DeviceRadixSort::SortPairsDescending(g_sort.tmp, tb, kin, kout, vin, vout, (int)n, 0, 32, st) != hipSuccess)
    return -1;
  *order = vout;
  return 0;
}
}  // namespace

// Lane-parse waves resident at once (CUs x waves per CU by LDS); the lane
// kernel deals the sorted units over groups of this many waves.
extern "C" uint32_t zs_lane_resident_waves(void) {
  static const uint32_t v = [] {
    const char *e = std::getenv("ZS_LANE_MAP");
    if (e) return (uint32_t)std::atoi(e);
    int dev = 0, cus = 0, lds = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || cus <= 0 ||
        lds <= 0)
      return 0u;
    return (uint32_t)cus * std::max<uint32_t>(1u, (uint32_t)lds / (uint32_t)sizeof(LaneLDS));
  }();
  return v;
}

namespace {
struct SplitWs {  // split parse state per unit slot; grown on demand (the library serializes batches)
  ZsWalkDev *walks = nullptr;
  uint2 *cps = nullptr;
  uint32_t *lists = nullptr;  // [0, cap) walked units, [cap, 2 cap) leftovers; then the two counts
  size_t cap = 0;
};
SplitWs g_splits[2];  // one per concurrent chunked group (zs_launch_chunked ctx)
int split_reserve(int ctx, uint32_t n) {
  SplitWs &g_split = g_splits[ctx & 1];
  if (n <= g_split.cap) return 0;
  if (g_split.walks) (void)hipFree(g_split.walks);
  if (g_split.cps) (void)hipFree(g_split.cps);
  if (g_split.lists) (void)hipFree(g_split.lists);
  g_split = SplitWs{};
  const size_t c = (size_t)n + n / 2;
  if (hipMalloc(&g_split.walks, c * sizeof(ZsWalkDev)) != hipSuccess ||
      hipMalloc(&g_split.cps, (c + 1) * WK_CP * sizeof(uint2)) != hipSuccess ||  // + idle lanes' slot (zs_walk_kernel)
      hipMalloc(&g_split.lists, (2 * c + 3) * sizeof(uint32_t)) != hipSuccess)
    return -1;
  g_split.cap = c;
  return 0;
}
// Grid of the split and leftover kernels (they loop over device-side lists):
// enough waves to fill every SIMD several times over.
uint32_t split_grid(uint32_t n) {
  static const uint32_t g = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return (uint32_t)cus * 32u;
  }();
  return std::max(1u, std::min(n, g));
}
}  // namespace

// wave_units: 0 = a lane per unit (zs_lane_kernel), 1 = a wave per unit
// (zs_unitw_kernel, for batches with few units), 2 = the split parse (walk +
// sub-unit decode + leftovers, for batches with many units).
extern "C" void zs_launch_parse(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, ZsChunkDev *d_chunks, uint32_t nchunks,
                                uint32_t *d_tokens, uint32_t *d_tables, const uint32_t *d_fixed, ZsTokPool pool, int d64,
                                int wave_units, hipStream_t st, int ctx) {
  if (!nchunks) return;
  SplitWs &g_split = g_splits[ctx & 1];
  if (wave_units == 2 && split_reserve(ctx, nchunks) != 0) {  // no room for the split state: the lane parse
    (void)hipGetLastError();
    wave_units = 0;
  }
  // the split parse reads only the compact and walk tables of a unit's first
  // block (a failed split decodes its header again): no zlib-layout copy
  const int zl_out = wave_units == 2 ? 0 : 1;
  if (d64)
    hipLaunchKernelGGL(zs_unit_header_kernel<true>, dim3(nchunks), dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, d_tables,
                       d_fixed, zl_out);
  else
    hipLaunchKernelGGL(zs_unit_header_kernel<false>, dim3(nchunks), dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, d_tables,
                       d_fixed, zl_out);
  uint32_t *order = nullptr;
  if (sort_units(ctx, d_jobs, d_chunks, nchunks, 0, &order, st)) return;
  if (wave_units == 2) {
    uint32_t *counts = g_split.lists + 2 * g_split.cap;
    uint32_t *lists = g_split.lists;
    (void)hipMemsetAsync(counts, 0, 3 * sizeof(uint32_t), st);  // splits, leftovers, the split's next unit
    // the walk deals its sorted units over the waves resident at once, as the lane parse
    static const uint32_t lane_map = [] {
      int dev = 0, cus = 0, lds = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
          cus <= 0 || lds <= 0)
        return 0u;
      return (uint32_t)cus * std::max<uint32_t>(1u, (uint32_t)lds / (uint32_t)sizeof(WalkLDS));
    }();
    const dim3 wgrid((nchunks + WAVE - 1) / WAVE), sgrid(split_grid(nchunks));
    // (tests) ZS_SPLIT_LEFT=1: every split unit fails its check and goes to the leftovers
    static const int force_left = getenv("ZS_SPLIT_LEFT") ? 1 : 0;
    // the leftover list lives at lists + nchunks: the kernels index it that way
    if (d64) {
      hipLaunchKernelGGL(zs_walk_kernel<true>, wgrid, dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, nchunks, d_tables,
                         order, pool, lane_map, g_split.walks, g_split.cps, lists, counts);
      hipLaunchKernelGGL(zs_split_kernel<true>, sgrid, dim3(WAVE), 0, st, d_jobs, d_chunks, nchunks, d_tokens, d_tables,
                         pool, g_split.walks, g_split.cps, lists, counts, force_left);
      hipLaunchKernelGGL(zs_unitw_list_kernel<true>, sgrid, dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, d_tokens,
                         d_tables, d_fixed, lists + nchunks, counts + 1, pool, g_split.walks);
    } else {
      hipLaunchKernelGGL(zs_walk_kernel<false>, wgrid, dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, nchunks, d_tables,
                         order, pool, lane_map, g_split.walks, g_split.cps, lists, counts);
      hipLaunchKernelGGL(zs_split_kernel<false>, sgrid, dim3(WAVE), 0, st, d_jobs, d_chunks, nchunks, d_tokens, d_tables,
                         pool, g_split.walks, g_split.cps, lists, counts, force_left);
      hipLaunchKernelGGL(zs_unitw_list_kernel<false>, sgrid, dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, d_tokens,
                         d_tables, d_fixed, lists + nchunks, counts + 1, pool, g_split.walks);
    }
    static const bool dbg = getenv("ZS_SPLIT_STATS") != nullptr;
    if (dbg) {  // (diagnostics) walked units and leftovers of this batch, on stderr
      uint32_t h[2] = {0, 0};
      if (hipMemcpyAsync(h, counts, sizeof h, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess)
        fprintf(stderr, "split: %u unit slots, %u walked, %u leftovers\n", nchunks, h[0], h[1]);
    }
    return;
  }
  if (wave_units) {
    if (d64)
      hipLaunchKernelGGL(zs_unitw_kernel<true>, dim3(nchunks), dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, nchunks,
                         d_tokens, d_tables, d_fixed, order, pool);
    else
      hipLaunchKernelGGL(zs_unitw_kernel<false>, dim3(nchunks), dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks, nchunks,
                         d_tokens, d_tables, d_fixed, order, pool);
    return;
  }
  // Units sorted longest first are dealt round-robin over the waves that can
  // be resident at once (CUs x waves per CU by LDS), then over the next such
  // group: every resident wave gets a share of the long units (C2 parse 18.7 ->
  // 17.8 ms, C5 73.8 -> 69.0 ms; spreading over more waves than fit made the
  // last ones wait a round, 28.6 ms).  Env ZS_LANE_MAP: group size, 0 = blocked.
  const uint32_t lane_map = zs_lane_resident_waves();
  if (d64)
    hipLaunchKernelGGL(zs_lane_kernel<true>, dim3((nchunks + WAVE - 1) / WAVE), dim3(WAVE), 0, st, d_jobs, d_heads,
                       d_chunks, nchunks, d_tokens, d_tables, d_fixed, order, pool, lane_map);
  else
    hipLaunchKernelGGL(zs_lane_kernel<false>, dim3((nchunks + WAVE - 1) / WAVE), dim3(WAVE), 0, st, d_jobs, d_heads,
                       d_chunks, nchunks, d_tokens, d_tables, d_fixed, order, pool, lane_map);
}

// ZS_EXPAND=1: the round-per-batch expand kernel for 32 KiB windows too (A/B)
static bool expand_v1() {
  static const bool v = [] {
    const char *e = getenv("ZS_EXPAND");
    return e && atoi(e) == 1;
  }();
  return v;
}

// expand the verified chain members (after zs_chain_kernel), longest first
extern "C" void zs_launch_expand(const ZsJobDev *d_jobs, ZsChunkDev *d_chunks, uint32_t nchunks, uint16_t *d_scratch,
                                 const uint32_t *d_tokens, ZsTokPool pool, uint32_t *d_fallback, int d64, hipStream_t st,
                                 int ctx) {
  if (!nchunks) return;
  uint32_t *order = nullptr;
  if (sort_units(ctx, d_jobs, d_chunks, nchunks, 1, &order, st)) return;
  if (d64)
    hipLaunchKernelGGL(zs_expand_kernel<true>, dim3(nchunks), dim3(EXP_T), 0, st, d_jobs, d_chunks, d_scratch, d_tokens,
                       order, pool, d_fallback);
  else if (expand_v1())
    hipLaunchKernelGGL(zs_expand_kernel<false>, dim3(nchunks), dim3(EXP_T), 0, st, d_jobs, d_chunks, d_scratch, d_tokens,
                       order, pool, d_fallback);
  else
    hipLaunchKernelGGL(zs_expand2_kernel, dim3(nchunks), dim3(EX2_T), 0, st, d_jobs, d_chunks, d_scratch, d_tokens,
                       order, pool);
}

extern "C" int zs_kprof_read_ck(uint64_t *out16, int reset);
extern "C" int zs_kprof_read_dz(uint64_t *out12, int reset);
// Counter readback (profiling builds only; product builds report 0 counters).
extern "C" int zs_kprof_read_w(uint64_t *out32, int reset);
extern "C" int zs_kprof_read(uint64_t *out, uint32_t n, int reset) {
#if KP_ON
  const uint32_t k = n < KP_TOTAL ? n : KP_TOTAL;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kprof), (k < KP_COUNT ? k : KP_COUNT) * sizeof(uint64_t)) != hipSuccess) return -1;
  if (k >= KP_TOTAL) {
    uint64_t w[32];
    if (zs_kprof_read_w(w, reset) == 32)
      for (int i = 0; i < 32; i++) out[64 + i] = w[i];
  }
  if (k >= 64) {
    uint64_t ck[16];
    if (zs_kprof_read_ck(ck, reset) == 16)
      for (int i = 0; i < 16; i++) out[48 + i] = ck[i];
    uint64_t dz[12];
    if (zs_kprof_read_dz(dz, reset) == 12)
      for (int i = 0; i < 12; i++) out[26 + i] = dz[i];
  }
  if (reset) {
    static const unsigned long long z[KP_COUNT] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_kprof), z, sizeof z) != hipSuccess) return -1;
  }
  return (int)k;
#else
  (void)out;
  (void)n;
  (void)reset;
  return 0;
#endif
}
