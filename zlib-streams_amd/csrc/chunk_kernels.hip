// chunk_kernels.hip -- speculative chunk-parallel inflate for large streams.
//
// Hot loop of the reference: src/inffast.c:100-287 (symbol decode + copy), fed
// by the block/table states of src/inflate.c:834-1033 and src/inftrees.c.
// MI355X design:
//   zs_find_kernel   one wave per chunk; each lane tests 32 bit offsets per
//                    step with bit-parallel filters (BFINAL=0, BTYPE=2, HLIT,
//                    HDIST, complete code-length code), survivors get a full
//                    header validation; the lowest valid offset wins.
//   zs_lane_kernel   ONE LANE PER CHUNK: 64 independent decoders per wave.
//                    Each lane decodes symbols with its own zlib-layout tables
//                    (global, per chunk) and writes u16 entries; matches that
//                    reach before the chunk start emit markers 256+w naming
//                    byte w of the unknown 32 KiB history.  Block headers and
//                    stored blocks are handled cooperatively: the whole wave
//                    works on one lane's header at a time (bits staged in LDS,
//                    ballot-parallel table build), then the lane resumes.
//   zs_link_kernel   one workgroup per stream: verifies the chunk chain,
//                    computes output offsets, resolves the 32 KiB history of
//                    every chunk in order (LDS double buffer).
//   zs_emit_kernel   one workgroup per chunk: entries -> bytes at their final
//                    offsets (markers looked up in the chunk's window in LDS).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zs_common.h"
#include "zs_device.h"

#define MARK_BASE 256u
#define HIST 32768u
#define STAGE_WORDS 256  // 1 KiB of staged header bits per cooperative step

// ---------------------------------------------------------------------------
// masked 32-bit input word (bytes at or past end_byte read as zero)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t in_word(const uint32_t *w, uint32_t wi, uint32_t end_byte) {
  uint32_t b = wi * 4u;
  if (b + 4u <= end_byte) return w[wi];
  if (b >= end_byte) return 0u;
  uint32_t keep = end_byte - b;  // 1..3
  return w[wi] & ((1u << (8u * keep)) - 1u);
}

// ---------------------------------------------------------------------------
// Full dynamic-header validation for one candidate (per lane, rare path).
// Mirrors the acceptance rules of src/inflate.c:905-1033 + src/inftrees.c
// (complete code-length code, repeat rules, end-of-block present, literal and
// distance codes complete or a single 1-bit code, empty distance code allowed).
// ---------------------------------------------------------------------------
__device__ bool validate_header(const uint32_t *w, uint32_t end_byte, uint32_t bit, uint8_t *lut) {
  const uint32_t limit = end_byte * 8u;
  uint32_t wi = bit >> 5;
  uint64_t hold = (uint64_t)in_word(w, wi, end_byte) >> (bit & 31);
  uint32_t n = 32 - (bit & 31);
  wi++;
  auto refill = [&]() {
    while (n <= 32) {
      hold |= (uint64_t)in_word(w, wi, end_byte) << n;
      n += 32;
      wi++;
    }
  };
  auto pos = [&]() { return wi * 32u - n; };
  refill();
  hold >>= 3;
  n -= 3;
  const uint32_t nlen = (uint32_t)(hold & 31) + 257, ndist = (uint32_t)((hold >> 5) & 31) + 1;
  const uint32_t ncode = (uint32_t)((hold >> 10) & 15) + 4;
  hold >>= 14;
  n -= 14;
  if (nlen > 286 || ndist > 30) return false;
  uint8_t cl[19];
#pragma unroll
  for (int i = 0; i < 19; i++) cl[i] = 0;
  const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
#pragma unroll
  for (int i = 0; i < 19; i++) {
    if ((uint32_t)i < ncode) {
      refill();
      cl[ord[i]] = (uint8_t)(hold & 7);
      hold >>= 3;
      n -= 3;
    }
  }
  // canonical codes of the code-length code -> 7-bit LUT (sym | len << 5)
  uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 19; i++) cnt[cl[i]]++;
  uint32_t nxt[8];
  nxt[0] = 0;
  nxt[1] = 0;
  uint32_t code = 0;
#pragma unroll
  for (int L = 1; L < 8; L++) {
    code = (code + (L > 1 ? cnt[L - 1] : 0)) << (L > 1 ? 1 : 0);
    nxt[L] = code;
  }
  for (int i = 0; i < 128; i++) lut[i] = 0;
#pragma unroll
  for (int s = 0; s < 19; s++) {
    uint32_t L = cl[s];
    if (L) {
      uint32_t c = 0;
#pragma unroll
      for (int x = 1; x < 8; x++)
        if ((uint32_t)x == L) c = nxt[x]++;
      uint32_t rev = __builtin_bitreverse32(c) >> (32 - L);
      for (uint32_t j = rev; j < 128; j += (1u << L)) lut[j] = (uint8_t)(s | (L << 5));
    }
  }
  const uint32_t total = nlen + ndist;
  uint32_t have = 0, prev = 0, eob = 0;
  uint32_t lk = 0, lmax = 0, dk = 0, dmax = 0, dn = 0;
  while (have < total) {
    refill();
    uint32_t e = lut[hold & 127];
    uint32_t L = e >> 5, sym = e & 31;
    if (L == 0) return false;
    hold >>= L;
    n -= L;
    uint32_t rep = 1, v = sym;
    if (sym == 16) {
      if (have == 0) return false;
      rep = 3 + (uint32_t)(hold & 3);
      hold >>= 2;
      n -= 2;
      v = prev;
    } else if (sym == 17) {
      rep = 3 + (uint32_t)(hold & 7);
      hold >>= 3;
      n -= 3;
      v = 0;
    } else if (sym == 18) {
      rep = 11 + (uint32_t)(hold & 127);
      hold >>= 7;
      n -= 7;
      v = 0;
    }
    if (pos() > limit) return false;
    if (have + rep > total) return false;
    if (v) {
      // split the run between the literal/length and distance code lengths
      uint32_t nl = have < nlen ? min(rep, nlen - have) : 0u;
      uint32_t nd = rep - nl;
      lk += nl << (15 - v);
      if (nl) lmax = max(lmax, v);
      dk += nd << (15 - v);
      dn += nd;
      if (nd) dmax = max(dmax, v);
      if (have <= 256 && 256 < have + rep) eob = v;
    }
    prev = v;
    have += rep;
  }
  if (eob == 0) return false;
  if (lk > 32768u || (lk < 32768u && lmax != 1)) return false;
  if (dn && (dk > 32768u || (dk < 32768u && dmax != 1))) return false;
  return true;
}

// ---------------------------------------------------------------------------
// Block finder
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) zs_find_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                      ZsChunkDev *__restrict__ chunks, const uint32_t *__restrict__ ids) {
  __shared__ uint8_t s_lut[WAVE][128];
  const uint32_t lane = threadIdx.x;
  const uint32_t c = ids[blockIdx.x];
  const ZsChunkDev ch = chunks[c];
  const ZsJobDev jb = jobs[ch.job];
  const ZsHeadDev hd = heads[ch.job];
  if (hd.code != ZD_END) {
    if (lane == 0) chunks[c].start_bit = ZS_NONE;
    return;
  }
  const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
  const uint32_t mis = (uint32_t)(ip & 3u);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(ip - mis);
  const uint32_t end_byte = mis + (uint32_t)jb.in_len;
  uint32_t lo = (mis + max(ch.s_byte, (uint32_t)hd.start_byte)) * 8u;
  const uint32_t hi = (mis + ch.e_byte) * 8u;
  for (uint32_t base = lo & ~31u; base < hi; base += WAVE * 32u) {
    const uint32_t b0 = base + lane * 32u;
    uint32_t found = ZS_NONE;
    if (b0 < hi) {
      const uint32_t wi = b0 >> 5;
      const uint64_t lo64 = (uint64_t)in_word(w, wi, end_byte) | ((uint64_t)in_word(w, wi + 1, end_byte) << 32);
      const uint64_t hi64 = (uint64_t)in_word(w, wi + 2, end_byte) | ((uint64_t)in_word(w, wi + 3, end_byte) << 32);
      // BFINAL = 0, BTYPE = 2 at offset p: bit p = 0, bit p+1 = 0, bit p+2 = 1
      uint32_t cand = (uint32_t)(~lo64 & ~(lo64 >> 1) & (lo64 >> 2));
      if (b0 < lo) cand &= ~0u << (lo - b0);
      if (hi - b0 < 32u) cand &= (1u << (hi - b0)) - 1u;
      while (cand) {
        const uint32_t p = __builtin_ctz(cand);
        cand &= cand - 1u;
        const uint64_t h = lo64 >> (p + 3);
        if ((h & 31) > 29 || ((h >> 5) & 31) > 29) continue;
        const uint32_t ncode = (uint32_t)((h >> 10) & 15) + 4;
        const uint32_t s = p + 17;  // 17..48
        const uint64_t clb = (lo64 >> s) | (hi64 << (64 - s));
        uint32_t kraft = 0;
#pragma unroll
        for (int i = 0; i < 19; i++) {
          uint32_t L = (uint32_t)(clb >> (3 * i)) & 7u;
          if ((uint32_t)i < ncode && L) kraft += 128u >> L;
        }
        if (kraft != 128u) continue;
        if (validate_header(w, end_byte, b0 + p, s_lut[lane])) {
          found = b0 + p;
          break;
        }
      }
    }
    const uint64_t m = __ballot(found != ZS_NONE);
    if (m) {
      const uint32_t first_lane = (uint32_t)__builtin_ctzll(m);
      const uint32_t f = __builtin_amdgcn_readlane(found, first_lane);
      if (lane == 0) chunks[c].start_bit = f;
      return;
    }
  }
  if (lane == 0) chunks[c].start_bit = ZS_NONE;
}

// ---------------------------------------------------------------------------
// Fixed tables (src/inflate.c:260-298) built once into global memory.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) zs_fixed_tables_kernel(uint32_t *__restrict__ fixed) {
  __shared__ uint32_t s_tab[544];
  __shared__ uint16_t s_lens[320];
  __shared__ uint16_t s_sorted[320];
  __shared__ uint32_t s_scr[32];
  const uint32_t lane = threadIdx.x;
  for (uint32_t s = lane; s < 288; s += WAVE) s_lens[s] = s < 144 ? 8 : (s < 256 ? 9 : (s < 280 ? 7 : 8));
  __builtin_amdgcn_wave_barrier();
  uint32_t r = 9;
  build_table(T_LENS, s_lens, 288, s_tab, &r, s_sorted, s_scr, 0);
  for (uint32_t s = lane; s < 32; s += WAVE) s_lens[s] = 5;
  __builtin_amdgcn_wave_barrier();
  r = 5;
  build_table(T_DISTS, s_lens, 32, s_tab + 512, &r, s_sorted, s_scr, 0);
  for (uint32_t i = lane; i < 544; i += WAVE) fixed[i] = s_tab[i];
}

// ---------------------------------------------------------------------------
// Lane decoder
// ---------------------------------------------------------------------------
enum { LM_SYM = 0, LM_BLOCK = 1, LM_DONE = 2 };

struct LaneState {
  const uint32_t *w;   // 4-byte aligned input base
  uint32_t end_byte, limit;
  uint32_t wi, nw, nbits;
  uint64_t hold;
  uint16_t *out;
  uint32_t pos, cap;
  const uint32_t *lt, *dt;
  uint32_t lmask, dmask;
  uint32_t stop, bit, whave;
  int mode, code, last;
};

__device__ __forceinline__ void lane_prime(LaneState &s, uint32_t bit) {
  s.wi = bit >> 5;
  uint32_t w0 = in_word(s.w, s.wi, s.end_byte);
  s.nw = in_word(s.w, s.wi + 1, s.end_byte);
  s.hold = (uint64_t)w0 >> (bit & 31);
  s.nbits = 32 - (bit & 31);
  s.wi += 1;
}
__device__ __forceinline__ void lane_refill(LaneState &s) {
  if (s.nbits < 32) {
    s.hold |= (uint64_t)s.nw << s.nbits;
    s.nbits += 32;
    s.wi++;
    s.nw = in_word(s.w, s.wi, s.end_byte);
  }
}
__device__ __forceinline__ uint32_t lane_pos(const LaneState &s) { return s.wi * 32u - s.nbits; }

// one symbol; returns true when the lane left symbol mode
__device__ __forceinline__ bool lane_step(LaneState &s) {
  lane_refill(s);
  uint32_t e = s.lt[(uint32_t)s.hold & s.lmask];
  uint32_t op = e_op(e);
  uint32_t used = e_bits(e);
  if (op != 0 && (op & 0xf0u) == 0) {
    e = s.lt[e_val(e) + ((uint32_t)(s.hold >> used) & ((1u << op) - 1u))];
    used += e_bits(e);
    op = e_op(e);
  }
  if (lane_pos(s) + used > s.limit) {
    s.code = ZD_TRUNC;
    s.mode = LM_DONE;
    return true;
  }
  s.hold >>= used;
  s.nbits -= used;
  if (op == 0) {
    if (s.pos >= s.cap) {
      s.code = ZD_FULL;
      s.mode = LM_DONE;
      return true;
    }
    s.out[s.pos++] = (uint16_t)e_val(e);
    return false;
  }
  if (op & 32) {  // end of block
    s.bit = lane_pos(s);
    s.mode = LM_BLOCK;
    return true;
  }
  if (op & 64) {
    s.code = ZD_ERROR | (ZM_LITLEN_CODE << 8);
    s.mode = LM_DONE;
    return true;
  }
  uint32_t len = e_val(e);
  const uint32_t xb = op & 15u;
  len += (uint32_t)s.hold & ((1u << xb) - 1u);
  s.hold >>= xb;
  s.nbits -= xb;
  lane_refill(s);
  uint32_t d = s.dt[(uint32_t)s.hold & s.dmask];
  uint32_t dop = e_op(d);
  uint32_t dused = e_bits(d);
  if ((dop & 0xf0u) == 0) {
    d = s.dt[e_val(d) + ((uint32_t)(s.hold >> dused) & ((1u << dop) - 1u))];
    dused += e_bits(d);
    dop = e_op(d);
  }
  const uint32_t dx = dop & 15u;
  if (lane_pos(s) + dused + dx > s.limit) {
    s.code = ZD_TRUNC;
    s.mode = LM_DONE;
    return true;
  }
  s.hold >>= dused;
  s.nbits -= dused;
  if (dop & 64) {
    s.code = ZD_ERROR | (ZM_DIST_CODE << 8);
    s.mode = LM_DONE;
    return true;
  }
  const uint32_t dist = e_val(d) + ((uint32_t)s.hold & ((1u << dx) - 1u));
  s.hold >>= dx;
  s.nbits -= dx;
  if (s.pos + len > s.cap) {
    s.code = ZD_FULL;
    s.mode = LM_DONE;
    return true;
  }
  const int q = (int)s.pos - (int)dist;
  if (q < -(int)s.whave) {
    s.code = ZD_ERROR | (ZM_TOO_FAR << 8);
    s.mode = LM_DONE;
    return true;
  }
  // copy: entry k comes from q + (k mod dist) (always before pos, so the group
  // loads never depend on this match's own stores); q < 0 -> history marker
  uint16_t *o = s.out + s.pos;
  uint32_t m = 0;
  for (uint32_t k = 0; k < len; k += 8) {
    uint16_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int idx = q + (int)m;
      v[i] = (idx < 0) ? (uint16_t)(MARK_BASE + HIST + idx) : ((k + i < len) ? s.out[idx] : (uint16_t)0);
      m = (m + 1 == dist) ? 0u : m + 1;
    }
#pragma unroll
    for (int i = 0; i < 8; i++)
      if (k + i < len) o[k + i] = v[i];
  }
  s.pos += len;
  return false;
}

// Wave-uniform bit reader over the LDS-staged header bits.
struct StageBits {
  const uint32_t *st;  // LDS words
  uint32_t base;       // bit index of st[0] in the input
  __device__ __forceinline__ uint32_t peek(uint32_t bit, uint32_t n) const {
    uint32_t r = bit - base;
    uint64_t v = (uint64_t)st[r >> 5] | ((uint64_t)st[(r >> 5) + 1] << 32);
    return (uint32_t)(v >> (r & 31)) & ((n >= 32) ? 0xffffffffu : ((1u << n) - 1u));
  }
};

struct CoopLDS {
  uint32_t stage[STAGE_WORDS + 4];
  uint32_t tab[TABLE_ENTRIES];
  uint16_t lens[320];
  uint16_t sorted[320];
  uint32_t scr[32];
};

// Stage 1 KiB of input starting at the 16-byte boundary at or below `bit`.
__device__ void stage_bits(CoopLDS &L, const uint32_t *w, uint32_t end_byte, uint32_t bit, StageBits &sb) {
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

// Cooperative block-boundary processing for lane `ln` (all lanes call it with
// the same ln).  Handles end/stop checks, stored blocks, fixed and dynamic
// headers; installs the lane's tables.  Mirrors src/inflate.c:834-1033.
__device__ void coop_block(LaneState &s, uint32_t ln, CoopLDS &L, uint32_t *lane_tab, const uint32_t *fixed) {
  const uint32_t lane = lane_id();
  const uint32_t *w = reinterpret_cast<const uint32_t *>(readlane_ptr(s.w, ln));
  uint16_t *out = reinterpret_cast<uint16_t *>(readlane_ptr(s.out, ln));
  uint32_t *tabg = reinterpret_cast<uint32_t *>(readlane_ptr(lane_tab, ln));
  const uint32_t end_byte = __builtin_amdgcn_readlane(s.end_byte, ln);
  const uint32_t limit = end_byte * 8u;
  const uint32_t stop = __builtin_amdgcn_readlane(s.stop, ln);
  const uint32_t cap = __builtin_amdgcn_readlane(s.cap, ln);
  uint32_t bit = __builtin_amdgcn_readlane(s.bit, ln);
  uint32_t pos = __builtin_amdgcn_readlane(s.pos, ln);
  int last = __builtin_amdgcn_readlane(s.last, ln);
  int mode = LM_DONE, code = 0;
  const uint32_t *lt = nullptr, *dt = nullptr;
  uint32_t lbits = 0, dbits = 0;
  for (;;) {
    if (last) {
      code = ZD_END;
      break;
    }
    if (bit >= stop) {
      code = ZD_STOP;
      break;
    }
    if (bit + 3 > limit) {
      code = ZD_TRUNC;
      break;
    }
    StageBits sb;
    stage_bits(L, w, end_byte, bit, sb);
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
      stage_bits(L, w, end_byte, bit, sb);
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
      const uint8_t *src = reinterpret_cast<const uint8_t *>(w) + bit / 8;
      for (uint32_t k = lane; k < n; k += WAVE) out[pos + k] = src[k];
      pos += n;
      bit += n * 8;
      continue;
    }
    if (type == 1) {
      lt = fixed;
      dt = fixed + 512;
      lbits = 9;
      dbits = 5;
      mode = LM_SYM;
      break;
    }
    if (type == 3) {
      code = ZD_ERROR | (ZM_BLOCK_TYPE << 8);
      break;
    }
    // dynamic header
    if (bit + 14 > limit) {
      code = ZD_TRUNC;
      break;
    }
    const uint32_t h = sb.peek(bit, 14);
    const uint32_t nlen = (h & 31) + 257, ndist = ((h >> 5) & 31) + 1, ncode = ((h >> 10) & 15) + 4;
    bit += 14;
    if (nlen > 286 || ndist > 30) {
      code = ZD_ERROR | (ZM_TOO_MANY << 8);
      break;
    }
    if (bit + 3 * ncode > limit) {
      code = ZD_TRUNC;
      break;
    }
    if (lane < 19) L.lens[c_clorder[lane]] = lane < ncode ? (uint16_t)sb.peek(bit + 3 * lane, 3) : (uint16_t)0;
    bit += 3 * ncode;
    __builtin_amdgcn_wave_barrier();
    uint32_t cbits = 7;
    if (build_table(T_CODES, L.lens, 19, L.tab, &cbits, L.sorted, L.scr, 0)) {
      code = ZD_ERROR | (ZM_CODE_LENGTHS << 8);
      break;
    }
    const uint32_t total = nlen + ndist;
    const uint32_t cmask = (1u << cbits) - 1u;
    uint32_t have = 0;
    bool bad = false;
    while (have < total) {
      if (bit - sb.base > (STAGE_WORDS - 2) * 32u - 64u) stage_bits(L, w, end_byte, bit, sb);
      const uint32_t x = sb.peek(bit, 14);
      const uint32_t e = L.tab[x & cmask];
      const uint32_t eb = e_bits(e), ev = e_val(e);
      if (ev < 16) {
        if (bit + eb > limit) { bad = true; code = ZD_TRUNC; break; }
        bit += eb;
        if (lane == 0) L.lens[have] = (uint16_t)ev;
        have++;
        continue;
      }
      const uint32_t xb = ev == 16 ? 2u : (ev == 17 ? 3u : 7u);
      if (bit + eb + xb > limit) { bad = true; code = ZD_TRUNC; break; }
      if (ev == 16 && have == 0) { bad = true; code = ZD_ERROR | (ZM_REPEAT << 8); break; }
      const uint32_t rep = (ev == 18 ? 11u : 3u) + ((x >> eb) & ((1u << xb) - 1u));
      bit += eb + xb;
      if (have + rep > total) { bad = true; code = ZD_ERROR | (ZM_REPEAT << 8); break; }
      __builtin_amdgcn_wave_barrier();
      const uint32_t fillv = ev == 16 ? uni(L.lens[have - 1]) : 0u;
      for (uint32_t k = lane; k < rep; k += WAVE) L.lens[have + k] = (uint16_t)fillv;
      __builtin_amdgcn_wave_barrier();
      have += rep;
    }
    if (bad) break;
    __builtin_amdgcn_wave_barrier();
    if (uni(L.lens[256]) == 0) {
      code = ZD_ERROR | (ZM_MISSING_EOB << 8);
      break;
    }
    lbits = 9;
    if (build_table(T_LENS, L.lens, nlen, L.tab, &lbits, L.sorted, L.scr, 0)) {
      code = ZD_ERROR | (ZM_LITLEN_SET << 8);
      break;
    }
    dbits = 6;
    if (build_table(T_DISTS, L.lens + nlen, ndist, L.tab + DIST_TABLE_OFF, &dbits, L.sorted, L.scr, 0)) {
      code = ZD_ERROR | (ZM_DIST_SET << 8);
      break;
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = lane; i < TABLE_ENTRIES; i += WAVE) tabg[i] = L.tab[i];
    lt = tabg;
    dt = tabg + DIST_TABLE_OFF;
    mode = LM_SYM;
    break;
  }
  if (lane == ln) {
    s.pos = pos;
    s.last = last;
    s.bit = bit;
    s.mode = mode;
    if (mode == LM_SYM) {
      s.lt = lt;
      s.dt = dt;
      s.lmask = (1u << lbits) - 1u;
      s.dmask = (1u << dbits) - 1u;
      lane_prime(s, bit);
    } else {
      s.code = code;
    }
  }
}

__global__ void __launch_bounds__(64) zs_lane_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                      ZsChunkDev *__restrict__ chunks, uint32_t nchunks,
                                                      uint16_t *__restrict__ scratch, uint32_t *__restrict__ tables,
                                                      const uint32_t *__restrict__ fixed) {
  __shared__ CoopLDS L;
  const uint32_t lane = threadIdx.x;
  const uint32_t c = blockIdx.x * WAVE + lane;
  LaneState s;
  s.mode = LM_DONE;
  s.code = ZD_SKIP;
  s.pos = 0;
  s.last = 0;
  s.bit = 0;
  s.stop = ZS_NONE;
  s.w = nullptr;
  s.out = nullptr;
  s.end_byte = 0;
  s.limit = 0;
  s.cap = 0;
  s.whave = 0;
  s.lt = s.dt = fixed;
  s.lmask = s.dmask = 0;
  s.wi = s.nw = s.nbits = 0;
  s.hold = 0;
  uint32_t *lane_tab = tables + (size_t)min(c, nchunks - 1) * TABLE_ENTRIES;
  if (c < nchunks) {
    const ZsChunkDev ch = chunks[c];
    const ZsHeadDev hd = heads[ch.job];
    const ZsJobDev jb = jobs[ch.job];
    const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
    const uint32_t mis = (uint32_t)(ip & 3u);
    uint32_t start = ch.ord == 0 ? (mis + (uint32_t)hd.start_byte) * 8u : ch.start_bit;
    if (hd.code == ZD_END && start != ZS_NONE) {
      s.w = reinterpret_cast<const uint32_t *>(ip - mis);
      s.end_byte = mis + (uint32_t)jb.in_len;
      s.limit = s.end_byte * 8u;
      s.out = scratch + ch.scratch;
      s.cap = ch.cap;
      s.whave = ch.ord == 0 ? 0u : HIST;
      s.bit = start;
      s.mode = LM_BLOCK;
      s.code = 0;
      for (uint32_t k = ch.ord + 1; k < ch.nchunks; k++) {
        uint32_t sb = chunks[ch.first + k].start_bit;
        if (sb != ZS_NONE) {
          s.stop = sb;
          break;
        }
      }
    }
  }
  for (;;) {
    uint64_t need = __ballot(s.mode == LM_BLOCK);
    while (need) {
      const uint32_t ln = (uint32_t)__builtin_ctzll(need);
      need &= need - 1;
      coop_block(s, ln, L, lane_tab, fixed);
    }
    if (__ballot(s.mode == LM_SYM) == 0) break;
    if (s.mode == LM_SYM) {
      for (int it = 0; it < 64; it++)
        if (lane_step(s)) break;
    }
  }
  if (c < nchunks) {
    ZsChunkDev *ch = &chunks[c];
    ch->code = s.code;
    ch->end_bit = (s.code == ZD_END || s.code == ZD_STOP) ? s.bit : 0u;
    ch->n_out = s.pos;
  }
}

// ---------------------------------------------------------------------------
// Link: verify the chain, offsets, history windows (one workgroup per stream)
// ---------------------------------------------------------------------------
#define LINK_THREADS 256
__global__ void __launch_bounds__(LINK_THREADS) zs_link_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                               ZsChunkDev *__restrict__ chunks, const ZsCJobDev *__restrict__ cjobs,
                                                               const uint16_t *__restrict__ scratch, uint8_t *__restrict__ windows,
                                                               ZsDecDev *__restrict__ decs, uint32_t *__restrict__ fallback) {
  __shared__ uint8_t s_win[2][HIST];
  __shared__ uint32_t s_ok, s_cur, s_next;
  __shared__ uint32_t s_end_bit;
  __shared__ uint64_t s_total;
  const uint32_t t = threadIdx.x;
  const ZsCJobDev cj = cjobs[blockIdx.x];
  const ZsJobDev jb = jobs[cj.job];
  const ZsHeadDev hd = heads[cj.job];
  if (hd.code != ZD_END) {
    if (t == 0) {
      fallback[cj.job] = 0;
      ZsDecDev d;
      d.code = ZD_SKIP;
      d.msg = 0;
      d.end_bits = 0;
      d.total_out = 0;
      decs[cj.job] = d;
    }
    return;
  }
  if (t == 0) {
    // walk the chain from chunk 0
    uint32_t c = cj.first;
    uint64_t total = 0;
    uint32_t ok = 1, end_bit = 0;
    for (;;) {
      ZsChunkDev ch = chunks[c];
      chunks[c].out_off = total;
      total += ch.n_out;
      const int code = ch.code & 0xff;
      if (code == ZD_END) {
        chunks[c].chain_next = ZS_NONE;
        end_bit = ch.end_bit;
        break;
      }
      if (code != ZD_STOP) {
        ok = 0;
        break;
      }
      uint32_t k = ZS_NONE;
      for (uint32_t o = ch.ord + 1; o < cj.nchunks; o++)
        if (chunks[cj.first + o].start_bit != ZS_NONE) {
          k = cj.first + o;
          break;
        }
      if (k == ZS_NONE || chunks[k].start_bit != ch.end_bit) {
        ok = 0;
        break;
      }
      chunks[c].chain_next = k;
      c = k;
    }
    if (total > jb.out_cap) ok = 0;
    s_ok = ok;
    s_total = total;
    s_end_bit = end_bit;
    s_cur = cj.first;
  }
  __syncthreads();
  if (!s_ok) {
    if (t == 0) fallback[cj.job] = 1;
    return;
  }
  // history windows in chain order: W holds the last HIST bytes before chunk c
  uint32_t wv = 0;  // valid bytes of history
  int cur = 0;
  uint32_t c = s_cur;
  for (;;) {
    const ZsChunkDev ch = chunks[c];
    uint8_t *W = s_win[cur];
    uint8_t *W2 = s_win[cur ^ 1];
    if (ch.ord != 0) {
      uint8_t *g = windows + (size_t)c * HIST;
      for (uint32_t i = t * 16; i < HIST; i += LINK_THREADS * 16)
        *reinterpret_cast<uint4 *>(g + i) = *reinterpret_cast<const uint4 *>(W + i);
    }
    const uint32_t n = ch.n_out;
    const uint16_t *e = scratch + ch.scratch;
    const uint32_t keep = n < HIST ? HIST - n : 0u;  // old history bytes still inside the new window
    for (uint32_t i = t; i < keep; i += LINK_THREADS) W2[i] = W[i + n];
    const uint32_t lowest = HIST - wv;  // first valid history index
    for (uint32_t i = keep + t; i < HIST; i += LINK_THREADS) {
      const uint32_t v = e[n - HIST + i];
      uint32_t b;
      if (v < MARK_BASE) {
        b = v;
      } else {
        const uint32_t wx = v - MARK_BASE;
        if (wx < lowest) s_ok = 0;  // reaches before the stream start
        b = W[wx & (HIST - 1)];
      }
      W2[i] = (uint8_t)b;
    }
    wv = min(HIST, wv + n);
    cur ^= 1;
    __syncthreads();
    if (ch.chain_next == ZS_NONE) break;
    c = ch.chain_next;
  }
  if (t == 0) {
    if (!s_ok) {
      fallback[cj.job] = 1;
    } else {
      fallback[cj.job] = 0;
      ZsDecDev d;
      d.code = ZD_END;
      d.msg = 0;
      const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(jb.in) & 3u);
      d.end_bits = s_end_bit - mis * 8u;
      d.total_out = s_total;
      decs[cj.job] = d;
      // mark chain members for the emit pass
      uint32_t k = cj.first;
      while (k != ZS_NONE) {
        chunks[k].in_chain = 1;
        k = chunks[k].chain_next;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Emit: u16 entries -> final bytes (one workgroup per chunk)
// ---------------------------------------------------------------------------
#define EMIT_THREADS 256
__global__ void __launch_bounds__(EMIT_THREADS) zs_emit_kernel(const ZsJobDev *__restrict__ jobs, const ZsChunkDev *__restrict__ chunks,
                                                               const uint16_t *__restrict__ scratch, const uint8_t *__restrict__ windows,
                                                               const uint32_t *__restrict__ fallback) {
  __shared__ uint8_t s_w[HIST];
  const uint32_t c = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const ZsChunkDev ch = chunks[c];
  if (!ch.in_chain || fallback[ch.job]) return;
  if (ch.ord != 0) {
    const uint8_t *g = windows + (size_t)c * HIST;
    for (uint32_t i = t * 16; i < HIST; i += EMIT_THREADS * 16)
      *reinterpret_cast<uint4 *>(s_w + i) = *reinterpret_cast<const uint4 *>(g + i);
    __syncthreads();
  }
  uint8_t *out = jobs[ch.job].out + ch.out_off;
  const uint16_t *e = scratch + ch.scratch;
  const uint32_t n = ch.n_out;
  // bytes [0, head) and the tail are written byte-wise so no 8-byte word is
  // shared with a neighbouring chunk; the body uses aligned 8-byte stores
  const uint32_t head = min(n, (uint32_t)((8u - (uint32_t)(reinterpret_cast<uintptr_t>(out) & 7u)) & 7u));
  for (uint32_t i = t; i < head; i += EMIT_THREADS) {
    uint32_t v = e[i];
    out[i] = (uint8_t)(v < MARK_BASE ? v : s_w[v - MARK_BASE]);
  }
  const uint32_t body = (n - head) & ~7u;
  for (uint32_t i = head + t * 8; i < head + body; i += EMIT_THREADS * 8) {
    uint64_t word = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t v = e[i + k];
      uint32_t b = v < MARK_BASE ? v : s_w[v - MARK_BASE];
      word |= (uint64_t)b << (8 * k);
    }
    *reinterpret_cast<uint64_t *>(out + i) = word;
  }
  for (uint32_t i = head + body + t; i < n; i += EMIT_THREADS) {
    uint32_t v = e[i];
    out[i] = (uint8_t)(v < MARK_BASE ? v : s_w[v - MARK_BASE]);
  }
}

// ---------------------------------------------------------------------------
// host launch helpers
// ---------------------------------------------------------------------------
extern "C" void zs_launch_fixed_tables(uint32_t *fixed, hipStream_t st) {
  hipLaunchKernelGGL(zs_fixed_tables_kernel, dim3(1), dim3(64), 0, st, fixed);
}

extern "C" void zs_launch_chunked(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, ZsChunkDev *d_chunks, uint32_t nchunks,
                                  const uint32_t *d_find_ids, uint32_t nfind, const ZsCJobDev *d_cjobs, uint32_t ncjobs,
                                  uint16_t *d_scratch, uint32_t *d_tables, const uint32_t *d_fixed, uint8_t *d_windows,
                                  ZsDecDev *d_decs, uint32_t *d_fallback, hipStream_t st, hipEvent_t *ev) {
  if (nfind) hipLaunchKernelGGL(zs_find_kernel, dim3(nfind), dim3(64), 0, st, d_jobs, d_heads, d_chunks, d_find_ids);
  if (ev) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(zs_lane_kernel, dim3((nchunks + WAVE - 1) / WAVE), dim3(WAVE), 0, st, d_jobs, d_heads, d_chunks,
                     nchunks, d_scratch, d_tables, d_fixed);
  if (ev) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(zs_link_kernel, dim3(ncjobs), dim3(LINK_THREADS), 0, st, d_jobs, d_heads, d_chunks, d_cjobs,
                     d_scratch, d_windows, d_decs, d_fallback);
  hipLaunchKernelGGL(zs_emit_kernel, dim3(nchunks), dim3(EMIT_THREADS), 0, st, d_jobs, d_chunks, d_scratch, d_windows,
                     d_fallback);
}
