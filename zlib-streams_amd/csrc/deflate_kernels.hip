// deflate_kernels.hip -- GPU deflate (LZ77 match-find + Huffman emission).
//
// Reference path: the deflate core of the zlib submodule (deflate.c, absent
// from /root/reference; pinned by host zlib 1.2.11) and
// src/trees.c (_tr_tally 1029-1053, _tr_flush_block 931-1023, build_tree 561,
// gen_bitlen 474, gen_codes 205, send_all_trees 767, compress_block 834-882).
// The output is a valid raw / zlib / gzip deflate stream that inflates to the
// input (tests/test_gpu_deflate.py checks every case); it is not
// byte-identical to zlib's (that needs zlib's sequential hash chains).
//
// MI355X design: every stream is cut into 64 KiB SEGMENTS, each compressed
// independently into one deflate block (matches may reach 32 KiB back into the
// previous segment: the input is all in HBM, so history is free):
//   zs_dz_match_kernel  one 256-thread workgroup per segment: an LDS hash table
//                       (8192 buckets x 4 ways of 16-bit positions, primed with
//                       the 32 KiB before the segment); 256 positions per step
//                       look up their 4 candidates, verify them 4 bytes at a
//                       time and keep the longest match (clamped to the segment);
//   zs_dz_parse_kernel  one LANE per segment: zlib-style lazy parse over the
//                       per-position matches, writing tokens in place (the
//                       inflate parse pass's token format);
//   zs_dz_block_kernel  one workgroup per segment: LDS histograms, length-
//                       limited Huffman codes (rank sort + two-queue build +
//                       count adjustment), dynamic header, fixed/dynamic/stored
//                       choice, then every token's bit length, a block scan for
//                       bit offsets and LDS atomicOr packing; the block's bits
//                       go to an aligned per-segment buffer;
//   zs_dz_stitch_kernel one workgroup per segment: shifts the block's bits to
//                       its offset in the job's stream (a per-job scan over
//                       segment bit lengths) with atomicOr on the two boundary
//                       words; zs_dz_frame_kernel writes the wrapper header,
//                       the checksum combine (CRC-32 / Adler-32 over segment
//                       pieces) and the trailer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zs_common.h"
#include "zs_device.h"
#include "zs_check.h"
#include "zs_kprof.h"

#if KP_ON
__device__ unsigned long long g_kprof_dz[12];  // KP_D_* - 26
#define KPD_ADD(i, v) atomicAdd(&g_kprof_dz[(i) - 26], (unsigned long long)(v))
#else
#define KPD_ADD(i, v) ((void)0)
#endif

#define DZ_SEG 65536u        // input bytes per segment
#define DZ_T 256u            // threads per workgroup
#define DZ_HB 8192u          // hash buckets
#define DZ_WAYS 4u
#define DZ_WIN 32768u        // deflate window
#define DZ_OUTW 18440u       // LDS output words per block: the fixed-code bound 3 + 9 x 64 Ki + 7 bits

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const uint8_t gcu8;  // global loads, not flat
__device__ __forceinline__ uint32_t dz_load32(gcu8 *p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
__device__ __forceinline__ uint4 dz_load128(gcu8 *p) {  // unaligned 16-byte load
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
// bytes equal at the start of a and b (0..16)
__device__ __forceinline__ uint32_t dz_eq16(uint4 a, uint4 b) {
  const uint32_t x0 = a.x ^ b.x, x1 = a.y ^ b.y, x2 = a.z ^ b.z, x3 = a.w ^ b.w;
  if (x0) return (uint32_t)__builtin_ctz(x0) >> 3;
  if (x1) return 4u + ((uint32_t)__builtin_ctz(x1) >> 3);
  if (x2) return 8u + ((uint32_t)__builtin_ctz(x2) >> 3);
  if (x3) return 12u + ((uint32_t)__builtin_ctz(x3) >> 3);
  return 16u;
}
__device__ __forceinline__ uint32_t dz_hash(uint32_t v) { return (v * 2654435761u) >> (32 - 13); }

// length 3..258 -> length code index 0..28 and its extra bits (inverse of the
// lbase/lext tables of src/inftrees.c:59-64)
// Deflate64 (inflate9 tables, src/inftrees.c:73-87): code 284 covers 227..258
// (5 extra bits), code 285 is 3 + a 16-bit extra (lengths 3..65538; used here
// for merged runs longer than 258).
__device__ __forceinline__ uint32_t dz_len_sym(uint32_t len, uint32_t *xb, uint32_t *xv, bool d64 = false) {
  const uint32_t l = len - 3u;
  if (d64 && len >= 258u) {
    *xb = len == 258u ? 5u : 16u;
    *xv = len == 258u ? 31u : l;
    return len == 258u ? 27u : 28u;
  }
  if (len == 258u) {
    *xb = 0;
    *xv = 0;
    return 28;
  }
  if (l < 8u) {
    *xb = 0;
    *xv = 0;
    return l;
  }
  const uint32_t e = (31u - __builtin_clz(l)) - 2u;
  *xb = e;
  *xv = l & ((1u << e) - 1u);
  return 4u + 4u * e + ((l >> e) - 4u);
}
// distance 1..32768 -> distance code 0..29 and extra bits (dbase/dext)
__device__ __forceinline__ uint32_t dz_dist_sym(uint32_t dist, uint32_t *xb, uint32_t *xv) {
  const uint32_t d = dist - 1u;
  if (d < 4u) {
    *xb = 0;
    *xv = 0;
    return d;
  }
  const uint32_t e = (31u - __builtin_clz(d)) - 1u;
  *xb = e;
  *xv = d & ((1u << e) - 1u);
  return 2u + 2u * e + ((d >> e) - 2u);
}

// ---------------------------------------------------------------------------
// D1: match finding
// ---------------------------------------------------------------------------
// One 512-thread workgroup per HALF segment (32 KiB of positions).  The half,
// the 32 KiB of history before it and the longest match past its end are
// staged in LDS next to the hash table (8192 buckets x 4 ways of 16-bit
// window offsets, 0 = empty): candidate compares read LDS, not HBM.  A step
// looks up 512 positions at once, then inserts them; positions 128 k ..
// 128 k + 127 of a step go to way k, the even wave of the pair first and the
// odd (later) one after a barrier, and within one store the higher lane lands
// last -- the table, and so the output, is deterministic.
#define DZ_MT 512u
#define DZ_HALF 32768u

__device__ __forceinline__ uint32_t dz_lds32(const uint32_t *w, uint32_t a) {
  return __builtin_amdgcn_alignbyte(w[(a >> 2) + 1], w[a >> 2], a & 3u);
}
__device__ __forceinline__ uint4 dz_lds128(const uint32_t *w, uint32_t a) {
  const uint32_t k = a >> 2, b = a & 3u;
  const uint32_t x0 = w[k], x1 = w[k + 1], x2 = w[k + 2], x3 = w[k + 3], x4 = w[k + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(x1, x0, b), __builtin_amdgcn_alignbyte(x2, x1, b),
                    __builtin_amdgcn_alignbyte(x3, x2, b), __builtin_amdgcn_alignbyte(x4, x3, b));
}

// Deflate64 (window_bits -16): a 64 KiB window, so one workgroup per QUARTER
// segment (16 KiB of positions after 64 KiB of history: 80 KiB + the table in
// LDS); table entries are then positions mod 2^16 (a candidate is rel minus
// the 16-bit difference; every candidate is verified byte by byte anyway).
template <bool D64>
__global__ void __launch_bounds__(DZ_MT) zs_dz_match_kernel(const ZsDJobDev *__restrict__ jobs,
                                                             const ZsDSegDev *__restrict__ segs,
                                                             uint16_t *__restrict__ dist16, uint8_t *__restrict__ len8) {
  constexpr uint32_t SPAN = D64 ? DZ_HALF / 2u : DZ_HALF;   // positions per workgroup
  constexpr uint32_t HIST = D64 ? 2u * DZ_WIN : DZ_WIN;     // history before them
  constexpr uint32_t PARTS = DZ_SEG / SPAN;
  __shared__ uint16_t tab[DZ_HB][DZ_WAYS];
  __shared__ __attribute__((aligned(16))) uint32_t win[(HIST + SPAN + 288u) / 4 + 8];
  const uint32_t tid = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x / PARTS];
  const uint32_t half = blockIdx.x % PARTS;
  const ZsDJobDev jb = jobs[sg.job];
  if ((jb.wbits == 16u) != D64) return;  // the other variant's job
  if (jb.level == 0 || jb.exact || half * SPAN >= sg.len) return;  // stored blocks / zlib-identical jobs / no positions
  gcu8 *in = (gcu8 *)jb.in;
  const uint64_t n = jb.in_len;
  const uint64_t s = sg.start + half * SPAN;
  const uint64_t segend = sg.start + sg.len;  // matches stop at the segment end
  const uint64_t e = min<uint64_t>(segend, s + SPAN);
  const uint64_t hs = s > HIST ? s - HIST : 0;
  const uint64_t we = min<uint64_t>(segend, e + 272u);
  // per position: length - 3 (4..258 -> 1..255; 0 = no match) and distance - 1
  uint16_t *do16 = dist16 + sg.tok + half * SPAN;
  uint8_t *lo8 = len8 + sg.tok + half * SPAN;
  for (uint32_t i = tid; i < DZ_HB * DZ_WAYS / 2; i += DZ_MT) reinterpret_cast<uint32_t *>(tab)[i] = 0u;
  {
    const uint32_t nb = (uint32_t)(we - hs), n16 = (nb + 15u) / 16u;
    for (uint32_t k = tid; k < n16; k += DZ_MT) {
      const uint64_t a = hs + 16ull * k;
      uint4 v;
      if (a + 16 <= n) {
        v = dz_load128(in + a);
      } else {
        uint32_t b[4] = {0, 0, 0, 0};
        for (uint32_t i = 0; a + i < n && i < 16; i++) b[i >> 2] |= (uint32_t)in[a + i] << (8u * (i & 3u));
        v = make_uint4(b[0], b[1], b[2], b[3]);
      }
      *reinterpret_cast<uint4 *>(&win[4 * k]) = v;
    }
  }
  __syncthreads();
  const uint32_t way = (tid >> 7) & 3u;
  const bool odd = (tid >> 6) & 1u;
  // prime with the history: 4 consecutive positions per thread and step (a
  // thread's stores land in order, the even wave of a pair before the odd)
  for (uint64_t P = hs; P < s; P += 4u * DZ_MT) {
    uint32_t hh[4];
    uint16_t tv[4];
    bool okk[4];
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) {
      const uint64_t p = P + 4u * tid + r;
      okk[r] = p < s && p + 4 <= n;
      const uint32_t rel = (uint32_t)(p - hs);
      hh[r] = okk[r] ? dz_hash(dz_lds32(win, rel)) : 0u;
      tv[r] = (uint16_t)(D64 ? rel : rel + 1u);
    }
    if (!odd)
#pragma unroll
      for (uint32_t r = 0; r < 4; r++)
        if (okk[r]) tab[hh[r]][way] = tv[r];
    __syncthreads();
    if (odd)
#pragma unroll
      for (uint32_t r = 0; r < 4; r++)
        if (okk[r]) tab[hh[r]][way] = tv[r];
    __syncthreads();
  }
  const uint32_t maxd = 1u << jb.wbits;
  for (uint64_t P = s; P < e; P += DZ_MT) {
    const uint64_t p = P + tid;
    const bool ok = p < e && p + 4 <= n;
    const uint32_t rel = (uint32_t)(p - hs);
    uint32_t h = 0, best = 0, bd = 0;
    if (ok) {
      const uint32_t lim = (uint32_t)min<uint64_t>(258u, segend - p);
      const uint4 cur = dz_lds128(win, rel);
      h = dz_hash(cur.x);
      const uint2 ent = *reinterpret_cast<const uint2 *>(&tab[h][0]);
      const uint32_t c4[4] = {ent.x & 0xffffu, ent.x >> 16, ent.y & 0xffffu, ent.y >> 16};
#pragma unroll
      for (uint32_t w = 0; w < DZ_WAYS; w++) {
        uint32_t crel, d;
        if (D64) {
          d = (rel - c4[w]) & 0xffffu;  // 0: empty, or exactly 2^16 back (skipped)
          if (d == 0 || d > rel) continue;
          crel = rel - d;
        } else {
          if (!c4[w]) continue;
          crel = c4[w] - 1u;
          d = rel - crel;
          if (crel >= rel || d > maxd) continue;
        }
        if (dz_lds32(win, crel) != cur.x) continue;  // 2 LDS words reject most candidates (hash collisions)
        uint32_t L = dz_eq16(dz_lds128(win, crel), cur);
        if (L < 4u) continue;
        if (L == 16u) {
          while (L + 16u <= lim) {
            const uint32_t k = dz_eq16(dz_lds128(win, crel + L), dz_lds128(win, rel + L));
            L += k;
            if (k < 16u) break;
          }
          if (L + 16u > lim && L < lim) L += dz_eq16(dz_lds128(win, crel + L), dz_lds128(win, rel + L));
        }
        L = min(L, lim);
        if (L > best || (L == best && d < bd)) {
          best = L;
          bd = d;
        }
      }
    }
    if (p < e) {  // candidates need 4 equal bytes; the segment-end clamp can leave fewer
      lo8[p - s] = (uint8_t)(best >= 4u ? best - 3u : 0u);
      do16[p - s] = (uint16_t)(best >= 4u ? bd - 1u : 0u);
    }
    const bool ins = ok && (D64 || rel + 1u <= 0xffffu);
    const uint16_t tv = (uint16_t)(D64 ? rel : rel + 1u);
    __syncthreads();  // every lookup of the step before its inserts
    if (ins && !odd) tab[h][way] = tv;
    __syncthreads();
    if (ins && odd) tab[h][way] = tv;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// D2: lazy parse (zlib deflate_slow semantics: a match is deferred by one byte
// when the next position has a longer one and the current is shorter than
// max_lazy; greedy below level 4), one workgroup per segment.
//
// The parse is the path from position 0 under next(p), a function of m[p] and
// m[p+1] only.  Thread i owns positions [256 i, 256 i + 256): it walks from
// its own first position (speculation) and marks the positions it visits.
// Paths under next() merge within a few tokens, so the exit of range i rarely
// depends on where the true path enters it: every thread re-walks from its
// predecessor's exit until it meets a marked position (then its speculative
// exit holds) or leaves the range, and the rounds repeat until no exit
// changes (usually one).  The result is two bitmaps per segment: token
// starts (S) and match starts (T), read by the block kernel.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const uint32_t gcu32;
#define DZ_BMW (DZ_SEG / 32u)  // start-bitmap words per segment

// next(p) over the LDS length stage (length - 3, 0 = no match)
__device__ __forceinline__ uint32_t dz_next(const uint8_t *sl, uint32_t p, uint32_t len, uint32_t max_lazy) {
  const uint32_t l8 = sl[p];
  const uint32_t n8 = p + 1 < len ? sl[p + 1] : 0u;
  const uint32_t L = l8 + 3u, NL8 = n8 + 3u;
  return (l8 && !(L < max_lazy && n8 && NL8 > L)) ? p + L : p + 1;
}

__global__ void __launch_bounds__(DZ_T) zs_dz_parse_kernel(const ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                            const uint8_t *__restrict__ len8, uint32_t *__restrict__ bm) {
  __shared__ __attribute__((aligned(16))) uint8_t s_len[DZ_SEG];
  __shared__ uint32_t s_vis[DZ_BMW];  // speculative marks, then the token starts
  __shared__ uint32_t s_ex[DZ_T];
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.level == 0 || jb.exact) return;
  const uint32_t len = sg.len;
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(len8 + sg.tok);
    uint4 *dst = reinterpret_cast<uint4 *>(s_len);
    const uint32_t n16 = (len + 15u) / 16u;
    for (uint32_t k = t; k < n16; k += DZ_T) dst[k] = src[k];
  }
  const uint32_t max_lazy = jb.level >= 4 ? 16u : 0u;
  const uint32_t a = t * 256u, b = min(len, a + 256u);
  const bool active = a < len;
  for (uint32_t k = 0; k < 8; k++) s_vis[t * 8 + k] = 0;
  __syncthreads();
  // speculative walk from the range start (own bitmap words only)
  uint32_t p = a;
  while (p < b) {
    s_vis[p >> 5] |= 1u << (p & 31u);
    p = dz_next(s_len, p, len, max_lazy);
  }
  const uint32_t spec = active ? p : a;
  s_ex[t] = spec;
  __syncthreads();
  for (;;) {
    const uint32_t e = t == 0 ? 0u : s_ex[t - 1];
    uint32_t r = s_ex[t];
    if (active) {
      uint32_t q = e;
      r = q;
      while (q < b) {
        if (s_vis[q >> 5] & (1u << (q & 31u))) {
          r = spec;
          break;
        }
        q = dz_next(s_len, q, len, max_lazy);
        r = q;
      }
    }
    __syncthreads();
    const bool changed = active && r != s_ex[t];
    if (changed) s_ex[t] = r;
    if (!__syncthreads_or(changed)) break;
  }
  // final walk from the true entry; the marks are the owner's alone, so they
  // are cleared and reused for the token starts
  for (uint32_t k = 0; k < 8; k++) s_vis[t * 8 + k] = 0;
  uint32_t cnt = 0;
  if (active) {
    uint32_t q = t == 0 ? 0u : s_ex[t - 1];
    while (q < b) {
      s_vis[q >> 5] |= 1u << (q & 31u);
      cnt++;
      q = dz_next(s_len, q, len, max_lazy);
    }
  }
  __syncthreads();
  uint32_t *o = bm + (uint64_t)blockIdx.x * DZ_BMW;
  for (uint32_t k = t; k < DZ_BMW; k += DZ_T) o[k] = s_vis[k];
  uint32_t c = cnt;  // token count: wave sums into segs[].ntok (zeroed by the host)
  for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off);
  if ((t & 63u) == 0) atomicAdd(&segs[blockIdx.x].ntok, c);
}

// the 16 positions q0 .. q0 + 15 of one block-kernel thread: token starts
// (S), match starts (a start whose successor position is not a start; the
// segment end counts as a start), lengths, distances (loaded only for the
// halves holding a match start) and literal bytes
// ---------------------------------------------------------------------------
// D2b (deflate64 only): long copies become ONE code-285 match (3 + a 16-bit
// extra: lengths up to 65538; src/inftrees.c:73-87).  From every 258-long
// match at p with distance d, the wave extends the copy while
// in[p + k] == in[p + k - d] (64 bytes per compare), then absorbs the
// following tokens that lie wholly inside the extension: their bytes are the
// copy's bytes, so the output is unchanged.  Absorbed starts leave the start
// bitmap and x16[p] holds the length beyond 258.  One wave per segment walks
// its tokens in order from an LDS copy of the bitmap and lengths (a
// test-vector path, not a hot one).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(WAVE) zs_dz_merge_kernel(const ZsDJobDev *__restrict__ jobs,
                                                            const ZsDSegDev *__restrict__ segs,
                                                            const uint16_t *__restrict__ dist16,
                                                            const uint8_t *__restrict__ len8, uint32_t *__restrict__ bm,
                                                            uint16_t *__restrict__ lx16) {
  __shared__ uint32_t sS[DZ_SEG / 32u];
  __shared__ __attribute__((aligned(16))) uint8_t sL[DZ_SEG];
  const uint32_t lane = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.wbits != 16u || jb.level == 0 || jb.exact) return;
  uint32_t *S = bm + (uint64_t)blockIdx.x * (DZ_SEG / 32u);
  const uint16_t *d16 = dist16 + sg.tok;
  uint16_t *x16 = lx16 + sg.tok;
  const uint8_t *in = jb.in + sg.start;
  const uint32_t len = sg.len;
  for (uint32_t k = lane; k < DZ_SEG / 32u; k += WAVE) sS[k] = S[k];
  for (uint32_t k = lane; k < (len + 15u) / 16u; k += WAVE)
    reinterpret_cast<uint4 *>(sL)[k] = reinterpret_cast<const uint4 *>(len8 + sg.tok)[k];
  __syncthreads();
  auto start = [&](uint32_t q) -> bool { return q >= len || ((sS[q >> 5] >> (q & 31u)) & 1u); };
  auto tlen = [&](uint32_t q) -> uint32_t { return (q + 1 < len && !start(q + 1)) ? sL[q] + 3u : 1u; };
  uint32_t p = 0;
  while (p < len) {  // p is a token start: tokens tile the segment
    const uint32_t L = tlen(p);
    if (L != 258u) {
      p += L;
      continue;
    }
    const uint32_t d = (uint32_t)d16[p] + 1u;
    const uint32_t lim = min(65538u, len - p);
    uint32_t M = 258u;
    while (M < lim) {
      const uint32_t k = M + lane;
      const bool bad = k < lim && in[p + k] != in[(int64_t)p + k - d];
      const uint64_t bm64 = __ballot(bad);
      if (bm64) {
        M += (uint32_t)__builtin_ctzll(bm64);
        break;
      }
      M = min(lim, M + WAVE);
    }
    uint32_t q = p + 258u;
    while (q < len) {
      const uint32_t Lq = tlen(q);
      if (q + Lq > p + M) break;
      if (lane == 0) sS[q >> 5] &= ~(1u << (q & 31u));
      __builtin_amdgcn_wave_barrier();
      q += Lq;
    }
    if (lane == 0) x16[p] = (uint16_t)(q - p - 258u);
    p = q;
  }
  __syncthreads();
  for (uint32_t k = lane; k < DZ_SEG / 32u; k += WAVE) S[k] = sS[k];
}

struct DzTok16 {
  uint32_t s16, t16;
  uint4 l8, lit;
  uint4 d[2];
  uint32_t q0;
  const uint16_t *x16;  // deflate64: length beyond 258 of merged runs (zs_dz_merge_kernel), else null
};
__device__ __forceinline__ void dz_load_tok16(DzTok16 &k, gcu32 *bS, gcu8 *l8, const uint16_t *d16, gcu8 *in, uint32_t q0,
                                              uint32_t len) {
  k.s16 = 0;
  k.t16 = 0;
  k.q0 = q0;
  if (q0 >= len) return;
  const uint32_t w = bS[q0 >> 5];
  const uint32_t sh = q0 & 16u;
  const uint32_t real = (w >> sh) & 0xffffu;  // positions >= len are 0
  const uint32_t nb = q0 + 16u < len ? (sh ? bS[(q0 >> 5) + 1] & 1u : (w >> 16) & 1u) : 0u;
  uint32_t s17 = real | (nb << 16);
  if (len - q0 <= 16u) s17 |= 1u << (len - q0);  // the segment end
  k.s16 = real;
  k.t16 = real & ~(s17 >> 1);
  __builtin_memcpy(&k.l8, l8 + q0, 16);
  typedef __attribute__((address_space(1))) const uint16_t gcu16;
  gcu16 *dp = (gcu16 *)(d16 + q0);
  if (k.t16 & 0x00ffu) __builtin_memcpy(&k.d[0], dp, 16);
  if (k.t16 & 0xff00u) __builtin_memcpy(&k.d[1], dp + 8, 16);
  if (q0 + 16u <= len) {
    k.lit = dz_load128(in + q0);
  } else {
    uint32_t b[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; q0 + i < len; i++) b[i >> 2] |= (uint32_t)in[q0 + i] << (8u * (i & 3u));
    k.lit = make_uint4(b[0], b[1], b[2], b[3]);
  }
}
__device__ __forceinline__ uint32_t dz_u4_byte(uint4 v, uint32_t i) {
  const uint32_t w = i < 4 ? v.x : i < 8 ? v.y : i < 12 ? v.z : v.w;
  return (w >> (8u * (i & 3u))) & 0xffu;
}
// the token word at position i: ((length - 2) << 16) | (distance - 1), or the literal
__device__ __forceinline__ uint32_t dz_tok16_at(const DzTok16 &k, uint32_t i) {
  if ((k.t16 >> i) & 1u) {
    const uint4 dv = k.d[i >> 3];
    const uint32_t j = i & 7u;
    const uint32_t w = j < 2 ? dv.x : j < 4 ? dv.y : j < 6 ? dv.z : dv.w;
    uint32_t L = dz_u4_byte(k.l8, i) + 3u;
    if (k.x16 && L == 258u) L += k.x16[k.q0 + i];
    return ((L - 2u) << 16) | ((w >> (16u * (j & 1u))) & 0xffffu);
  }
  return dz_u4_byte(k.lit, i);
}

// ---------------------------------------------------------------------------
// D3: Huffman codes and block emission (src/trees.c _tr_flush_block 931-1023),
// three kernels:
//   zs_dz_hist_kernel   one workgroup per segment: symbol histograms, extra
//                       bits and the fixed-code cost;
//   zs_dz_codes_kernel  one THREAD per segment: the serial code build (sort,
//                       two-queue Huffman, length limit, canonical codes),
//                       header RLE and code-length code, the dynamic / fixed
//                       choice and the header bits.  Every segment builds at
//                       once (scratch rows laid out SoA in HBM, so a wave's
//                       accesses coalesce), instead of one thread per
//                       workgroup holding a CU's LDS;
//   zs_dz_emit_kernel   one workgroup per segment: token bits at scanned
//                       offsets, atomicOr-packed into a 16 KiB LDS ring that
//                       is flushed to the segment's output after every chunk.
// ---------------------------------------------------------------------------
#define NL 286
#define ND 32  // 30 deflate distance codes + deflate64's 30/31 (zero for deflate streams)
#define NC 19
#define DZ_HROWS 320u  // histogram rows per segment (SoA): lit/len 0..285, dist 286..317, extra bits 318, fixed bits 319
#define DZ_ROW_XBITS (NL + ND)
#define DZ_ROW_FIX (NL + ND + 1)
#define DZ_CROW 320u   // code words per segment (AoS): lit/len 0..285, dist 286..317 (code | len << 16, code bit-reversed)
#define DZ_HDRW 192u   // header words per segment (AoS); word 191 = header bit count
#define DZ_SCR 2400u   // build scratch rows per segment (SoA)
#define DZ_AUXW (DZ_HROWS + DZ_CROW + DZ_HDRW + DZ_SCR)  // aux words per segment
#define DZ_RING 4096u  // emit ring words (16 KiB); a chunk emits <= 4096 x 15 bits
typedef __attribute__((address_space(1))) uint32_t gu32;

__device__ __forceinline__ uint32_t dz_scan_excl(uint32_t v, uint32_t *s_tmp, uint32_t *total) {
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  uint32_t x = v;
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  if (lane == WAVE - 1) s_tmp[wv] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (uint32_t k = 0; k < DZ_T / WAVE; k++) {
    const uint32_t y = s_tmp[k];
    before += k < wv ? y : 0u;
    all += y;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

__device__ __forceinline__ uint32_t dz_tok_bits(uint32_t tk, const uint32_t *cl, const uint32_t *cd, uint32_t *v0,
                                                uint32_t *n0, uint32_t *v1, uint32_t *n1, bool d64) {
  // returns total bits; emits as up to two (value, bits) pieces of <= 32 bits
  if ((tk >> 16) == 0) {
    const uint32_t c = cl[tk & 0xffu];
    *v0 = c & 0xffffu;
    *n0 = c >> 16;
    *v1 = 0;
    *n1 = 0;
    return *n0;
  }
  uint32_t lx, lv, dx, dv;
  const uint32_t ls = dz_len_sym((tk >> 16) + 2u, &lx, &lv, d64);
  const uint32_t ds = dz_dist_sym((tk & 0xffffu) + 1u, &dx, &dv);
  const uint32_t c1 = cl[257 + ls], c2 = cd[ds];
  const uint32_t b1 = c1 >> 16, b2 = c2 >> 16;
  *v0 = (c1 & 0xffffu) | (lv << b1);  // <= 15 + 16 bits
  *n0 = b1 + lx;
  *v1 = (c2 & 0xffffu) | (dv << b2);  // <= 15 + 14 bits
  *n1 = b2 + dx;
  return *n0 + *n1;
}

__device__ __forceinline__ void dz_put_ring(uint32_t *ring, uint32_t bit, uint32_t v, uint32_t nb) {  // nb <= 32
  if (!nb) return;
  const uint64_t x = (uint64_t)(v & (nb == 32 ? 0xffffffffu : ((1u << nb) - 1u))) << (bit & 31);
  const uint32_t w = bit >> 5;
  atomicOr(&ring[w & (DZ_RING - 1)], (uint32_t)x);
  if ((bit & 31) + nb > 32) atomicOr(&ring[(w + 1) & (DZ_RING - 1)], (uint32_t)(x >> 32));
}

// D3a: histograms
__global__ void __launch_bounds__(DZ_T) zs_dz_hist_kernel(const ZsDJobDev *__restrict__ jobs, const ZsDSegDev *__restrict__ segs,
                                                           uint32_t nseg, const uint16_t *__restrict__ dist16,
                                                           const uint8_t *__restrict__ len8, const uint32_t *__restrict__ bm,
                                                           uint32_t *__restrict__ hist, const uint16_t *__restrict__ lx16) {
  __shared__ uint32_t fl[NL + 2], fd[ND + 2];
  __shared__ uint64_t s_red[16];
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.level == 0 || jb.exact) return;
  gcu8 *l8 = (gcu8 *)(len8 + sg.tok);
  const uint16_t *d16 = dist16 + sg.tok;
  gcu8 *in = (gcu8 *)(jb.in + sg.start);
  gcu32 *bS = (gcu32 *)(bm + (uint64_t)blockIdx.x * DZ_BMW);
  const uint32_t nch = (sg.len + 4095u) / 4096u;
  for (uint32_t i = t; i < NL + 2; i += DZ_T) fl[i] = 0;
  if (t < ND + 2) fd[t] = 0;
  __syncthreads();
  uint32_t xbits = 0, fix = 0;  // length/distance extra bits; fixed-code cost
  const bool d64 = jb.wbits == 16u;
  const uint16_t *x16 = d64 ? lx16 + sg.tok : nullptr;
  for (uint32_t c = 0; c < nch; c++) {
    DzTok16 k;
    k.x16 = x16;
    dz_load_tok16(k, bS, l8, d16, in, c * 4096u + 16u * t, sg.len);
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
      if (!((k.s16 >> i) & 1u)) continue;
      const uint32_t x = dz_tok16_at(k, i);
      if ((x >> 16) == 0) {
        atomicAdd(&fl[x], 1u);
        fix += x < 144u ? 8u : 9u;
      } else {
        uint32_t lx, lv, dx, dv;
        const uint32_t ls = dz_len_sym((x >> 16) + 2u, &lx, &lv, d64);
        atomicAdd(&fl[257 + ls], 1u);
        atomicAdd(&fd[dz_dist_sym((x & 0xffffu) + 1u, &dx, &dv)], 1u);
        xbits += lx + dx;
        fix += (257u + ls < 280u ? 7u : 8u) + lx + 5u + dx;
      }
    }
  }
  const uint64_t xs = zs_block_sum(xbits, s_red);
  const uint64_t fs = zs_block_sum(fix, s_red);
  gu32 *h = (gu32 *)hist + blockIdx.x;  // row r at h[r * nseg]
  for (uint32_t i = t; i < NL; i += DZ_T) h[(uint64_t)i * nseg] = i == 256 ? 1u : fl[i];  // one end-of-block
  if (t < ND) h[(uint64_t)(NL + t) * nseg] = fd[t];
  if (t == 0) {
    h[(uint64_t)DZ_ROW_XBITS * nseg] = (uint32_t)xs;
    h[(uint64_t)DZ_ROW_FIX * nseg] = (uint32_t)fs;
  }
}

// D3b: one thread per segment
struct DzRows {  // SoA rows of one segment
  gu32 *b;
  uint64_t stride;
  __device__ __forceinline__ gu32 &operator[](uint32_t r) const { return b[(uint64_t)r * stride]; }
};
#define DZS_KEY 0u
#define DZS_TMP 288u
#define DZS_W 576u
#define DZS_P 1152u
#define DZS_LEN 1728u  // lit/len 1728..2013, dist 2014..2045, code-length 2046..2064
#define DZS_RLE 2068u  // header symbols: sym | extra << 8

// Code lengths (1..maxbits, 0 = unused) of the n frequencies freq(i) into
// scratch rows LEN0 .. LEN0 + n: at least two symbols used (trees.c:610-620),
// leaves sorted by (freq, symbol), two-queue Huffman, depth limit by the
// bl_count adjustment (cf. gen_bitlen, trees.c:474-559), longest codes to the
// least frequent symbols.  cnt: 32 words of LDS.
template <typename F>
__device__ void dz_huff_lengths(const DzRows &S, F freq, uint32_t n, uint32_t maxbits, uint32_t len0, uint32_t *cnt) {
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t f = freq(i);
    S[len0 + i] = 0;
    if (f) S[DZS_KEY + m++] = (f << 9) | i;
  }
  for (uint32_t i = 0; m < 2 && i < n; i++)
    if (!freq(i)) S[DZS_KEY + m++] = (1u << 9) | i;
  // bottom-up merge sort of the keys (unique: the symbol is in the low bits)
  uint32_t src = DZS_KEY, dst = DZS_TMP;
  for (uint32_t w = 1; w < m; w <<= 1) {
    for (uint32_t lo = 0; lo < m; lo += 2 * w) {
      const uint32_t mid = min(lo + w, m), hi = min(lo + 2 * w, m);
      uint32_t i = lo, j = mid;
      uint32_t a = i < mid ? S[src + i] : 0xffffffffu, b = j < hi ? S[src + j] : 0xffffffffu;
      for (uint32_t k = lo; k < hi; k++) {
        if (a <= b) {
          S[dst + k] = a;
          i++;
          a = i < mid ? S[src + i] : 0xffffffffu;
        } else {
          S[dst + k] = b;
          j++;
          b = j < hi ? S[src + j] : 0xffffffffu;
        }
      }
    }
    const uint32_t x = src;
    src = dst;
    dst = x;
  }
  // two-queue Huffman: leaves 0..m-1 (sorted weights), internal nodes from m
  for (uint32_t i = 0; i < m; i++) S[DZS_W + i] = S[src + i] >> 9;
  uint32_t li = 0, ii = m, end = m;
  uint32_t wl = S[DZS_W], wi = 0;
  for (uint32_t k = 0; k + 1 < m; k++) {
    uint32_t x[2], wx[2];
    for (int q = 0; q < 2; q++) {
      if (li < m && (ii >= end || wl <= wi)) {
        x[q] = li;
        wx[q] = wl;
        li++;
        wl = li < m ? S[DZS_W + li] : 0u;
      } else {
        x[q] = ii;
        wx[q] = wi;
        ii++;
        wi = ii < end ? S[DZS_W + ii] : 0u;
      }
    }
    const uint32_t sum = wx[0] + wx[1];
    S[DZS_W + end] = sum;
    S[DZS_P + x[0]] = end;
    S[DZS_P + x[1]] = end;
    if (ii == end) wi = sum;
    end++;
  }
  // depths (parents have higher indices); W is reused for them
  const uint32_t root = end - 1;
  S[DZS_W + root] = 0;
  for (uint32_t x = root; x-- > 0;) S[DZS_W + x] = min(31u, S[DZS_W + S[DZS_P + x]] + 1u);
  for (uint32_t b = 0; b < 32; b++) cnt[b] = 0;
  uint32_t maxd = 0;
  for (uint32_t i = 0; i < m; i++) {
    const uint32_t d = S[DZS_W + i];
    cnt[d]++;
    maxd = max(maxd, d);
  }
  for (uint32_t i = maxd; i > maxbits; i--) {
    while (cnt[i] > 0) {
      uint32_t j = i - 2;
      while (cnt[j] == 0) j--;
      cnt[i] -= 2;
      cnt[i - 1] += 1;
      cnt[j + 1] += 2;
      cnt[j] -= 1;
    }
  }
  uint32_t k = 0;
  for (uint32_t b = min(maxd, maxbits); b >= 1; b--)
    for (uint32_t c = 0; c < cnt[b]; c++) S[len0 + (S[src + k++] & 511u)] = b;
}

// canonical codes (gen_codes, trees.c:205) of lengths len(i), bit-reversed for
// LSB-first output; put(i, code | len << 16).  bl: 16 words of LDS.
template <typename L, typename P>
__device__ void dz_canonical(L len, P put, uint32_t n, uint32_t *bl) {
  for (uint32_t b = 0; b < 16; b++) bl[b] = 0;
  for (uint32_t i = 0; i < n; i++) bl[len(i)]++;
  bl[0] = 0;
  uint32_t code = 0, prev = 0;
  for (uint32_t b = 1; b < 16; b++) {
    code = (code + prev) << 1;
    prev = bl[b];
    bl[b] = code;  // next code of length b
  }
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t l = len(i);
    if (!l) {
      put(i, 0u);
      continue;
    }
    const uint32_t cv = bl[l]++;
    put(i, (l << 16) | (__builtin_bitreverse32(cv) >> (32 - l)));
  }
}

struct DzBitW {  // LSB-first bit writer into global words
  gu32 *o;
  uint64_t acc;
  uint32_t n, w;
  __device__ __forceinline__ void put(uint32_t v, uint32_t nb) {
    acc |= (uint64_t)(v & ((1u << nb) - 1u)) << n;
    n += nb;
    if (n >= 32) {
      o[w++] = (uint32_t)acc;
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ __forceinline__ uint32_t flush() {
    const uint32_t bits = w * 32u + n;
    if (n) o[w] = (uint32_t)acc;
    return bits;
  }
};

__global__ void __launch_bounds__(WAVE) zs_dz_codes_kernel(const ZsDJobDev *__restrict__ jobs, const ZsDSegDev *__restrict__ segs,
                                                            uint32_t nseg, uint32_t *__restrict__ aux) {
  __shared__ uint32_t s_cnt[WAVE][32];
  __shared__ uint32_t s_bl[WAVE][16];
  __shared__ uint32_t s_fc[WAVE][20];
  __shared__ uint32_t s_cc[WAVE][20];
  const uint32_t s = blockIdx.x * WAVE + threadIdx.x;
  if (s >= nseg) return;
  const ZsDSegDev sg = segs[s];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.level == 0 || jb.exact) return;
  const uint32_t lane = threadIdx.x;
  gu32 *A = (gu32 *)aux;
  const DzRows H{A + s, nseg};                                              // histograms
  gu32 *C = A + (uint64_t)DZ_HROWS * nseg + (uint64_t)s * DZ_CROW;          // codes (AoS)
  gu32 *HB = A + (uint64_t)(DZ_HROWS + DZ_CROW) * nseg + (uint64_t)s * DZ_HDRW;  // header bits (AoS)
  const DzRows S{A + (uint64_t)(DZ_HROWS + DZ_CROW + DZ_HDRW) * nseg + s, nseg};  // scratch
  uint32_t *cnt = s_cnt[lane], *bl = s_bl[lane], *fc = s_fc[lane], *cc = s_cc[lane];
  dz_huff_lengths(S, [&](uint32_t i) -> uint32_t { return H[i]; }, NL, 15, DZS_LEN, cnt);
  dz_huff_lengths(S, [&](uint32_t i) -> uint32_t { return H[NL + i]; }, ND, 15, DZS_LEN + NL, cnt);
  // header: lengths RLE (scan_tree / send_tree, trees.c:682-766)
  uint32_t hlit = NL;
  while (hlit > 257 && S[DZS_LEN + hlit - 1] == 0) hlit--;
  uint32_t hdist = ND;
  while (hdist > 1 && S[DZS_LEN + NL + hdist - 1] == 0) hdist--;
  const uint32_t tot = hlit + hdist;
  auto lenat = [&](uint32_t i) -> uint32_t { return i < hlit ? S[DZS_LEN + i] : S[DZS_LEN + NL + (i - hlit)]; };
  for (uint32_t i = 0; i < 20; i++) fc[i] = 0;
  uint32_t nr = 0;
  for (uint32_t i = 0; i < tot;) {
    const uint32_t v = lenat(i);
    uint32_t r = 1;
    while (i + r < tot && r < 138 && lenat(i + r) == v) r++;
    if (v == 0 && r >= 3) {
      const uint32_t sym = r >= 11 ? 18u : 17u;
      S[DZS_RLE + nr++] = sym | ((r - (sym == 18 ? 11u : 3u)) << 8);
      fc[sym]++;
      i += r;
    } else if (v != 0 && r >= 4) {
      S[DZS_RLE + nr++] = v;
      fc[v]++;
      uint32_t rem = r - 1;
      i += 1;
      while (rem >= 3) {
        const uint32_t q = min(rem, 6u);
        S[DZS_RLE + nr++] = 16u | ((q - 3u) << 8);
        fc[16]++;
        rem -= q;
        i += q;
      }
    } else {
      S[DZS_RLE + nr++] = v;
      fc[v]++;
      i++;
    }
  }
  dz_huff_lengths(S, [&](uint32_t i) -> uint32_t { return fc[i]; }, NC, 7, DZS_LEN + NL + ND, cnt);
  dz_canonical([&](uint32_t i) -> uint32_t { return S[DZS_LEN + NL + ND + i]; }, [&](uint32_t i, uint32_t c) { cc[i] = c; },
               NC, bl);
  static constexpr uint8_t ordr[NC] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  uint32_t hclen = NC;
  while (hclen > 4 && (cc[ordr[hclen - 1]] >> 16) == 0) hclen--;
  uint32_t hb = 3 + 5 + 5 + 4 + 3 * hclen;
  for (uint32_t i = 0; i < nr; i++) {
    const uint32_t sym = S[DZS_RLE + i] & 0xffu;
    hb += (cc[sym] >> 16) + (sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u);
  }
  uint64_t dyn = (uint64_t)hb + H[DZ_ROW_XBITS];
  for (uint32_t i = 0; i < NL; i++) dyn += (uint64_t)H[i] * S[DZS_LEN + i];
  for (uint32_t i = 0; i < ND; i++) dyn += (uint64_t)H[NL + i] * S[DZS_LEN + NL + i];
  const uint64_t fix = 3ull + H[DZ_ROW_FIX] + 7ull;
  DzBitW bw{HB, 0, 0, 0};
  bw.put(sg.last ? 1u : 0u, 1);
  if (dyn < fix) {
    dz_canonical([&](uint32_t i) -> uint32_t { return S[DZS_LEN + i]; }, [&](uint32_t i, uint32_t c) { C[i] = c; }, NL, bl);
    dz_canonical([&](uint32_t i) -> uint32_t { return S[DZS_LEN + NL + i]; }, [&](uint32_t i, uint32_t c) { C[NL + i] = c; },
                 ND, bl);
    bw.put(2u, 2);
    bw.put(hlit - 257u, 5);
    bw.put(hdist - 1u, 5);
    bw.put(hclen - 4u, 4);
    for (uint32_t i = 0; i < hclen; i++) bw.put(cc[ordr[i]] >> 16, 3);
    for (uint32_t i = 0; i < nr; i++) {
      const uint32_t e = S[DZS_RLE + i];
      const uint32_t sym = e & 0xffu, c = cc[sym];
      bw.put(c & 0xffffu, c >> 16);
      const uint32_t xb = sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u;
      if (xb) bw.put(e >> 8, xb);
    }
  } else {
    // fixed codes (src/trees.c tr_static_init): lit 0-143 8 bits from 0x30,
    // 144-255 9 bits from 0x190, 256-279 7 bits from 0, 280-287 8 bits from
    // 0xc0; distances 5 bits
    for (uint32_t i = 0; i < NL; i++) {
      const uint32_t len = i < 144 ? 8u : i < 256 ? 9u : i < 280 ? 7u : 8u;
      const uint32_t code = i < 144 ? 0x30u + i : i < 256 ? 0x190u + (i - 144u) : i < 280 ? i - 256u : 0xc0u + (i - 280u);
      C[i] = (len << 16) | (__builtin_bitreverse32(code) >> (32 - len));
    }
    for (uint32_t i = 0; i < ND; i++) C[NL + i] = (5u << 16) | (__builtin_bitreverse32(i) >> 27);
    bw.put(1u, 2);
  }
  HB[DZ_HDRW - 1] = bw.flush();
}

// D3c: emission
__global__ void __launch_bounds__(DZ_T) zs_dz_emit_kernel(const ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                           uint32_t nseg, const uint16_t *__restrict__ dist16,
                                                           const uint8_t *__restrict__ len8, const uint32_t *__restrict__ bm,
                                                           const uint32_t *__restrict__ aux, uint32_t *__restrict__ obuf,
                                                           const uint16_t *__restrict__ lx16) {
  __shared__ uint32_t ring[DZ_RING];
  __shared__ uint32_t s_cl[NL + 2], s_cd[ND + 2];
  __shared__ uint32_t s_scan[DZ_T / WAVE + 1];
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.exact) return;  // zlib-identical jobs: deflate_zlib.hip
  uint32_t *gout = obuf + sg.obuf / 4;
  if (jb.level == 0) {
    // zlib's deflate_stored for one deflate(Z_FINISH) with room for the whole
    // output: stored blocks of MAX_STORED = 65535 bytes from the stream's
    // start (the last one shorter; an empty stream is one empty block), each
    // a byte-aligned 5-byte header + its bytes.  Blocks do not align with the
    // 64 KiB segments: a segment writes the tail of the block open at its start,
    // then a header + bytes for each block that starts inside it.
    const uint64_t S = sg.start, N = jb.in_len;
    const uint32_t n = sg.len;
    const uint8_t *in = jb.in + S;
    uint8_t *ob = reinterpret_cast<uint8_t *>(gout);
    const uint64_t k0 = (S + 65534u) / 65535u;  // first block starting at or after S
    const uint64_t kend = N ? (S + n + 65534u) / 65535u : 1u;  // blocks starting before S + n (an empty stream: block 0)
    const uint32_t nst = (uint32_t)(kend > k0 ? kend - k0 : 0u);
    const uint32_t lead = (uint32_t)min<uint64_t>(n, k0 * 65535u - S);  // tail of the block open at S
    for (uint32_t i = t; i < lead; i += DZ_T) ob[i] = in[i];
    for (uint32_t j = 0; j < nst; j++) {
      const uint64_t bs = (k0 + j) * 65535u;  // block start (stream position)
      const uint32_t bl = (uint32_t)min<uint64_t>(65535u, N - bs);
      const uint32_t seg_bl = (uint32_t)min<uint64_t>(bl, S + n - bs);  // its bytes inside this segment
      uint8_t *hp = ob + (bs - S) + 5u * j;
      if (t == 0) {
        hp[0] = (uint8_t)((jb.term == ZS_DT_FINAL && bs + bl == N) ? 1u : 0u);  // the final block may start a segment early
        hp[1] = (uint8_t)bl;
        hp[2] = (uint8_t)(bl >> 8);
        hp[3] = (uint8_t)~bl;
        hp[4] = (uint8_t)(~bl >> 8);
      }
      for (uint32_t i = t; i < seg_bl; i += DZ_T) hp[5 + i] = in[bs - S + i];
    }
    if (t == 0) segs[blockIdx.x].nbits = 8u * (n + 5u * nst);
    return;
  }
  const uint32_t *C = aux + (uint64_t)DZ_HROWS * nseg + (uint64_t)blockIdx.x * DZ_CROW;
  const uint32_t *HB = aux + (uint64_t)(DZ_HROWS + DZ_CROW) * nseg + (uint64_t)blockIdx.x * DZ_HDRW;
  const uint32_t hbits = HB[DZ_HDRW - 1];
  for (uint32_t i = t; i < NL; i += DZ_T) s_cl[i] = C[i];
  if (t < ND) s_cd[t] = C[NL + t];
  for (uint32_t i = t; i < DZ_RING; i += DZ_T) ring[i] = i < (hbits + 31u) / 32u ? HB[i] : 0u;
  __syncthreads();
  gcu8 *l8 = (gcu8 *)(len8 + sg.tok);
  const uint16_t *d16 = dist16 + sg.tok;
  gcu8 *in = (gcu8 *)(jb.in + sg.start);
  gcu32 *bS = (gcu32 *)(bm + (uint64_t)blockIdx.x * DZ_BMW);
  const uint32_t nch = (sg.len + 4095u) / 4096u;
  uint32_t base = hbits, flushed = 0;  // bits emitted; words written to gout
  const bool d64 = jb.wbits == 16u;
  const uint16_t *x16 = d64 ? lx16 + sg.tok : nullptr;
  for (uint32_t c = 0; c < nch; c++) {
    DzTok16 k;
    k.x16 = x16;
    dz_load_tok16(k, bS, l8, d16, in, c * 4096u + 16u * t, sg.len);
    uint32_t nb = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
      if (!((k.s16 >> i) & 1u)) continue;
      uint32_t v0, n0, v1, n1;
      nb += dz_tok_bits(dz_tok16_at(k, i), s_cl, s_cd, &v0, &n0, &v1, &n1, d64);
    }
    uint32_t all;
    uint32_t off = dz_scan_excl(nb, s_scan, &all) + base;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
      if (!((k.s16 >> i) & 1u)) continue;
      uint32_t v0, n0, v1, n1;
      dz_tok_bits(dz_tok16_at(k, i), s_cl, s_cd, &v0, &n0, &v1, &n1, d64);
      dz_put_ring(ring, off, v0, n0);
      dz_put_ring(ring, off + n0, v1, n1);
      off += n0 + n1;
    }
    base += all;
    __syncthreads();
    const uint32_t full = base >> 5;  // words complete after this chunk
    for (uint32_t w = flushed + t; w < full; w += DZ_T) {
      gout[w] = ring[w & (DZ_RING - 1)];
      ring[w & (DZ_RING - 1)] = 0;
    }
    flushed = full;
    __syncthreads();
  }
  if (t == 0) {
    const uint32_t e = s_cl[256];
    dz_put_ring(ring, base, e & 0xffffu, e >> 16);
    segs[blockIdx.x].nbits = base + (e >> 16);
  }
  __syncthreads();
  const uint32_t endw = (base + (s_cl[256] >> 16) + 31u) >> 5;
  for (uint32_t w = flushed + t; w < endw; w += DZ_T) gout[w] = ring[w & (DZ_RING - 1)];
}

// ---------------------------------------------------------------------------
// D4: checksums of the input (zs_check.h: every segment adds its contribution
// to the job's accumulators, in any order) and per-job bit offsets
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(DZ_T) zs_dz_check_kernel(ZsDJobDev *__restrict__ jobs, const ZsDSegDev *__restrict__ segs) {
  __shared__ uint32_t s_tab[4][256];
  __shared__ ZsCkTabs s_ck;
  __shared__ uint64_t s_red[16];
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  // the check covers in[ck0, in_len): the bytes before ck0 are history the
  // check of an earlier segment of the stream already took
  const uint8_t *in = jb.in + jb.ck0;
  const uint64_t n = jb.in_len - jb.ck0;
  const uint64_t s_lo = max(sg.start, jb.ck0) - jb.ck0, s_hi = sg.start + sg.len;
  if (jb.wrap == 0 || s_hi <= jb.ck0) return;
  const uint64_t s_len = s_hi - jb.ck0 - s_lo;
  if ((reinterpret_cast<uintptr_t>(in + s_lo) & 15u) == 0) {  // coalesced 4 KiB steps (zs_check.h)
    static_assert(DZ_T == ZS_CK_T, "zs_check.h block checks run 256 threads");
    zs_ck_tables(s_ck);
    if (jb.wrap == 2) {
      const uint32_t v = zs_crc_block(in, s_lo, s_lo + s_len, n, s_ck, reinterpret_cast<uint32_t *>(s_red));
      if (t == 0 && v) atomicXor(reinterpret_cast<unsigned long long *>(&jobs[sg.job].ck_a), (unsigned long long)v);
    } else {
      uint64_t sa, sb;
      zs_adler_block(in, s_lo, s_lo + s_len, n, s_red, &sa, &sb);
      if (t == 0) {
        atomicAdd(reinterpret_cast<unsigned long long *>(&jobs[sg.job].ck_a), (unsigned long long)sa);
        atomicAdd(reinterpret_cast<unsigned long long *>(&jobs[sg.job].ck_b), (unsigned long long)sb);
      }
    }
    return;
  }
  const uint64_t per = ((s_len + DZ_T - 1) / DZ_T + 3u) & ~3ull;
  const uint64_t lo = s_lo + min(s_len, per * t), hi = s_lo + min(s_len, per * (t + 1));
  if (jb.wrap == 2) {
    zs_crc_tables(s_tab);
    const uint32_t v = zs_block_xor(zs_crc_piece(in, lo, hi, n, s_tab), reinterpret_cast<uint32_t *>(s_red));
    if (t == 0 && v) atomicXor(reinterpret_cast<unsigned long long *>(&jobs[sg.job].ck_a), (unsigned long long)v);
  } else {
    uint32_t A = 0, B = 0;
    if (hi > lo) zs_adler_piece(in, lo, hi, n, &A, &B);
    const uint64_t sa = zs_block_sum(A, s_red);
    const uint64_t sb = zs_block_sum(B, s_red);
    if (t == 0) {
      atomicAdd(reinterpret_cast<unsigned long long *>(&jobs[sg.job].ck_a), (unsigned long long)sa);
      atomicAdd(reinterpret_cast<unsigned long long *>(&jobs[sg.job].ck_b), (unsigned long long)sb);
    }
  }
}

// per job (one workgroup): segment bit offsets, combined checksum, header and
// trailer sizes -> job total bytes; writes the wrapper header into the staging
#define DZ_JT 1024u
__global__ void __launch_bounds__(DZ_JT) zs_dz_offsets_kernel(ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                               uint8_t *__restrict__ stage) {
  __shared__ uint64_t s_sum[DZ_JT];
  const uint32_t t = threadIdx.x;
  ZsDJobDev jb = jobs[blockIdx.x];
  if (jb.exact) return;  // zs_zd_layout_kernel
  const uint32_t hdr = !jb.hdr ? 0u : jb.wrap == 2 ? 10u : (jb.wrap == 1 ? 2u : 0u);
  // segment k of the job: jb.seg0 + k; per-thread contiguous ranges
  const uint32_t ns = jb.nseg;
  const uint32_t per = (ns + DZ_JT - 1) / DZ_JT;
  const uint32_t k0 = min(ns, per * t), k1 = min(ns, per * (t + 1));
  uint64_t sum = 0;
  for (uint32_t k = k0; k < k1; k++) sum += segs[jb.seg0 + k].nbits;
  s_sum[t] = sum;
  __syncthreads();
  if (t == 0) {  // small serial exclusive scan over 1024 partial sums
    uint64_t acc = jb.bit0 + 8ull * hdr;
    for (uint32_t k = 0; k < DZ_JT; k++) {
      const uint64_t x = s_sum[k];
      s_sum[k] = acc;
      acc += x;
    }
    jobs[blockIdx.x].endbit = acc;
    jobs[blockIdx.x].total_out = zs_dz_total_bytes(jb, acc);
  }
  __syncthreads();
  uint64_t off = s_sum[t];
  for (uint32_t k = k0; k < k1; k++) {
    segs[jb.seg0 + k].bitoff = off;
    off += segs[jb.seg0 + k].nbits;
  }
  if (t == 0)
    jobs[blockIdx.x].check = jb.wrap == 2   ? zs_crc_final((uint32_t)jb.ck_a, jb.in_len - jb.ck0)
                             : jb.wrap == 1 ? zs_adler_final(jb.ck_a, jb.ck_b, jb.in_len - jb.ck0)
                                            : 0u;
  if (t == 0 && hdr) {
    uint8_t *o = stage + jb.stage;
    if (jb.wrap == 2) {  // gzip header as zlib writes it with no options (mtime 0, OS 3)
      const uint8_t gz[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, (uint8_t)(jb.level == 9 ? 2 : (jb.level < 2 ? 4 : 0)), 3};
      for (int i = 0; i < 10; i++) o[i] = gz[i];
    } else if (jb.wrap == 1) {  // CMF/FLG with FLEVEL as deflate.c sets it, FCHECK % 31
      const uint32_t flevel = jb.level < 2 ? 0u : (jb.level < 6 ? 1u : (jb.level == 6 ? 2u : 3u));
      uint32_t h = ((((jb.wbits - 8u) << 4) | 8u) << 8) | (flevel << 6);
      h += 31u - (h % 31u);
      o[0] = (uint8_t)(h >> 8);
      o[1] = (uint8_t)h;
    }
  }
}

// shift each segment's block bits to its stream offset (masked at the block's
// last bit); the staging area is zeroed; the first and last
// destination words may be shared with the neighbouring blocks (or the
// wrapper header): atomicOr; interior words are this block's alone.
__global__ void __launch_bounds__(DZ_T) zs_dz_stitch_kernel(const ZsDJobDev *__restrict__ jobs, const ZsDSegDev *__restrict__ segs,
                                                             const uint32_t *__restrict__ obuf, uint8_t *__restrict__ stage) {
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  const uint32_t nbits = sg.nbits;
  if (nbits == 0 || jb.exact) return;
  uint32_t *dst = reinterpret_cast<uint32_t *>(stage + jb.stage);  // 4 KiB aligned
  const uint32_t *src = obuf + sg.obuf / 4;
  const uint64_t off = sg.bitoff;
  const uint32_t sh = (uint32_t)(off & 31u);
  const uint64_t d0 = off >> 5;
  const uint32_t last = (uint32_t)(((off + nbits - 1) >> 5) - d0);  // last destination word (relative)
  const uint32_t nw = (nbits + 31u) / 32u;
  const uint32_t tailm = (nbits & 31u) ? ((1u << (nbits & 31u)) - 1u) : 0xffffffffu;  // bits past the block are not zero for stored blocks
  auto word = [&](uint32_t i) -> uint32_t { return i < nw ? (i + 1 == nw ? src[i] & tailm : src[i]) : 0u; };
  for (uint32_t i = t; i <= last; i += DZ_T) {
    const uint32_t a = word(i);
    const uint32_t b = (i > 0 && sh) ? word(i - 1) : 0u;
    const uint32_t v = (a << sh) | (sh ? (b >> (32u - sh)) : 0u);
    if (i == 0 || i == last) {
      if (v) atomicOr(&dst[d0 + i], v);
    } else {
      dst[d0 + i] = v;
    }
  }
}

// trailer (after all stitching): CRC-32 + ISIZE (gzip) or Adler-32 big-endian (zlib)
__global__ void zs_dz_trailer_kernel(const ZsDJobDev *__restrict__ jobs, uint32_t njobs, uint8_t *__restrict__ stage,
                                     uint32_t exact) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  const ZsDJobDev jb = jobs[j];
  if ((jb.exact != 0) != (exact != 0)) return;
  uint8_t *o = stage + jb.stage;
  if (jb.term == ZS_DT_SYNC) {  // the empty stored block's LEN / NLEN (its header bits and padding are zero)
    uint8_t *p = o + jb.total_out - 4;
    p[0] = 0;
    p[1] = 0;
    p[2] = 0xff;
    p[3] = 0xff;
    return;
  }
  if (jb.term == ZS_DT_PARTIAL) {  // trees.c _tr_align: BFINAL 0, BTYPE 01, static END_BLOCK (7 zero bits)
    const uint64_t b = jb.endbit + 1;
    o[b >> 3] |= (uint8_t)(1u << (b & 7u));
    return;
  }
  if (jb.term != ZS_DT_FINAL || !jb.trl) return;
  const uint64_t tr = jb.wrap == 2 ? 8u : (jb.wrap == 1 ? 4u : 0u);
  uint8_t *p = o + jb.total_out - tr;
  if (jb.wrap == 2) {
    const uint32_t c = jb.check, n = (uint32_t)(jb.in_len - jb.ck0);
    p[0] = (uint8_t)c;
    p[1] = (uint8_t)(c >> 8);
    p[2] = (uint8_t)(c >> 16);
    p[3] = (uint8_t)(c >> 24);
    p[4] = (uint8_t)n;
    p[5] = (uint8_t)(n >> 8);
    p[6] = (uint8_t)(n >> 16);
    p[7] = (uint8_t)(n >> 24);
  } else if (jb.wrap == 1) {
    const uint32_t c = jb.check;
    p[0] = (uint8_t)(c >> 24);
    p[1] = (uint8_t)(c >> 16);
    p[2] = (uint8_t)(c >> 8);
    p[3] = (uint8_t)c;
  }
}

// ---------------------------------------------------------------------------
// Level-0 stream calls (zs_capi.cpp ds_stored_call).  zlib's deflate_stored
// sizes every stored block from the call's avail_out, flush and window
// (deflate.c, 1.2.11); the host replays that arithmetic and hands the call's
// output as copy pieces of the staged source [pieces | unframed window bytes |
// new input | header / marker bytes].  A workgroup per 16 KiB of output writes
// it; the last workgroup computes the check of the new input (zs_check.h).
// ---------------------------------------------------------------------------
#define ZS_SC_TILE 16384u
__global__ void __launch_bounds__(DZ_T) zs_stored_call_kernel(const uint8_t *__restrict__ src,
                                                              const ZsPiece *__restrict__ pc, uint32_t np, uint64_t total,
                                                              uint8_t *__restrict__ dst, uint64_t ck_lo, uint64_t ck_hi,
                                                              uint32_t wrap, uint32_t *__restrict__ res) {
  __shared__ ZsCkTabs s_ck;
  __shared__ uint32_t s_red32[16];
  __shared__ uint64_t s_red[16];
  const uint32_t t = threadIdx.x;
  const uint64_t ntile = (total + ZS_SC_TILE - 1) / ZS_SC_TILE;
  if (blockIdx.x < ntile) {
    const uint64_t lo = (uint64_t)blockIdx.x * ZS_SC_TILE, hi = min(total, lo + ZS_SC_TILE);
    uint32_t a = 0, b = np;  // the last piece starting at or before lo
    while (b - a > 1) {
      const uint32_t m = (a + b) / 2;
      if (pc[m].dst <= lo) a = m;
      else b = m;
    }
    for (uint32_t k = a; k < np && pc[k].dst < hi; k++) {
      const ZsPiece q = pc[k];
      const uint64_t s0 = max(lo, q.dst), e = min(hi, q.dst + q.len);
      for (uint64_t i = s0 + t; i < e; i += DZ_T) dst[i] = src[q.src + (i - q.dst)];
    }
    return;
  }
  const uint64_t n = ck_hi > ck_lo ? ck_hi - ck_lo : 0u;
  if (wrap == 2) {
    zs_ck_tables(s_ck);
    const uint32_t acc = zs_crc_block(src + ck_lo, 0, n, n, s_ck, s_red32);
    if (t == 0) res[0] = zs_crc_final(acc, n);
  } else if (wrap == 1) {
    uint64_t A, B;
    zs_adler_block(src + ck_lo, 0, n, n, s_red, &A, &B);
    if (t == 0) res[0] = zs_adler_final(A, B, n);
  } else if (t == 0) {
    res[0] = 1u;
  }
}

extern "C" void zs_launch_stored_call(const uint8_t *d_src, const ZsPiece *d_pc, uint32_t np, uint64_t total,
                                      uint8_t *d_dst, uint64_t ck_lo, uint64_t ck_hi, uint32_t wrap, uint32_t *d_res,
                                      hipStream_t st) {
  const uint64_t ntile = (total + ZS_SC_TILE - 1) / ZS_SC_TILE;
  hipLaunchKernelGGL(zs_stored_call_kernel, dim3((uint32_t)ntile + 1u), dim3(DZ_T), 0, st, d_src, d_pc, np, total, d_dst,
                     ck_lo, ck_hi, wrap, d_res);
}

// ---------------------------------------------------------------------------
// launcher
// ---------------------------------------------------------------------------
// per segment: d_dist16 / d_len8 DZ_SEG entries, d_bm DZ_BMW bitmap words, d_aux DZ_AUXW words
// d_lx16: DZ_SEG u16 per segment when the batch has deflate64 jobs (has_d64), else unused
extern "C" void zs_launch_deflate(ZsDJobDev *d_jobs, uint32_t njobs, ZsDSegDev *d_segs, uint32_t nseg, uint16_t *d_dist16,
                                  uint8_t *d_len8, uint32_t *d_bm, uint32_t *d_aux, uint32_t *d_obuf, uint8_t *d_stage,
                                  uint16_t *d_lx16, int has_std, int has_d64, hipStream_t st, hipEvent_t *ev) {
  if (ev) (void)hipEventRecord(ev[0], st);
  if (has_std)
    hipLaunchKernelGGL(zs_dz_match_kernel<false>, dim3(2 * nseg), dim3(DZ_MT), 0, st, d_jobs, d_segs, d_dist16, d_len8);
  if (has_d64)
    hipLaunchKernelGGL(zs_dz_match_kernel<true>, dim3(4 * nseg), dim3(DZ_MT), 0, st, d_jobs, d_segs, d_dist16, d_len8);
  if (ev) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(zs_dz_parse_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs, d_len8, d_bm);
  if (has_d64) hipLaunchKernelGGL(zs_dz_merge_kernel, dim3(nseg), dim3(64), 0, st, d_jobs, d_segs, d_dist16, d_len8, d_bm, d_lx16);
  if (ev) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(zs_dz_hist_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs, nseg, d_dist16, d_len8, d_bm, d_aux,
                     d_lx16);
  hipLaunchKernelGGL(zs_dz_codes_kernel, dim3((nseg + WAVE - 1) / WAVE), dim3(WAVE), 0, st, d_jobs, d_segs, nseg, d_aux);
  hipLaunchKernelGGL(zs_dz_emit_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs, nseg, d_dist16, d_len8, d_bm, d_aux,
                     d_obuf, d_lx16);
  hipLaunchKernelGGL(zs_dz_check_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs);
  if (ev) (void)hipEventRecord(ev[3], st);
  hipLaunchKernelGGL(zs_dz_offsets_kernel, dim3(njobs), dim3(DZ_JT), 0, st, d_jobs, d_segs, d_stage);
  hipLaunchKernelGGL(zs_dz_stitch_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs, d_obuf, d_stage);
  hipLaunchKernelGGL(zs_dz_trailer_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, d_jobs, njobs, d_stage, 0u);
  if (ev) (void)hipEventRecord(ev[4], st);
}

// trailers of the zlib-identical jobs, after their layout
extern "C" void zs_launch_dz_trailer(ZsDJobDev *d_jobs, uint32_t njobs, uint8_t *d_stage, hipStream_t st) {
  hipLaunchKernelGGL(zs_dz_trailer_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, d_jobs, njobs, d_stage, 1u);
}

// block-kernel counters of the profiling build (merged into zs_kprof_read's 26..37)
extern "C" int zs_kprof_read_dz(uint64_t *out12, int reset) {
#if KP_ON
  if (hipMemcpyFromSymbol(out12, HIP_SYMBOL(g_kprof_dz), 12 * sizeof(uint64_t)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[12] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_kprof_dz), z, sizeof z) != hipSuccess) return -1;
  }
  return 12;
#else
  (void)out12;
  (void)reset;
  return 0;
#endif
}
