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
__device__ __forceinline__ uint32_t dz_len_sym(uint32_t len, uint32_t *xb, uint32_t *xv) {
  const uint32_t l = len - 3u;
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
__global__ void __launch_bounds__(DZ_T) zs_dz_match_kernel(const ZsDJobDev *__restrict__ jobs,
                                                            const ZsDSegDev *__restrict__ segs,
                                                            uint32_t *__restrict__ matches) {
  __shared__ uint16_t tab[DZ_HB][DZ_WAYS];
  const uint32_t tid = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.level == 0) return;  // stored blocks: no matches
  gcu8 *in = (gcu8 *)jb.in;
  const uint64_t n = jb.in_len;
  const uint64_t s = sg.start, e = s + sg.len;
  uint32_t *mo = matches + sg.tok;
  for (uint32_t i = tid; i < DZ_HB * DZ_WAYS / 2; i += DZ_T) reinterpret_cast<uint32_t *>(tab)[i] = 0xffffffffu;
  __syncthreads();
  // Way w of a bucket belongs to wave w: the waves of a step never store to
  // the same slot, and within one store instruction the higher lane (the later
  // position) lands last, so the table -- and the output -- is deterministic.
  const uint32_t way = tid / WAVE;
  // prime with the window before the segment
  const uint64_t hs = s > DZ_WIN ? s - DZ_WIN : 0;
  for (uint64_t P = hs; P < s; P += DZ_T) {
    const uint64_t p = P + tid;
    if (p < s && p + 4 <= n) tab[dz_hash(dz_load32(in + p))][way] = (uint16_t)p;
  }
  __syncthreads();
  const uint32_t maxd = 1u << jb.wbits;
  for (uint64_t P = s; P < e; P += DZ_T) {
    const uint64_t p = P + tid;
    uint32_t h = 0;
    uint32_t best = 0, bd = 0;
    if (p < e && p + 4 <= n) {
      const uint32_t lim = (uint32_t)min<uint64_t>(258u, e - p);
      if (p + 16 <= n) {
        // 16-byte compares: one load round for the common (short) match
        const uint4 cur = dz_load128(in + p);
        h = dz_hash(cur.x);
        const uint2 ent = *reinterpret_cast<const uint2 *>(&tab[h][0]);
        const uint32_t c4[4] = {ent.x & 0xffffu, ent.x >> 16, ent.y & 0xffffu, ent.y >> 16};
        uint32_t dd[4];
        uint4 cv[4];
#pragma unroll
        for (uint32_t w = 0; w < DZ_WAYS; w++) {
          const uint32_t d = ((uint32_t)p - c4[w]) & 0xffffu;
          dd[w] = (c4[w] == 0xffffu || d == 0 || d > maxd || d > p) ? 0u : d;
          if (dd[w]) cv[w] = dz_load128(in + (p - dd[w]));
        }
#pragma unroll
        for (uint32_t w = 0; w < DZ_WAYS; w++) {
          if (!dd[w]) continue;
          uint32_t L = dz_eq16(cv[w], cur);
          if (L < 4u) continue;
          if (L == 16u) {
            gcu8 *q = in + (p - dd[w]);
            while (L + 16u <= lim) {
              const uint32_t k = dz_eq16(dz_load128(q + L), dz_load128(in + p + L));
              L += k;
              if (k < 16u) break;
            }
            if (L + 16u > lim)
              while (L < lim && q[L] == in[p + L]) L++;
          }
          L = min(L, lim);
          if (L > best || (L == best && dd[w] < bd)) {
            best = L;
            bd = dd[w];
          }
        }
      } else {  // the last 15 bytes of the input: byte compares
        const uint32_t v = dz_load32(in + p);
        h = dz_hash(v);
#pragma unroll
        for (uint32_t w = 0; w < DZ_WAYS; w++) {
          const uint32_t c16 = tab[h][w];
          if (c16 == 0xffffu) continue;
          const uint32_t d = ((uint32_t)p - c16) & 0xffffu;
          if (d == 0 || d > maxd || d > p) continue;
          gcu8 *q = in + (p - d);
          uint32_t L = 0;
          while (L < lim && q[L] == in[p + L]) L++;
          if (L < 4u) continue;
          if (L > best || (L == best && d < bd)) {
            best = L;
            bd = d;
          }
        }
      }
    }
    if (p < e) mo[p - s] = best >= 3u ? ((best << 16) | (bd - 1u)) : 0u;
    __syncthreads();  // every lookup of the step before its inserts
    if (p < e && p + 4 <= n) tab[h][way] = (uint16_t)p;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// D2: lazy parse (one lane per segment), tokens written over the matches
// (zlib deflate_slow semantics: a match is deferred by one byte when the next
// position has a longer one and the current is shorter than max_lazy)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) zs_dz_parse_kernel(const ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                          uint32_t nseg, uint32_t *__restrict__ matches) {
  const uint32_t c = blockIdx.x * 64u + threadIdx.x;
  if (c >= nseg) return;
  const ZsDSegDev sg = segs[c];
  const ZsDJobDev jb = jobs[sg.job];
  uint32_t *m = matches + sg.tok;
  const uint8_t *in = jb.in + sg.start;
  const uint32_t len = sg.len;
  uint32_t nt = 0;
  if (jb.level == 0) {
    segs[c].ntok = 0;
    return;
  }
  const uint32_t max_lazy = jb.level >= 4 ? 16u : 0u;
  uint32_t p = 0;
  uint32_t cur = len ? m[0] : 0u;
  while (p < len) {
    const uint32_t nxt = p + 1 < len ? m[p + 1] : 0u;
    const uint32_t L = cur >> 16;
    if (L >= 3u && !(L < max_lazy && (nxt >> 16) > L)) {
      m[nt++] = cur;
      p += L;
      cur = p < len ? m[p] : 0u;
    } else {
      m[nt++] = in[p];
      p++;
      cur = nxt;
    }
  }
  segs[c].ntok = nt;
}

// ---------------------------------------------------------------------------
// D3: Huffman codes + block emission (one workgroup per segment)
// ---------------------------------------------------------------------------
#define NL 286
#define ND 30
#define NC 19

struct DzLDS {
  union {
    uint32_t out[DZ_OUTW];     // block bits (LSB-first), atomicOr-packed (zeroed after the code builds)
    struct {                   // code-build scratch, dead before out is used
      uint16_t order[NL + 2];  // symbols by (freq, symbol)
      uint32_t w[2 * (NL + 2)];
      uint16_t par[2 * (NL + 2)];
      uint8_t depth[2 * (NL + 2)];
    };
  };
  uint32_t fl[NL + 2], fd[ND + 2], fc[NC + 1];
  uint32_t cl[NL + 2], cd[ND + 2], cc[NC + 1];  // code | len << 16 (code bit-reversed)
  uint8_t lens[NL + ND + 4]; // concatenated lit + dist lengths for the header
  uint16_t rle[NL + ND + 4]; // header symbols: sym | extra << 8
  uint32_t scan[DZ_T / WAVE + 1];
  uint32_t misc[16];
};

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

// Length-limited Huffman code lengths for freq[0..n) (every used symbol gets a
// length 1..maxbits; at least two symbols are forced used, as trees.c:610-620
// does, so every code is complete), then canonical codes (gen_codes,
// trees.c:205) bit-reversed for LSB-first output.  Whole workgroup.
__device__ void dz_build_code(DzLDS &L, uint32_t *freq, uint32_t n, uint32_t maxbits, uint32_t *codes) {
  const uint32_t t = threadIdx.x;
  if (t == 0) {
    uint32_t used = 0;
    for (uint32_t i = 0; i < n; i++) used += freq[i] != 0;
    for (uint32_t i = 0; used < 2 && i < n; i++)
      if (freq[i] == 0) {
        freq[i] = 1;
        used++;
      }
  }
  __syncthreads();
  // rank sort of the used symbols by (freq, symbol)
  uint32_t nu = 0;
  for (uint32_t i = 0; i < n; i++) nu += freq[i] != 0;
  for (uint32_t i = t; i < n; i += DZ_T) {
    const uint32_t f = freq[i];
    if (!f) continue;
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t g = freq[j];
      r += (g != 0) && (g < f || (g == f && j < i));
    }
    L.order[r] = (uint16_t)i;
  }
  __syncthreads();
  if (t == 0) {
    // two-queue Huffman: leaves 0..nu-1 (sorted), internal nodes nu.. in order
    for (uint32_t i = 0; i < nu; i++) L.w[i] = freq[L.order[i]];
    uint32_t li = 0, ii = nu, in_end = nu;
    for (uint32_t k = 0; k + 1 < nu; k++) {
      uint32_t a, b;
      for (int pick = 0; pick < 2; pick++) {
        uint32_t x;
        if (li < nu && (ii >= in_end || L.w[li] <= L.w[ii])) x = li++;
        else x = ii++;
        if (pick == 0) a = x;
        else b = x;
      }
      L.w[in_end] = L.w[a] + L.w[b];
      L.par[a] = (uint16_t)in_end;
      L.par[b] = (uint16_t)in_end;
      in_end++;
    }
    // depths: root = in_end - 1
    const uint32_t root = in_end - 1;
    L.depth[root] = 0;
    for (int x = (int)root - 1; x >= 0; x--) L.depth[x] = (uint8_t)min(255u, L.depth[L.par[x]] + 1u);
    uint32_t count[32];
    for (int b = 0; b < 32; b++) count[b] = 0;
    uint32_t maxd = 0;
    for (uint32_t i = 0; i < nu; i++) {
      const uint32_t d = min(31u, (uint32_t)L.depth[i]);
      count[d]++;
      maxd = max(maxd, d);
    }
    // limit to maxbits (bl_count adjustment; cf. gen_bitlen overflow, trees.c:474-559)
    for (uint32_t i = maxd; i > maxbits; i--) {
      while (count[i] > 0) {
        uint32_t j = i - 2;
        while (count[j] == 0) j--;
        count[i] -= 2;
        count[i - 1] += 1;
        count[j + 1] += 2;
        count[j] -= 1;
      }
    }
    // least frequent symbols get the longest codes
    uint32_t k = 0;
    for (uint32_t b = min(maxd, maxbits); b >= 1; b--)
      for (uint32_t c = 0; c < count[b]; c++) codes[L.order[k++]] = b << 16;
    for (uint32_t i = 0; i < n; i++)
      if (freq[i] == 0) codes[i] = 0;
    // canonical codes
    uint32_t bl[16];
    for (int b = 0; b < 16; b++) bl[b] = 0;
    for (uint32_t i = 0; i < n; i++) bl[codes[i] >> 16]++;
    bl[0] = 0;
    uint32_t nextc[16], code = 0;
    for (int b = 1; b < 16; b++) {
      code = (code + bl[b - 1]) << 1;
      nextc[b] = code;
    }
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t len = codes[i] >> 16;
      if (!len) continue;
      const uint32_t cv = nextc[len]++;
      codes[i] = (len << 16) | (__builtin_bitreverse32(cv) >> (32 - len));
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void dz_put(uint32_t *out, uint32_t bit, uint32_t v, uint32_t nb) {  // nb <= 32
  if (!nb) return;
  const uint64_t x = (uint64_t)(v & (nb == 32 ? 0xffffffffu : ((1u << nb) - 1u))) << (bit & 31);
  atomicOr(&out[bit >> 5], (uint32_t)x);
  if ((bit & 31) + nb > 32) atomicOr(&out[(bit >> 5) + 1], (uint32_t)(x >> 32));
}

__device__ __forceinline__ uint32_t dz_tok_bits(uint32_t tk, const uint32_t *cl, const uint32_t *cd, uint32_t *v0,
                                                uint32_t *n0, uint32_t *v1, uint32_t *n1) {
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
  const uint32_t ls = dz_len_sym(tk >> 16, &lx, &lv);
  const uint32_t ds = dz_dist_sym((tk & 0xffffu) + 1u, &dx, &dv);
  const uint32_t c1 = cl[257 + ls], c2 = cd[ds];
  const uint32_t b1 = c1 >> 16, b2 = c2 >> 16;
  *v0 = (c1 & 0xffffu) | (lv << b1);  // <= 15 + 5 bits
  *n0 = b1 + lx;
  *v1 = (c2 & 0xffffu) | (dv << b2);  // <= 15 + 13 bits
  *n1 = b2 + dx;
  return *n0 + *n1;
}

__global__ void __launch_bounds__(DZ_T) zs_dz_block_kernel(const ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                            const uint32_t *__restrict__ tokens, uint32_t *__restrict__ obuf) {
  __shared__ DzLDS L;
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  const uint32_t *tk = tokens + sg.tok;
  const uint32_t nt = sg.ntok;
  uint32_t *gout = obuf + sg.obuf / 4;
  const uint32_t last = sg.last;
  if (jb.level == 0) {  // stored blocks of <= 65535 bytes, byte-aligned (every block is stored)
    const uint8_t *in = jb.in + sg.start;
    uint8_t *ob = reinterpret_cast<uint8_t *>(gout);
    const uint32_t n = sg.len;
    const uint32_t nblk = n ? (n + 65534u) / 65535u : 1u;
    for (uint32_t b = 0; b < nblk; b++) {
      const uint32_t off = b * 65535u, bl = min(65535u, n - off);
      uint8_t *hp = ob + off + 5u * b;
      if (t == 0) {
        hp[0] = (uint8_t)((last && b + 1 == nblk) ? 1u : 0u);
        hp[1] = (uint8_t)bl;
        hp[2] = (uint8_t)(bl >> 8);
        hp[3] = (uint8_t)~bl;
        hp[4] = (uint8_t)(~bl >> 8);
      }
      for (uint32_t i = t; i < bl; i += DZ_T) hp[5 + i] = in[off + i];
    }
    if (t == 0) segs[blockIdx.x].nbits = 8u * (n + 5u * nblk);
    return;
  }
  for (uint32_t i = t; i < NL + 2; i += DZ_T) L.fl[i] = 0;
  if (t < ND + 2) L.fd[t] = 0;
  if (t < NC + 1) L.fc[t] = 0;
  __syncthreads();
  for (uint32_t i = t; i < nt; i += DZ_T) {
    const uint32_t x = tk[i];
    if ((x >> 16) == 0) {
      atomicAdd(&L.fl[x & 0xffu], 1u);
    } else {
      uint32_t a, b;
      atomicAdd(&L.fl[257 + dz_len_sym(x >> 16, &a, &b)], 1u);
      atomicAdd(&L.fd[dz_dist_sym((x & 0xffffu) + 1u, &a, &b)], 1u);
    }
  }
  if (t == 0) L.fl[256] = 1;
  __syncthreads();
  // fixed-code cost (src/trees.c static_ltree / static_dtree) vs dynamic
  dz_build_code(L, L.fl, NL, 15, L.cl);
  dz_build_code(L, L.fd, ND, 15, L.cd);
  // dynamic header: lengths RLE (send_tree/scan_tree, trees.c:682-766)
  if (t == 0) {
    uint32_t hlit = NL;
    while (hlit > 257 && (L.cl[hlit - 1] >> 16) == 0) hlit--;
    uint32_t hdist = ND;
    while (hdist > 1 && (L.cd[hdist - 1] >> 16) == 0) hdist--;
    const uint32_t tot = hlit + hdist;
    for (uint32_t i = 0; i < hlit; i++) L.lens[i] = (uint8_t)(L.cl[i] >> 16);
    for (uint32_t i = 0; i < hdist; i++) L.lens[hlit + i] = (uint8_t)(L.cd[i] >> 16);
    uint32_t nr = 0;
    for (uint32_t i = 0; i < tot;) {
      const uint32_t v = L.lens[i];
      uint32_t r = 1;
      while (i + r < tot && L.lens[i + r] == v) r++;
      if (v == 0 && r >= 3) {
        const uint32_t k = min(r, 138u);
        if (k >= 11) L.rle[nr++] = (uint16_t)(18 | ((k - 11) << 8));
        else L.rle[nr++] = (uint16_t)(17 | ((k - 3) << 8));
        i += k;
      } else if (v != 0 && r >= 4) {
        L.rle[nr++] = (uint16_t)v;
        uint32_t rem = r - 1, used = 1;
        while (rem >= 3) {
          const uint32_t k = min(rem, 6u);
          L.rle[nr++] = (uint16_t)(16 | ((k - 3) << 8));
          rem -= k;
          used += k;
        }
        i += used;
      } else {
        L.rle[nr++] = (uint16_t)v;
        i++;
      }
    }
    for (uint32_t i = 0; i < nr; i++) L.fc[L.rle[i] & 0xffu]++;
    L.misc[0] = hlit;
    L.misc[1] = hdist;
    L.misc[2] = nr;
  }
  __syncthreads();
  dz_build_code(L, L.fc, NC, 7, L.cc);
  for (uint32_t i = t; i < DZ_OUTW; i += DZ_T) L.out[i] = 0;
  __syncthreads();
  // sizes
  uint32_t dyn_tok = 0, fix_tok = 0;
  for (uint32_t i = t; i < nt; i += DZ_T) {
    const uint32_t x = tk[i];
    uint32_t a, b, c, d;
    dyn_tok += dz_tok_bits(x, L.cl, L.cd, &a, &b, &c, &d);
    if ((x >> 16) == 0) {
      fix_tok += (x & 0xffu) < 144u ? 8u : 9u;
    } else {
      uint32_t lx, lv, dx, dv;
      const uint32_t ls = dz_len_sym(x >> 16, &lx, &lv);
      dz_dist_sym((x & 0xffffu) + 1u, &dx, &dv);
      fix_tok += (257u + ls < 280u ? 7u : 8u) + lx + 5u + dx;
    }
  }
  uint32_t dyn_all, fix_all;
  dz_scan_excl(dyn_tok, L.scan, &dyn_all);
  dz_scan_excl(fix_tok, L.scan, &fix_all);
  __shared__ uint32_t s_hdr_bits, s_dynamic;
  if (t == 0) {
    static const uint8_t ordr[NC] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t hclen = NC;
    while (hclen > 4 && (L.cc[ordr[hclen - 1]] >> 16) == 0) hclen--;
    uint32_t hb = 3 + 5 + 5 + 4 + 3 * hclen;
    for (uint32_t i = 0; i < L.misc[2]; i++) {
      const uint32_t sym = L.rle[i] & 0xffu;
      hb += (L.cc[sym] >> 16) + (sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u);
    }
    const uint64_t dyn = (uint64_t)hb + dyn_all + (L.cl[256] >> 16);
    const uint64_t fix = 3ull + fix_all + 7ull;
    s_dynamic = dyn < fix;
    // block header + (dynamic) code description
    uint32_t bit = 0;
    dz_put(L.out, bit, last ? 1u : 0u, 1);
    bit += 1;
    if (s_dynamic) {
      dz_put(L.out, bit, 2u, 2);
      bit += 2;
      dz_put(L.out, bit, L.misc[0] - 257u, 5);
      bit += 5;
      dz_put(L.out, bit, L.misc[1] - 1u, 5);
      bit += 5;
      dz_put(L.out, bit, hclen - 4u, 4);
      bit += 4;
      for (uint32_t i = 0; i < hclen; i++) {
        dz_put(L.out, bit, L.cc[ordr[i]] >> 16, 3);
        bit += 3;
      }
      for (uint32_t i = 0; i < L.misc[2]; i++) {
        const uint32_t sym = L.rle[i] & 0xffu, xv = L.rle[i] >> 8;
        const uint32_t c = L.cc[sym];
        dz_put(L.out, bit, c & 0xffffu, c >> 16);
        bit += c >> 16;
        const uint32_t xb = sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u;
        dz_put(L.out, bit, xv, xb);
        bit += xb;
      }
    } else {
      dz_put(L.out, bit, 1u, 2);
      bit += 2;
      // fixed codes (src/trees.c tr_static_init): lit 0-143: 8 bits 0x30+, 144-255: 9 bits
      // 0x190+, 256-279: 7 bits 0+, 280-287: 8 bits 0xc0+; distances 5 bits
      for (uint32_t i = 0; i < NL; i++) {
        uint32_t len, code;
        if (i < 144) {
          len = 8;
          code = 0x30 + i;
        } else if (i < 256) {
          len = 9;
          code = 0x190 + (i - 144);
        } else if (i < 280) {
          len = 7;
          code = i - 256;
        } else {
          len = 8;
          code = 0xc0 + (i - 280);
        }
        L.cl[i] = (len << 16) | (__builtin_bitreverse32(code) >> (32 - len));
      }
      for (uint32_t i = 0; i < ND; i++) L.cd[i] = (5u << 16) | (__builtin_bitreverse32(i) >> 27);
    }
    s_hdr_bits = bit;
  }
  __syncthreads();
  // tokens: bit offsets by a block scan over 256-token batches
  uint32_t base = s_hdr_bits;
  for (uint32_t b0 = 0; b0 < nt; b0 += DZ_T) {
    const uint32_t i = b0 + t;
    uint32_t v0 = 0, n0 = 0, v1 = 0, n1 = 0, nb = 0;
    if (i < nt) nb = dz_tok_bits(tk[i], L.cl, L.cd, &v0, &n0, &v1, &n1);
    uint32_t all;
    const uint32_t off = dz_scan_excl(nb, L.scan, &all) + base;
    if (i < nt) {
      dz_put(L.out, off, v0, n0);
      dz_put(L.out, off + n0, v1, n1);
    }
    base += all;
  }
  if (t == 0) {
    const uint32_t c = L.cl[256];
    dz_put(L.out, base, c & 0xffffu, c >> 16);
    segs[blockIdx.x].nbits = base + (c >> 16);
  }
  __syncthreads();
  const uint32_t nw = (base + 32u + 31u) / 32u;
  for (uint32_t i = t; i < nw; i += DZ_T) gout[i] = L.out[i];
}

// ---------------------------------------------------------------------------
// D4: checksums of the input (zs_check.h: every segment adds its contribution
// to the job's accumulators, in any order) and per-job bit offsets
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(DZ_T) zs_dz_check_kernel(ZsDJobDev *__restrict__ jobs, const ZsDSegDev *__restrict__ segs) {
  __shared__ uint32_t s_tab[4][256];
  __shared__ uint64_t s_red[16];
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.wrap == 0 || sg.len == 0) return;
  const uint32_t per = ((sg.len + DZ_T - 1) / DZ_T + 3u) & ~3u;
  const uint64_t lo = sg.start + min(sg.len, per * t), hi = sg.start + min(sg.len, per * (t + 1));
  if (jb.wrap == 2) {
    zs_crc_tables(s_tab);
    const uint32_t v = zs_block_xor(zs_crc_piece(jb.in, lo, hi, jb.in_len, s_tab), reinterpret_cast<uint32_t *>(s_red));
    if (t == 0 && v) atomicXor(reinterpret_cast<unsigned long long *>(&jobs[sg.job].ck_a), (unsigned long long)v);
  } else {
    uint32_t A = 0, B = 0;
    if (hi > lo) zs_adler_piece(jb.in, lo, hi, jb.in_len, &A, &B);
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
  const uint32_t hdr = jb.wrap == 2 ? 10u : (jb.wrap == 1 ? 2u : 0u);
  // segment k of the job: jb.seg0 + k; per-thread contiguous ranges
  const uint32_t ns = jb.nseg;
  const uint32_t per = (ns + DZ_JT - 1) / DZ_JT;
  const uint32_t k0 = min(ns, per * t), k1 = min(ns, per * (t + 1));
  uint64_t sum = 0;
  for (uint32_t k = k0; k < k1; k++) sum += segs[jb.seg0 + k].nbits;
  s_sum[t] = sum;
  __syncthreads();
  if (t == 0) {  // small serial exclusive scan over 1024 partial sums
    uint64_t acc = 8ull * hdr;
    for (uint32_t k = 0; k < DZ_JT; k++) {
      const uint64_t x = s_sum[k];
      s_sum[k] = acc;
      acc += x;
    }
    const uint64_t body_bytes = (acc + 7) / 8;
    const uint32_t tr = jb.wrap == 2 ? 8u : (jb.wrap == 1 ? 4u : 0u);
    jobs[blockIdx.x].total_out = body_bytes + tr;
  }
  __syncthreads();
  uint64_t off = s_sum[t];
  for (uint32_t k = k0; k < k1; k++) {
    segs[jb.seg0 + k].bitoff = off;
    off += segs[jb.seg0 + k].nbits;
  }
  if (t == 0)
    jobs[blockIdx.x].check = jb.wrap == 2   ? zs_crc_final((uint32_t)jb.ck_a, jb.in_len)
                             : jb.wrap == 1 ? zs_adler_final(jb.ck_a, jb.ck_b, jb.in_len)
                                            : 0u;
  if (t == 0) {
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
  if (nbits == 0) return;
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
__global__ void zs_dz_trailer_kernel(const ZsDJobDev *__restrict__ jobs, uint32_t njobs, uint8_t *__restrict__ stage) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  const ZsDJobDev jb = jobs[j];
  uint8_t *o = stage + jb.stage;
  const uint64_t tr = jb.wrap == 2 ? 8u : (jb.wrap == 1 ? 4u : 0u);
  uint8_t *p = o + jb.total_out - tr;
  if (jb.wrap == 2) {
    const uint32_t c = jb.check, n = (uint32_t)jb.in_len;
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
// launcher
// ---------------------------------------------------------------------------
extern "C" void zs_launch_deflate(ZsDJobDev *d_jobs, uint32_t njobs, ZsDSegDev *d_segs, uint32_t nseg, uint32_t *d_tokens,
                                  uint32_t *d_obuf, uint8_t *d_stage, hipStream_t st, hipEvent_t *ev) {
  if (ev) (void)hipEventRecord(ev[0], st);
  hipLaunchKernelGGL(zs_dz_match_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs, d_tokens);
  if (ev) (void)hipEventRecord(ev[1], st);
  hipLaunchKernelGGL(zs_dz_parse_kernel, dim3((nseg + 63) / 64), dim3(64), 0, st, d_jobs, d_segs, nseg, d_tokens);
  if (ev) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(zs_dz_block_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs, d_tokens, d_obuf);
  hipLaunchKernelGGL(zs_dz_check_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs);
  if (ev) (void)hipEventRecord(ev[3], st);
  hipLaunchKernelGGL(zs_dz_offsets_kernel, dim3(njobs), dim3(DZ_JT), 0, st, d_jobs, d_segs, d_stage);
  hipLaunchKernelGGL(zs_dz_stitch_kernel, dim3(nseg), dim3(DZ_T), 0, st, d_jobs, d_segs, d_obuf, d_stage);
  hipLaunchKernelGGL(zs_dz_trailer_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, d_jobs, njobs, d_stage);
  if (ev) (void)hipEventRecord(ev[4], st);
}
