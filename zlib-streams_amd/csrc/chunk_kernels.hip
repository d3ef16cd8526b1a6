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
// Link: verify the chain, offsets, history windows (one workgroup per stream)
// ---------------------------------------------------------------------------
#define LINK_THREADS 1024
#define LINK_PER (HIST / LINK_THREADS)  // window entries per thread and chain step
__global__ void __launch_bounds__(LINK_THREADS) zs_link_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                               ZsChunkDev *__restrict__ chunks, const ZsCJobDev *__restrict__ cjobs,
                                                               const uint16_t *__restrict__ scratch, uint8_t *__restrict__ windows,
                                                               ZsDecDev *__restrict__ decs, uint32_t *__restrict__ fallback) {
  __shared__ uint8_t s_win[2][HIST];
  __shared__ uint32_t s_ok, s_cur;
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
    const uint32_t lowest = HIST - wv;                // first valid history index
    // window index i = k * LINK_THREADS + t; all LINK_PER loads are issued
    // before any is consumed (one memory latency per chain step)
    uint16_t v[LINK_PER];
#pragma unroll
    for (int k = 0; k < LINK_PER; k++) {
      const uint32_t i = (uint32_t)k * LINK_THREADS + t;
      v[k] = (i >= keep) ? e[n - HIST + i] : (uint16_t)0;
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < LINK_PER; k++) {
      const uint32_t i = (uint32_t)k * LINK_THREADS + t;
      uint32_t b;
      if (i < keep) {
        b = W[i + n];
      } else if (v[k] < MARK_BASE) {
        b = v[k];
      } else {
        const uint32_t wx = v[k] - MARK_BASE;
        bad |= wx < lowest;  // reaches before the stream start
        b = W[wx & (HIST - 1)];
      }
      W2[i] = (uint8_t)b;
    }
    if (bad) s_ok = 0;
    if (t == 0) chunks[c].in_chain = 1;
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

extern "C" void zs_launch_lane(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, ZsChunkDev *d_chunks, uint32_t nchunks,
                               uint16_t *d_scratch, uint32_t *d_tokens, uint32_t *d_tables, const uint32_t *d_fixed,
                               hipStream_t st, hipEvent_t *ev);

extern "C" void zs_launch_chunked(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, ZsChunkDev *d_chunks, uint32_t nchunks,
                                  const uint32_t *d_find_ids, uint32_t nfind, const ZsCJobDev *d_cjobs, uint32_t ncjobs,
                                  uint16_t *d_scratch, uint32_t *d_tokens, uint32_t *d_tables, const uint32_t *d_fixed,
                                  uint8_t *d_windows, ZsDecDev *d_decs, uint32_t *d_fallback, hipStream_t st,
                                  hipEvent_t *ev) {
  // ev (profiling, optional): [0] before find, [1] after find, [2] after parse,
  // [3] after expand, [4] after link, [5] after emit
  if (ev) (void)hipEventRecord(ev[0], st);
  if (nfind) hipLaunchKernelGGL(zs_find_kernel, dim3(nfind), dim3(64), 0, st, d_jobs, d_heads, d_chunks, d_find_ids);
  if (ev) (void)hipEventRecord(ev[1], st);
  zs_launch_lane(d_jobs, d_heads, d_chunks, nchunks, d_scratch, d_tokens, d_tables, d_fixed, st, ev ? ev + 2 : nullptr);
  hipLaunchKernelGGL(zs_link_kernel, dim3(ncjobs), dim3(LINK_THREADS), 0, st, d_jobs, d_heads, d_chunks, d_cjobs,
                     d_scratch, d_windows, d_decs, d_fallback);
  if (ev) (void)hipEventRecord(ev[4], st);
  hipLaunchKernelGGL(zs_emit_kernel, dim3(nchunks), dim3(EMIT_THREADS), 0, st, d_jobs, d_chunks, d_scratch, d_windows,
                     d_fallback);
  if (ev) (void)hipEventRecord(ev[5], st);
}
