// deflate_zlib.hip -- GPU deflate that writes zlib's bytes (levels 4..9).
//
// Reference path: the deflate core of the zlib submodule (deflate.c
// deflate_slow + longest_match, absent from /root/reference; pinned by host
// zlib 1.2.11) called as deflateInit2(level, Z_DEFLATED,
// -15|31, 8, Z_DEFAULT_STRATEGY) (src/wasm/deflate_stream_wasm.c:31-49), and
// src/trees.c (_tr_tally 1029-1053, _tr_flush_block 931-1023, build_tree 561,
// gen_bitlen 474, gen_codes 205, scan_tree / send_tree, build_bl_tree 734,
// send_all_trees 767, compress_block 834-882, _tr_stored_block 794).
//
// deflate_slow inserts every position into its hash chains, so the chain of
// position p is a function of the input alone: every earlier position q >= 1
// whose 15-bit hash of in[q..q+2] equals p's.  That makes the search
// data-parallel; the stages (their semantics pinned on the CPU by
// tests/tools/dz_model.c against host zlib) are:
//   zs_zd_prev_kernel   four waves per 128 Ki positions: previous same-hash
//                       distance of every position (u16 head table in LDS,
//                       64 positions per step, same-hash lanes found with 15
//                       ballots; entries aged out every 16 Ki positions);
//   zs_zd_match_kernel  one 1024-thread workgroup per 8 Ki positions (the
//                       32 KiB window's bytes and chain links in LDS): the
//                       longest match of every position under the level's
//                       chain budget -- max_chain, and max_chain >> 2 (used when
//                       prev_length >= good_length) -- as longest_match finds
//                       it (first candidate reaching the best length, the
//                       first reaching nice_length ending the walk); lanes
//                       take a new position as soon as their walk ends;
//   zs_zd_parse_kernel  one workgroup per 64 KiB region: deflate_slow's loop
//                       replayed over those tables, 256-position pieces
//                       walked speculatively and re-walked from their
//                       predecessor's exit until the walks merge (a shared
//                       position in the "just emitted a match" state);
//                       zs_zd_fix_kernel does the same across regions;
//   zs_zd_count / blocks / tree / layout / emit kernels: blocks of 16383
//                       symbols, each flushed as _tr_flush_block does (stored /
//                       static / dynamic by the same bit counts, trees built
//                       with the same heap order and overflow repair), bit
//                       offsets per job, then the bits.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "zs_check.h"
#include "zs_common.h"
#include "zs_device.h"

#define ZD_MINM 3u
#define ZD_MAXM 258u
#define ZD_LOOK (ZD_MAXM + ZD_MINM + 1u)  // MIN_LOOKAHEAD
#define ZD_TOO_FAR 4096u
#define ZD_BLOCK 16383u                   // symbols per block: lit_bufsize - 1 (memLevel 8)
#define ZD_S1 131072u                     // zs_zd_prev_kernel positions per wave
#define ZD_SWEEP 16384u                   // head-table ageing period
#define ZD_S2 8192u                       // zs_zd_match_kernel positions per workgroup
#define ZD_MT 1024u
#define ZD_REG 65536u                     // parse region (one ZsDSegDev segment)
#ifndef ZD_PT
#define ZD_PT 256u  // parse threads per region
#endif
#define ZD_PIECE (ZD_REG / ZD_PT)  // positions per parse piece (a multiple of zs_zd_msearch_kernel's start spacing)
#define ZD_AUX 352u                       // per-block table words: 286 lit/len + 30 dist + 19 bit-length (+ pad)

// zlib deflate.c configuration_table rows (good, lazy, nice, chain), levels 4..9
__constant__ uint16_t zd_cfg[10][4] = {{0, 0, 0, 0},      {0, 0, 0, 0},        {0, 0, 0, 0},        {0, 0, 0, 0},
                                       {4, 4, 16, 16},    {8, 16, 32, 32},     {8, 16, 128, 128},   {8, 32, 128, 256},
                                       {32, 128, 258, 1024}, {32, 258, 258, 4096}};

struct ZsZWorkDev {  // one K1 / K2 work item
  uint32_t job;
  uint32_t len;
  uint64_t start;
};

__device__ __forceinline__ uint32_t zd_max_dist(const ZsDJobDev &jb) { return (1u << jb.wbits) - ZD_LOOK; }

// deflate_slow state A (avail 0, prev_len 2): after every match, and the stream start (K3)
#define ZD_STATE_A (2u << 1)

// bitmaps of a job: S (token starts), V (variant of match starts), M (state-A
// marks), I (deflate_fast: positions inserted into the hash chains), A / B
// (deflate_slow: positions whose match under max_chain / max_chain >> 2 the
// search kernel wrote)
struct ZdBm {
  uint32_t *S, *V, *M, *I, *A, *B;
};
__device__ __forceinline__ uint64_t zd_bm_words(uint64_t L) { return (L + 32u) / 32u + 1u; }
__device__ __forceinline__ ZdBm zd_bm(uint32_t *bm, const ZsDJobDev &jb) {
  const uint64_t words = zd_bm_words(jb.in_len);
  ZdBm b;
  b.S = bm + jb.bm0;
  b.V = b.S + words;
  b.M = b.V + words;
  b.I = b.M + words;
  b.A = b.I + words;
  b.B = b.A + words;
  return b;
}

// ---------------------------------------------------------------------------
// K1: previous same-hash distance (0: none within 32767, or position 0 = NIL)
// ---------------------------------------------------------------------------
// Four waves per work item, 256 positions per step: each wave finds, for its
// 64 positions, the earlier same-hash lanes of its own wave (15 ballots: the
// bulk of the work, in parallel across the waves); then, in wave order, the
// lanes with none read the head table and each hash group's last lane writes
// it (four short phases between barriers).  Occupancy: 2 work items (8 waves)
// per CU instead of 2 waves.
#define ZD_PT1 256u
#define ZD_HB (ZD_PT1 * 16u)  // positions whose hashes are computed together
__global__ void __launch_bounds__(ZD_PT1) zs_zd_prev_kernel(const ZsDJobDev *__restrict__ jobs,
                                                             const ZsZWorkDev *__restrict__ work, uint16_t *__restrict__ prevd) {
  __shared__ uint16_t head[32768];
  __shared__ __attribute__((aligned(16))) uint16_t s_h[ZD_HB];
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  const ZsZWorkDev wk = work[blockIdx.x];
  const ZsDJobDev jb = jobs[wk.job];
  const uint8_t *in = jb.in;
  const uint64_t L = jb.in_len;
  const uint64_t start = wk.start, to = wk.start + wk.len;
  const uint64_t from = start >= 32768u ? start - 32768u : 0u;
  // entries hold position & 0xffff; an entry whose age could exceed 32767 is
  // reset every ZD_SWEEP positions to a position 40000 back (age stays in
  // 40000 .. 56384 < 65536 until the next sweep: decoded as "none")
  auto sweep = [&](uint64_t b) {
    const uint32_t sent = (uint32_t)((b - 40000u) & 0xffffu);
    for (uint32_t i = t * 8; i < 32768u; i += ZD_PT1 * 8) {
      uint4 v = *reinterpret_cast<const uint4 *>(&head[i]);
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint32_t lo = w[k] & 0xffffu, hi = w[k] >> 16;
        if (((uint32_t)(b - lo) & 0xffffu) > 32768u) lo = sent;
        if (((uint32_t)(b - hi) & 0xffffu) > 32768u) hi = sent;
        w[k] = lo | (hi << 16);
      }
      *reinterpret_cast<uint4 *>(&head[i]) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  };
  {
    const uint32_t sent = (uint32_t)((from - 40000u) & 0xffffu);
    for (uint32_t i = t; i < 32768u / 2; i += ZD_PT1) reinterpret_cast<uint32_t *>(head)[i] = sent | (sent << 16);
  }
  __syncthreads();
  uint16_t *po = prevd + jb.pos0;
  static_assert(ZD_SWEEP % ZD_PT1 == 0, "sweeps fall on step boundaries");
  static_assert(ZD_SWEEP % ZD_HB == 0, "hash blocks fall on sweep boundaries");
  for (uint64_t base = from; base < to; base += ZD_PT1) {
    if (((base - from) % ZD_HB) == 0) {
      // the next ZD_HB positions' hashes into LDS, 16 per thread from 20 input
      // bytes (one batch of loads per 16 steps instead of three byte loads in
      // every step, each waiting on memory)
      __syncthreads();
      const uint64_t q0 = base + (uint64_t)t * 16u;
      uint8_t b[20];
      const uintptr_t a = reinterpret_cast<uintptr_t>(in + q0);
      if (q0 + 24u <= L && q0 >= 4u) {  // six aligned words cover the 20 bytes
        const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3u);
        uint32_t x[6];
#pragma unroll
        for (int k = 0; k < 6; k++) x[k] = w[k];
#pragma unroll
        for (int k = 0; k < 5; k++) {
          const uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
          b[4 * k] = (uint8_t)v;
          b[4 * k + 1] = (uint8_t)(v >> 8);
          b[4 * k + 2] = (uint8_t)(v >> 16);
          b[4 * k + 3] = (uint8_t)(v >> 24);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 20; k++) b[k] = q0 + k < L ? in[q0 + k] : 0;
      }
      uint32_t hv[8];
#pragma unroll
      for (int k = 0; k < 16; k += 2) {
        const uint32_t h0 = (((uint32_t)b[k] << 10) ^ ((uint32_t)b[k + 1] << 5) ^ b[k + 2]) & 0x7fffu;
        const uint32_t h1 = (((uint32_t)b[k + 1] << 10) ^ ((uint32_t)b[k + 2] << 5) ^ b[k + 3]) & 0x7fffu;
        hv[k / 2] = h0 | (h1 << 16);
      }
      uint4 *hd = reinterpret_cast<uint4 *>(s_h + t * 16u);
      hd[0] = make_uint4(hv[0], hv[1], hv[2], hv[3]);
      hd[1] = make_uint4(hv[4], hv[5], hv[6], hv[7]);
      if (base != from && ((base - from) % ZD_SWEEP) == 0) sweep(base);
      __syncthreads();
    }
    const uint64_t p = base + (uint64_t)wv * WAVE + lane;
    const bool valid = p + 2 < L && p < to;
    uint32_t h = 0;
    if (valid) h = s_h[(uint32_t)((base - from) % ZD_HB) + wv * WAVE + lane];
    // lanes of this wave with the same hash: 15 ballots
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 15; b++) {
      const uint64_t B = __ballot(valid && ((h >> b) & 1u));
      m &= ((h >> b) & 1u) ? B : ~B;
    }
    const uint64_t below = m & ((1ull << lane) - 1ull);
    const uint64_t above = lane == 63 ? 0ull : (m & ~((2ull << lane) - 1ull));
    uint32_t d = below ? lane - (63u - (uint32_t)__builtin_clzll(below)) : 0u;
    // head table in wave order: earlier waves' positions of this step first
#pragma unroll
    for (uint32_t ph = 0; ph < ZD_PT1 / WAVE; ph++) {
      if (wv == ph) {
        if (!below) d = (uint32_t)(p - head[h]) & 0xffffu;
        __builtin_amdgcn_wave_barrier();
        if (valid && !above) head[h] = (uint16_t)(p & 0xffffu);  // the group's latest position
      }
      __syncthreads();
    }
    if (p >= start && p < to) po[p] = (valid && d < 32768u && p != d) ? (uint16_t)d : (uint16_t)0;
  }
}

// The same table for small jobs (a stream segment: a window of history and the
// call's new input) in short work items: the window before an item enters the
// head table in one parallel pass (the latest position of each hash by LDS
// atomicMax, u32 entries relative to the window start), instead of the 32 Ki
// ordered steps the long items spend on it, so an item costs its own length.
// Work items of at most ZD_S1S positions (the relative positions stay below
// 2^16 + 1 with no ageing).
#define ZD_S1S 8192u
__global__ void __launch_bounds__(ZD_PT1) zs_zd_prev_small_kernel(const ZsDJobDev *__restrict__ jobs,
                                                                   const ZsZWorkDev *__restrict__ work,
                                                                   uint16_t *__restrict__ prevd) {
  __shared__ uint32_t head[32768];  // relative position + 1 of the latest occurrence (0: none)
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  const ZsZWorkDev wk = work[blockIdx.x];
  const ZsDJobDev jb = jobs[wk.job];
  const uint8_t *in = jb.in;
  const uint64_t L = jb.in_len;
  const uint64_t start = wk.start, to = wk.start + wk.len;
  const uint64_t from = start >= 32768u ? start - 32768u : 0u;
  for (uint32_t i = t; i < 32768u; i += ZD_PT1) head[i] = 0;
  __syncthreads();
  for (uint64_t r = from + t; r < start; r += ZD_PT1) {
    if (r + 2 < L) {
      const uint32_t h = (((uint32_t)in[r] << 10) ^ ((uint32_t)in[r + 1] << 5) ^ in[r + 2]) & 0x7fffu;
      atomicMax(&head[h], (uint32_t)(r - from + 1u));
    }
  }
  __syncthreads();
  uint16_t *po = prevd + jb.pos0;
  for (uint64_t base = start; base < to; base += ZD_PT1) {
    const uint64_t p = base + (uint64_t)wv * WAVE + lane;
    const bool valid = p + 2 < L && p < to;
    uint32_t h = 0;
    if (valid) h = (((uint32_t)in[p] << 10) ^ ((uint32_t)in[p + 1] << 5) ^ in[p + 2]) & 0x7fffu;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 15; b++) {
      const uint64_t B = __ballot(valid && ((h >> b) & 1u));
      m &= ((h >> b) & 1u) ? B : ~B;
    }
    const uint64_t below = m & ((1ull << lane) - 1ull);
    const uint64_t above = lane == 63 ? 0ull : (m & ~((2ull << lane) - 1ull));
    uint32_t d = below ? lane - (63u - (uint32_t)__builtin_clzll(below)) : 0u;
#pragma unroll
    for (uint32_t ph = 0; ph < ZD_PT1 / WAVE; ph++) {
      if (wv == ph) {
        if (!below) {
          const uint32_t e = head[h];
          d = e ? (uint32_t)(p - from - (e - 1u)) : 0xffffffffu;
        }
        __builtin_amdgcn_wave_barrier();
        if (valid && !above) head[h] = (uint32_t)(p - from + 1u);
      }
      __syncthreads();
    }
    if (p < to) po[p] = (valid && d < 32768u && p != d) ? (uint16_t)d : (uint16_t)0;
  }
}

// ---------------------------------------------------------------------------
// K2: longest match per position, two chain budgets
// ---------------------------------------------------------------------------
#define ZD_WB (ZD_S2 + 32768u + 272u)  // window bytes in LDS

__device__ __forceinline__ uint32_t zd_lw(const uint32_t *w, uint32_t a) {  // 4 bytes at byte a
  const uint32_t lo = w[a >> 2], hi = w[(a >> 2) + 1];
  return __builtin_amdgcn_alignbyte(hi, lo, a & 3u);
}

__global__ void __launch_bounds__(ZD_MT) zs_zd_match_kernel(const ZsDJobDev *__restrict__ jobs,
                                                             const ZsZWorkDev *__restrict__ work,
                                                             const uint16_t *__restrict__ prevd, uint32_t *__restrict__ ma,
                                                             uint32_t *__restrict__ mb, uint32_t *__restrict__ bm) {
  __shared__ __attribute__((aligned(16))) uint32_t s_w[ZD_WB / 4 + 4];
  __shared__ __attribute__((aligned(16))) uint16_t s_pd[ZD_S2 + 32768u];
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  const ZsZWorkDev wk = work[blockIdx.x];
  const ZsDJobDev jb = jobs[wk.job];
  const uint64_t L = jb.in_len, s = wk.start;
  const int64_t B = (int64_t)s - 32768;  // LDS index of position q: q - B
  // stage window bytes [max(0, B), min(L, s + n + 272)) and chain links [max(0, B), s + n)
  {
    uint8_t *wb = reinterpret_cast<uint8_t *>(s_w);
    const uint64_t lo = B < 0 ? 0u : (uint64_t)B;
    const uint64_t hi_b = s + wk.len + 272u;
    for (uint32_t i = t; i < ZD_WB / 4 + 4; i += ZD_MT) s_w[i] = 0;
    __syncthreads();
    for (uint64_t q = lo + t; q < hi_b && q < L; q += ZD_MT) wb[q - B] = jb.in[q];
    const uint16_t *pd = prevd + jb.pos0;
    for (uint64_t q = lo + t; q < s + wk.len; q += ZD_MT) s_pd[q - B] = pd[q];
  }
  __syncthreads();
  const uint32_t level = (uint32_t)jb.level;
  const uint32_t nice = zd_cfg[level][2], chain = zd_cfg[level][3], chain_b = chain >> 2;
  const uint32_t max_dist = zd_max_dist(jb);
  uint32_t *oa = ma + jb.pos0, *ob = mb + jb.pos0;
  // each wave owns a 16th of the item (512 positions of a full one; short
  // items -- small jobs, for latency -- at least 64); a lane takes the next
  // position when its walk ends
  const uint32_t per_w = max(64u, ((wk.len + ZD_MT / WAVE - 1) / (ZD_MT / WAVE) + 63u) & ~63u);
  const uint64_t q_beg = s + (uint64_t)wv * per_w;
  const uint64_t q_end = min(s + wk.len, q_beg + per_w);
  uint64_t nextp = q_beg + WAVE;
  uint64_t p = q_beg + lane;
  bool active = p < q_end, fin = false;
  uint32_t c = 0, k = 0, best = 0, bdist = 0, bl = 0, bd = 0, cap = 0, nicep = 0, ow = 0, pi = 0;
  // the common prefix of the strings at LDS bytes a and pi, capped at cap:
  // 16 bytes of both per iteration (10 independent LDS dword reads, one round
  // trip; a 4-byte step paid one per 4 bytes)
  auto cmp_len = [&](uint32_t a0) -> uint32_t {
    uint32_t n = 0;
    for (;;) {
      const uint32_t a = a0 + n, b = pi + n;
      const uint32_t wa = a >> 2, wb = b >> 2, sa = a & 3u, sb = b & 3u;
      uint32_t ua[5], ub[5];
#pragma unroll
      for (int q = 0; q < 5; q++) {
        ua[q] = s_w[wa + q];
        ub[q] = s_w[wb + q];
      }
      uint32_t x = 0, g = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t d = __builtin_amdgcn_alignbyte(ua[q + 1], ua[q], sa) ^ __builtin_amdgcn_alignbyte(ub[q + 1], ub[q], sb);
        if (x == 0) {
          x = d;
          g = (uint32_t)q;
        }
      }
      if (x) {
        n += 4 * g + ((uint32_t)__builtin_ctz(x) >> 3);
        break;
      }
      n += 16;
      if (n >= cap) break;
    }
    return min(n, cap);
  };
  // a walk starts at position p: its first candidate, or done at once
  auto start = [&]() {
    best = bdist = bl = bd = 0;
    k = 0;
    fin = true;
    if (!active) return;
    pi = (uint32_t)(p - B);
    const uint32_t d0 = s_pd[pi];
    if (p + ZD_MINM <= L && d0 != 0 && d0 <= max_dist) {
      const uint64_t look = L - p;
      cap = look < ZD_MAXM ? (uint32_t)look : ZD_MAXM;
      nicep = look < nice ? (uint32_t)look : nice;
      c = pi - d0;  // LDS byte index of the candidate
      fin = false;
    }
  };
  start();
  // One chain step per iteration for every walking lane, written with selects
  // (the per-step exec-mask bookkeeping of nested branches cost as many scalar
  // instructions as the step's vector work); only the full compare branches.
  auto step = [&]() {
    const bool walking = active && !fin;
    const uint32_t cc = walking ? c : 0u;
    const uint32_t nd = s_pd[cc];  // next link, in flight during the compare
    const uint32_t se = zd_lw(s_w, cc + (best >= 3 ? best - 3 : 0u));
    if (walking && (best < 3 || se == ow)) {
      const uint32_t n = cmp_len(c);
      if (n > best) {
        best = n;
        bdist = pi - c;
        if (best >= 3) ow = zd_lw(s_w, pi + best - 3);
      }
    }
    k += walking ? 1u : 0u;
    // the chain_b budget's result: at its last candidate, or at an earlier stop
    // zlib: stop at nice, at the chain budget, at a missing link, or when the
    // next candidate is not above strstart - MAX_DIST
    const uint32_t cn = c - nd;
    const bool stop = walking && (best >= nicep || k >= chain || nd == 0 || (pi - cn) >= max_dist);
    const bool snap = walking && (k == chain_b || (stop && k < chain_b));
    bl = snap ? best : bl;
    bd = snap ? bdist : bd;
    c = walking && !stop ? cn : c;
    fin = fin || stop;
  };
  for (;;) {
    // sixteen steps between refills: the ballot / refill bookkeeping is paid
    // every sixteenth step (a lane that stops early idles the rest; 8 steps:
    // 161 ms, 16: 154, 32: 171 per 16 x 64 MiB)
#pragma unroll
    for (int r = 0; r < 16; r++) step();
    const bool done = active && fin;
    if (done) {
      oa[p] = best | (bdist << 9);
      ob[p] = bl | (bd << 9);
    }
    const uint64_t fm = __ballot(done);
    if (fm) {
      if (done) {
        p = nextp + (uint64_t)__builtin_popcountll(fm & ((1ull << lane) - 1ull));
        active = p < q_end;
        start();
      }
      nextp += (uint64_t)__builtin_popcountll(fm);
    }
    if (!__ballot(active)) break;
  }
  // every position of the item has both results (items start 32-aligned)
  const ZdBm Bm = zd_bm(bm, jb);
  for (uint32_t i = t; i < (wk.len + 31u) / 32u; i += ZD_MT) Bm.A[s / 32u + i] = Bm.B[s / 32u + i] = ~0u;
}

// ---------------------------------------------------------------------------
// K2 (default): longest matches only where deflate_slow's parse looks for them.
// The parse searches at a loop top only while prev_length < max_lazy, never
// inside the matches it emits: ~0.2-0.3 searches per byte of text, and the
// positions it skips are the expensive ones (inside repeats, the full chain
// budget runs): tools/zd_search_probe.c, C2 text at L6, zs_zd_match_kernel
// walks 43 (Zipf) / 98 (lines) chain candidates per byte, the true parse 4.8 /
// 3.3.  Which loop tops the parse reaches depends on the matches, so the
// kernel walks the parse itself: one workgroup per 16 KiB item (window bytes
// and chain links in LDS, as zs_zd_match_kernel), a walk starting in state A
// at every 16th position (and at the job's parse entry), each lane taking the
// next start when its walk ends.  A walk stops at a state-A loop top another
// walk already claimed (both would continue identically) or at the item's
// end, so every path from a start is walked once up to the item end -- the
// paths the parse kernel's pieces (state A at every 256th position) and
// re-walks follow.  A search runs the budget the state asks for, as
// longest_match does; its result goes to ma / mb and its bit to the job's A / B
// bitmap.  Searches the walks did not make (a parse path entering an item from
// the previous one, until it meets a walked path) run on demand in the parse
// (zd_lookup).  Probe: 0.41 (Zipf) / 0.49 (lines) searches per byte, 8.9 /
// 20.8 candidates; with one start per lane a workgroup lasts as long as its
// longest walk (~1 K chain steps against ~300 on average: lanes busy 25 / 37%
// of its time).  Measured on 16 x 64 MiB L6 (tools/gpu_msearch.sh): search
// 118 ms (zs_zd_match_kernel) -> 66 ms; 512 threads 80.7 ms (half the waves
// to cover the LDS latency of a chain step), a start every 8th position
// (more starts per lane, 14% more searches) 109 / 85 ms, 8 chain steps per
// walk update 103 ms.  Measured in the probe and not built: an LDS ring that
// streams a span through one workgroup (the slowest walk holds the ring: lanes
// busy 26-47% at 1024 threads), cheap-budget prefixes for the walks that start
// off the parse kernel's piece grid (fewer searches, the same tail).  In-kernel
// timeline (ZD_MS_PROF=1, 16 x 64 MiB L6): every start is handed out within
// the first ~18% of a workgroup's time, 28 of 64 lanes search per wave-step on
// average, a chain step costs ~1 250 cycles per wave (issue-bound: ~120
// instructions, 4 waves per SIMD).  Measured and dropped: the step as a fixed
// sequence (filter, then one 16-byte compare block per step for every
// comparing lane, no divergent compare loop): 66 -> 78 ms.
// ---------------------------------------------------------------------------
#define ZD_S3 16384u  // positions per workgroup (zs_capi.cpp ZD_S3_HOST)
#ifndef ZD_MT3
#define ZD_MT3 1024u  // threads per workgroup (512: 80.7 ms, 1024: 66 ms per 16 x 64 MiB L6)
#endif
#ifndef ZD_PL3
#define ZD_PL3 16u  // a walk starts at every 16th position
#endif
#ifndef ZD_MSU
#define ZD_MSU 16  // chain steps between walk updates
#endif
#ifndef ZD_MS_PROF
#define ZD_MS_PROF 0  // per-workgroup timeline printed for a few items (tools/build_variant.sh ... -DZD_MS_PROF=1)
#endif
#ifndef ZD_XT3
#define ZD_XT3 512u  // walks go on this far past the item's end (parse paths entering the next item)
#endif
#define ZD_WB3 (ZD_S3 + ZD_XT3 + 32768u + 272u)  // window bytes in LDS

__global__ void __launch_bounds__(ZD_MT3) zs_zd_msearch_kernel(const ZsDJobDev *__restrict__ jobs,
                                                                const ZsZWorkDev *__restrict__ work,
                                                                const uint16_t *__restrict__ prevd,
                                                                uint32_t *__restrict__ ma, uint32_t *__restrict__ mb,
                                                                uint32_t *__restrict__ bm) {
  __shared__ __attribute__((aligned(16))) uint32_t s_w[ZD_WB3 / 4 + 4];
  __shared__ __attribute__((aligned(16))) uint16_t s_pd[ZD_S3 + ZD_XT3 + 32768u];
  __shared__ uint32_t s_claim[(ZD_S3 + ZD_XT3) / 32], s_sa[(ZD_S3 + ZD_XT3) / 32], s_sb[(ZD_S3 + ZD_XT3) / 32];
  __shared__ uint32_t s_next;
#if ZD_MS_PROF
  __shared__ uint32_t pf_iters, pf_lanes, pf_titers, pf_tlanes, pf_tail_at, pf_end, pf_stage;
  const uint64_t pf_t0 = clock64();
  if (threadIdx.x == 0) pf_iters = pf_lanes = pf_titers = pf_tlanes = pf_tail_at = pf_end = pf_stage = 0;
#endif
  const uint32_t t = threadIdx.x;
  const ZsZWorkDev wk = work[blockIdx.x];
  const ZsDJobDev jb = jobs[wk.job];
  const uint64_t L = jb.in_len, s = wk.start;
  const uint32_t len = wk.len;
  if (jb.pstart >= s + len) return;  // history only: the parse never searches here
  // walks continue ZD_XT3 positions into the next item, with starts there as
  // well: the paths the parse kernel's pieces and the region fix-ups follow
  // across the item's end are searched here until they meet one of those
  // starts' paths (= the next item's own walks).  Measured on 16 x 64 MiB L6:
  // without the extension the parse made on-demand searches (parse 10.8 ->
  // 16.5 ms); with it but no starts in it, a path crossing the end was one
  // lane's serial 512-position walk, the workgroup's new tail (search 66 ->
  // 167 ms); with both: search 66 ms, parse 10.85 ms, 9 915 MiB/s.
  const uint32_t lenx = (uint32_t)min<uint64_t>(len + ZD_XT3, L - s);
  const int64_t B = (int64_t)s - 32768;  // LDS index of position q: q - B
  {
    uint8_t *wb = reinterpret_cast<uint8_t *>(s_w);
    const uint64_t lo = B < 0 ? 0u : (uint64_t)B;
    const uint64_t hi_b = s + lenx + 272u;
    for (uint32_t i = t; i < ZD_WB3 / 4 + 4; i += ZD_MT3) s_w[i] = 0;
    for (uint32_t i = t; i < (ZD_S3 + ZD_XT3) / 32; i += ZD_MT3) s_claim[i] = s_sa[i] = s_sb[i] = 0;
    if (t == 0) s_next = 0;
    __syncthreads();
    // 16-byte loads (lo and its LDS index are multiples of 16; the job's link
    // array starts 64-position aligned); byte loads for an unaligned input
    const uint64_t hb = min(hi_b, L);
    uint64_t q16 = lo;
    if ((reinterpret_cast<uintptr_t>(jb.in) & 15u) == 0) {
      const uint64_t nq = (hb - lo) / 16u;
      const uint4 *src = reinterpret_cast<const uint4 *>(jb.in + lo);
      uint4 *dst = reinterpret_cast<uint4 *>(wb + (lo - B));
      for (uint64_t i = t; i < nq; i += ZD_MT3) dst[i] = src[i];
      q16 = lo + nq * 16u;
    }
    for (uint64_t q = q16 + t; q < hb; q += ZD_MT3) wb[q - B] = jb.in[q];
    const uint16_t *pd = prevd + jb.pos0;
    const uint64_t he = s + lenx, nl = (he - lo) / 8u;
    const uint4 *ps = reinterpret_cast<const uint4 *>(pd + lo);
    uint4 *pdst = reinterpret_cast<uint4 *>(s_pd + (lo - B));
    for (uint64_t i = t; i < nl; i += ZD_MT3) pdst[i] = ps[i];
    for (uint64_t q = lo + nl * 8u + t; q < he; q += ZD_MT3) s_pd[q - B] = pd[q];
  }
  __syncthreads();
#if ZD_MS_PROF
  if (t == 0) pf_stage = (uint32_t)(clock64() - pf_t0);
#endif
  const uint32_t level = (uint32_t)jb.level;
  const uint32_t good = zd_cfg[level][0], lazy = zd_cfg[level][1], nice = zd_cfg[level][2], chain = zd_cfg[level][3];
  const uint32_t max_dist = zd_max_dist(jb);
  uint32_t *oa = ma + jb.pos0 + s, *ob = mb + jb.pos0 + s;
  // starts: the job's parse entry when it lies in this item, then every 16th
  // position after it
  const bool ent = jb.pstart >= s;
  const uint32_t k0 = ent ? (uint32_t)((jb.pstart - s) / ZD_PL3) + 1u : 0u;
  const uint32_t npl = (lenx + ZD_PL3 - 1u) / ZD_PL3;  // (starts in the extension too: a crossing path meets one within ~64 positions)
  const uint32_t nst = (ent ? 1u : 0u) + (npl > k0 ? npl - k0 : 0u);
  // walk: loop top iq (item offset) in state st; search: at iq, budget svar
  uint32_t iq = 0, st = 0, svar = 0;
  bool walking = false, idle = false, srch = false, have = false;
  uint32_t c = 0, k = 0, best = 0, bdist = 0, cap = 0, nicep = 0, ow = 0, pi = 0, clim = 0;
  auto cmp_len = [&](uint32_t a0) -> uint32_t {  // as zs_zd_match_kernel
    uint32_t n = 0;
    for (;;) {
      const uint32_t a = a0 + n, b = pi + n;
      const uint32_t wa = a >> 2, wb = b >> 2, sa = a & 3u, sb = b & 3u;
      uint32_t ua[5], ub[5];
#pragma unroll
      for (int q = 0; q < 5; q++) {
        ua[q] = s_w[wa + q];
        ub[q] = s_w[wb + q];
      }
      uint32_t x = 0, g = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t d = __builtin_amdgcn_alignbyte(ua[q + 1], ua[q], sa) ^ __builtin_amdgcn_alignbyte(ub[q + 1], ub[q], sb);
        if (x == 0) {
          x = d;
          g = (uint32_t)q;
        }
      }
      if (x) {
        n += 4 * g + ((uint32_t)__builtin_ctz(x) >> 3);
        break;
      }
      n += 16;
      if (n >= cap) break;
    }
    return min(n, cap);
  };
  // one chain step of a searching lane (zs_zd_match_kernel's step, one budget)
  auto cstep = [&]() {
    const uint32_t cc = srch ? c : 0u;
    const uint32_t nd = s_pd[cc];
    const uint32_t se = zd_lw(s_w, cc + (best >= 3 ? best - 3 : 0u));
    if (srch && (best < 3 || se == ow)) {
      const uint32_t n = cmp_len(c);
      if (n > best) {
        best = n;
        bdist = pi - c;
        if (best >= 3) ow = zd_lw(s_w, pi + best - 3);
      }
    }
    k += srch ? 1u : 0u;
    const uint32_t cn = c - nd;
    const bool stop = srch && (best >= nicep || k >= clim || nd == 0 || (pi - cn) >= max_dist);
    c = srch && !stop ? cn : c;
    have = have || stop;
    srch = srch && !stop;
  };
  // deflate_slow's iteration at iq with match m (zd_step)
  auto advance = [&](uint32_t m) {
    const uint32_t pl = (st >> 1) & 511u;
    uint32_t mlen = 2, mdist = 0, mvar = 0;
    if (pl < lazy) {
      mvar = pl >= good ? 1u : 0u;
      const uint32_t ml = m & 511u;
      if (ml > pl) {
        mlen = ml;
        mdist = m >> 9;
      } else if (ml) {
        mlen = pl;
      }
      if (mlen == ZD_MINM && mdist > ZD_TOO_FAR) mlen = 2;
    }
    if (pl >= ZD_MINM && mlen <= pl) {
      iq = iq - 1u + pl;
      st = ZD_STATE_A;
    } else {
      st = 1u | (mlen << 1) | (mvar << 10) | (mdist << 11);
      iq += 1u;
    }
  };
  auto record = [&](uint32_t m) {
    (svar ? ob : oa)[iq] = m;
    atomicOr(&(svar ? s_sb : s_sa)[iq >> 5], 1u << (iq & 31u));
  };
  for (;;) {
    if (!idle && !srch) {
      if (have) {  // the search at iq ended
        const uint32_t m = best | (bdist << 9);
        record(m);
        advance(m);
        have = false;
      }
      // step the walk to its next search, taking new starts as walks end
      for (;;) {
        if (!walking) {
          const uint32_t i = atomicAdd(&s_next, 1u);
          if (i >= nst) {
            idle = true;
            break;
          }
          if (ent && i == 0) {
            iq = (uint32_t)(jb.pstart - s);
            st = jb.pstate;
          } else {
            iq = (k0 + i - (ent ? 1u : 0u)) * ZD_PL3;
            st = ZD_STATE_A;
          }
          walking = true;
        }
        if (iq >= lenx) {  // ZD_XT3 past the item's end: the next item's walks cover what follows
          walking = false;
          continue;
        }
        if (st == ZD_STATE_A) {
          const uint32_t bit = 1u << (iq & 31u);
          if (atomicOr(&s_claim[iq >> 5], bit) & bit) {  // another walk goes on from here
            walking = false;
            continue;
          }
        }
        const uint32_t pl = (st >> 1) & 511u;
        if (pl >= lazy) {  // no search: the pending match is emitted
          advance(0);
          continue;
        }
        svar = pl >= good ? 1u : 0u;
        pi = iq + 32768u;
        best = bdist = k = 0;
        clim = svar ? chain >> 2 : chain;
        const uint32_t d0 = s_pd[pi];
        const uint64_t look = L - s - iq;
        if (look < ZD_MINM || d0 == 0 || d0 > max_dist) {  // no candidate
          record(0);
          advance(0);
          continue;
        }
        cap = look < ZD_MAXM ? (uint32_t)look : ZD_MAXM;
        nicep = look < nice ? (uint32_t)look : nice;
        c = pi - d0;
        srch = true;
        break;
      }
    }
    if (!__ballot(!idle)) break;
#if ZD_MS_PROF
    {
      const uint64_t am = __ballot(srch);
      if ((t & 63u) == 0) {
        atomicAdd(&pf_iters, 1u);
        atomicAdd(&pf_lanes, (uint32_t)__builtin_popcountll(am));
        if (s_next >= nst && pf_tail_at == 0) atomicMax(&pf_tail_at, (uint32_t)(clock64() - pf_t0));
        if (s_next >= nst) {
          atomicAdd(&pf_titers, 1u);
          atomicAdd(&pf_tlanes, (uint32_t)__builtin_popcountll(am));
        }
      }
    }
#endif
    // sixteen chain steps between walk updates (zs_zd_match_kernel's refill rhythm)
#pragma unroll
    for (int r = 0; r < ZD_MSU; r++) cstep();
  }
#if ZD_MS_PROF
  if ((t & 63u) == 0) atomicMax(&pf_end, (uint32_t)(clock64() - pf_t0));
#endif
  __syncthreads();
#if ZD_MS_PROF
  if (t == 0 && (blockIdx.x % 512u) == 7u)
    printf("msprof blk %u len %u nst %u: stage %u cyc, walks %u cyc (tail from %u), wave-iters %u (tail %u), active lanes/iter %.1f (tail %.1f)\n",
           blockIdx.x, len, nst, pf_stage, pf_end, pf_tail_at, pf_iters, pf_titers, (double)pf_lanes / max(pf_iters, 1u),
           (double)pf_tlanes / max(pf_titers, 1u));
#endif
  const ZdBm Bm = zd_bm(bm, jb);
  // words the previous item's walks may also set ([0, ZD_XT3)) and the ones
  // past this item's end are OR-ed in; the rest belong to this item alone
  for (uint32_t i = t; i < (lenx + 31u) / 32u; i += ZD_MT3) {
    if (i < ZD_XT3 / 32u || i >= len / 32u) {
      if (s_sa[i]) atomicOr(&Bm.A[s / 32u + i], s_sa[i]);
      if (s_sb[i]) atomicOr(&Bm.B[s / 32u + i], s_sb[i]);
    } else {
      Bm.A[s / 32u + i] = s_sa[i];
      Bm.B[s / 32u + i] = s_sb[i];
    }
  }
}

// ---------------------------------------------------------------------------
// K3: deflate_slow's loop over the match tables.
// State at a loop top: avail (a literal is pending at p - 1), prev_length,
// prev_match distance, and which table gave it (the V bit a match start
// records).  Packed: bit 0 avail, 1-9 prev_len, 10 variant, 11-25 prev_dist.
// State A (avail 0, prev_len 2) follows every match and starts the stream.
// ---------------------------------------------------------------------------

struct ZdTabs {
  const uint32_t *ma, *mb;
  const uint8_t *in;
  uint64_t L;
  uint32_t good, lazy;
  // the parse walks (zd_step): which (position, budget) zs_zd_msearch_kernel
  // searched (bitmaps A / B), and what an on-demand search needs
  const uint32_t *sa, *sb;
  uint32_t *wa, *wb;  // ma / mb, written by on-demand searches
  const uint16_t *pd;
  uint32_t nice, chain, max_dist;
};

// longest_match at p under one chain budget (var 1: max_chain >> 2), from
// global memory: the parse's searches zs_zd_msearch_kernel did not make (a
// walk entering an item from its predecessor, until it meets a searched path).
// Same rules and result as the kernel's LDS walk: candidates along the same-hash
// chain while the chain budget lasts, the link exists and the candidate is
// within max_dist; strictly longer matches only; nice_length ends the walk.
__device__ __noinline__ uint32_t zd_search_g(const ZdTabs &T, uint64_t p, uint32_t var) {
  const uint32_t d0 = T.pd[p];
  if (p + ZD_MINM > T.L || d0 == 0 || d0 > T.max_dist) return 0;
  const uint64_t look = T.L - p;
  const uint32_t cap = look < ZD_MAXM ? (uint32_t)look : ZD_MAXM;
  const uint32_t nicep = look < T.nice ? (uint32_t)look : T.nice;
  const uint32_t clim = var ? T.chain >> 2 : T.chain;
  const uint8_t *in = T.in;
  uint64_t c = p - d0;
  uint32_t best = 0, bdist = 0;
  for (uint32_t k = 0;;) {
    if (best < 3 || (in[c + best] == in[p + best] && in[c + best - 1] == in[p + best - 1])) {
      uint32_t n = 0;
      while (n < cap && in[c + n] == in[p + n]) n++;
      if (n > best) {
        best = n;
        bdist = (uint32_t)(p - c);
      }
    }
    k++;
    const uint32_t nd = T.pd[c];
    if (best >= nicep || k >= clim || nd == 0) break;
    const uint64_t cn = c - nd;
    if (p - cn >= T.max_dist) break;
    c = cn;
  }
  return best | (bdist << 9);
}

// the match table entry the parse reads at p (budget var): searched by
// zs_zd_msearch_kernel, or searched here and stored for the token kernels
__device__ __forceinline__ uint32_t zd_lookup(const ZdTabs &T, uint64_t p, uint32_t var) {
  const uint32_t m = (var ? T.mb : T.ma)[p];
  if (((var ? T.sb : T.sa)[p >> 5] >> (p & 31u)) & 1u) return m;
  const uint32_t x = zd_search_g(T, p, var);
  (var ? T.wb : T.wa)[p] = x;
  return x;
}

// one loop iteration at p; returns the token emitted (start, kind) via out
// params: tok = 0 none, 1 literal at p - 1, 2 match at p - 1 (variant in *var)
__device__ __forceinline__ uint32_t zd_step(const ZdTabs &T, uint64_t &p, uint32_t &st, uint32_t *var) {
  const uint32_t avail = st & 1u, pl = (st >> 1) & 511u;
  uint32_t mlen = 2, mdist = 0, mvar = 0;
  if (pl < T.lazy) {
    mvar = pl >= T.good ? 1u : 0u;
    const uint32_t m = zd_lookup(T, p, mvar);
    const uint32_t ml = m & 511u;
    if (ml > pl) {
      mlen = ml;
      mdist = m >> 9;
    } else if (ml) {
      mlen = pl;  // longest_match returns best_len = prev_length
    }
    if (mlen == ZD_MINM && mdist > ZD_TOO_FAR) mlen = 2;
  }
  if (pl >= ZD_MINM && mlen <= pl) {
    *var = (st >> 10) & 1u;
    p = p - 1 + pl;
    st = ZD_STATE_A;
    return 2;
  }
  const uint32_t tok = avail ? 1u : 0u;
  *var = 0;
  st = 1u | (mlen << 1) | (mvar << 10) | (mdist << 11);
  p += 1;
  return tok;
}

// A loop-top state with no match pending (prev_length 2: state A, or a literal
// pending after a search that found nothing) walks on exactly as state A: the
// next iteration reads only prev_length, and avail / the variant / a too-far
// distance only decide the token at p - 1.  Walks that meet in such states at the
// same position walk the same path from there (merge points of the parse,
// re-walks and region fix-ups; on text with literal runs they meet far sooner
// than at state A, and on incompressible data -- no state A at all -- at once).
__device__ __forceinline__ bool zd_free(uint32_t st) { return ((st >> 1) & 511u) == 2u; }

__device__ __forceinline__ void zd_setbit(uint32_t *w, uint64_t i) { w[i >> 5] |= 1u << (i & 31u); }
__device__ __forceinline__ void zd_putbit(uint32_t *w, uint64_t i, bool v) {
  if (v) w[i >> 5] |= 1u << (i & 31u);
}
__device__ __forceinline__ bool zd_getbit(const uint32_t *w, uint64_t i) { return (w[i >> 5] >> (i & 31u)) & 1u; }

// the tables a parse walk reads (zd_step): match tables, searched bitmaps and
// what an on-demand search needs
__device__ __forceinline__ ZdTabs zd_tabs(const ZsDJobDev &jb, uint32_t *ma, uint32_t *mb, const uint16_t *prevd,
                                          uint32_t *bm) {
  ZdTabs T;
  T.ma = T.wa = ma + jb.pos0;
  T.mb = T.wb = mb + jb.pos0;
  T.in = jb.in;
  T.L = jb.in_len;
  T.good = zd_cfg[jb.level][0];
  T.lazy = zd_cfg[jb.level][1];
  T.nice = zd_cfg[jb.level][2];
  T.chain = zd_cfg[jb.level][3];
  T.max_dist = zd_max_dist(jb);
  T.pd = prevd + jb.pos0;
  const ZdBm b = zd_bm(bm, jb);
  T.sa = b.A;
  T.sb = b.B;
  return T;
}

// Token bits of a walk over [lo, hi): every loop top q with a literal pending
// (avail) makes q - 1 a token start -- a literal, or the match deflate_slow
// emits there, whose table is the state's variant bit.  A walk records
// pending positions from its second loop top on, and the one pending when it
// leaves (then q == hi): so each walk writes only positions in [lo, hi).
// (rec_first: also the literal pending at the first loop top -- a job's parse
// entry, whose pending literal no earlier walk of the job records)
template <typename SetF>
__device__ __forceinline__ void zd_walk_record(const ZdTabs &T, uint64_t &q, uint32_t &qs, uint64_t hi, SetF set,
                                               uint32_t *marks, uint64_t mark0, bool rec_first = false) {
  uint32_t var;
  bool first = !rec_first;
  while (q < hi) {
    if (marks && zd_free(qs)) zd_setbit(marks, q - mark0);
    if ((qs & 1u) && !first) set(q - 1, (qs >> 10) & 1u);
    first = false;
    (void)zd_step(T, q, qs, &var);
  }
  if (qs & 1u) set(q - 1, (qs >> 10) & 1u);
}

__global__ void __launch_bounds__(ZD_PT) zs_zd_parse_kernel(const ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                             uint32_t *__restrict__ ma, uint32_t *__restrict__ mb,
                                                             const uint16_t *__restrict__ prevd, uint32_t *__restrict__ bm) {
  __shared__ uint32_t s_S[ZD_REG / 32], s_V[ZD_REG / 32], s_M[ZD_REG / 32];
  __shared__ uint64_t s_xp[ZD_PT];
  __shared__ uint32_t s_xs[ZD_PT];
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.exact != ZD_SLOW) return;
  const ZdTabs T = zd_tabs(jb, ma, mb, prevd, bm);
  const uint64_t r0 = sg.start, rend = sg.start + sg.len;
  const uint64_t a = r0 + (uint64_t)t * ZD_PIECE, b = min(rend, a + ZD_PIECE);
  // the job's parse entry (pstart, pstate) lies in its first region (the
  // history before it is at most one window); pieces before it hold no tokens
  // and the piece holding it starts there, in that state
  const bool has_ent = r0 == 0 && jb.pstart < rend;
  const uint32_t ent_t = has_ent ? (uint32_t)(jb.pstart / ZD_PIECE) : 0u;
  const uint64_t ent_p = has_ent ? jb.pstart : r0;
  const uint32_t ent_s = has_ent ? jb.pstate : ZD_STATE_A;
  const bool act = a < rend && t >= ent_t && (r0 != 0 || jb.pstart < rend);
  for (uint32_t i = t; i < ZD_REG / 32; i += ZD_PT) s_S[i] = s_V[i] = s_M[i] = 0;
  __syncthreads();
  uint32_t var;
  // speculative walk of the piece from (a, A), recording as the final walk
  // would: its state-A positions, token starts and variants (kept from the
  // point where the true parse meets it, below)
  auto rec = [&](uint64_t x, uint32_t v) {
    zd_setbit(s_S, x - r0);
    zd_putbit(s_V, x - r0, v != 0);
  };
  uint64_t p = t == ent_t ? ent_p : a;
  uint32_t st = t == ent_t ? ent_s : ZD_STATE_A;
  if (act) zd_walk_record(T, p, st, b, rec, s_M, r0, has_ent && t == ent_t);
  const uint64_t spec_p = act ? p : a;
  const uint32_t spec_s = act ? st : ZD_STATE_A;
  s_xp[t] = spec_p;
  s_xs[t] = spec_s;
  __syncthreads();
  for (;;) {  // re-walk from the predecessor's exit until meeting a marked state-A position
    uint64_t q = t == ent_t ? ent_p : s_xp[t - 1];
    uint32_t qs = t == ent_t ? ent_s : s_xs[t - 1];
    uint64_t rp = s_xp[t];
    uint32_t rs = s_xs[t];
    if (act) {
      bool merged = false;
      while (q < b) {
        if (zd_free(qs) && zd_getbit(s_M, q - r0)) {
          merged = true;
          break;
        }
        (void)zd_step(T, q, qs, &var);
      }
      rp = merged ? spec_p : q;
      rs = merged ? spec_s : qs;
    }
    __syncthreads();
    const bool changed = act && (rp != s_xp[t] || rs != s_xs[t]);
    if (changed) {
      s_xp[t] = rp;
      s_xs[t] = rs;
    }
    if (!__syncthreads_or(changed)) break;
  }
  // final walk from the true entry, only up to where it meets the speculative
  // walk (a marked state-A loop top: from there both walk the same path, whose
  // tokens and marks the speculative walk recorded); the piece's bits below
  // that point are cleared and rewritten (each piece owns its 32-aligned words)
  if (act) {
    uint64_t q = t == ent_t ? ent_p : s_xp[t - 1];
    uint32_t qs = t == ent_t ? ent_s : s_xs[t - 1];
    uint64_t mq = q;
    uint32_t mqs = qs;
    while (mq < b && !(zd_free(mqs) && zd_getbit(s_M, mq - r0))) (void)zd_step(T, mq, mqs, &var);
    const uint64_t mp = min(mq, b);
    for (uint64_t x = a; x < mp; x += 32u) {
      const uint32_t wi = (uint32_t)((x - r0) >> 5);
      const uint32_t n = (uint32_t)min<uint64_t>(32u, mp - x);
      const uint32_t keep = n == 32u ? 0u : ~0u << n;
      s_S[wi] &= keep;
      s_V[wi] &= keep;
      s_M[wi] &= keep;
    }
    zd_walk_record(T, q, qs, mp, rec, s_M, r0, has_ent && t == ent_t);
  }
  __syncthreads();
  ZdBm Bm = zd_bm(bm, jb);
  const uint64_t w0 = r0 / 32u;
  const uint32_t nw = (uint32_t)((sg.len + 31u) / 32u);
  for (uint32_t i = t; i < nw; i += ZD_PT) {
    Bm.S[w0 + i] = s_S[i];
    Bm.V[w0 + i] = s_V[i];
    Bm.M[w0 + i] = s_M[i];
  }
  const uint32_t lastp = sg.len ? (uint32_t)((sg.len + ZD_PIECE - 1u) / ZD_PIECE) - 1u : 0u;
  if (t == lastp) {
    segs[blockIdx.x].zx0 = s_xp[t];
    segs[blockIdx.x].zs0 = s_xs[t];
    segs[blockIdx.x].zx[0] = segs[blockIdx.x].zx[1] = s_xp[t];
    segs[blockIdx.x].zs[0] = segs[blockIdx.x].zs[1] = s_xs[t];
    segs[blockIdx.x].zfix = r0;
  }
}

// ---------------------------------------------------------------------------
// K3b: across regions.  Region r's true entry is region r-1's current exit;
// when it differs from the assumed one (region start, state A) the region is
// re-walked from it until the walk meets a state-A position of the region's
// own parse (and reaches past earlier rewrites), its tokens before that point
// rewritten.  zs_zd_fix_kernel: one round, every region at once (exits
// double-buffered: read [cur], write [cur ^ 1]); the host repeats rounds while
// exits change, up to a bound.  A correction moves one region per round, so a
// long periodic run (zeros, a repeated pattern: the true parse and each
// region's own parse step in 258s from offsets that never line up) would need
// a round per region; past the bound zs_zd_fix_seq_kernel finishes the job in
// ONE pass, a thread per job walking its regions in order, each region's
// entry being the exit its predecessor just got.
// ---------------------------------------------------------------------------
// region i from entry (ep, es): rewrites its tokens where they change, returns
// its exit in (xp, xs)
__device__ void zd_fix_region(const ZsDJobDev &jb, ZsDSegDev *__restrict__ segs, uint32_t i, uint32_t *__restrict__ ma,
                              uint32_t *__restrict__ mb, const uint16_t *__restrict__ prevd, uint32_t *__restrict__ bm,
                              uint64_t ep, uint32_t es, uint64_t &xp, uint32_t &xs) {
  const ZsDSegDev sg = segs[i];
  const uint64_t r0 = sg.start, rend = sg.start + sg.len;
  xp = sg.zx0;
  xs = sg.zs0;
  if (ep == r0 && zd_free(es) && sg.zfix == r0) return;  // its own parse stands (a pending literal at r0 - 1 is the predecessor's)
  const ZdTabs T = zd_tabs(jb, ma, mb, prevd, bm);
  ZdBm Bm = zd_bm(bm, jb);
  // 1. where does the walk from the entry merge with the region's own parse?
  uint64_t q = ep;
  uint32_t qs = es, var;
  bool merged = false;
  while (q < rend) {
    if (zd_free(qs) && q >= sg.zfix && zd_getbit(Bm.M, q)) {
      merged = true;
      break;
    }
    (void)zd_step(T, q, qs, &var);
  }
  const uint64_t conv = merged ? q : rend;
  if (!merged) {
    xp = q;
    xs = qs;
  }
  // 2. rewrite the tokens of [r0, conv)
  for (uint64_t x = r0; x < conv; x += 32u) {
    const uint64_t w = x >> 5;
    const uint32_t n = (uint32_t)min<uint64_t>(32u, conv - x);
    const uint32_t keep = n == 32u ? 0u : ~0u << n;  // region words start 32-aligned
    Bm.S[w] &= keep;
    Bm.V[w] &= keep;
  }
  q = ep;
  qs = es;
  zd_walk_record(
      T, q, qs, conv,
      [&](uint64_t x, uint32_t v) {
        Bm.S[x >> 5] |= 1u << (x & 31u);
        if (v) Bm.V[x >> 5] |= 1u << (x & 31u);
      },
      (uint32_t *)nullptr, 0);
  segs[i].zfix = conv;
}

__global__ void zs_zd_fix_kernel(const ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs, uint32_t nseg,
                                 uint32_t *__restrict__ ma, uint32_t *__restrict__ mb, const uint16_t *__restrict__ prevd,
                                 uint32_t *__restrict__ bm, uint32_t cur, uint32_t *__restrict__ changed) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  const ZsDSegDev sg = segs[i];
  const ZsDJobDev jb = jobs[sg.job];
  if (jb.exact != ZD_SLOW) return;
  uint64_t ep = sg.start;
  uint32_t es = ZD_STATE_A;
  if (sg.start != 0) {
    ep = segs[i - 1].zx[cur];
    es = segs[i - 1].zs[cur];
  }
  uint64_t xp;
  uint32_t xs;
  zd_fix_region(jb, segs, i, ma, mb, prevd, bm, ep, es, xp, xs);
  segs[i].zx[cur ^ 1u] = xp;
  segs[i].zs[cur ^ 1u] = xs;
  if (xp != sg.zx[cur] || xs != sg.zs[cur]) atomicOr(changed, 1u);
}

// one thread per job: its regions in order from the job's start, so every
// entry is final when its region is walked (no rounds)
__global__ void zs_zd_fix_seq_kernel(const ZsDJobDev *__restrict__ jobs, uint32_t njobs, ZsDSegDev *__restrict__ segs,
                                     uint32_t *__restrict__ ma, uint32_t *__restrict__ mb,
                                     const uint16_t *__restrict__ prevd, uint32_t *__restrict__ bm) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  const ZsDJobDev jb = jobs[j];
  if (jb.exact != ZD_SLOW) return;
  uint64_t ep = 0;
  uint32_t es = ZD_STATE_A;
  for (uint32_t i = jb.seg0; i < jb.seg0 + jb.nseg; i++) {
    if (segs[i].start == 0) {
      ep = 0;
      es = ZD_STATE_A;
    }
    uint64_t xp;
    uint32_t xs;
    zd_fix_region(jb, segs, i, ma, mb, prevd, bm, ep, es, xp, xs);
    segs[i].zx[0] = segs[i].zx[1] = xp;
    segs[i].zs[0] = segs[i].zs[1] = xs;
    ep = xp;
    es = xs;
  }
}

// ---------------------------------------------------------------------------
// K3c: levels 1..3, deflate_fast (zlib deflate.c, configuration_table rows
// 1..3).  deflate_fast inserts a match's inner positions into the hash chains
// only when the match is at most max_insert_length (= max_lazy) long, so the
// chain a search walks depends on every earlier parse decision -- and on
// periodic text that dependence never dies out: started mid-stream from a
// different insertion history, the parse of `line-%08d` text still differs
// 4 MiB later (13% of decisions; tools/fast_resync_probe.c), so no
// speculative split of a stream can be verified locally.  The parse is
// therefore serial per stream, and the parallelism is inside one step: one
// wave per job, zlib's head / prev tables in LDS, and 64 consecutive positions
// searched at once against the tables as they stand before those positions.
// A position's search is the one zlib makes there unless an earlier position
// of the same 64 with the same hash gets inserted first (its chain would then
// start there): the wave walks the loop tops in order, commits searches until
// the first such one, inserts what it committed, and starts the next step at
// that position.  Positions are kept as (absolute & 0xffff), entries older
// than a window reset every 16 Ki positions (as zs_zd_prev_kernel), so a
// stored position decodes as `q - ((q - e) & 0xffff)` without aliasing.
// Output: token starts (S), match length | distance << 9 at each match start
// (ma), the insertion bits (I) -- the format of the deflate_slow parse, read by
// the same block kernels.
// ---------------------------------------------------------------------------
// zlib deflate.c configuration_table rows 1..3: good, lazy (max_insert_length), nice, chain
__constant__ uint16_t zd_cfgf[4][4] = {{0, 0, 0, 0}, {4, 4, 8, 4}, {4, 5, 16, 8}, {4, 6, 32, 32}};
#define ZF_SWEEP 16384u
#ifndef ZF_PROF
#define ZF_PROF 0  // per-step phase clocks, printed per job (tools/build_variant.sh ... -DZF_PROF=1)
#endif

// the job's input read as aligned words (unaligned caller buffers; word
// indices clamped to the buffer's own words)
struct ZfIn {
  const uint32_t *w;
  uint32_t sh;
  uint64_t nw;
  __device__ void init(const uint8_t *in, uint64_t L) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(in);
    w = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
    sh = (uint32_t)(a & 3u);
    nw = (sh + L + 3) / 4;
    if (nw == 0) nw = 1;
  }
  __device__ __forceinline__ uint32_t ld4(uint64_t pos) const {  // bytes pos..pos+3 (past the end: unspecified)
    const uint64_t a = pos + sh, k = a >> 2;
    const uint32_t lo = w[min(k, nw - 1)], hi = w[min(k + 1, nw - 1)];
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(a & 3u));
  }
};

__device__ __forceinline__ uint32_t zf_hash3(uint32_t v) {
  return (((v & 0xffu) << 10) ^ (((v >> 8) & 0xffu) << 5) ^ ((v >> 16) & 0xffu)) & 0x7fffu;
}
__device__ __forceinline__ uint32_t zf_hash(const ZfIn &X, uint64_t q) { return zf_hash3(X.ld4(q)); }

// The window in LDS: a 32 KiB ring of input words (slot = position mod
// 32768) holding [fend - 32768, fend).  A step at p reads positions < p + 340
// and advances <= 321, so the ring is refilled ZF_FILL bytes at a time (loads
// issued before the step's searches, stored after them) while fend - p <
// 661 + ZF_FILL; a candidate older than the ring's start (the oldest ~2 K
// positions of the window) is compared from global memory instead.
#define ZF_RING_WORDS 8192u
#define ZF_FILL 1024u
struct ZfWin {
  const uint32_t *r;
  uint64_t lo;  // first position held
  __device__ __forceinline__ uint32_t rd4(uint64_t pos) const {
    const uint32_t a = (uint32_t)pos, w = (a >> 2) & (ZF_RING_WORDS - 1u);
    return __builtin_amdgcn_alignbyte(r[(w + 1u) & (ZF_RING_WORDS - 1u)], r[w], a & 3u);
  }
};

// common prefix of the strings at c and q, capped (16 bytes of both per step);
// RING: the candidate's bytes from the LDS ring, else from global memory
template <bool RING>
__device__ __forceinline__ uint32_t zf_cmp(const ZfWin &Wn, const ZfIn &X, uint64_t c, uint64_t q, uint32_t cap) {
  uint32_t n = 0;
  for (;;) {
    uint32_t x = 0, g = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint64_t cp = c + n + 4 * i;
      const uint32_t d = (RING ? Wn.rd4(cp) : X.ld4(cp)) ^ Wn.rd4(q + n + 4 * i);
      if (x == 0) {
        x = d;
        g = (uint32_t)i;
      }
    }
    if (x) {
      n += 4 * g + ((uint32_t)__builtin_ctz(x) >> 3);
      break;
    }
    n += 16;
    if (n >= cap) break;
  }
  return min(n, cap);
}

// age out entries more than a window old (see zs_zd_prev_kernel's sweep)
__device__ void zf_sweep(uint16_t *tab, uint64_t b, uint32_t lane) {
  const uint32_t sent = (uint32_t)((b - 40000u) & 0xffffu);
  for (uint32_t i = lane * 8; i < 65536u; i += WAVE * 8) {
    uint4 v = *reinterpret_cast<const uint4 *>(&tab[i]);
    uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t lo = wv[k] & 0xffffu, hi = wv[k] >> 16;
      if (((uint32_t)(b - lo) & 0xffffu) > 32768u) lo = sent;
      if (((uint32_t)(b - hi) & 0xffffu) > 32768u) hi = sent;
      wv[k] = lo | (hi << 16);
    }
    *reinterpret_cast<uint4 *>(&tab[i]) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
  }
}

// lanes of the wave with the same 15-bit hash (among `on` lanes)
__device__ __forceinline__ uint64_t zf_same(uint32_t h, bool on) {
  uint64_t m = __ballot(on);
#pragma unroll
  for (int b = 0; b < 15; b++) {
    const uint64_t B = __ballot(on && ((h >> b) & 1u));
    m &= ((h >> b) & 1u) ? B : ~B;
  }
  return on ? m : 0ull;
}

// INSERT_STRING for every lane with `ins` set, in lane (position) order:
// prev[q] = the latest earlier inserted position of its hash (an earlier lane
// of this step, else the head), head = the group's last inserted lane
__device__ __forceinline__ void zf_insert(uint16_t *head, uint16_t *prev, uint64_t q, uint32_t h, bool ins,
                                          uint64_t same, uint32_t lane) {
  const uint64_t insm = __ballot(ins);
  const uint64_t below = same & insm & ((1ull << lane) - 1ull);
  const uint64_t above = lane == 63 ? 0ull : (same & insm & ~((2ull << lane) - 1ull));
  uint32_t pv = 0;
  if (ins) pv = below ? (uint32_t)((q - lane + (63u - (uint32_t)__builtin_clzll(below))) & 0xffffu) : head[h];
  __builtin_amdgcn_wave_barrier();
  if (ins) {
    prev[q & 0x7fffu] = (uint16_t)pv;
    if (!above) head[h] = (uint16_t)(q & 0xffffu);
  }
  __builtin_amdgcn_wave_barrier();
}

// longest_match at q (prev_length = MIN_MATCH - 1, the full chain budget):
// candidates from head entry e0, best length and the distance of the first
// candidate reaching it
__device__ __forceinline__ void zf_search(const ZfWin &Wn, const ZfIn &X, const uint16_t *prev, uint64_t q, uint64_t L,
                                          uint32_t e0,
                                          uint32_t max_dist, uint32_t nice, uint32_t chain, uint32_t &olen,
                                          uint32_t &odist) {
  olen = 0;
  odist = 0;
  uint32_t age = (uint32_t)(q - e0) & 0xffffu;
  if (age > max_dist || age == 0 || q == age) return;  // NIL, out of range, or position 0 (zlib's NIL)
  const uint64_t look = L - q;
  const uint32_t cap = look < ZD_MAXM ? (uint32_t)look : ZD_MAXM;
  const uint32_t nicep = look < nice ? (uint32_t)look : nice;
  uint32_t best = ZD_MINM - 1, bdist = 0;
  for (uint32_t k = 0;;) {
    const uint64_t c = q - age;
    const uint32_t n = c >= Wn.lo ? zf_cmp<true>(Wn, X, c, q, cap) : zf_cmp<false>(Wn, X, c, q, cap);
    if (n > best) {
      best = n;
      bdist = age;
      if (n >= nicep) break;
    }
    if (++k >= chain) break;
    const uint32_t e = prev[c & 0x7fffu];
    age = (uint32_t)(q - e) & 0xffffu;
    if (age >= max_dist || q == age) break;  // cur_match <= strstart - MAX_DIST, or NIL
  }
  if (best >= ZD_MINM) {
    olen = best;
    odist = bdist;
  }
}

__global__ void __launch_bounds__(WAVE) zs_zd_fast_kernel(ZsDJobDev *__restrict__ jobs, uint32_t *__restrict__ bm,
                                                           uint32_t *__restrict__ ma) {
  __shared__ __attribute__((aligned(16))) uint16_t s_tab[65536];  // head[32768] | prev[32768]
  __shared__ __attribute__((aligned(16))) uint32_t s_ring[ZF_RING_WORDS];
  uint16_t *s_head = s_tab, *s_prev = s_tab + 32768;
  const uint32_t lane = threadIdx.x;
  const ZsDJobDev jb = jobs[blockIdx.x];
  if (jb.exact != ZD_FAST) return;
  const uint64_t L = jb.in_len;
  ZfIn X;
  X.init(jb.in, L);
  const ZdBm B = zd_bm(bm, jb);
  uint32_t *om = ma + jb.pos0;
  const uint32_t level = (uint32_t)jb.level;
  const uint32_t max_ins = zd_cfgf[level][1], nice = zd_cfgf[level][2], chain = zd_cfgf[level][3];
  const uint32_t max_dist = zd_max_dist(jb);
  const bool cut = jb.term == ZS_DT_CUT;
  {
    const uint32_t sent = (uint32_t)((0u - 40000u) & 0xffffu);
    for (uint32_t i = lane; i < 32768u / 2; i += WAVE) {
      reinterpret_cast<uint32_t *>(s_head)[i] = sent | (sent << 16);
      reinterpret_cast<uint32_t *>(s_prev)[i] = sent | (sent << 16);
    }
  }
  __builtin_amdgcn_wave_barrier();
  uint64_t next_sweep = ZF_SWEEP;
  auto sweep_to = [&](uint64_t p) {
    if (p < next_sweep) return;
    __builtin_amdgcn_wave_barrier();
    zf_sweep(s_tab, p, lane);
    __builtin_amdgcn_wave_barrier();
    next_sweep = p + ZF_SWEEP;
  };
  // the history before the parse entry: its inserted positions, in order
  // (a stream segment's window; the bits come from the previous segment)
#if ZF_PROF
  const uint64_t zh0 = __builtin_amdgcn_s_memtime();
#endif
  for (uint64_t p = 0; p < jb.pstart; p += WAVE) {
    sweep_to(p);
    const uint64_t q = p + lane;
    const bool on = q < jb.pstart && q + ZD_MINM <= L && zd_getbit(B.I, q);
    const uint32_t h = q + ZD_MINM <= L ? zf_hash(X, q) : 0u;
    zf_insert(s_head, s_prev, q, h, on, zf_same(h, on), lane);
  }
  uint64_t p = jb.pstart;
  bool stop = false;
#if ZF_PROF
  const uint64_t zhist = __builtin_amdgcn_s_memtime() - zh0;
  uint64_t zt[6] = {0, 0, 0, 0, 0, 0}, zsteps = 0, zt0 = __builtin_amdgcn_s_memtime();
#define ZF_T(i)                                         \
  do {                                                  \
    const uint64_t n_ = __builtin_amdgcn_s_memtime();   \
    zt[i] += n_ - zt0;                                  \
    zt0 = n_;                                           \
  } while (0)
#else
#define ZF_T(i) ((void)0)
#endif
  ZfWin Wn;
  Wn.r = s_ring;
  uint64_t fend = (p + 661u + ZF_FILL + 3u) & ~3ull;
  for (uint32_t i = lane; i < ZF_RING_WORDS; i += WAVE) {
    const bool neg = fend < 32768u && 4ull * i < 32768u - fend;  // before the input: never read
    const uint64_t pos = fend + 4ull * i - 32768u;
    s_ring[(uint32_t)(pos >> 2) & (ZF_RING_WORDS - 1u)] = neg ? 0u : X.ld4(pos);
  }
  __builtin_amdgcn_wave_barrier();
  while (p < L && !stop) {
    sweep_to(p);
    ZF_T(0);
    Wn.lo = fend < 32768u ? 0u : fend - 32768u;
    const bool refill = fend - p < 661u + ZF_FILL;
    uint32_t fw[ZF_FILL / 4 / WAVE];
    if (refill) {
#pragma unroll
      for (uint32_t i = 0; i < ZF_FILL / 4 / WAVE; i++) fw[i] = X.ld4(fend + 4ull * (lane + WAVE * i));
    }
    const uint64_t q = p + lane;
    const bool insq = q + ZD_MINM <= L;  // zlib inserts and searches only with lookahead >= MIN_MATCH
    const uint32_t h = insq ? zf_hash3(Wn.rd4(q)) : 0u;
    const uint64_t same = zf_same(h, insq);
    const uint64_t below = same & ((1ull << lane) - 1ull);
    uint32_t mlen = 0, mdist = 0;
    ZF_T(1);
    if (insq) zf_search(Wn, X, s_prev, q, L, s_head[h], max_dist, nice, chain, mlen, mdist);
    ZF_T(2);
    // commit loop tops in order (wave-uniform): stop at the end, at a cut
    // job's first short lookahead, or at the first search an earlier inserted
    // position of this step invalidates.  The walk goes match to match: the
    // literal run before the next match start is committed at once (every
    // position of it is a loop top), its stops found by one ballot.
    const bool valid = q < L, cutq = cut && valid && L - q < ZD_LOOK;
    const bool ism = valid && mlen >= ZD_MINM;
    const bool shrtq = ism && mlen <= max_ins && L - (q + mlen) >= ZD_MINM;
    const uint64_t Mm = __ballot(ism), Im = __ballot(insq), Sm = __ballot(shrtq);
    const uint64_t lt_me = (1ull << lane) - 1ull;
    auto below_from = [](uint32_t a) -> uint64_t { return a >= 64u ? ~0ull : ((1ull << a) - 1ull); };
    uint32_t t = 0;
    uint64_t insm = 0, tokm = 0;
    while (t < WAVE) {
      const uint64_t from_t = ~below_from(t);
      const uint64_t mt = Mm & from_t;
      const uint32_t m = mt ? (uint32_t)__builtin_ctzll(mt) : WAVE;  // next match start (WAVE: none)
      // loop tops t .. m (m included when < WAVE): any stop among them?
      const uint64_t run = from_t & below_from(m + 1u);
      const bool inrun = (run >> lane) & 1ull;
      const bool conf = (below & (insm | (Im & run & lt_me))) != 0ull;
      const uint64_t stops = __ballot(inrun && (!valid || cutq || conf));
      const uint64_t lits = from_t & below_from(m);  // the literal loop tops t .. m - 1
      if (stops) {
        const uint32_t x = (uint32_t)__builtin_ctzll(stops);
        const uint64_t done = lits & below_from(x);
        tokm |= done;
        insm |= Im & done;
        stop = stop || (((__ballot(cutq) >> x) & 1ull) && p + x < L);
        t = x;
        break;
      }
      tokm |= lits;
      insm |= Im & lits;
      if (m >= WAVE) {
        t = WAVE;
        break;
      }
      const uint32_t lm = __builtin_amdgcn_readlane(mlen, m);
      const bool shrt = (Sm >> m) & 1ull;
      if (shrt && m + lm > WAVE) {  // its inner inserts would pass this step
        t = m;
        break;
      }
      tokm |= 1ull << m;
      if (shrt) insm |= below_from(lm) << m;
      else insm |= Im & (1ull << m);
      t = m + lm;
    }
    ZF_T(3);
    const bool tok = (tokm >> lane) & 1ull, ins = (insm >> lane) & 1ull;
    if (tok && mlen >= ZD_MINM) om[q] = mlen | (mdist << 9);
    if (lane < 3) {  // token starts and insertion bits of [p, p + 64): three words
      const uint32_t sh = (uint32_t)(p & 31u);
      const uint64_t w0 = p >> 5;
      const uint32_t k = lane;
      uint32_t vs, vi;
      if (k == 0) {
        vs = (uint32_t)(tokm << sh);
        vi = (uint32_t)(insm << sh);
      } else if (k == 1) {
        vs = (uint32_t)(sh ? (tokm >> (32 - sh)) : (tokm >> 32));
        vi = (uint32_t)(sh ? (insm >> (32 - sh)) : (insm >> 32));
      } else {
        vs = sh ? (uint32_t)(tokm >> (64 - sh)) : 0u;
        vi = sh ? (uint32_t)(insm >> (64 - sh)) : 0u;
      }
      if (vs) atomicOr(&B.S[w0 + k], vs);
      if (vi) atomicOr(&B.I[w0 + k], vi);
    }
    zf_insert(s_head, s_prev, q, h, ins, same, lane);
    if (refill) {
#pragma unroll
      for (uint32_t i = 0; i < ZF_FILL / 4 / WAVE; i++)
        s_ring[(uint32_t)((fend >> 2) + lane + WAVE * i) & (ZF_RING_WORDS - 1u)] = fw[i];
      fend += ZF_FILL;
      __builtin_amdgcn_wave_barrier();
    }
    ZF_T(4);
#if ZF_PROF
    zsteps++;
#endif
    p += t;
  }
#if ZF_PROF
  if (lane == 0)
    printf("zf job %u L=%lu pstart %lu history clk %lu steps %lu pos/step %.1f clk/step: sweep %lu hash+same %lu search %lu commit %lu out+ins %lu\n",
           blockIdx.x, (unsigned long)L, (unsigned long)jb.pstart, (unsigned long)zhist, (unsigned long)zsteps,
           (double)(p - jb.pstart) / (double)(zsteps ? zsteps : 1),
           (unsigned long)(zt[0] / (zsteps ? zsteps : 1)), (unsigned long)(zt[1] / (zsteps ? zsteps : 1)),
           (unsigned long)(zt[2] / (zsteps ? zsteps : 1)), (unsigned long)(zt[3] / (zsteps ? zsteps : 1)),
           (unsigned long)(zt[4] / (zsteps ? zsteps : 1)));
#endif
  if (lane == 0) jobs[blockIdx.x].cut_pos = p;  // where the parse stopped (zs_zd_cut_kernel)
}

// ---------------------------------------------------------------------------
// K4: blocks.  Symbols per region, then per job a prefix over regions and
// the block list: block k holds symbols [16383 k, 16383 k + 16383); the last
// one the rest -- or none, when a symbol of deflate_slow's loop filled the
// previous block exactly (its pending final literal is tallied without a
// flush check, trees.c _tr_tally + deflate.c FLUSH_BLOCK(s, 1)).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) zs_zd_count_kernel(const ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                           const uint32_t *__restrict__ bm) {
  __shared__ uint32_t s_red[4];
  const uint32_t t = threadIdx.x;
  const ZsDSegDev sg = segs[blockIdx.x];
  const ZsDJobDev jb = jobs[sg.job];
  if (!jb.exact) return;
  const uint32_t *S = bm + jb.bm0;
  const uint64_t w0 = sg.start / 32u;
  const uint32_t nw = (uint32_t)((sg.len + 31u) / 32u);
  uint32_t c = 0;
  for (uint32_t k = t; k < nw; k += 256) c += (uint32_t)__builtin_popcount(S[w0 + k]);
  for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
  if ((t & 63) == 0) s_red[t / 64] = c;
  __syncthreads();
  if (t == 0) segs[blockIdx.x].nsym = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

// zlib's window slides at a loop top t when the lookahead is short of
// MIN_LOOKAHEAD and strstart >= wsize + MAX_DIST (deflate.c fill_window):
// the slides done by loop top t of an L-byte input
__device__ __forceinline__ uint64_t zd_slides(uint64_t t, uint64_t L, uint64_t wsize, uint64_t max_dist) {
  uint64_t k = 0;
  for (;;) {
    const uint64_t base = k * wsize;
    const uint64_t wend = min(L, base + 2 * wsize);
    if (t >= base && wend - min(wend, t) < ZD_LOOK && t - base >= wsize + max_dist) k++;
    else return k;
  }
}

// position of symbol number `sym` of a job (sym < its symbol count)
__device__ uint64_t zd_sym_pos(const ZsDSegDev *segs, const ZsDJobDev &jb, const uint32_t *S, uint64_t sym) {
  // region: last one whose sym0 <= sym (binary search over the job's regions)
  uint32_t lo = 0, hi = jb.nseg - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) / 2;
    if (segs[jb.seg0 + mid].sym0 <= sym) lo = mid;
    else hi = mid - 1;
  }
  const ZsDSegDev &sg = segs[jb.seg0 + lo];
  uint64_t rem = sym - sg.sym0;
  uint64_t w = sg.start / 32u;
  // 64 words (2 K positions) per iteration while the symbol lies past them:
  // 16 independent 16-byte loads in flight (a word at a time paid a memory
  // round trip per 32 positions -- the latency of a stream segment's blocks);
  // region words start 4-aligned and the bitmaps are padded past the input
  for (;;) {
    const uint4 *v = reinterpret_cast<const uint4 *>(S + w);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint4 x = v[i];
      c += (uint32_t)(__builtin_popcount(x.x) + __builtin_popcount(x.y) + __builtin_popcount(x.z) +
                      __builtin_popcount(x.w));
    }
    if (rem < c) break;
    rem -= c;
    w += 64;
  }
  for (;; w++) {
    const uint32_t x = S[w];
    const uint32_t c = (uint32_t)__builtin_popcount(x);
    if (rem < c) {
      uint32_t y = x;
      for (uint64_t k = 0; k < rem; k++) y &= y - 1u;
      return w * 32u + (uint32_t)__builtin_ctz(y);
    }
    rem -= c;
  }
}

// one workgroup per job: symbol prefix over regions, block count
__global__ void __launch_bounds__(1024) zs_zd_blocks_kernel(ZsDJobDev *__restrict__ jobs, ZsDSegDev *__restrict__ segs,
                                                             const uint32_t *__restrict__ bm) {
  __shared__ uint64_t s_sum[1024];
  const uint32_t t = threadIdx.x;
  const ZsDJobDev jb = jobs[blockIdx.x];
  if (!jb.exact) return;
  const uint32_t ns = jb.nseg, per = (ns + 1023) / 1024;
  const uint32_t k0 = min(ns, per * t), k1 = min(ns, per * (t + 1));
  uint64_t sum = 0;
  for (uint32_t k = k0; k < k1; k++) sum += segs[jb.seg0 + k].nsym;
  s_sum[t] = sum;
  __syncthreads();
  if (t == 0) {
    uint64_t acc = 0;
    for (uint32_t k = 0; k < 1024; k++) {
      const uint64_t x = s_sum[k];
      s_sum[k] = acc;
      acc += x;
    }
    const uint32_t *S = bm + jb.bm0;
    const uint64_t L = jb.in_len;
    const uint64_t eff = acc - min(acc, jb.skip);  // symbols of this job's blocks
    // deflate_slow tallies its pending last literal after the loop without a
    // flush check; deflate_fast tallies every symbol inside it
    const bool end_lit = jb.exact == ZD_SLOW && eff && zd_getbit(S, L - 1);
    const uint64_t nfull = eff / ZD_BLOCK;
    const bool empty_last = eff % ZD_BLOCK == 0 && !end_lit;
    // Z_FINISH flushes an empty last block; a flush mid-stream only a
    // non-empty one (deflate.c deflate_slow: `if (s->sym_next) FLUSH_BLOCK(s, 0)`)
    jobs[blockIdx.x].nzblk =
        (uint32_t)(empty_last ? nfull + (jb.term == ZS_DT_FINAL ? 1u : 0u) : (eff + ZD_BLOCK - 1) / ZD_BLOCK);
    s_sum[1023] = s_sum[1023];  // keep the scan in LDS
  }
  __syncthreads();
  uint64_t off = s_sum[t];
  for (uint32_t k = k0; k < k1; k++) {
    segs[jb.seg0 + k].sym0 = off;
    off += segs[jb.seg0 + k].nsym;
  }
}

// one thread per block slot: byte range, BFINAL, stored eligibility
__global__ void zs_zd_blist_kernel(const ZsDJobDev *__restrict__ jobs, uint32_t njobs, const ZsDSegDev *__restrict__ segs,
                                   const uint32_t *__restrict__ bm, ZsZBlkDev *__restrict__ blks, uint32_t nslots,
                                   const uint32_t *__restrict__ slot_job) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nslots) return;
  const uint32_t j = slot_job[i];
  const ZsDJobDev jb = jobs[j];
  const uint32_t k = i - jb.zblk0;
  ZsZBlkDev b{};
  b.job = j;
  if (!jb.exact || k >= jb.nzblk) {
    b.nsym = 0xffffffffu;  // unused slot
    blks[i] = b;
    return;
  }
  const uint32_t *S = bm + jb.bm0;
  const uint64_t L = jb.in_len;
  const ZsDSegDev &lastseg = segs[jb.seg0 + jb.nseg - 1];
  const uint64_t ns = lastseg.sym0 + lastseg.nsym;
  const uint64_t s0 = jb.skip + (uint64_t)k * ZD_BLOCK;
  const uint64_t s1 = min(ns, s0 + ZD_BLOCK);
  const bool final_blk = k + 1 == jb.nzblk;
  b.last = final_blk && jb.term == ZS_DT_FINAL;
  b.nsym = (uint32_t)(s1 > s0 ? s1 - s0 : 0);
  b.first = b.nsym ? zd_sym_pos(segs, jb, S, s0) : L;
  b.end = s1 < ns ? zd_sym_pos(segs, jb, S, s1) : L;
  // deflate_slow flushes in the iteration whose loop top followed the block's
  // last symbol start, deflate_fast in that symbol's own iteration; the last
  // block of a flushed job flushes after the loop (top = L)
  uint64_t top = L;
  if (b.nsym && (!final_blk || jb.term == ZS_DT_CUT)) {
    uint64_t x = b.end - 1;
    while (!zd_getbit(S, x)) x--;
    top = jb.exact == ZD_FAST ? x : x + 1;
  }
  b.top = top;
  // window slides counted in stream positions since zlib's window last restarted
  const uint64_t wsize = 1ull << jb.wbits;
  b.stored_ok = jb.abs0 + b.first >= zd_slides(jb.abs0 + top, jb.abs0 + L, wsize, wsize - ZD_LOOK) * wsize;
  blks[i] = b;
}

// symbols whose start lies in [0, y) (regions' symbol prefix, then the start
// bitmap of y's region)
__device__ uint64_t zd_syms_before(const ZsDSegDev *segs, const ZsDJobDev &jb, const uint32_t *S, uint64_t y) {
  if (y >= jb.in_len) {
    const ZsDSegDev &l = segs[jb.seg0 + jb.nseg - 1];
    return l.sym0 + l.nsym;
  }
  const ZsDSegDev &sg = segs[jb.seg0 + (uint32_t)(y / ZD_REG)];
  uint64_t c = sg.sym0;
  uint64_t w = sg.start / 32u;
  for (; (w + 64) * 32u <= y; w += 64) {  // 64 words per iteration (see zd_sym_pos)
    const uint4 *v = reinterpret_cast<const uint4 *>(S + w);
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint4 x = v[i];
      c += (uint64_t)(__builtin_popcount(x.x) + __builtin_popcount(x.y) + __builtin_popcount(x.z) + __builtin_popcount(x.w));
    }
  }
  for (; (w + 1) * 32u <= y; w++) c += (uint64_t)__builtin_popcount(S[w]);
  if (y & 31u) c += (uint64_t)__builtin_popcount(S[w] & ((1u << (y & 31u)) - 1u));
  return c;
}

// ZS_DT_CUT jobs (Z_NO_FLUSH calls of a stream), one thread per job: zlib
// processes loop tops t while the lookahead in_len - t >= MIN_LOOKAHEAD, so
// the blocks it completes are the leading full blocks whose flush loop top
// is <= in_len - 262; only those are emitted.  The next segment restarts at
// the last region exit at or before the first unsent symbol whose walk saw
// full lookahead (an exact loop top and state, from the fix-up), with the
// symbols from there to the first unsent one as its skip; with none, at this
// job's own entry.
// where the next segment of a stream resumes when the first K blocks of job
// jb (nb of them parsed) are sent: a loop top T in state sT with `skip`
// symbols from T already sent (deflate_slow: the last region exit at or before
// the first unsent symbol whose walk saw full lookahead, from the fix-up; with
// none, the job's own entry)
__device__ void zd_cut_at(const ZsDJobDev &jb, uint32_t nb, uint32_t K, const ZsDSegDev *__restrict__ segs,
                          const uint32_t *__restrict__ S, const ZsZBlkDev *__restrict__ blks, uint64_t *T_out,
                          uint32_t *sT_out, uint64_t *skip_out) {
  const uint64_t L = jb.in_len;
  if (jb.exact == ZD_FAST) {  // every token start is a loop top: restart at the first unsent symbol
    *T_out = K < nb ? blks[jb.zblk0 + K].first : jb.fstop;
    *sT_out = ZD_STATE_A;
    *skip_out = 0;
    return;
  }
  uint64_t T = jb.pstart, sT = jb.pstate, skip = jb.skip + (uint64_t)K * ZD_BLOCK;
  if (K < nb) {
    const uint64_t P0 = blks[jb.zblk0 + K].first;
    for (int32_t r = (int32_t)min<uint64_t>(jb.nseg - 1, P0 / ZD_REG); r >= 0; r--) {
      const ZsDSegDev &sg = segs[jb.seg0 + r];
      const uint64_t x = sg.zx[0];
      const uint32_t xs = sg.zs[0];
      if (sg.start + sg.len + ZD_LOOK + ZD_MAXM <= L && x - (xs & 1u) <= P0 && x >= jb.pstart) {
        T = x;
        sT = xs;
        skip = jb.skip + (uint64_t)K * ZD_BLOCK - zd_syms_before(segs, jb, S, x - (xs & 1u));
        break;
      }
    }
  }
  *T_out = T;
  *sT_out = (uint32_t)sT;
  *skip_out = skip;
}

__global__ void zs_zd_cut_kernel(ZsDJobDev *__restrict__ jobs, uint32_t njobs, const ZsDSegDev *__restrict__ segs,
                                 const uint32_t *__restrict__ bm, ZsZBlkDev *__restrict__ blks) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  const ZsDJobDev jb = jobs[j];
  if (!jb.exact) return;
  jobs[j].nzblk0 = jb.nzblk;
  if (jb.exact == ZD_FAST) jobs[j].fstop = jb.cut_pos;
  if (jb.term != ZS_DT_CUT) return;
  const uint32_t *S = bm + jb.bm0;
  const uint64_t L = jb.in_len;
  if (jb.exact == ZD_FAST) {
    // deflate_fast stopped at its first loop top with a short lookahead
    // (jb.cut_pos, zs_zd_fast_kernel): every symbol before it is tallied and
    // its full blocks are sent.  Every token start is a loop top, so the next
    // segment restarts at the first unsent symbol with nothing to skip (its
    // hash chains rebuilt from the insertion bits before it).
    uint32_t K = 0;
    while (K < jb.nzblk && blks[jb.zblk0 + K].nsym == ZD_BLOCK) K++;
    const ZsDSegDev &ls = segs[jb.seg0 + jb.nseg - 1];
    const uint64_t done = ls.sym0 + ls.nsym;
    for (uint32_t k = K; k < jb.nzblk; k++) blks[jb.zblk0 + k].nsym = 0xffffffffu;
    jobs[j].cut_open = done - (uint64_t)K * ZD_BLOCK;
    jobs[j].cut_pos = K < jb.nzblk ? blks[jb.zblk0 + K].first : jb.cut_pos;
    jobs[j].nzblk = K;
    jobs[j].cut_state = ZD_STATE_A;
    jobs[j].cut_skip = 0;
    return;
  }
  uint32_t K = 0;
  while (K < jb.nzblk && blks[jb.zblk0 + K].nsym == ZD_BLOCK && blks[jb.zblk0 + K].top + ZD_LOOK <= L) K++;
  uint64_t T = jb.pstart, sT = jb.pstate, skip = jb.skip + (uint64_t)K * ZD_BLOCK;
  if (K < jb.nzblk) {
    const uint64_t P0 = blks[jb.zblk0 + K].first;
    for (int32_t r = (int32_t)min<uint64_t>(jb.nseg - 1, P0 / ZD_REG); r >= 0; r--) {
      const ZsDSegDev &sg = segs[jb.seg0 + r];
      const uint64_t x = sg.zx[0];
      const uint32_t xs = sg.zs[0];
      if (sg.start + sg.len + ZD_LOOK + ZD_MAXM <= L && x - (xs & 1u) <= P0 && x >= jb.pstart) {
        T = x;
        sT = xs;
        skip = jb.skip + (uint64_t)K * ZD_BLOCK - zd_syms_before(segs, jb, S, x - (xs & 1u));
        break;
      }
    }
  }
  // symbols zlib has tallied by its last loop top (a token at x is tallied at x + 1)
  const uint64_t done = L >= ZD_LOOK ? zd_syms_before(segs, jb, S, L - ZD_LOOK) : 0;
  const uint64_t sent = jb.skip + (uint64_t)K * ZD_BLOCK;
  for (uint32_t k = K; k < jb.nzblk; k++) blks[jb.zblk0 + k].nsym = 0xffffffffu;  // not sent by this call
  jobs[j].cut_open = done > sent ? done - sent : 0;
  jobs[j].nzblk = K;
  jobs[j].cut_pos = T;
  jobs[j].cut_state = (uint32_t)sT;
  jobs[j].cut_skip = skip;
}

// first loop top at or after y of the job's parse (L if none).  deflate_slow
// (zlib deflate.c): a literal or match starting at s is tallied in the
// iteration at s + 1 and an emitted match moves the loop to its end, so the
// loop tops are {y : y - 1 or y is a token start}.  deflate_fast: the token
// starts (its CUT jobs know them up to fstop, their stop).
__device__ uint64_t zd_looptop_ge(const ZsDJobDev &jb, const uint32_t *__restrict__ S, uint64_t y) {
  const uint64_t L = jb.in_len;
  const bool fast = jb.exact == ZD_FAST;
  const uint64_t lim = fast && jb.term == ZS_DT_CUT ? min(L, jb.fstop) : L;
  if (y >= lim) return fast ? max(y, lim) : L;
  if (!fast && y > 0 && zd_getbit(S, y - 1)) return y;
  uint64_t w = y >> 5;
  uint32_t m = S[w] & (~0u << (y & 31u));
  while (!m) {
    if (++w * 32u >= lim) return lim;
    m = S[w];
  }
  return min(lim, w * 32u + (uint64_t)__builtin_ctz(m));
}

// zlib's reading during one deflate() call up to loop top t_lim (fill_window at
// every loop top whose lookahead is < MIN_LOOKAHEAD: slide by w_size once
// strstart - window start >= w_size + MAX_DIST, then read up to window_size);
// returns the read end (job offset) and moves *zb (stream offset).  A call that
// runs out of input stops at its first loop top with a short lookahead (NO_FLUSH,
// zs_zd_cut_kernel's rule) or processes every loop top to the end (a flush),
// attempting the fill (so the slide) at each.
__device__ uint64_t zd_read_model(const ZsDJobDev &jb, const uint32_t *__restrict__ S, uint64_t t_lim, bool early,
                                  uint64_t *zb_io) {
  const uint64_t L = jb.in_len, W = 1ull << jb.wbits, TH = 2 * W - ZD_LOOK, a0 = jb.abs0;
  uint64_t zb = *zb_io, rd = jb.rd0, lo = 0;
  if (jb.rtop == ~0ull) {
    rd = min(L, zb + 2 * W - a0);  // the fill at the call's first loop top (its slide already decided)
  } else {
    lo = jb.rtop;
    if (rd - min(rd, jb.rtop) < ZD_LOOK && jb.rtop <= t_lim) {
      if (a0 + jb.rtop >= zb + TH) zb += W;
      rd = min(L, zb + 2 * W - a0);
    }
  }
  for (int guard = 0; guard < (1 << 20); guard++) {
    const uint64_t y = max(lo, rd >= ZD_LOOK - 1 ? rd - (ZD_LOOK - 1) : 0ull);
    const uint64_t t = zd_looptop_ge(jb, S, y);
    if (t > t_lim) break;
    if (rd < L) {
      if (a0 + t >= zb + TH) zb += W;
      rd = min(L, zb + 2 * W - a0);
      lo = t + 1;
      continue;
    }
    // no input left: fill attempts (slide checks) at every loop top from t on
    const uint64_t tc = early ? t_lim : (jb.term == ZS_DT_CUT ? t : L);
    if (a0 + tc >= zb + TH) zb += W;
    break;
  }
  *zb_io = zb;
  return rd;
}

// zlib's pull-on-demand (after the layout: block bit ends are known): the
// first block whose flush leaves at least lim_bytes of the job's output makes
// deflate() return right there -- blocks flushed inside the loop (all of a
// CUT job's, all but the last of a flushing job's).  The job then ends as a
// CUT after that block (no terminator, no trailer), resuming where the next
// loop top is, and the read model gives what zlib had read.
__global__ void zs_zd_limit_kernel(ZsDJobDev *__restrict__ jobs, uint32_t njobs, const ZsDSegDev *__restrict__ segs,
                                   const uint32_t *__restrict__ bm, const ZsZBlkDev *__restrict__ blks) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  const ZsDJobDev jb = jobs[j];
  if (!jb.exact || jb.rd0 == ~0ull) return;  // not a stream segment (the batch API)
  const uint32_t *S = bm + jb.bm0;
  const uint32_t nb = jb.nzblk;
  uint32_t stop = 0xffffffffu;
  if (jb.lim_bytes != ~0ull) {
    const uint32_t ncand = jb.term == ZS_DT_CUT ? nb : (nb ? nb - 1u : 0u);
    for (uint32_t i = 0; i < ncand; i++) {
      const uint64_t e = i + 1 < nb ? blks[jb.zblk0 + i + 1].bitoff : jb.endbit;
      if (e / 8u >= jb.lim_bytes) {
        stop = i;
        break;
      }
    }
  }
  uint64_t zb = jb.zb;
  if (stop == 0xffffffffu) {
    jobs[j].early = 0;
    jobs[j].rd_out = zd_read_model(jb, S, jb.in_len, false, &zb);
    jobs[j].zb = zb;
    return;
  }
  const ZsZBlkDev &b = blks[jb.zblk0 + stop];
  const uint64_t t_i = b.top;
  jobs[j].early = 1;
  jobs[j].early_k = stop + 1;
  jobs[j].rd_out = zd_read_model(jb, S, t_i, true, &zb);
  jobs[j].zb = zb;
  jobs[j].next_top = zd_looptop_ge(jb, S, t_i + 1);
  jobs[j].endbit = stop + 1 < nb ? blks[jb.zblk0 + stop + 1].bitoff : jb.endbit;
  jobs[j].term = ZS_DT_CUT;
  jobs[j].trl = 0;
  jobs[j].total_out = (jobs[j].endbit + 7u) / 8u;
  uint64_t T, skip;
  uint32_t sT;
  zd_cut_at(jb, jb.nzblk0, stop + 1, segs, S, blks, &T, &sT, &skip);
  jobs[j].cut_pos = T;
  jobs[j].cut_state = sT;
  jobs[j].cut_skip = skip;
  jobs[j].cut_open = 0;
  jobs[j].nzblk = stop + 1;
}

// ---------------------------------------------------------------------------
// K4c: one workgroup per block: symbol frequencies, then (thread 0) the trees
// and the choice of _tr_flush_block, restated from trees.c:
//   build_tree   -- leaves in a heap ordered by (freq, depth), two nodes
//                   joined per step, a third parent numbered from `elems`;
//   gen_bitlen   -- lengths from the root down, overflow past max_length
//                   repaired by moving leaves as zlib does;
//   gen_codes    -- canonical codes (bit-reversed here for LSB-first output);
//   build_bl_tree / scan_tree -- the code-length code;
// opt_len / static_len accumulate exactly as zlib's (including its forced
// second leaf), so the stored / static / dynamic choice is zlib's.
// ---------------------------------------------------------------------------
#define ZD_HEAP 573
#define ZD_TT 256

__constant__ uint8_t zd_xl[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint8_t zd_xd[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t zd_xb[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
__constant__ uint8_t zd_blord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ uint32_t zd_lcode(uint32_t len) {  // 3..258 -> 0..28
  if (len == 258) return 28;
  const uint32_t l = len - 3;
  if (l < 8) return l;
  const uint32_t e = 29u - (uint32_t)__builtin_clz(l);
  return 4 * (e + 1) + ((l >> e) & 3u);
}
__device__ __forceinline__ uint32_t zd_lbase(uint32_t c) { return c == 28 ? 258u : c < 8 ? c + 3 : ((4u + (c & 3u)) << (c / 4 - 1)) + 3u; }
__device__ __forceinline__ uint32_t zd_dcode(uint32_t d) {  // 1..32768 -> 0..29
  const uint32_t x = d - 1;
  if (x < 4) return x;
  const uint32_t e = 30u - (uint32_t)__builtin_clz(x);
  return 2 * (e + 1) + ((x >> e) & 1u);
}
__device__ __forceinline__ uint32_t zd_dbase(uint32_t c) { return c < 4 ? c + 1 : ((2u + (c & 1u)) << (c / 2 - 1)) + 1u; }
__device__ __forceinline__ uint32_t zd_rev(uint32_t c, uint32_t n) { return __builtin_bitreverse32(c) >> (32u - n); }

struct ZdTreeLDS {
  uint32_t freq[ZD_HEAP];
  uint16_t dl[ZD_HEAP];  // parent while building, then code length (zlib's Dad / Len union)
  uint8_t depth[ZD_HEAP];
  int16_t heap[ZD_HEAP];  // the nodes in extraction order (heap[heap_max..])
  uint64_t hk[ZD_HEAP];   // the live heap: (freq << 8 | depth) << 10 | node
  uint16_t blc[16];
  uint32_t next[16];      // gen_codes' next code per length
  uint32_t blf[19];       // bit-length code frequencies (scan_tree)
};

// trees.c tr_static_init's static code lengths: literal/length (kind 1) 8 / 9 /
// 7 / 8 by symbol range, distance (kind 2) 5 -- computed, not a private array
// (dynamically indexed private arrays live in scratch memory)
__device__ __forceinline__ uint32_t zd_stat_len(int kind, int n) {
  return kind == 2 ? 5u : (n < 144 ? 8u : n < 256 ? 9u : n < 280 ? 7u : 8u);
}

// zlib's smaller(): freq, then depth, as one key -- the heap holds its
// entries' keys, so a sift level is one LDS round trip (two children), not
// two (the children, then their freq and depth)
__device__ __forceinline__ uint64_t zd_key(const ZdTreeLDS &w, int n) {
  return ((uint64_t)((w.freq[n] << 8) | w.depth[n]) << 10) | (uint64_t)n;
}
__device__ void zd_sift(ZdTreeLDS &w, int hl, int k) {
  const uint64_t v = w.hk[k];
  for (int j = k << 1; j <= hl; j <<= 1) {
    uint64_t a = w.hk[j];
    if (j < hl) {
      const uint64_t b = w.hk[j + 1];
      if ((b >> 10) <= (a >> 10)) {
        j++;
        a = b;
      }
    }
    if ((v >> 10) <= (a >> 10)) break;
    w.hk[k] = a;
    k = j;
  }
  w.hk[k] = v;
}

// freq[0..elems) in w.freq; lens out in len_out[0..elems), canonical LSB-first
// codes in code_out; returns max_code.  stat: static lengths (nullptr: none).
__device__ int zd_build(ZdTreeLDS &w, int elems, int stat, const uint8_t *xb, int xbase, int maxlen,
                        uint64_t &opt_len, uint64_t &static_len, uint16_t *len_out, uint16_t *code_out) {
  int max_code = -1, hl = 0, hmax = ZD_HEAP;
  for (int n = 0; n < elems; n++) {
    if (w.freq[n]) {
      max_code = n;
      w.depth[n] = 0;
      w.hk[++hl] = zd_key(w, n);
    } else {
      w.dl[n] = 0;
    }
  }
  while (hl < 2) {
    const int node = max_code < 2 ? ++max_code : 0;
    w.freq[node] = 1;
    w.depth[node] = 0;
    w.hk[++hl] = zd_key(w, node);
    opt_len--;
    if (stat) static_len -= zd_stat_len(stat, node);
  }
  for (int n = hl / 2; n >= 1; n--) zd_sift(w, hl, n);
  int node = elems;
  do {
    const int n = (int)(w.hk[1] & 1023u);
    w.hk[1] = w.hk[hl--];
    zd_sift(w, hl, 1);
    const int m = (int)(w.hk[1] & 1023u);
    w.heap[--hmax] = (int16_t)n;
    w.heap[--hmax] = (int16_t)m;
    w.freq[node] = w.freq[n] + w.freq[m];
    w.depth[node] = (uint8_t)((w.depth[n] >= w.depth[m] ? w.depth[n] : w.depth[m]) + 1);
    w.dl[n] = w.dl[m] = (uint16_t)node;
    w.hk[1] = zd_key(w, node++);
    zd_sift(w, hl, 1);
  } while (hl >= 2);
  w.heap[--hmax] = (int16_t)(w.hk[1] & 1023u);
  for (int b = 0; b < 16; b++) w.blc[b] = 0;
  w.dl[w.heap[hmax]] = 0;
  int overflow = 0, h;
  for (h = hmax + 1; h < ZD_HEAP; h++) {
    const int n = w.heap[h];
    int bits = w.dl[w.dl[n]] + 1;
    if (bits > maxlen) bits = maxlen, overflow++;
    w.dl[n] = (uint16_t)bits;
    if (n > max_code) continue;
    w.blc[bits]++;
    const int x = n >= xbase ? xb[n - xbase] : 0;
    opt_len += (uint64_t)w.freq[n] * (uint64_t)(bits + x);
    if (stat) static_len += (uint64_t)w.freq[n] * (uint64_t)(zd_stat_len(stat, n) + x);
  }
  if (overflow) {
    do {
      int bits = maxlen - 1;
      while (w.blc[bits] == 0) bits--;
      w.blc[bits]--;
      w.blc[bits + 1] += 2;
      w.blc[maxlen]--;
      overflow -= 2;
    } while (overflow > 0);
    for (int bits = maxlen; bits != 0; bits--) {
      int n = w.blc[bits];
      while (n != 0) {
        const int m = w.heap[--h];
        if (m > max_code) continue;
        if (w.dl[m] != bits) {
          opt_len += ((uint64_t)bits - w.dl[m]) * w.freq[m];
          w.dl[m] = (uint16_t)bits;
        }
        n--;
      }
    }
  }
  uint32_t code = 0;
  for (int b = 1; b <= 15; b++) w.next[b] = code = (code + w.blc[b - 1]) << 1;
  for (int n = 0; n < elems; n++) {
    const uint32_t len = n <= max_code ? w.dl[n] : 0u;
    len_out[n] = (uint16_t)len;
    code_out[n] = len ? (uint16_t)zd_rev(w.next[len]++, len) : (uint16_t)0;
  }
  return max_code;
}

// run-length coding of a code-length array (scan_tree / send_tree): mode 0
// counts into freq[], mode 1 returns the bits it would send with (bl_len, bl_code)
template <typename Emit>
__device__ void zd_rle(const uint16_t *lens, int max_code, Emit emit) {
  int prevlen = -1, nextlen = lens[0], count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) max_count = 138, min_count = 3;
  for (int n = 0; n <= max_code; n++) {
    const int curlen = nextlen;
    nextlen = n + 1 <= max_code ? lens[n + 1] : 0xffff;
    if (++count < max_count && curlen == nextlen) continue;
    if (count < min_count) {
      for (; count; count--) emit(curlen, 0u, 0u);
    } else if (curlen != 0) {
      if (curlen != prevlen) {
        emit(curlen, 0u, 0u);
        count--;
      }
      emit(16, (uint32_t)count - 3u, 2u);
    } else if (count <= 10) {
      emit(17, (uint32_t)count - 3u, 3u);
    } else {
      emit(18, (uint32_t)count - 11u, 7u);
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) max_count = 138, min_count = 3;
    else if (curlen == nextlen) max_count = 6, min_count = 3;
    else max_count = 7, min_count = 4;
  }
}

// token at position q (S bit set): literal, or match (len, dist) from its table
struct ZdTok {
  uint32_t len;  // 0: literal
  uint32_t dist;
  uint32_t lit;
};
__device__ __forceinline__ ZdTok zd_tok(const ZdTabs &T, const ZdBm &B, uint64_t q) {
  ZdTok k;
  const bool lit = q + 1 >= T.L || zd_getbit(B.S, q + 1);
  if (lit) {
    k.len = 0;
    k.dist = 0;
    k.lit = T.in[q];
  } else {
    const uint32_t m = (zd_getbit(B.V, q) ? T.mb : T.ma)[q];
    k.len = m & 511u;
    k.dist = m >> 9;
    k.lit = 0;
  }
  return k;
}

// f(token) for every token start in [q0, q1), in order: the start bitmap is
// read a word at a time and walked by its set bits (a per-position test read
// a bitmap word per input byte)
template <typename F>
__device__ __forceinline__ void zd_for_tokens(const ZdTabs &T, const ZdBm &B, uint64_t q0, uint64_t q1, F f) {
  for (uint64_t wq = q0 & ~31ull; wq < q1; wq += 32) {
    uint32_t sw = B.S[wq >> 5];
    if (wq < q0) sw &= ~0u << (q0 - wq);
    if (q1 - wq < 32) sw &= (1u << (q1 - wq)) - 1u;
    if (!sw) continue;
    const uint32_t s_all = B.S[wq >> 5], s_next = B.S[(wq >> 5) + 1], vw = B.V[wq >> 5];
    while (sw) {
      const uint32_t b = (uint32_t)__builtin_ctz(sw);
      sw &= sw - 1u;
      const uint64_t q = wq + b;
      const bool next_start = b < 31 ? ((s_all >> (b + 1)) & 1u) : (s_next & 1u);
      ZdTok k;
      if (q + 1 >= T.L || next_start) {  // as zd_tok
        k.len = 0;
        k.dist = 0;
        k.lit = T.in[q];
      } else {
        const uint32_t m = ((vw >> b) & 1u ? T.mb : T.ma)[q];
        k.len = m & 511u;
        k.dist = m >> 9;
        k.lit = 0;
      }
      f(k);
    }
  }
}

// per-block tables in global memory (ZD_AUX words): [0, 286) lit/len code |
// len << 16, [286, 316) distance, [316, 335) bit-length code
__global__ void __launch_bounds__(ZD_TT) zs_zd_tree_kernel(const ZsDJobDev *__restrict__ jobs, ZsZBlkDev *__restrict__ blks,
                                                            const uint32_t *__restrict__ ma, const uint32_t *__restrict__ mb,
                                                            uint32_t *__restrict__ bm, uint32_t *__restrict__ aux) {
  __shared__ uint32_t s_lf[288], s_df[32];
  __shared__ ZdTreeLDS W;
  __shared__ uint16_t s_ll[288], s_lc[288], s_dlen[32], s_dc[32], s_bl[19], s_bc[19];
  const uint32_t t = threadIdx.x;
  const ZsZBlkDev bk = blks[blockIdx.x];
  if (bk.nsym == 0xffffffffu) return;
  const ZsDJobDev jb = jobs[bk.job];
  ZdTabs T;
  T.ma = ma + jb.pos0;
  T.mb = mb + jb.pos0;
  T.in = jb.in;
  T.L = jb.in_len;
  const ZdBm B = zd_bm(bm, jb);
#ifndef ZD_TREE_PROF
#define ZD_TREE_PROF 0  // per-block phase clocks, printed for a few blocks (tools/build_variant.sh ... -DZD_TREE_PROF=1)
#endif
#if ZD_TREE_PROF
  const uint64_t tp0 = clock64();
#endif
  for (uint32_t i = t; i < 288; i += ZD_TT) s_lf[i] = 0;
  if (t < 32) s_df[t] = 0;
  __syncthreads();
  const uint64_t n = bk.end - bk.first, per = (n + ZD_TT - 1) / ZD_TT;
  const uint64_t q0 = bk.first + min(n, per * t), q1 = bk.first + min(n, per * (t + 1));
  zd_for_tokens(T, B, q0, q1, [&](const ZdTok &k) {
    if (!k.len) {
      atomicAdd(&s_lf[k.lit], 1u);
    } else {
      atomicAdd(&s_lf[257 + zd_lcode(k.len)], 1u);
      atomicAdd(&s_df[zd_dcode(k.dist)], 1u);
    }
  });
  __syncthreads();
  if (t != 0) return;
#if ZD_TREE_PROF
  const uint64_t tp1 = clock64();
#endif
  uint64_t opt = 0, stat = 0;
  for (int i = 0; i < ZD_HEAP; i++) W.freq[i] = i < 286 ? s_lf[i] : 0u;
  W.freq[256] = 1;  // end of block
  const int lmax = zd_build(W, 286, 1, zd_xl, 257, 15, opt, stat, s_ll, s_lc);
  for (int i = 0; i < ZD_HEAP; i++) W.freq[i] = i < 30 ? s_df[i] : 0u;
  const int dmax = zd_build(W, 30, 2, zd_xd, 0, 15, opt, stat, s_dlen, s_dc);
  for (int i = 0; i < 19; i++) W.blf[i] = 0;
  auto count = [&](int sym, uint32_t, uint32_t) { W.blf[sym]++; };
  zd_rle(s_ll, lmax, count);
  zd_rle(s_dlen, dmax, count);
  for (int i = 0; i < ZD_HEAP; i++) W.freq[i] = i < 19 ? W.blf[i] : 0u;
  uint64_t dummy = 0;
  (void)zd_build(W, 19, 0, zd_xb, 0, 7, opt, dummy, s_bl, s_bc);
  int blmax = 18;
  for (; blmax >= 3; blmax--)
    if (s_bl[zd_blord[blmax]] != 0) break;
  opt += 3 * ((uint64_t)blmax + 1) + 5 + 5 + 4;
  uint64_t opt_b = (opt + 3 + 7) >> 3;
  const uint64_t stat_b = (stat + 3 + 7) >> 3;
  if (stat_b <= opt_b) opt_b = stat_b;
  const uint64_t nbytes = bk.end - bk.first;
  ZsZBlkDev o = bk;
  o.lmax = (uint32_t)lmax;
  o.dmax = (uint32_t)dmax;
  o.blmax = (uint32_t)blmax;
  o.hbits = 0;
  // exact bits (zlib's opt_len counts its forced leaves; the stream does not)
  uint64_t body_dyn = 0, body_fix = 0;
  for (int i = 0; i < 286; i++) {
    const uint64_t f = s_lf[i] + (i == 256 ? 1u : 0u);
    const uint32_t x = i >= 257 ? zd_xl[i - 257] : 0u;
    body_dyn += f * (s_ll[i] + x);
    body_fix += f * (zd_stat_len(1, i) + x);
  }
  for (int i = 0; i < 30; i++) {
    body_dyn += (uint64_t)s_df[i] * (s_dlen[i] + zd_xd[i]);
    body_fix += (uint64_t)s_df[i] * (5u + zd_xd[i]);
  }
  if (nbytes + 4 <= opt_b && bk.stored_ok) {
    o.type = 0;
    o.bits = 32 + 8 * nbytes;  // + alignment, known at layout
  } else if (stat_b == opt_b) {
    o.type = 1;
    o.bits = body_fix;
  } else {
    o.type = 2;
    uint32_t hb = 5 + 5 + 4 + 3 * ((uint32_t)blmax + 1);
    auto bits = [&](int sym, uint32_t, uint32_t xn) { hb += s_bl[sym] + xn; };
    zd_rle(s_ll, lmax, bits);
    zd_rle(s_dlen, dmax, bits);
    o.hbits = hb;
    o.bits = hb + body_dyn;
  }
  blks[blockIdx.x] = o;
#if ZD_TREE_PROF
  if (blockIdx.x < 4)
    printf("zd_tree blk %u syms %lu type %u: count %lu cyc, build %lu cyc (lmax %d)\n", blockIdx.x, (unsigned long)n, o.type,
           (unsigned long)(tp1 - tp0), (unsigned long)(clock64() - tp1), lmax);
#endif
  uint32_t *ax = aux + (size_t)blockIdx.x * ZD_AUX;
  if (o.type == 1) {
    for (int i = 0; i < 286; i++) {
      const uint32_t L = zd_stat_len(1, i);
      uint32_t c;  // static code of symbol i (trees.c tr_static_init: canonical over 288 lengths)
      if (i < 144) c = 0x30 + i;
      else if (i < 256) c = 0x190 + (i - 144);
      else if (i < 280) c = i - 256;
      else c = 0xc0 + (i - 280);
      ax[i] = zd_rev(c, L) | (L << 16);
    }
    for (int i = 0; i < 30; i++) ax[286 + i] = zd_rev((uint32_t)i, 5) | (5u << 16);
  } else if (o.type == 2) {
    for (int i = 0; i < 286; i++) ax[i] = s_lc[i] | ((uint32_t)s_ll[i] << 16);
    for (int i = 0; i < 30; i++) ax[286 + i] = s_dc[i] | ((uint32_t)s_dlen[i] << 16);
    for (int i = 0; i < 19; i++) ax[316 + i] = s_bc[i] | ((uint32_t)s_bl[i] << 16);
  }
}

// ---------------------------------------------------------------------------
// K4d: one workgroup per job: block bit offsets.  A block takes 3 type bits
// plus its body; a stored block also aligns to a byte after the type bits
// (trees.c _tr_stored_block: bi_windup), so with stored blocks the offsets
// are summed in order by one thread.  Then the wrapper header and the check.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) zs_zd_layout_kernel(ZsDJobDev *__restrict__ jobs, ZsZBlkDev *__restrict__ blks,
                                                             uint8_t *__restrict__ stage) {
  __shared__ uint64_t s_sum[1024];
  __shared__ uint32_t s_stored;
  const uint32_t t = threadIdx.x;
  ZsDJobDev jb = jobs[blockIdx.x];
  if (!jb.exact) return;
  const uint32_t nb = jb.nzblk, per = (nb + 1023) / 1024;
  const uint32_t k0 = min(nb, per * t), k1 = min(nb, per * (t + 1));
  const uint32_t hdr = !jb.hdr ? 0u : jb.wrap == 2 ? 10u : (jb.wrap == 1 ? 2u : 0u);
  if (t == 0) s_stored = 0;
  __syncthreads();
  uint64_t sum = 0;
  bool stored = false;
  for (uint32_t k = k0; k < k1; k++) {
    const ZsZBlkDev &b = blks[jb.zblk0 + k];
    sum += 3 + b.bits;
    stored |= b.type == 0;
  }
  if (stored) atomicOr(&s_stored, 1u);
  s_sum[t] = sum;
  __syncthreads();
  uint64_t endbit = 0;
  if (!s_stored) {
    if (t == 0) {
      uint64_t acc = jb.bit0 + 8ull * hdr;
      for (uint32_t k = 0; k < 1024; k++) {
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
      blks[jb.zblk0 + k].bitoff = off;
      off += 3 + blks[jb.zblk0 + k].bits;
    }
  } else if (t == 0) {
    uint64_t off = jb.bit0 + 8ull * hdr;
    for (uint32_t k = 0; k < nb; k++) {
      ZsZBlkDev &b = blks[jb.zblk0 + k];
      b.bitoff = off;
      off += 3;
      if (b.type == 0) off = (off + 7) & ~7ull;
      off += b.bits;
    }
    endbit = off;
    jobs[blockIdx.x].endbit = endbit;
    jobs[blockIdx.x].total_out = zs_dz_total_bytes(jb, endbit);
  }
  if (t == 0) {
    jobs[blockIdx.x].check = jb.wrap == 2   ? zs_crc_final((uint32_t)jb.ck_a, jb.in_len - jb.ck0)
                             : jb.wrap == 1 ? zs_adler_final(jb.ck_a, jb.ck_b, jb.in_len - jb.ck0)
                                            : 0u;
  }
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

// ---------------------------------------------------------------------------
// K5: one workgroup per block: the bits.  Threads own contiguous position
// ranges; a count pass and a block scan give each its bit offset, then each
// writes its bits -- whole words with plain stores, its first and last
// partial words with atomicOr (the staging area is zeroed).
// ---------------------------------------------------------------------------
struct ZdBits {
  uint32_t *w;   // staging words
  uint64_t wi;   // current word
  uint64_t acc;  // pending bits, LSB first
  uint32_t n;    // pending bit count (first word: the bits before our start count as zeros)
  bool first;
  __device__ void init(uint32_t *base, uint64_t bit) {
    w = base;
    wi = bit >> 5;
    acc = 0;
    n = (uint32_t)(bit & 31u);
    first = true;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t nb) {
    acc |= (uint64_t)v << n;
    n += nb;
    if (n >= 32) {
      const uint32_t x = (uint32_t)acc;
      if (first) atomicOr(&w[wi], x);
      else w[wi] = x;
      first = false;
      wi++;
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ void done() {
    if (n) atomicOr(&w[wi], (uint32_t)acc);
  }
};

__global__ void __launch_bounds__(ZD_TT) zs_zd_emit_kernel(const ZsDJobDev *__restrict__ jobs, const ZsZBlkDev *__restrict__ blks,
                                                            const uint32_t *__restrict__ ma, const uint32_t *__restrict__ mb,
                                                            uint32_t *__restrict__ bm, const uint32_t *__restrict__ aux,
                                                            uint8_t *__restrict__ stage) {
  __shared__ uint32_t s_l[288], s_d[32];
  __shared__ uint64_t s_off[ZD_TT];
  const uint32_t t = threadIdx.x;
  const ZsZBlkDev bk = blks[blockIdx.x];
  if (bk.nsym == 0xffffffffu) return;
  const ZsDJobDev jb = jobs[bk.job];
  uint8_t *o8 = stage + jb.stage;  // 4 KiB aligned
  uint32_t *o32 = reinterpret_cast<uint32_t *>(o8);
  const uint64_t n = bk.end - bk.first;
  if (bk.type == 0) {  // stored: 3 type bits, align, LEN, NLEN, the bytes
    if (t == 0) {
      const uint64_t b = bk.bitoff;
      const uint64_t v = (uint64_t)bk.last << (b & 31u);
      if (v) {
        atomicOr(&o32[b >> 5], (uint32_t)v);
        if (v >> 32) atomicOr(&o32[(b >> 5) + 1], (uint32_t)(v >> 32));
      }
    }
    const uint64_t P = (bk.bitoff + 3 + 7) / 8;
    const uint32_t len = (uint32_t)n;
    if (t < 4) o8[P + t] = (uint8_t)((t < 2 ? len : ~len) >> (8 * (t & 1)));
    for (uint64_t i = t; i < n; i += ZD_TT) o8[P + 4 + i] = jb.in[bk.first + i];
    return;
  }
  const uint32_t *ax = aux + (size_t)blockIdx.x * ZD_AUX;
  for (uint32_t i = t; i < 286; i += ZD_TT) s_l[i] = ax[i];
  if (t < 30) s_d[t] = ax[286 + t];
  __syncthreads();
  ZdTabs T;
  T.ma = ma + jb.pos0;
  T.mb = mb + jb.pos0;
  T.in = jb.in;
  T.L = jb.in_len;
  const ZdBm B = zd_bm(bm, jb);
  const uint64_t per = (n + ZD_TT - 1) / ZD_TT;
  const uint64_t q0 = bk.first + min(n, per * t), q1 = bk.first + min(n, per * (t + 1));
  auto sym_bits = [&](const ZdTok &k) -> uint32_t {
    if (!k.len) return s_l[k.lit] >> 16;
    const uint32_t lc = zd_lcode(k.len), dc = zd_dcode(k.dist);
    return (s_l[257 + lc] >> 16) + zd_xl[lc] + (s_d[dc] >> 16) + zd_xd[dc];
  };
  uint64_t mine = t == 0 ? 3u + bk.hbits : 0u;
  zd_for_tokens(T, B, q0, q1, [&](const ZdTok &k) { mine += sym_bits(k); });
  if (t == ZD_TT - 1) mine += s_l[256] >> 16;  // end of block
  s_off[t] = mine;
  __syncthreads();
  if (t == 0) {
    uint64_t acc = bk.bitoff;
    for (uint32_t k = 0; k < ZD_TT; k++) {
      const uint64_t x = s_off[k];
      s_off[k] = acc;
      acc += x;
    }
  }
  __syncthreads();
  ZdBits W;
  W.init(o32, s_off[t]);
  if (t == 0) {
    W.put(bk.last | (bk.type << 1), 3);
    if (bk.type == 2) {
      W.put(bk.lmax + 1 - 257, 5);
      W.put(bk.dmax + 1 - 1, 5);
      W.put(bk.blmax + 1 - 4, 4);
      const uint32_t *bl = ax + 316;
      for (uint32_t r = 0; r <= bk.blmax; r++) W.put(bl[zd_blord[r]] >> 16, 3);
      uint16_t lens[286];
      auto send = [&](int sym, uint32_t xv, uint32_t xn) {
        W.put(bl[sym] & 0xffffu, bl[sym] >> 16);
        if (xn) W.put(xv, xn);
      };
      for (uint32_t i = 0; i <= bk.lmax; i++) lens[i] = (uint16_t)(s_l[i] >> 16);
      zd_rle(lens, (int)bk.lmax, send);
      for (uint32_t i = 0; i <= bk.dmax; i++) lens[i] = (uint16_t)(s_d[i] >> 16);
      zd_rle(lens, (int)bk.dmax, send);
    }
  }
  zd_for_tokens(T, B, q0, q1, [&](const ZdTok &k) {
    if (!k.len) {
      W.put(s_l[k.lit] & 0xffffu, s_l[k.lit] >> 16);
    } else {
      const uint32_t lc = zd_lcode(k.len), dc = zd_dcode(k.dist);
      W.put(s_l[257 + lc] & 0xffffu, s_l[257 + lc] >> 16);
      if (zd_xl[lc]) W.put(k.len - zd_lbase(lc), zd_xl[lc]);
      W.put(s_d[dc] & 0xffffu, s_d[dc] >> 16);
      if (zd_xd[dc]) W.put(k.dist - zd_dbase(dc), zd_xd[dc]);
    }
  });
  if (t == ZD_TT - 1) W.put(s_l[256] & 0xffffu, s_l[256] >> 16);
  W.done();
}

// ---------------------------------------------------------------------------
// host launch: everything up to the bits (the check and trailer kernels of
// deflate_kernels.hip run beside it); returns after the fix-up rounds, which
// need the host (a flag read per round)
// ---------------------------------------------------------------------------
// parallel fix-up rounds before the in-order pass (env ZS_ZD_ROUNDS, read per
// batch so tests can force the in-order pass on small inputs)
static int zd_fix_rounds() {
  const char *e = getenv("ZS_ZD_ROUNDS");
  const int v = e ? atoi(e) : 8;
  return v < 0 ? 0 : v;
}

extern "C" int zs_launch_zdeflate(ZsDJobDev *d_jobs, uint32_t njobs, ZsDSegDev *d_segs, uint32_t nseg,
                                  const ZsZWorkDev *d_w1, uint32_t n1, const ZsZWorkDev *d_w1s, uint32_t n1s,
                                  const ZsZWorkDev *d_w2, uint32_t n2, const ZsZWorkDev *d_w3, uint32_t n3,
                                  uint16_t *d_prevd, uint32_t *d_ma, uint32_t *d_mb, uint32_t *d_bm, ZsZBlkDev *d_blks,
                                  uint32_t nblk_slots, const uint32_t *d_slot_job, uint32_t *d_aux, uint8_t *d_stage,
                                  uint32_t *d_flag, int has_slow, int has_fast, uint32_t max_regions, hipStream_t st,
                                  hipEvent_t *ev) {
  if (ev) (void)hipEventRecord(ev[0], st);
  if (n1) hipLaunchKernelGGL(zs_zd_prev_kernel, dim3(n1), dim3(ZD_PT1), 0, st, d_jobs, d_w1, d_prevd);
  if (n1s) hipLaunchKernelGGL(zs_zd_prev_small_kernel, dim3(n1s), dim3(ZD_PT1), 0, st, d_jobs, d_w1s, d_prevd);
  if (n2) hipLaunchKernelGGL(zs_zd_match_kernel, dim3(n2), dim3(ZD_MT), 0, st, d_jobs, d_w2, d_prevd, d_ma, d_mb, d_bm);
  if (n3) hipLaunchKernelGGL(zs_zd_msearch_kernel, dim3(n3), dim3(ZD_MT3), 0, st, d_jobs, d_w3, d_prevd, d_ma, d_mb, d_bm);
  if (ev) (void)hipEventRecord(ev[1], st);
  if (has_fast) hipLaunchKernelGGL(zs_zd_fast_kernel, dim3(njobs), dim3(WAVE), 0, st, d_jobs, d_bm, d_ma);
  if (has_slow)
    hipLaunchKernelGGL(zs_zd_parse_kernel, dim3(nseg), dim3(ZD_PT), 0, st, d_jobs, d_segs, d_ma, d_mb, d_prevd, d_bm);
  // parallel fix-up rounds while exits change (nearly every input settles in
  // one or two), then, if a cascade is still moving, the in-order pass
  // (jobs of a few regions -- stream segments -- go straight to the in-order
  // pass: no host round trip per round)
  const int max_rounds = has_slow && max_regions > 4 ? zd_fix_rounds() : 0;
  uint32_t cur = 0;
  bool settled = !has_slow;  // (max_rounds 0 with slow jobs: the in-order pass below)
  for (int round = 0; round < max_rounds; round++) {
    uint32_t changed = 0;
    if (hipMemsetAsync(d_flag, 0, sizeof(uint32_t), st) != hipSuccess) return -1;
    hipLaunchKernelGGL(zs_zd_fix_kernel, dim3((nseg + 255) / 256), dim3(256), 0, st, d_jobs, d_segs, nseg, d_ma, d_mb, d_prevd, d_bm,
                       cur, d_flag);
    if (hipMemcpyAsync(&changed, d_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return -1;
    cur ^= 1u;
    if (!changed) {
      settled = true;
      break;
    }
  }
  if (!settled) {
    hipLaunchKernelGGL(zs_zd_fix_seq_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, d_jobs, njobs, d_segs, d_ma, d_mb, d_prevd,
                       d_bm);
  }
  if (ev) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(zs_zd_count_kernel, dim3(nseg), dim3(256), 0, st, d_jobs, d_segs, d_bm);
  hipLaunchKernelGGL(zs_zd_blocks_kernel, dim3(njobs), dim3(1024), 0, st, d_jobs, d_segs, d_bm);
  hipLaunchKernelGGL(zs_zd_blist_kernel, dim3((nblk_slots + 255) / 256), dim3(256), 0, st, d_jobs, njobs, d_segs, d_bm,
                     d_blks, nblk_slots, d_slot_job);
  hipLaunchKernelGGL(zs_zd_cut_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, d_jobs, njobs, d_segs, d_bm, d_blks);
  hipLaunchKernelGGL(zs_zd_tree_kernel, dim3(nblk_slots), dim3(ZD_TT), 0, st, d_jobs, d_blks, d_ma, d_mb, d_bm, d_aux);
  hipLaunchKernelGGL(zs_zd_layout_kernel, dim3(njobs), dim3(1024), 0, st, d_jobs, d_blks, d_stage);
  hipLaunchKernelGGL(zs_zd_emit_kernel, dim3(nblk_slots), dim3(ZD_TT), 0, st, d_jobs, d_blks, d_ma, d_mb, d_bm, d_aux,
                     d_stage);
  hipLaunchKernelGGL(zs_zd_limit_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, d_jobs, njobs, d_segs, d_bm, d_blks);
  if (ev) (void)hipEventRecord(ev[3], st);
  return 0;
}
