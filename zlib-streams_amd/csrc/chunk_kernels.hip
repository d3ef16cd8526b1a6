// chunk_kernels.hip -- speculative chunk-parallel inflate for large streams.
//
// Hot loop of the reference: src/inffast.c:100-287 (symbol decode + copy), fed
// by the block/table states of src/inflate.c:834-1033 and src/inftrees.c.
// MI355X design:
//   zs_find_kernel   one wave per search segment: bit-parallel filters queue
//                    candidate block starts in LDS; the queue is validated 64
//                    at a time (one candidate per lane); up to SEG_SLOTS starts
//                    are recorded per segment.
//   zs_plan_kernel   one workgroup per stream: stream start + recorded starts
//                    -> ordered decode units with stops and scratch ranges.
//   zs_lane_kernel / zs_expand_kernel (lane_decode.hip): one lane per unit
//                    parses symbols to tokens; one workgroup per unit expands
//                    tokens to u16 entries (markers 256+w for the unknown
//                    32 KiB history before the unit).
//   zs_link_kernel   one workgroup per stream: follows the unit chain,
//                    computes output offsets, resolves the 32 KiB history of
//                    every chained unit in order (LDS double buffer).
//   zs_emit_kernel   one workgroup per unit: entries -> bytes at their final
//                    offsets (markers looked up in the unit's window in LDS).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "zs_common.h"
#include "zs_device.h"
#include "zs_kprof.h"

#if KP_ON
__device__ unsigned long long g_kprof_ck[16];  // KP_L_* - 48
#define KPC_ADD(i, v) atomicAdd(&g_kprof_ck[(i) - 48], (unsigned long long)(v))
#define KPC_MAX(i, v) atomicMax(&g_kprof_ck[(i) - 48], (unsigned long long)(v))
#endif

#define MARK_BASE 256u
#define HIST 32768u
#define STAGE_WORDS 256  // 1 KiB of staged header bits per cooperative step

// ---------------------------------------------------------------------------
// Full dynamic-header validation for one candidate (per lane, rare path).
// Mirrors the acceptance rules of src/inflate.c:905-1033 + src/inftrees.c
// (complete code-length code, repeat rules, end-of-block present, literal and
// distance codes complete or a single 1-bit code, empty distance code allowed).
// ---------------------------------------------------------------------------
// The input comes from a per-lane window of VWIN words in LDS (win: the
// lane's column of a [VWIN][WAVE] array, lane-interleaved), loaded by 16-byte
// loads when the validation starts and again whenever the reader leaves it
// (a long header): a global load per 32 bits made some lane of the wave
// refill on nearly every code-length symbol.  The symbol loop is straight
// line (selects, one reload site): the round-5 loop (a bit buffer refilled by
// an unrolled inner loop, branches per repeat code) compiled to ~2 000
// instructions of exec-mask branches and cost ~1 500-2 000 cycles per symbol
// of the wave's longest lane (profiling build, C2).
#ifndef VWIN
#define VWIN 32u
#endif
// One candidate's validation state (a lane of zs_findval_kernel).
// The code-length code is decoded canonically from registers (no per-lane
// LUT: filling 128 LUT bytes per candidate cost ~60% of the pool's time, and
// its 8 KiB per wave capped the occupancy): lim_L, the left-justified end of
// the length-L codes in the 7-bit code space (= the partial Kraft sums), as
// bytes P1 (L = 1..4) / P2 (5..6); the code's length is 1 + the number of
// lim_L <= the next 7 bits read first-bit-first (a SWAR byte compare); BA/BB
// the start of each length's range and OA/OB the rank of its first symbol
// (bytes, L = 1..4 / 5..7); SL/SH the symbols in canonical order (5 bits
// each, ranks 0..11 / 12..18).
struct VState {
  const uint32_t *w;  // input (4-byte-aligned base)
  uint32_t end_byte, wb;  // input length from w; window base word
  uint32_t p, have, prev, eob, lk, lmax, dk, dmax, dn, nlen, total;
  uint32_t P1, P2, BA, BB, OA, OB;
  uint64_t SL, SH;
};
// the lane's window: VWIN words of input from word `at` rounded down to 4
__device__ __forceinline__ void vwin_load(VState &v, uint32_t at, uint32_t *win) {
  v.wb = at & ~3u;
  if (v.wb + VWIN <= (v.end_byte >> 2)) {
    const uint32_t *src = v.w + v.wb;
#pragma unroll
    for (uint32_t h = 0; h < VWIN / 16u; h++) {  // 16 words at a time (fewer registers in flight)
      uint4 x[4];
#pragma unroll
      for (uint32_t q = 0; q < 4u; q++) __builtin_memcpy(&x[q], src + 16u * h + 4u * q, 16);
#pragma unroll
      for (uint32_t q = 0; q < 4u; q++) {
        win[(16u * h + 4u * q) * WAVE] = x[q].x;
        win[(16u * h + 4u * q + 1u) * WAVE] = x[q].y;
        win[(16u * h + 4u * q + 2u) * WAVE] = x[q].z;
        win[(16u * h + 4u * q + 3u) * WAVE] = x[q].w;
      }
    }
  } else {
#pragma unroll 1
    for (uint32_t q = 0; q < VWIN; q++) win[q * WAVE] = in_word(v.w, v.wb + q, v.end_byte);
  }
}
enum { VS_RUN = 0, VS_OK = 1, VS_BAD = 2 };
// header, code-length code and its LUT of the candidate at `bit`
template <bool D64>
__device__ uint32_t val_setup(VState &v, uint32_t bit, uint32_t *win) {
  vwin_load(v, bit >> 5, win);
  // the header's 14 + 3 * 19 bits lie in the window's first 5 words
  const uint32_t r0 = (bit >> 5) - v.wb, sh = bit & 31u;
  const uint32_t h0 = __builtin_amdgcn_alignbit(win[(r0 + 1u) * WAVE], win[r0 * WAVE], sh);
  const uint32_t h1 = __builtin_amdgcn_alignbit(win[(r0 + 2u) * WAVE], win[(r0 + 1u) * WAVE], sh);
  const uint32_t h2 = __builtin_amdgcn_alignbit(win[(r0 + 3u) * WAVE], win[(r0 + 2u) * WAVE], sh);
  v.nlen = ((h0 >> 3) & 31u) + 257u;
  const uint32_t ndist = ((h0 >> 8) & 31u) + 1u, ncode = ((h0 >> 13) & 15u) + 4u;
  if (v.nlen > 286 || ndist > (D64 ? 32u : 30u)) return VS_BAD;
  // the 19 3-bit code-length-code lengths from bit 17, in stream order, masked to ncode
  const uint64_t cls_s = ((((uint64_t)h1 << 32) | h0) >> 17 | ((uint64_t)h2 << 47)) & (~0ull >> (64u - 3u * ncode));
  // ... in symbol order (src/inflate.c:975-983 order[])
  constexpr uint8_t inv[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};
  uint64_t cls = 0;
  uint64_t cntp = 0;  // 5-bit count of each length 1..7 at bits 5L (length 0 not counted)
#pragma unroll
  for (int sy = 0; sy < 19; sy++) {
    const uint32_t L = (uint32_t)(cls_s >> (3 * inv[sy])) & 7u;
    cls |= (uint64_t)L << (3 * sy);
    cntp += (1ull << (5u * L)) & ~31ull;
  }
  // complete code-length code (src/inftrees.c:137-140 rejects any other for CODES)
  uint32_t lim = 0, offs = 0;
  v.P1 = v.P2 = v.BA = v.BB = v.OA = v.OB = 0;
#pragma unroll
  for (int L = 1; L < 8; L++) {
    const uint32_t c = (uint32_t)(cntp >> (5 * L)) & 31u;
    if (L < 5) {
      v.BA |= lim << (8 * (L - 1));
      v.OA |= offs << (8 * (L - 1));
    } else {
      v.BB |= lim << (8 * (L - 5));
      v.OB |= offs << (8 * (L - 5));
    }
    lim += c << (7 - L);
    offs += c;
    if (L < 5) v.P1 |= min(lim, 255u) << (8 * (L - 1));
    else if (L < 7) v.P2 |= min(lim, 255u) << (8 * (L - 5));
  }
  if (lim != 128u) return VS_BAD;
  // the symbols in canonical order: symbol order within each length
  uint64_t seen = 0;
  v.SL = v.SH = 0;
#pragma unroll
  for (int sy = 0; sy < 19; sy++) {
    const uint32_t L = (uint32_t)(cls >> (3 * sy)) & 7u;
    const uint32_t sh8 = 8u * ((L - 1u) & 3u);
    const uint32_t rank = ((((L < 5u) ? v.OA : v.OB) >> sh8) & 255u) + ((uint32_t)(seen >> (5u * L)) & 31u);
    seen += 1ull << (5u * L);
    const uint64_t put = L ? (uint64_t)sy : 0ull;
    v.SL |= rank < 12u ? put << (5u * rank) : 0ull;
    v.SH |= rank < 12u ? 0ull : put << (5u * (rank - 12u));
  }
  v.total = v.nlen + ndist;
  v.p = bit + 17u + 3u * ncode;
  v.have = v.prev = v.eob = v.lk = v.lmax = v.dk = v.dmax = v.dn = 0;
  return VS_RUN;
}
// one code-length symbol (src/inflate.c:1000-1033); at the last one, the
// completeness checks (src/inftrees.c:131-140, as zlib's table builds)
template <bool D64>
__device__ __forceinline__ uint32_t val_step(VState &v, uint32_t *win) {
  uint32_t i = (v.p >> 5) - v.wb;
  if (i + 1u >= VWIN) {
    vwin_load(v, v.p >> 5, win);
    i = (v.p >> 5) - v.wb;
  }
  const uint32_t x = __builtin_amdgcn_alignbit(win[(i + 1u) * WAVE], win[i * WAVE], v.p & 31u);
  // canonical decode of the next code-length symbol (the VState registers)
  const uint32_t c7 = __builtin_bitreverse32(x) >> 25;
  const uint32_t L = 1u + (uint32_t)__builtin_popcount(((0x80808080u | (c7 * 0x01010101u)) - v.P1) & 0x80808080u) +
                     (uint32_t)__builtin_popcount(((0x8080u | (c7 * 0x0101u)) - v.P2) & 0x8080u);
  const uint32_t sh8 = 8u * ((L - 1u) & 3u);
  const uint32_t base = (((L < 5u) ? v.BA : v.BB) >> sh8) & 255u, offs = (((L < 5u) ? v.OA : v.OB) >> sh8) & 255u;
  const uint32_t idx = offs + ((c7 - base) >> (7u - L));
  const uint32_t sym = idx < 12u ? (uint32_t)(v.SL >> (5u * idx)) & 31u : (uint32_t)(v.SH >> (5u * (idx - 12u))) & 31u;
  // repeat codes 16 / 17 / 18: 2 / 3 / 7 extra bits, 3 / 3 / 11 + extra copies
  const uint32_t xb = sym < 16u ? 0u : (sym == 16u ? 2u : (sym == 17u ? 3u : 7u));
  const uint32_t rep = sym < 16u ? 1u : (sym == 18u ? 11u : 3u) + __builtin_amdgcn_ubfe(x, L, xb);
  const uint32_t val = sym < 16u ? sym : (sym == 16u ? v.prev : 0u);
  v.p += L + xb;
  if (L == 0u || (sym == 16u && v.have == 0u) || v.p > v.end_byte * 8u || v.have + rep > v.total) return VS_BAD;
  // the run's lengths split between the literal/length and distance codes;
  // partial Kraft sums only grow, so an over-subscribed code fails now
  const uint32_t nl = v.have < v.nlen ? min(rep, v.nlen - v.have) : 0u;
  const uint32_t nd = rep - nl;
  const uint32_t sv = 15u - val;
  v.lk += val ? nl << sv : 0u;
  v.dk += val ? nd << sv : 0u;
  v.dn += val ? nd : 0u;
  v.lmax = (val && nl) ? max(v.lmax, val) : v.lmax;
  v.dmax = (val && nd) ? max(v.dmax, val) : v.dmax;
  v.eob = (v.have <= 256u && 256u < v.have + rep) ? val : v.eob;
  if (v.lk > 32768u || v.dk > 32768u) return VS_BAD;
  v.prev = val;
  v.have += rep;
  if (v.have < v.total) return VS_RUN;
  if (v.eob == 0) return VS_BAD;
  if (v.lk > 32768u || (v.lk < 32768u && v.lmax != 1)) return VS_BAD;
  if (v.dn && (v.dk > 32768u || (v.dk < 32768u && v.dmax != 1))) return VS_BAD;
  if (D64 && v.dn == 0) return VS_BAD;  // deflate64 rejects an empty distance code (src/inftrees.c:131-132)
  return VS_OK;
}

// ---------------------------------------------------------------------------
// Block finder, two kernels (round 6):
//   zs_find_kernel     one wave per search segment: every lane tests 32 bit
//                      offsets per step with bit-parallel filters (BFINAL = 0
//                      -- or 1 in a stream's last segments --, BTYPE = 2,
//                      HLIT <= 29, HDIST <= 29), the survivors go through an LDS
//                      queue (one candidate per lane) to the code-length-code
//                      completeness check, and what passes that is appended, in
//                      offset order, to the segment's survivor list in global
//                      memory (<= FV_LIST - 1 per segment; hints only).
//   zs_findval_kernel  the survivors of all segments, one per lane, through the
//                      full header validation (a pool: lanes refilled as they
//                      finish); zs_findsel_kernel keeps each segment's first
//                      SEG_SLOTS that pass.
// Measured (C2, round 5, one kernel): the full validation's long per-lane LDS
// and global chains ran inside the scan loop at 4 waves per SIMD (its 8 KiB of
// LUTs), 40% of the wave cycles waiting; split, the scan runs at 3.9 KiB of
// LDS and the validation has its own occupancy.  A C2 segment holds ~220
// filter candidates per 2048-bit step, ~0.3-0.9 pass the completeness check,
// a validation decodes ~40-80 code-length symbols (tools/find_probe.c).
// ---------------------------------------------------------------------------
#ifndef FIND_WG
#define FIND_WG 4u  // segments (waves) per finder workgroup: one-wave workgroups left CUs at ~12 resident waves
#endif
#define FQ_LIST 256u  // u32 per segment in the survivor lists: [0] count, then <= FQ_LIST - 1 bit offsets

__device__ __forceinline__ uint32_t find_scan_excl(uint32_t v, uint32_t *total) {
  uint32_t x = v;
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  *total = __builtin_amdgcn_readlane(x, WAVE - 1);
  return x - v;
}

// code-length-code completeness (Kraft sum == 2^7) of the candidate header at
// bit p (p - base < 2048): HCLEN at p+13, 3-bit lengths from p+17; the bits
// come from the step's LDS stage st (words of the input from bit base).  The
// lengths past HCLEN + 4 are masked off, then the sum goes three lengths at a
// time through k9 (k9[x] = the Kraft weights 2^(7-L) of the three 3-bit
// lengths of x, 0 for L = 0): 7 independent LDS reads instead of 19 serial
// extract/shift/select/add steps.
__device__ __forceinline__ bool cl_complete(const uint32_t *st, uint32_t base, uint32_t p, const uint8_t *k9) {
  // the 64 bits from p + 13 (HCLEN, then the 19 lengths) from three stage words
  const uint32_t r = p + 13u - base, wi = r >> 5;
  const uint32_t a = st[wi], b = st[wi + 1], c = st[wi + 2];
  const uint32_t lo = __builtin_amdgcn_alignbit(b, a, r), hi = __builtin_amdgcn_alignbit(c, b, r);
  const uint32_t ncode = (lo & 15u) + 4u;
  const uint64_t clb = ((((uint64_t)hi << 32) | lo) >> 4) & (~0ull >> (64u - 3u * ncode));
  const uint32_t l = (uint32_t)clb, h = (uint32_t)(clb >> 32);
  const uint32_t kraft = k9[l & 511u] + k9[__builtin_amdgcn_ubfe(l, 9, 9)] + k9[__builtin_amdgcn_ubfe(l, 18, 9)] +
                         k9[__builtin_amdgcn_alignbit(h, l, 27) & 511u] + k9[__builtin_amdgcn_ubfe(h, 4, 9)] +
                         k9[__builtin_amdgcn_ubfe(h, 13, 9)] + k9[__builtin_amdgcn_ubfe(h, 22, 9)];
  return kraft == 128u;
}

// position of this lane among the set lanes of m below it
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <bool D64>
__global__ void __launch_bounds__(FIND_WG * WAVE) zs_find_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                                const ZsSegDev *__restrict__ segs, uint32_t *__restrict__ vlist,
                                                                uint32_t nseg) {
  __shared__ uint32_t s_st_all[FIND_WG][WAVE + 8];  // this step's input words (2048 bits + overlap)
  // this step's candidates passing the bit-parallel filters: ~11% of random
  // bits; past FQC (adversarial bit patterns) the rest of the step is dropped
  // -- starts are hints, the chain check keeps results exact
  constexpr uint32_t FQC = WAVE * 12;
  __shared__ uint32_t s_q_all[FIND_WG][FQC];
  __shared__ uint8_t s_k9[512];  // Kraft weights of 3 code-length-code lengths (cl_complete), <= 192
  const uint32_t lane = threadIdx.x & (WAVE - 1u), wv = threadIdx.x / WAVE;
  uint32_t *const s_st = s_st_all[wv];
  uint32_t *const s_q = s_q_all[wv];
  __shared__ uint32_t s_l_all[FIND_WG][FQ_LIST - 1u];  // the segment's survivors (stored to vlist at the end)
  uint32_t *const s_l = s_l_all[wv];
  for (uint32_t x = threadIdx.x; x < 512; x += FIND_WG * WAVE) {
    uint32_t k = 0;
    for (int f = 0; f < 3; f++) {
      const uint32_t L = (x >> (3 * f)) & 7u;
      k += L ? 128u >> L : 0u;
    }
    s_k9[x] = (uint8_t)k;
  }
  __syncthreads();
  const uint32_t sg = blockIdx.x * FIND_WG + wv;
  if (sg >= nseg) return;
  const ZsSegDev seg = segs[sg];
  const ZsJobDev jb = jobs[seg.job];
  const ZsHeadDev hd = heads[seg.job];
  uint32_t *const out = vlist + (size_t)sg * FQ_LIST;
  uint32_t nv = 0;  // survivors listed
  if (hd.code == ZD_END) {
    const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
    const uint32_t mis = (uint32_t)(ip & 3u);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(ip - mis);
    const uint32_t end_byte = mis + (uint32_t)jb.in_len;
    // strictly after the stream's first block (that start is unit 0)
    const uint32_t lo = max((mis + seg.s_byte) * 8u, (mis + (uint32_t)hd.start_byte) * 8u + jb.sbit + 1u);
    const uint32_t hi = (mis + seg.e_byte) * 8u;
    // input words of a step: lane word (base/32 + lane), the next one, and 8
    // overlap words (lanes < 8), loaded two steps ahead.  The loads are
    // unconditional (index clamped to the last word, bytes past the input
    // zeroed when used) and no global store sits in the loop: a conditional
    // load, or a store after the prefetch, made the compiler wait vmcnt(0) at
    // the loop top -- one full memory latency per step (C2 scan 2.2 ms)
    const uint32_t lastw = (end_byte - 1u) >> 2;
    // (global, not flat: flat loads count in lgkmcnt, so every LDS wait would wait for them)
    typedef __attribute__((address_space(1))) const uint32_t gcu32f;
    const gcu32f *gw = (const gcu32f *)w;
    auto fetch = [&](uint32_t bs, uint32_t &a0, uint32_t &a1, uint32_t &a2) {
      const uint32_t wi = (bs >> 5) + lane;
      a0 = gw[min(wi, lastw)];
      a1 = gw[min(wi + 1u, lastw)];
      a2 = gw[min((bs >> 5) + WAVE + (lane & 7u), lastw)];
    };
    auto mask = [&](uint32_t v, uint32_t wi) {
      const uint32_t b = wi * 4u;
      const uint32_t keep = b >= end_byte ? 0u : end_byte - b;
      return keep >= 4u ? v : __builtin_amdgcn_ubfe(v, 0, 8u * keep);
    };
    uint32_t nx0, nx1, nx2, ny0, ny1, ny2;
    fetch(lo & ~31u, nx0, nx1, nx2);
    fetch((lo & ~31u) + WAVE * 32u, ny0, ny1, ny2);
    // one step over the 2048 bits at base from buffer (a0, a1, a2), which
    // then takes the words of the step after next; the loop alternates the two
    // buffers (a register move between them made the loop wait for the
    // next step's loads)
    auto step = [&](uint32_t base, uint32_t &a0, uint32_t &a1, uint32_t &a2) {
      const uint32_t b0 = base + lane * 32u;
      const uint32_t wl = b0 >> 5;
      const uint32_t x0 = mask(a0, wl), x1 = mask(a1, wl + 1u), x2 = mask(a2, (base >> 5) + WAVE + (lane & 7u));
      fetch(base + 2u * WAVE * 32u, a0, a1, a2);
      s_st[lane] = x0;
      if (lane < 8) s_st[WAVE + lane] = x2;
      uint32_t cand = 0;
      if (b0 < hi) {
        const uint64_t x = (uint64_t)x0 | ((uint64_t)x1 << 32);
        // bit-parallel over the lane's 32 offsets p: BTYPE = 2 (bit p+1 = 0,
        // bit p+2 = 1), BFINAL (bit p) = 0 unless this is one of the stream's
        // last segments, HLIT <= 29 (not bits p+4..p+7 all set), HDIST <= 29
        // (not bits p+9..p+12 all set)
        const uint64_t bt = ~(x >> 1) & (x >> 2);
        const uint64_t hlit_bad = (x >> 4) & (x >> 5) & (x >> 6) & (x >> 7);
        // (deflate64 allows HDIST 30 and 31: 32 distance codes)
        const uint64_t hdist_bad = D64 ? 0ull : (x >> 9) & (x >> 10) & (x >> 11) & (x >> 12);
        cand = (uint32_t)((seg.final_ok ? bt : (bt & ~x)) & ~hlit_bad & ~hdist_bad);
        if (b0 < lo) cand &= ~0u << (lo - b0);
        if (hi - b0 < 32u) cand &= (1u << (hi - b0)) - 1u;
      }
      uint32_t tot;
      const uint32_t at = find_scan_excl((uint32_t)__builtin_popcount(cand), &tot);
      // two candidates per iteration (the loop runs for the wave's largest
      // count, ~9 of a lane's 32 offsets): find 5.12 -> 4.98 ms on C2
      for (uint32_t k = 0; cand && at + k < FQC; k += 2) {
        const uint32_t c1 = cand & (cand - 1u);
        s_q[at + k] = b0 + (uint32_t)__builtin_ctz(cand);
        if (c1 && at + k + 1 < FQC) s_q[at + k + 1] = b0 + (uint32_t)__builtin_ctz(c1);
        cand = c1 & (c1 - 1u);
      }
      tot = min(tot, FQC);
      __builtin_amdgcn_wave_barrier();
      // completeness check, one candidate per lane, four rounds of the queue
      // at once (their LDS reads in flight together, not four serial chains);
      // survivors keep their order in the list
      for (uint32_t q0 = 0; q0 < tot; q0 += 4u * WAVE) {
        uint32_t cb[4];
        bool ok[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
          const uint32_t q = q0 + j * WAVE + lane;
          const uint32_t v = s_q[min(q, FQC - 1u)];
          cb[j] = q < tot ? v : base;
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) ok[j] = cl_complete(s_st, base, cb[j], s_k9) && q0 + j * WAVE + lane < tot;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
          const uint64_t m = __ballot(ok[j]);
          const uint32_t pos = nv + lanes_below(m);
          if (ok[j] && pos < FQ_LIST - 1u) s_l[pos] = cb[j];
          nv = min(nv + (uint32_t)__builtin_popcountll(m), FQ_LIST - 1u);
        }
      }
      __builtin_amdgcn_wave_barrier();
    };
    for (uint32_t base = lo & ~31u; base < hi;) {
      step(base, nx0, nx1, nx2);
      base += WAVE * 32u;
      if (base >= hi) break;
      step(base, ny0, ny1, ny2);
      base += WAVE * 32u;
    }
  }
  __builtin_amdgcn_wave_barrier();
  for (uint32_t i = lane; i < nv; i += WAVE) out[1u + i] = s_l[i];
  if (lane == 0) out[0] = nv;
  if (lane < 8u) vlist[(size_t)nseg * FQ_LIST + sg * 8u + lane] = 0u;  // zs_findval_kernel's accepted bitmap
  if (sg == 0 && lane == 0) vlist[(size_t)nseg * (FQ_LIST + 8u)] = 0u;  // its segment counter
}

// Full header validation of every survivor, one per lane, from ONE pool:
// each wave takes whole segments' lists from a global counter into an LDS
// queue, and a lane whose candidate is decided takes the next one; lanes are
// refilled together once FV_REFILL of them are idle (a setup costs the wave
// the same whatever number of lanes run it).  Measured (profiling build, C2,
// round 6): with a wave per segment and 64 candidates per batch, a batch
// lasted as long as its longest lane (~170 code-length symbols) while the
// lanes averaged ~40 -- 22% of lane-steps did work.  Accepted candidates set
// their bit in the segment's bitmap; zs_findsel_kernel keeps the first
// SEG_SLOTS of each segment (in offset order, as one wave per segment did).
#define FV_QN 256u     // queue entries per wave (a segment lists <= FQ_LIST - 1)
#ifndef FV_REFILL
#define FV_REFILL 24u  // idle lanes that trigger a refill
#endif
#define FV_WAVES_PER_CU 16u
template <bool D64>
__global__ void __launch_bounds__(WAVE) zs_findval_kernel(const ZsJobDev *__restrict__ jobs, const ZsSegDev *__restrict__ segs,
                                                         uint32_t *__restrict__ vlist, uint32_t nseg) {
  __shared__ uint32_t s_win[VWIN][WAVE];  // per-lane input windows
  __shared__ uint32_t s_qi[FV_QN], s_qb[FV_QN], s_qj[FV_QN];  // queue: segment << 8 | index, bit, job
  const uint32_t lane = threadIdx.x;
  uint32_t *const ctr = vlist + (size_t)nseg * (FQ_LIST + 8u);
  uint32_t *const bmp = vlist + (size_t)nseg * FQ_LIST;
  uint32_t *win = &s_win[0][lane];
  uint32_t qh = 0, qt = 0;  // queue head / tail (uniform, monotonic)
  bool more = true, act = false;
  uint32_t cur = 0;  // the lane's candidate: segment << 8 | index
  VState v;
  v.w = nullptr;
  v.end_byte = v.wb = v.p = v.have = v.prev = v.eob = v.lk = v.lmax = v.dk = v.dmax = v.dn = v.nlen = v.total = 0;
  v.P1 = v.P2 = v.BA = v.BB = v.OA = v.OB = 0;
  v.SL = v.SH = 0;
#if KP_ON
  const uint64_t kt0 = KP_NOW();
  uint64_t kp_st = 0;
  uint32_t kp_rounds = 0, kp_wsteps = 0, kp_lsteps = 0;
#endif
  for (;;) {
    // whole segments into the queue while one fits
    while (more && qt - qh + (FQ_LIST - 1u) <= FV_QN) {
      uint32_t sg = 0;
      if (lane == 0) sg = atomicAdd(ctr, 1u);
      sg = __builtin_amdgcn_readfirstlane(sg);
      if (sg >= nseg) {
        more = false;
        break;
      }
      const uint32_t *lst = vlist + (size_t)sg * FQ_LIST;
      const uint32_t n = min(lst[0], FQ_LIST - 1u), job = segs[sg].job;
      for (uint32_t i = lane; i < n; i += WAVE) {
        const uint32_t k = (qt + i) & (FV_QN - 1u);
        s_qi[k] = (sg << 8) | i;
        s_qb[k] = lst[1u + i];
        s_qj[k] = job;
      }
      qt += n;
    }
    __builtin_amdgcn_wave_barrier();
    // idle lanes take the next candidates, in lane order
    {
      const uint64_t m = __ballot(!act);
      const uint32_t k = lanes_below(m), avail = qt - qh;
      if (!act && k < avail) {
        const uint32_t e = (qh + k) & (FV_QN - 1u);
        cur = s_qi[e];
        const uint32_t bit = s_qb[e];
        const ZsJobDev jb = jobs[s_qj[e]];
        const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
        const uint32_t mis = (uint32_t)(ip & 3u);
        v.w = reinterpret_cast<const uint32_t *>(ip - mis);
        v.end_byte = mis + (uint32_t)jb.in_len;
        act = val_setup<D64>(v, bit, win) == VS_RUN;
      }
      qh += min((uint32_t)__builtin_popcountll(m), avail);
#if KP_ON
      kp_rounds++;
#endif
    }
    const bool drain = !more && qh == qt;
    if (__ballot(act) == 0) {
      if (drain) break;
      continue;
    }
#if KP_ON
    const uint64_t ks0 = KP_NOW();
#endif
    // steps until enough lanes are idle (or, with nothing left to take, all)
    const uint32_t keep = drain ? 0u : WAVE - FV_REFILL;
    do {
#if KP_ON
      kp_wsteps++;
      kp_lsteps += act ? 1u : 0u;
#endif
      if (act) {
        const uint32_t r = val_step<D64>(v, win);
        if (r != VS_RUN) {
          act = false;
          if (r == VS_OK) atomicOr(&bmp[(cur >> 8) * 8u + ((cur & 255u) >> 5)], 1u << (cur & 31u));
        }
      }
    } while ((uint32_t)__builtin_popcountll(__ballot(act)) > keep);
#if KP_ON
    kp_st += KP_NOW() - ks0;
#endif
  }
#if KP_ON
  {
    uint32_t ls = kp_lsteps;
    for (uint32_t o = 1; o < WAVE; o <<= 1) ls += (uint32_t)__shfl_xor((int)ls, (int)o);
    if (lane == 0) {
      KPC_ADD(58, 1);
      KPC_ADD(59, kp_rounds);
      KPC_ADD(60, kp_st);
      KPC_ADD(61, kp_wsteps);
      KPC_ADD(62, ls);
      KPC_ADD(63, KP_NOW() - kt0);
    }
  }
#endif
}

// The first SEG_SLOTS validated starts of each segment (lowest bitmap bits:
// the list is in offset order), one thread per segment.
__global__ void __launch_bounds__(256) zs_findsel_kernel(ZsSegDev *__restrict__ segs, const uint32_t *__restrict__ vlist,
                                                         uint32_t nseg) {
  const uint32_t sg = blockIdx.x * 256u + threadIdx.x;
  if (sg >= nseg) return;
  const uint32_t *lst = vlist + (size_t)sg * FQ_LIST;
  const uint32_t *bm = vlist + (size_t)nseg * FQ_LIST + sg * 8u;
  uint32_t nf = 0;
  for (uint32_t k = 0; k < 8u && nf < SEG_SLOTS; k++) {
    uint32_t b = bm[k];
    while (b && nf < SEG_SLOTS) {
      const uint32_t i = 32u * k + (uint32_t)__builtin_ctz(b);
      b &= b - 1u;
      segs[sg].cand[nf++] = lst[1u + i];
    }
  }
  segs[sg].ncand = nf;
}

// ---------------------------------------------------------------------------
// Fixed-Huffman block finder (src/inflate.c:834-869, BTYPE = 1), for search
// segments in which zs_find_kernel recorded no dynamic start (streams written
// with Z_FIXED, or long runs of fixed blocks).  A fixed block has no header
// to validate, so a candidate bit p must (a) follow a fixed-code end of block
// (the 7-bit code 0000000 at p-7..p-1), (b) carry BTYPE = 01 (BFINAL = 0 unless
// this is one of the stream's last segments), and (c) decode FIXED_CHECK
// fixed-code symbols (or reach an end of block after at least FIXED_MIN of
// them) without an invalid literal/length (286, 287) or distance (30, 31)
// code.  The chain check of zs_chain_kernel keeps results exact whatever is
// recorded; (c) only keeps false starts rare.
// ---------------------------------------------------------------------------
#define FIXED_CHECK 256
#define FIXED_MIN 64
#define FIXED_LOOKBACK 2048  // bits decoded before a candidate

// One fixed-code symbol (literal/length + length extra + distance + extra)
// from `hold`; returns its bit length, 0 for an invalid code; *eob on 256.
__device__ __forceinline__ uint32_t fixed_symbol(uint64_t hold, bool *eob) {
  const uint32_t r9 = __builtin_bitreverse32((uint32_t)hold) >> 23;  // next 9 bits, first bit highest
  const uint32_t c7 = r9 >> 2, c8 = r9 >> 1;
  uint32_t sym, used;
  if (c7 < 24u) {
    sym = 256 + c7;
    used = 7;
  } else if (c8 < 0xc0u) {
    sym = c8 - 0x30u;
    used = 8;
  } else if (c8 < 0xc8u) {
    sym = 280 + (c8 - 0xc0u);
    used = 8;
  } else {
    sym = 144 + (r9 - 0x190u);
    used = 9;
  }
  *eob = sym == 256;
  if (sym > 285) return 0;
  if (sym > 256) {
    const uint32_t ls = sym - 257;
    used += (ls >= 8 && ls < 28) ? (ls >> 2) - 1 : 0u;
    const uint32_t d = __builtin_bitreverse32((uint32_t)(hold >> used)) >> 27;
    if (d >= 30) return 0;
    used += 5 + (d < 4 ? 0u : (d >> 1) - 1);
  }
  return used;  // <= 9 + 5 + 5 + 13 = 32
}

// Fixed-code decode from bit `from`: true when it reaches bit `to` exactly
// on a symbol boundary with an end-of-block code ending there (mode 0), or
// decodes FIXED_CHECK symbols from `from` (mode 1: `to` unused; an end of
// block after FIXED_MIN symbols also passes).
__device__ bool fixed_walk(const uint32_t *w, uint32_t end_byte, uint32_t from, uint32_t to, int mode) {
  const uint32_t limit = end_byte * 8u;
  uint32_t wi = from >> 5;
  uint64_t hold = (uint64_t)in_word(w, wi, end_byte) >> (from & 31);
  uint32_t n = 32 - (from & 31);
  wi++;
  uint32_t pos = from;
  for (uint32_t k = 0; k < 4096; k++) {
    while (n <= 32) {
      hold |= (uint64_t)in_word(w, wi, end_byte) << n;
      n += 32;
      wi++;
    }
    bool eob;
    uint32_t used = fixed_symbol(hold, &eob);
    if (!used) return false;
    if (mode == 0) {
      if (eob && pos + 7 == to) return true;
      if (pos + used > to) return false;  // ran over `to`: no symbol boundary there
      if (eob) {  // an earlier block end: skip its successor's header (fixed blocks only)
        used += 3;
        if (((hold >> 7) & 6u) != 2u) return false;
      }
    } else {
      if (eob) return k >= FIXED_MIN;
      if (k + 1 >= FIXED_CHECK) return true;
    }
    hold >>= used;
    n -= used;
    pos += used;
    if (pos > limit) return false;
  }
  return false;
}

// Candidate fixed block start at bit p (header at p, data from `data_bit`):
// a fixed-code decode from FIXED_LOOKBACK bits earlier must land exactly on an
// end of block ending at p -- fixed codes resynchronise within a few symbols,
// so a real boundary is met on a symbol boundary while a false candidate (7
// zero bits inside other codes) is run over -- and the block must decode.
__device__ bool fixed_plausible(const uint32_t *w, uint32_t end_byte, uint32_t data_bit, uint32_t p) {
  const uint32_t from = p >= data_bit + 3u + FIXED_LOOKBACK ? p - FIXED_LOOKBACK : data_bit + 3u;
  if (from + 7u > p) return false;
  return fixed_walk(w, end_byte, from, p, 0) && fixed_walk(w, end_byte, p + 3u, 0, 1);
}

__global__ void __launch_bounds__(64) zs_find_fixed_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                            ZsSegDev *__restrict__ segs, uint32_t nseg) {
  __shared__ uint32_t s_q[WAVE * 32];
  const uint32_t lane = threadIdx.x;
  const uint32_t sg = blockIdx.x;
  const ZsSegDev seg = segs[sg];
  if (seg.ncand != 0) return;
  // a segment between segments with dynamic starts lies inside a long dynamic
  // block: no fixed-block search there (the neighbours are this job's when
  // their ordinals are adjacent)
  if (seg.ord > 0 && segs[sg - 1].ncand != 0) return;
  if (sg + 1 < nseg && segs[sg + 1].job == seg.job && segs[sg + 1].ncand != 0) return;
  const ZsJobDev jb = jobs[seg.job];
  const ZsHeadDev hd = heads[seg.job];
  if (hd.code != ZD_END) return;
  const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
  const uint32_t mis = (uint32_t)(ip & 3u);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(ip - mis);
  const uint32_t end_byte = mis + (uint32_t)jb.in_len;
  const uint32_t lo = max((mis + seg.s_byte) * 8u, (mis + (uint32_t)hd.start_byte) * 8u + jb.sbit + 8u);
  const uint32_t hi = (mis + seg.e_byte) * 8u;
  uint32_t nfound = 0;
  for (uint32_t base = lo & ~31u; base < hi && nfound < SEG_SLOTS; base += WAVE * 32u) {
    const uint32_t b0 = base + lane * 32u;
    uint32_t cand = 0;
    if (b0 < hi) {
      const uint32_t wi = b0 >> 5;
      const uint32_t pw = wi ? in_word(w, wi - 1, end_byte) : 0u;
      const uint64_t lw = (uint64_t)pw | ((uint64_t)in_word(w, wi, end_byte) << 32);
      const uint64_t y = (lw >> 25) | ((uint64_t)in_word(w, wi + 1, end_byte) << 39);  // bit k = stream bit b0 - 7 + k
      const uint64_t z = ~y;
      const uint64_t eob = z & (z >> 1) & (z >> 2) & (z >> 3) & (z >> 4) & (z >> 5) & (z >> 6);
      const uint64_t bt = (y >> 8) & ~(y >> 9);
      cand = (uint32_t)(eob & bt & (seg.final_ok ? ~0ull : ~(y >> 7)));
      if (b0 < lo) cand &= lo - b0 >= 32u ? 0u : ~0u << (lo - b0);
      if (hi - b0 < 32u) cand &= (1u << (hi - b0)) - 1u;
    }
    uint32_t tot;
    const uint32_t at = find_scan_excl((uint32_t)__builtin_popcount(cand), &tot);
    for (uint32_t k = 0; cand; k++) {
      s_q[at + k] = b0 + (uint32_t)__builtin_ctz(cand);
      cand &= cand - 1u;
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t q0 = 0; q0 < tot && nfound < SEG_SLOTS; q0 += WAVE) {
      const uint32_t take = min(tot - q0, (uint32_t)WAVE);
      uint32_t cb = 0;
      bool ok = false;
      if (lane < take) {
        cb = s_q[q0 + lane];
        ok = fixed_plausible(w, end_byte, (mis + (uint32_t)hd.start_byte) * 8u + jb.sbit, cb);
      }
      uint64_t m = __ballot(ok);
      while (m && nfound < SEG_SLOTS) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint32_t f = __builtin_amdgcn_readlane(cb, l);
        if (lane == 0) segs[sg].cand[nfound] = f;
        nfound++;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0) segs[sg].nfixed = nfound;
}

// ---------------------------------------------------------------------------
// Plan: one workgroup per chunked job.  Units = the stream's first block +
// every recorded start, in order; each unit's stop is the next unit's start.
// Each unit gets a primary token region sized from its own compressed span
// (TOK_PER_BYTE tokens per span byte + TOK_SLACK), carved from the job's
// host-reserved range; tokens beyond it go to pool pages taken on demand by
// the parse pass (ZsTokPool), so a unit never fails for an underestimated
// size.  Output entries are not reserved here at all: zs_chain_kernel places
// every verified unit at its exact output offset.  Unused slots are marked
// inactive.
// ---------------------------------------------------------------------------
#define PLAN_T 256

__device__ uint32_t plan_block_scan(uint32_t v, uint32_t *s_tmp, uint32_t *total) {  // exclusive, PLAN_T threads
  const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  uint32_t wt;
  const uint32_t ex = find_scan_excl(v, &wt);
  if (lane == 0) s_tmp[wv] = wt;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (uint32_t k = 0; k < PLAN_T / WAVE; k++) {
    const uint32_t x = s_tmp[k];
    before += k < wv ? x : 0u;
    all += x;
  }
  __syncthreads();
  *total = all;
  return before + ex;
}

__global__ void __launch_bounds__(PLAN_T) zs_plan_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                          const ZsSegDev *__restrict__ segs, ZsCJobDev *__restrict__ cjobs,
                                                          ZsChunkDev *__restrict__ units, ZsTokPool pool) {
  __shared__ uint32_t s_tmp[PLAN_T / WAVE];
  __shared__ uint64_t s_cap_base;
  __shared__ uint64_t s_c[PLAN_T];
  const uint32_t t = threadIdx.x;
  const ZsCJobDev cj = cjobs[blockIdx.x];
  const ZsJobDev jb = jobs[cj.job];
  const ZsHeadDev hd = heads[cj.job];
  const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(jb.in) & 3u);
  const uint32_t end_bit = (mis + (uint32_t)jb.in_len) * 8u;
  const uint32_t ecap = (uint32_t)min<uint64_t>(jb.out_cap, 0xfff00000ull);
  uint32_t nunits = 0;
  if (hd.code == ZD_END) {
    // unit index of each segment's first candidate (unit 0 = stream start)
    uint32_t run = 1;
    if (t == 0) s_cap_base = 0;
    for (uint32_t s0 = 0; s0 < cj.nseg; s0 += PLAN_T) {
      const uint32_t sg = s0 + t;
      const ZsSegDev *sgp = segs + cj.first_seg + sg;
      const uint32_t c = sg < cj.nseg ? (sgp->ncand ? sgp->ncand : sgp->nfixed) : 0u;
      uint32_t tot;
      const uint32_t ex = plan_block_scan(c, s_tmp, &tot);
      for (uint32_t k = 0; k < c; k++) {
        ZsChunkDev u{};
        u.start_bit = segs[cj.first_seg + sg].cand[k];
        units[cj.unit0 + run + ex + k] = u;  // start only; completed below
      }
      run += tot;
    }
    nunits = run;
    if (t == 0) {
      ZsChunkDev u{};
      u.start_bit = (mis + (uint32_t)hd.start_byte) * 8u + jb.sbit;
      units[cj.unit0] = u;
    }
    __syncthreads();
    // stops, spans, primary token regions (scanned in u64 through per-thread sums)
    for (uint32_t u0 = 0; u0 < nunits; u0 += PLAN_T) {
      const uint32_t i = u0 + t;
      uint64_t cap = 0;
      uint32_t st = 0, sp = ZS_NONE;
      if (i < nunits) {
        st = units[cj.unit0 + i].start_bit;
        sp = i + 1 < nunits ? units[cj.unit0 + i + 1].start_bit : ZS_NONE;
        const uint32_t span_bytes = ((sp == ZS_NONE ? end_bit : sp) - st + 7u) / 8u;
        // whole 128-byte lines: every unit's token region starts line-aligned (the split
        // decode writes 64-byte halves, round 6)
        cap = ((uint64_t)span_bytes * ZS_TOK_PER_BYTE + ZS_TOK_SLACK + 31u) & ~31ull;
      }
      // exclusive u64 prefix of the regions (thread 0 walks the tile)
      s_c[t] = cap;
      __syncthreads();
      if (t == 0) {
        uint64_t acc = s_cap_base;
        for (uint32_t k = 0; k < PLAN_T; k++) {
          const uint64_t x = s_c[k];
          s_c[k] = acc;
          acc += x;
        }
        s_cap_base = acc;
      }
      __syncthreads();
      const uint64_t pre = s_c[t];
      if (i < nunits) {
        ZsChunkDev u{};
        u.job = cj.job;
        u.ord = i;
        u.first = cj.unit0;
        u.nunits = nunits;
        u.start_bit = st;
        u.stop_bit = sp;
        u.end_bit = 0;
        u.code = ZD_SKIP;
        u.cap = ecap;
        u.tcap = (uint32_t)cap;
        u.scratch = 0;
        u.tok = cj.tok0 + pre;
        u.chain_next = ZS_NONE;
        u.in_chain = 0;
        units[cj.unit0 + i] = u;  // start_bit unchanged: neighbours' reads stay valid
        uint4 *pt = reinterpret_cast<uint4 *>(pool.ptab + (size_t)(cj.unit0 + i) * ZS_TP_MAXPG);
#pragma unroll
        for (int k = 0; k < ZS_TP_MAXPG / 4; k++) pt[k] = make_uint4(0, 0, 0, 0);
      }
      __syncthreads();
    }
  }
  __syncthreads();
  for (uint32_t i = nunits + t; i < cj.max_units; i += PLAN_T) {
    ZsChunkDev u{};
    u.job = cj.job;
    u.start_bit = ZS_NONE;
    u.stop_bit = ZS_NONE;
    u.code = ZD_SKIP;
    u.chain_next = ZS_NONE;
    units[cj.unit0 + i] = u;
  }
  if (t == 0) {
    cjobs[blockIdx.x].nunits = nunits;
    cjobs[blockIdx.x].nchain = 0;
    cjobs[blockIdx.x].ok = 0;
  }
}

// ---------------------------------------------------------------------------
// Fixed tables (src/inflate.c:260-298) built once into global memory.
// ---------------------------------------------------------------------------
// (d64: the deflate64 set -- length code 285 = 3 + 16 extra bits, distance
// codes 30 and 31 valid, src/inftrees.c:73-87)
__global__ void __launch_bounds__(64) zs_fixed_tables_kernel(uint32_t *__restrict__ fixed, int d64) {
  __shared__ uint32_t s_tab[544];
  __shared__ uint16_t s_lens[320];
  __shared__ uint16_t s_sorted[320];
  __shared__ uint32_t s_scr[32];
  const uint32_t lane = threadIdx.x;
  for (uint32_t s = lane; s < 288; s += WAVE) s_lens[s] = s < 144 ? 8 : (s < 256 ? 9 : (s < 280 ? 7 : 8));
  __builtin_amdgcn_wave_barrier();
  uint32_t r = 9;
  build_table(T_LENS, s_lens, 288, s_tab, &r, s_sorted, s_scr, d64);
  for (uint32_t s = lane; s < 32; s += WAVE) s_lens[s] = 5;
  __builtin_amdgcn_wave_barrier();
  r = 5;
  build_table(T_DISTS, s_lens, 32, s_tab + 512, &r, s_sorted, s_scr, d64);
  for (uint32_t i = lane; i < 544; i += WAVE) fixed[i] = s_tab[i];
}

// ---------------------------------------------------------------------------
// Chain (one 1024-thread workgroup per stream), between parse and expand:
//   A. in parallel, every unit finds its successor: the first later unit whose
//      start is its end bit (recorded starts that are not block boundaries
//      are skipped; starts ascend, so the search stops early);
//   B. thread 0 walks the successors (in LDS for up to LINK_MAXU units),
//      assigning output offsets and writing the chain in order to `info`;
//      every chain member's u16 entries are placed at the job's entry base +
//      its output offset, so entry space is exact (no per-unit estimate) and
//      the expand pass runs only on chain members.
// Any break (a unit that did not end at a block boundary, no successor, more
// output than out_cap) sends the stream to the exact serial decoder.
// ---------------------------------------------------------------------------
#define LINK_THREADS 1024
#define LINK_PER (HIST / LINK_THREADS)  // window entries per thread and chain step
#define LINK_MAXU 4096                  // units per stream with the successor walk in LDS

struct ZsLinkInfo {
  uint64_t scratch;
  uint32_t n_out;
  uint32_t unit;  // unit index (ord 0 <=> first of the job)
};

// Per stream: each unit's successor (the first later unit starting at its end
// bit), then the chain from the stream's first unit: exact output offsets and
// entry ranges of its members.  Round 6: with every unit field staged in LDS,
// the chain is a parallel prefix over predecessor links (pointer jumping,
// <= 12 rounds: each unit learns its chain's head, rank and offsets; members
// are the units headed by the first unit), unless a unit has two
// predecessors (a false start that resynchronised onto the true symbol grid
// ends where a true unit ends) or the stream has more than LINK_MAXU units:
// then thread 0 walks the chain as before.  The walk took 0.38-0.46 ms per C2
// batch (~720 dependent steps per stream).
__global__ void __launch_bounds__(LINK_THREADS) zs_chain_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                                ZsChunkDev *__restrict__ chunks, ZsCJobDev *__restrict__ cjobs,
                                                                ZsLinkInfo *__restrict__ info, ZsDecDev *__restrict__ decs,
                                                                uint32_t *__restrict__ fallback) {
  __shared__ uint16_t s_succ[LINK_MAXU];  // successor - unit (0: none / end)
  __shared__ uint8_t s_code[LINK_MAXU];
  __shared__ uint32_t s_nout[LINK_MAXU], s_endb[LINK_MAXU], s_sb[LINK_MAXU];
  __shared__ uint32_t s_pj[LINK_MAXU];  // jump pointer (predecessor 2^r back; NONE) | head << 16
  __shared__ uint32_t s_rk[LINK_MAXU], s_sa[LINK_MAXU], s_st[LINK_MAXU];  // exclusive sums: members, entries (8-aligned), bytes
  __shared__ uint32_t s_merge, s_r1, s_r2, s_flag;
  const uint32_t t = threadIdx.x;
  const ZsCJobDev cj = cjobs[blockIdx.x];
  const ZsJobDev jb = jobs[cj.job];
  const ZsHeadDev hd = heads[cj.job];
  if (hd.code != ZD_END || cj.nunits == 0) {
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
  const uint32_t u0 = cj.unit0, nu = cj.nunits, last = u0 + nu;
  const bool small = nu <= LINK_MAXU;
  const bool part = (jb.flags & ZS_JF_PART) != 0;
  constexpr uint32_t PNONE = 0xffffu;
  if (small) {
    for (uint32_t i = t; i < nu; i += LINK_THREADS) {
      s_sb[i] = chunks[u0 + i].start_bit;
      s_pj[i] = PNONE;
    }
    if (t == 0) {
      s_merge = 0;
      s_flag = 0;
    }
    __syncthreads();
  }
  // A: successors (and, staged, every field the chain needs)
  for (uint32_t i = u0 + t; i < last; i += LINK_THREADS) {
    const ZsChunkDev ch = chunks[i];
    const int code = ch.code & 0xff;
    uint32_t k = ZS_NONE;
    if (code == ZD_STOP) {
      for (uint32_t o = i + 1; o < last; o++) {
        const uint32_t sb = small ? s_sb[o - u0] : chunks[o].start_bit;
        if (sb == ch.end_bit) {
          k = o;
          break;
        }
        if (sb > ch.end_bit) break;
      }
    }
    chunks[i].chain_next = k;
    if (small) {
      s_succ[i - u0] = (k == ZS_NONE || k - i > 0xffffu) ? (uint16_t)0 : (uint16_t)(k - i);
      s_code[i - u0] = (uint8_t)code;
      s_nout[i - u0] = ch.n_out;
      s_endb[i - u0] = ch.end_bit;
      if (k != ZS_NONE && atomicCAS(&s_pj[k - u0], PNONE, i - u0) != PNONE) s_merge = 1;
    }
  }
  __syncthreads();
  if (small && !s_merge && cj.scratch_n < 0xf0000000ull) {
    // initial sums: the predecessor's own values; head = self until resolved
    for (uint32_t i = t; i < nu; i += LINK_THREADS) {
      const uint32_t p = s_pj[i];
      s_rk[i] = p != PNONE ? 1u : 0u;
      s_sa[i] = p != PNONE ? (s_nout[p] + 7u) & ~7u : 0u;
      s_st[i] = p != PNONE ? s_nout[p] : 0u;
      s_pj[i] = p | ((p != PNONE ? p : i) << 16);  // jump | head (the farthest node reached)
    }
    __syncthreads();
    // pointer jumping: read a round's values, then write them (<= 4 units per thread)
    for (uint32_t r = 0; r < 12; r++) {
      uint32_t nj[LINK_MAXU / LINK_THREADS], ar[LINK_MAXU / LINK_THREADS], aa[LINK_MAXU / LINK_THREADS],
          at[LINK_MAXU / LINK_THREADS];
      bool any = false;
#pragma unroll
      for (uint32_t q = 0; q < LINK_MAXU / LINK_THREADS; q++) {
        const uint32_t i = t + q * LINK_THREADS;
        nj[q] = 0xffffffffu;
        if (i < nu) {
          const uint32_t pj = s_pj[i], j = pj & 0xffffu;
          if (j != PNONE) {
            nj[q] = s_pj[j];
            ar[q] = s_rk[j];
            aa[q] = s_sa[j];
            at[q] = s_st[j];
            any = true;
          }
        }
      }
      if (!__syncthreads_or(any)) break;
#pragma unroll
      for (uint32_t q = 0; q < LINK_MAXU / LINK_THREADS; q++) {
        const uint32_t i = t + q * LINK_THREADS;
        if (nj[q] != 0xffffffffu) {
          s_rk[i] += ar[q];
          s_sa[i] += aa[q];
          s_st[i] += at[q];
          s_pj[i] = nj[q];  // its jump and its head (the head of what j reached)
        }
      }
      __syncthreads();
    }
    // the walk's stop, in rank order: r1 = first member rejected before it is
    // taken (not a block end, or past the entry / piece budget), r2 = first
    // member after which the chain ends (end of stream, or no successor)
    if (t == 0) {
      s_r1 = 0xffffffffu;
      s_r2 = 0xffffffffu;
    }
    __syncthreads();
    for (uint32_t i = t; i < nu; i += LINK_THREADS) {
      if ((s_pj[i] >> 16) != 0u) continue;  // not headed by the stream's first unit
      const uint32_t code = s_code[i], n = s_nout[i], rk = s_rk[i];
      const uint64_t spos = s_sa[i];
      if ((code != ZD_STOP && code != ZD_END) || spos + n > cj.scratch_n || (part && (uint64_t)s_st[i] + n > ZS_PART_OUT))
        atomicMin(&s_r1, rk);
      if (code == ZD_END || s_succ[i] == 0) atomicMin(&s_r2, rk);
    }
    __syncthreads();
    const uint32_t r1 = s_r1, r2 = s_r2;
    const uint32_t len = r1 <= r2 ? r1 : r2 + 1u;  // members taken (ranks 0 .. len - 1)
    for (uint32_t i = t; i < nu; i += LINK_THREADS) {
      if ((s_pj[i] >> 16) != 0u || s_rk[i] >= len) continue;
      ZsLinkInfo li;
      li.scratch = cj.scratch0 + (uint64_t)cj.esz * s_sa[i];
      li.n_out = s_nout[i];
      li.unit = u0 + i;
      info[u0 + s_rk[i]] = li;
      chunks[u0 + i].out_off = s_st[i];
      chunks[u0 + i].scratch = li.scratch;
      if (s_rk[i] + 1u == len) s_flag = i;  // the last member taken
    }
    __syncthreads();
    if (t == 0) {
      uint32_t ok = 1, cut = 0, end_bit = 0;
      uint64_t total = 0;
      if (len) {
        const uint32_t m = s_flag;
        total = (uint64_t)s_st[m] + s_nout[m];
        end_bit = s_endb[m];
      }
      if (r1 <= r2) {  // stopped before member r1
        if (part && len) cut = 1;
        else ok = 0;
      } else if (s_code[s_flag] != ZD_END) {  // member r2 has no successor
        if (part) cut = 1;
        else ok = 0;
      }
      if (total > jb.out_cap) ok = 0;
      if (ok) {
        ZsDecDev d;
        d.code = cut ? ZD_STOP : ZD_END;
        d.msg = 0;
        const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(jb.in) & 3u);
        d.end_bits = end_bit - mis * 8u;
        d.total_out = total;
        decs[cj.job] = d;
      }
      fallback[cj.job] = ok ? 0u : 1u;
      cjobs[blockIdx.x].nchain = ok ? len : 0u;
      cjobs[blockIdx.x].ok = ok;
      s_r1 = ok;  // (reused: the members are flagged below)
    }
    __syncthreads();
    if (s_r1)
      for (uint32_t i = t; i < nu; i += LINK_THREADS)
        if ((s_pj[i] >> 16) == 0u && s_rk[i] < len) chunks[u0 + i].in_chain = 1;
    return;
  }
  // B: walk the chain.  A piece of a longer stream (ZS_JF_PART) ends its
  // chain at the last verified block boundary instead of failing: before a
  // member that did not stop at a block boundary (the unit cut off by the
  // piece's end) or that would pass the piece's output budget, or after a
  // member with no successor; the next piece resumes there (ZD_STOP).
  if (t == 0) {
    const bool part = (jb.flags & ZS_JF_PART) != 0;
    uint32_t c = u0, len = 0, ok = 1, end_bit = 0, cut = 0, last_end = 0;
    uint64_t total = 0, spos = 0;  // output bytes; entries used (each member starts 8-entry aligned)
    for (;;) {
      const ZsChunkDev ch = chunks[c];
      const int code = ch.code & 0xff;
      spos = (spos + 7u) & ~7ull;
      if ((code != ZD_STOP && code != ZD_END) || spos + ch.n_out > cj.scratch_n ||
          (part && total + ch.n_out > ZS_PART_OUT)) {
        if (part && len) {
          cut = 1;
          end_bit = last_end;
        } else {
          ok = 0;
        }
        break;
      }
      ZsLinkInfo li;
      li.scratch = cj.scratch0 + (uint64_t)cj.esz * spos;
      li.n_out = ch.n_out;
      li.unit = c;
      info[u0 + len] = li;
      len++;
      chunks[c].out_off = total;
      chunks[c].scratch = li.scratch;
      total += ch.n_out;
      spos += ch.n_out;
      last_end = ch.end_bit;
      if (code == ZD_END) {
        end_bit = ch.end_bit;
        break;
      }
      uint32_t k;
      if (small) {
        const uint32_t d = s_succ[c - u0];
        k = d ? c + d : ZS_NONE;
      } else {
        k = ch.chain_next;
      }
      if (k == ZS_NONE) {
        if (part) {
          cut = 1;
          end_bit = last_end;
        } else {
          ok = 0;
        }
        break;
      }
      c = k;
    }
    if (total > jb.out_cap) ok = 0;
    if (ok) {  // members are flagged only once the whole chain holds
      for (uint32_t j = 0; j < len; j++) chunks[info[u0 + j].unit].in_chain = 1;
      ZsDecDev d;
      d.code = cut ? ZD_STOP : ZD_END;
      d.msg = 0;
      const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(jb.in) & 3u);
      d.end_bits = end_bit - mis * 8u;
      d.total_out = total;
      decs[cj.job] = d;
    }
    fallback[cj.job] = ok ? 0u : 1u;
    cjobs[blockIdx.x].nchain = ok ? len : 0u;
    cjobs[blockIdx.x].ok = ok;
  }
}

// ---------------------------------------------------------------------------
// Link (one 1024-thread workgroup per verified stream), after expand: the
// 32 KiB history windows are resolved in chain order from each unit's last
// HIST entries; the entries of the next chain member are loaded into
// registers while the current one resolves (one memory latency per step is
// hidden behind the LDS work).
// ---------------------------------------------------------------------------
// thread t owns window entries 4t + 4096 g + {0..3}, g < LINK_PER / 4; entry
// pairs are packed in u32 (2 per word, 2 words per group)
template <uint32_t HN>
__device__ __forceinline__ void link_load(const uint16_t *__restrict__ scratch, const ZsLinkInfo &li, uint32_t t,
                                          uint2 (&lo)[HN / LINK_THREADS / 4], uint2 (&hi)[HN / LINK_THREADS / 4]) {
  // window entry i is the unit's entry n - HN + i (0 before the unit: a short
  // unit).  Two aligned 8-byte loads per 4 entries whatever the unit, and the
  // funnel shift left to link_take: the same loads every step and no use of
  // them before the next step lets the compiler wait for exactly the loads it
  // needs (vmcnt is in order; a branchy, immediately consumed load sequence
  // made it wait for everything, the prefetch included)
  constexpr int LINK_G = HN / LINK_THREADS / 4;
  const int64_t b0 = (int64_t)li.scratch + (int64_t)li.n_out - (int64_t)HN;  // entry index of window entry 0
  const uint32_t m = (uint32_t)((uint64_t)b0 & 3u);
#pragma unroll
  for (int g = 0; g < LINK_G; g++) {
    const int64_t e = b0 + (int64_t)((uint32_t)g * (LINK_THREADS * 4) + t * 4);
    const uint2 *al = reinterpret_cast<const uint2 *>(scratch + (e < 0 ? 0u : (uint64_t)(e - (int64_t)m)));
    lo[g] = al[0];
    hi[g] = al[1];
  }
}
template <uint32_t HN>
__device__ __forceinline__ uint2 link_take(const ZsLinkInfo &li, uint32_t t, int g, uint2 lo, uint2 hi) {
  const int64_t b0 = (int64_t)li.scratch + (int64_t)li.n_out - (int64_t)HN;
  const uint32_t m = (uint32_t)((uint64_t)b0 & 3u);
  const uint64_t x = (uint64_t)lo.x | ((uint64_t)lo.y << 32), c = (uint64_t)hi.x | ((uint64_t)hi.y << 32);
  uint64_t r = (x >> (16 * m)) | ((c << 1) << (63 - 16 * m));  // m = 0: c contributes nothing
  if (li.n_out < HN) {  // short unit: entries before it read as 0 (the keep rule replaces them)
    const int64_t e = b0 + (int64_t)((uint32_t)g * (LINK_THREADS * 4) + t * 4);
    const int64_t first = (int64_t)li.scratch - e;  // entries of this group before the unit
    if (first >= 4) r = 0;
    else if (first > 0) r &= ~0ull << (16 * first);
  }
  return make_uint2((uint32_t)r, (uint32_t)(r >> 32));
}

#define LS_SEGS_MAX 8u  // segments per chain at most (segmented link)
template <uint32_t HN>
__global__ void __launch_bounds__(LINK_THREADS) zs_link_kernel(const ZsJobDev *__restrict__ jobs, ZsCJobDev *__restrict__ cjobs,
                                                               const uint16_t *__restrict__ scratch, uint8_t *__restrict__ windows,
                                                               const ZsLinkInfo *__restrict__ info, uint32_t *__restrict__ fallback,
                                                               uint32_t nseg_per = 1, const uint16_t *__restrict__ sstart = nullptr,
                                                               const ZsChunkDev *__restrict__ chunks = nullptr) {
  constexpr int LINK_G = HN / LINK_THREADS / 4;
  constexpr uint32_t MB = HN == 65536u ? 0u : MARK_BASE;  // marker of history byte w: MB + w (deflate64: w)
  __shared__ uint8_t s_win[2][HN];
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x;
  // segments (pass 2 of the segmented link): workgroup (chain b, segment k)
  // links members [m0, m1) from the segment's start window (zs_linkseg_join_kernel)
  const uint32_t b = blockIdx.x / nseg_per, k = blockIdx.x % nseg_per;
  const ZsCJobDev cj = cjobs[b];
  if (!cj.ok) return;
  const uint32_t m0 = (uint32_t)((uint64_t)k * cj.nchain / nseg_per);
  const uint32_t m1 = (uint32_t)((uint64_t)(k + 1) * cj.nchain / nseg_per);
  if (m0 >= m1) return;
  const uint32_t u0 = cj.unit0 + m0;
  const uint32_t len = m1 - m0;
#if KP_ON
  const uint64_t kt0 = KP_NOW();
  uint64_t kt_ww = 0, kt_res = 0, kt_bar = 0;
  uint32_t kmark = 0;
#endif
  if (t == 0) s_bad = 0;
  // W holds the last HN bytes before unit c; a later piece of a long stream
  // (ZS_JF_CONT) starts with the earlier pieces' output before its own
  const ZsJobDev jb = jobs[cj.job];
  const bool cont = (jb.flags & ZS_JF_CONT) != 0;
  uint32_t wv = cont ? min(jb.hist, HN) : 0u;  // valid bytes of history
  if (k > 0) {  // a later segment: its start window, valid as far as output precedes it
    const uint16_t *S = sstart + ((size_t)b * LS_SEGS_MAX + (k - 1u)) * HN;
    wv = (uint32_t)min<uint64_t>(HN, chunks[info[u0].unit].out_off + (cont ? jb.hist : 0u));
    for (uint32_t i = t; i < HN; i += LINK_THREADS) s_win[0][i] = (uint8_t)S[i];
  } else if (cont) {
    for (uint32_t i = HN - wv + t; i < HN; i += LINK_THREADS) s_win[0][i] = jb.out[(int64_t)i - (int64_t)HN];
  }
  __syncthreads();
  int cur = 0;
  uint2 la[LINK_G], ha[LINK_G], lb[LINK_G], hb[LINK_G];
  bool bad = false;
  // member j's entries were loaded one step earlier; each step first issues
  // the next member's loads, then resolves, then stores the window (two
  // register sets, swapped by unrolling by two: no copies of loaded registers)
  link_load<HN>(scratch, info[u0], t, la, ha);
  auto step = [&](uint32_t j, const uint2 (&vl)[LINK_G], const uint2 (&vh)[LINK_G], uint2 (&nl)[LINK_G],
                  uint2 (&nh)[LINK_G]) {
    const ZsLinkInfo li = info[u0 + j];
    link_load<HN>(scratch, info[u0 + min(j + 1, len - 1)], t, nl, nh);
    __builtin_amdgcn_sched_barrier(0);  // nothing that uses this step's entries moves above the next loads
    uint2 v[LINK_G];
#pragma unroll
    for (int g = 0; g < LINK_G; g++) v[g] = link_take<HN>(li, t, g, vl[g], vh[g]);
    const uint32_t c = li.unit;
    uint8_t *W = s_win[cur];
    uint8_t *W2 = s_win[cur ^ 1];
#if KP_ON
    const uint64_t kb = KP_NOW();
#endif
    const uint32_t n = li.n_out;
    const uint32_t keep = n < HN ? HN - n : 0u;  // old history bytes still inside the new window
    const uint32_t lowest = HN - wv;                // first valid history index
    if (keep == 0 && lowest == 0) {
      // common case (full window, unit >= 32 KiB): branch-free gather, every
      // entry reads the window and selects literal or history byte
#pragma unroll
      for (int g = 0; g < LINK_G; g++) {
        const uint32_t i = (uint32_t)g * (LINK_THREADS * 4) + t * 4;
        const uint32_t x0 = v[g].x & 0xffffu, x1 = v[g].x >> 16, x2 = v[g].y & 0xffffu, x3 = v[g].y >> 16;
        const uint32_t r0 = W[(x0 - MB) & (HN - 1)], r1 = W[(x1 - MB) & (HN - 1)];
        const uint32_t r2 = W[(x2 - MB) & (HN - 1)], r3 = W[(x3 - MB) & (HN - 1)];
        const uint32_t b0 = x0 < MARK_BASE ? x0 : r0, b1 = x1 < MARK_BASE ? x1 : r1;
        const uint32_t b2 = x2 < MARK_BASE ? x2 : r2, b3 = x3 < MARK_BASE ? x3 : r3;
        *reinterpret_cast<uint32_t *>(W2 + i) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
#if KP_ON
        kmark += (x0 >= MARK_BASE) + (x1 >= MARK_BASE) + (x2 >= MARK_BASE) + (x3 >= MARK_BASE);
#endif
      }
    } else {
#pragma unroll
      for (int g = 0; g < LINK_G; g++) {
        const uint32_t xs[4] = {v[g].x & 0xffffu, v[g].x >> 16, v[g].y & 0xffffu, v[g].y >> 16};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t i = (uint32_t)g * (LINK_THREADS * 4) + t * 4 + k;
          const uint32_t x = xs[k];
          uint32_t b;
          if (i < keep) {
            b = W[i + n];
          } else if (x < MARK_BASE) {
            b = x;
          } else {
            const uint32_t wx = x - MB;
            bad |= wx < lowest;  // reaches before the stream start
            b = W[wx & (HN - 1)];
          }
          W2[i] = (uint8_t)b;
        }
      }
    }
#if KP_ON
    const uint64_t ka = KP_NOW();
    kt_res += ka - kb;
#endif
    // the window before unit c (for the first unit of a stream it is unused)
    {
      uint8_t *g = windows + (size_t)c * HN;
#pragma unroll
      for (uint32_t i = t * 16; i < HN; i += LINK_THREADS * 16)
        *reinterpret_cast<uint4 *>(g + i) = *reinterpret_cast<const uint4 *>(W + i);
    }
#if KP_ON
    const uint64_t kc = KP_NOW();
    kt_ww += kc - ka;
#endif
    wv = min(HN, wv + n);
    cur ^= 1;
    __syncthreads();
#if KP_ON
    kt_bar += KP_NOW() - kc;
#endif
  };
  for (uint32_t j = 0; j < len; j += 2) {
    step(j, la, ha, lb, hb);
    if (j + 1 < len) step(j + 1, lb, hb, la, ha);
  }
  if (bad) s_bad = 1;
  __syncthreads();
#if KP_ON
  if ((t & 63) == 0) KPC_ADD(KP_L_MARKERS, kmark);  // lane 0 of each wave: a sample
  if (t == 0) {
    const uint64_t tot = KP_NOW() - kt0;
    KPC_ADD(KP_L_STREAMS, 1);
    KPC_ADD(KP_L_STEPS, len);
    KPC_ADD(KP_L_CYC_WINWRITE, kt_ww);
    KPC_ADD(KP_L_CYC_RESOLVE, kt_res);
    KPC_ADD(KP_L_CYC_BARRIER, kt_bar);
    KPC_ADD(KP_L_CYC_TOTAL, tot);
    KPC_MAX(KP_L_CYC_MAX, tot);
  }
#endif
  if (t == 0 && s_bad) {  // a marker reached before the stream start: the serial decoder reports it
    fallback[cj.job] = 1;
    cjobs[b].ok = 0;
  }
}

// ---------------------------------------------------------------------------
// Segmented link (5..64 streams; zs_link_kernel alone links one chain per
// workgroup, a serial chain of ~3.5 us steps per member while most CUs idle):
// each chain is cut into S segments.  Pass 1 (zs_linkseg_kernel) links every
// segment at once from an unknown start window, as MAPS: u16 windows whose
// entries are a byte or MARK_BASE + w, "byte w of the segment's start window"
// (segment 0 starts from the stream's real history, so its map is bytes); only
// the map after a segment's last member is kept (M_end[k]).
// zs_linkseg_join_kernel resolves the segments' start windows in order (S - 1
// map applications per stream).  Pass 2 (zs_link_kernel with segments) links
// every segment again from its real start window, writing the members' byte
// windows as the serial link does, and the emit is unchanged.  Bytes before
// the stream start stay unresolved (0), as in zs_link_kernel: the emit's
// `lowest` check reports any marker into them.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(LINK_THREADS) zs_linkseg_kernel(const ZsJobDev *__restrict__ jobs,
                                                                  const ZsCJobDev *__restrict__ cjobs, uint32_t nseg_per,
                                                                  const uint16_t *__restrict__ scratch,
                                                                  uint16_t *__restrict__ mend,
                                                                  const ZsLinkInfo *__restrict__ info) {
  constexpr uint32_t HN = HIST;
  constexpr int LINK_G = HN / LINK_THREADS / 4;
  __shared__ __attribute__((aligned(16))) uint16_t s_map[2][HN];
  const uint32_t t = threadIdx.x;
  const uint32_t b = blockIdx.x / nseg_per, k = blockIdx.x % nseg_per;
  const ZsCJobDev cj = cjobs[b];
  if (!cj.ok) return;
  const uint32_t u0 = cj.unit0, len = cj.nchain;
  const uint32_t m0 = (uint32_t)((uint64_t)k * len / nseg_per), m1 = (uint32_t)((uint64_t)(k + 1) * len / nseg_per);
  const ZsJobDev jb = jobs[cj.job];
  // start map: segment 0 the stream's history (a later piece's earlier output),
  // else the identity (entry i = byte i of the start window)
  if (k == 0) {
    const bool cont = (jb.flags & ZS_JF_CONT) != 0;
    const uint32_t wv = cont ? min(jb.hist, HN) : 0u;
    for (uint32_t i = t; i < HN; i += LINK_THREADS)
      s_map[0][i] = i >= HN - wv ? (uint16_t)jb.out[(int64_t)i - (int64_t)HN] : (uint16_t)0;
  } else {
    for (uint32_t i = t; i < HN; i += LINK_THREADS) s_map[0][i] = (uint16_t)(MARK_BASE + i);
  }
  __syncthreads();
  int cur = 0;
  uint2 la[LINK_G], ha[LINK_G], lb[LINK_G], hb[LINK_G];
  if (m0 < m1) link_load<HN>(scratch, info[u0 + m0], t, la, ha);
  auto step = [&](uint32_t j, const uint2 (&vl)[LINK_G], const uint2 (&vh)[LINK_G], uint2 (&nl)[LINK_G],
                  uint2 (&nh)[LINK_G]) {
    const ZsLinkInfo li = info[u0 + j];
    link_load<HN>(scratch, info[u0 + min(j + 1, m1 - 1)], t, nl, nh);
    __builtin_amdgcn_sched_barrier(0);
    const uint16_t *W = s_map[cur];
    uint16_t *W2 = s_map[cur ^ 1];
    const uint32_t n = li.n_out;
    const uint32_t keep = n < HN ? HN - n : 0u;
#pragma unroll
    for (int g = 0; g < LINK_G; g++) {
      const uint2 v = link_take<HN>(li, t, g, vl[g], vh[g]);
      const uint32_t xs[4] = {v.x & 0xffffu, v.x >> 16, v.y & 0xffffu, v.y >> 16};
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t i = (uint32_t)g * (LINK_THREADS * 4) + t * 4 + q;
        const uint32_t x = xs[q];
        o[q] = i < keep ? W[i + n] : (x < MARK_BASE ? x : W[(x - MARK_BASE) & (HN - 1)]);
      }
      *reinterpret_cast<uint2 *>(W2 + (uint32_t)g * (LINK_THREADS * 4) + t * 4) =
          make_uint2(o[0] | (o[1] << 16), o[2] | (o[3] << 16));
    }
    cur ^= 1;
    __syncthreads();
  };
  for (uint32_t j = m0; j < m1; j += 2) {
    step(j, la, ha, lb, hb);
    if (j + 1 < m1) step(j + 1, lb, hb, la, ha);
  }
  // the map after the segment's last member (the next segment's start window)
  uint16_t *g = mend + ((size_t)b * LS_SEGS_MAX + k) * HN;
  for (uint32_t i = t * 8; i < HN; i += LINK_THREADS * 8)
    *reinterpret_cast<uint4 *>(g + i) = *reinterpret_cast<const uint4 *>(&s_map[cur][i]);
}

// start windows of every segment: S(0) unused (segment 0's maps are bytes),
// S(1) = M_end(0), S(k) = M_end(k - 1) applied to S(k - 1); written over the
// chain's M_end slots (M_end(k - 1) -> S(k)), one workgroup per chain (slots
// indexed by the chain's place in the group)
__global__ void __launch_bounds__(LINK_THREADS) zs_linkseg_join_kernel(const ZsCJobDev *__restrict__ cjobs, uint32_t nseg_per,
                                                                       uint16_t *__restrict__ mend) {
  constexpr uint32_t HN = HIST;
  __shared__ __attribute__((aligned(16))) uint16_t s_prev[HN];
  const uint32_t t = threadIdx.x;
  const ZsCJobDev cj = cjobs[blockIdx.x];
  if (!cj.ok) return;
  uint16_t *base = mend + (size_t)blockIdx.x * LS_SEGS_MAX * HN;
  // S(1) = M_end(0): bytes already
  for (uint32_t i = t; i < HN; i += LINK_THREADS) s_prev[i] = base[i];
  __syncthreads();
  for (uint32_t k = 1; k + 1 < nseg_per; k++) {
    uint16_t *m = base + (size_t)k * HN;  // M_end(k) -> S(k + 1)
    uint16_t r[HN / LINK_THREADS];
#pragma unroll
    for (uint32_t q = 0; q < HN / LINK_THREADS; q++) {
      const uint32_t v = m[t + q * LINK_THREADS];
      r[q] = v < MARK_BASE ? (uint16_t)v : s_prev[(v - MARK_BASE) & (HN - 1)];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < HN / LINK_THREADS; q++) {
      m[t + q * LINK_THREADS] = r[q];
      s_prev[t + q * LINK_THREADS] = r[q];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Emit: u16 entries -> final bytes (one workgroup per chunk)
// ---------------------------------------------------------------------------
#ifndef EMIT_THREADS
#define EMIT_THREADS 256
#endif
template <uint32_t HN>
__global__ void __launch_bounds__(EMIT_THREADS) zs_emit_kernel(const ZsJobDev *__restrict__ jobs, const ZsChunkDev *__restrict__ chunks,
                                                               const uint16_t *__restrict__ scratch, const uint8_t *__restrict__ windows,
                                                               uint32_t *__restrict__ fallback) {
  constexpr uint32_t MB = HN == 65536u ? 0u : MARK_BASE;
  __shared__ uint8_t s_w[HN];
  const uint32_t c = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const ZsChunkDev ch = chunks[c];
  if (!ch.in_chain || fallback[ch.job]) return;
  const ZsJobDev jb = jobs[ch.job];
  const uint64_t hist = (jb.flags & ZS_JF_CONT) ? jb.hist : 0u;  // output before the piece
  if (ch.ord != 0 || hist) {
    const uint8_t *g = windows + (size_t)c * HN;
    for (uint32_t i = t * 16; i < HN; i += EMIT_THREADS * 16)
      *reinterpret_cast<uint4 *>(s_w + i) = *reinterpret_cast<const uint4 *>(g + i);
    __syncthreads();
  }
  uint8_t *out = jb.out + ch.out_off;
  const uint16_t *e = scratch + ch.scratch;
  const uint32_t n = ch.n_out;
  // window bytes below `lowest` lie before the stream start: a marker into
  // them is a too-far distance (the parallel-prefix link leaves that check here)
  const uint32_t lowest = HN - (uint32_t)min<uint64_t>(HN, ch.out_off + hist);
  bool bad = false;
  // 16-byte output groups aligned in memory; group g covers unit bytes
  // [16 g - mis, 16 g - mis + 16).  Groups straddling the unit's ends are
  // written bytewise (neighbouring units own the other bytes).
  const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(out) & 15u);
  const uint32_t ngroups = (n + mis + 15u) / 16u;
  for (uint32_t g = t; g < ngroups; g += EMIT_THREADS) {
    const int32_t i0 = (int32_t)(g * 16u) - (int32_t)mis;  // unit byte of the group's first byte
    uint32_t b[16];
    if (i0 >= 0 && (uint32_t)i0 + 16u <= n) {
      uint4 lo, hi;
      __builtin_memcpy(&lo, e + i0, 16);
      __builtin_memcpy(&hi, e + i0 + 8, 16);
      const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t v = (w[k >> 1] >> (16 * (k & 1))) & 0xffffu;
        b[k] = v < MARK_BASE ? v : s_w[v - MB];
        bad |= v >= MARK_BASE && v - MB < lowest;
      }
      uint4 o;
      o.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
      o.y = b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24);
      o.z = b[8] | (b[9] << 8) | (b[10] << 16) | (b[11] << 24);
      o.w = b[12] | (b[13] << 8) | (b[14] << 16) | (b[15] << 24);
      *reinterpret_cast<uint4 *>(out + i0) = o;
    } else {
      for (int k = 0; k < 16; k++) {
        const int32_t i = i0 + k;
        if (i < 0 || (uint32_t)i >= n) continue;
        const uint32_t v = e[i];
        out[i] = (uint8_t)(v < MARK_BASE ? v : s_w[v - MB]);
        bad |= v >= MARK_BASE && v - MB < lowest;
      }
    }
  }
  if (__syncthreads_or(bad) && t == 0) fallback[ch.job] = 1;
}

// ---------------------------------------------------------------------------
// Deflate64 link and emit: 64 KiB windows, 17-bit entries stored as u32
// (literal byte, or 256 + w for byte w of the unit's 64 KiB history).
// ---------------------------------------------------------------------------
#define H64 65536u
// Thread t owns window entries 4t + 4096 g + {0..3}, g < 16: its 64 entries
// of a chain member are loaded together (16 x 16 B, issued back to back) so a
// step pays one memory latency, not one per entry.
#define L64_G (H64 / LINK_THREADS / 4)
__device__ __forceinline__ void link64_load(const uint16_t *__restrict__ scratch, const ZsLinkInfo &li, uint32_t t,
                                            uint4 (&v)[L64_G]) {
  const uint32_t *E = reinterpret_cast<const uint32_t *>(scratch + li.scratch);
  const uint32_t n = li.n_out;
  if (n >= H64) {
    const uint32_t *b = E + (n - H64);  // 4-byte aligned
#pragma unroll
    for (int g = 0; g < L64_G; g++) __builtin_memcpy(&v[g], b + (uint32_t)g * (LINK_THREADS * 4) + t * 4, 16);
  } else {  // short unit: entry i exists only for i >= H64 - n
#pragma unroll
    for (int g = 0; g < L64_G; g++) {
      const uint32_t i = (uint32_t)g * (LINK_THREADS * 4) + t * 4;
      uint32_t x[4];
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = (i + k + n >= H64) ? E[i + k + n - H64] : 0u;
      v[g] = make_uint4(x[0], x[1], x[2], x[3]);
    }
  }
}

__global__ void __launch_bounds__(LINK_THREADS) zs_link64_kernel(const ZsJobDev *__restrict__ jobs, ZsCJobDev *__restrict__ cjobs,
                                                                 const uint16_t *__restrict__ scratch,
                                                                 uint8_t *__restrict__ windows, const ZsLinkInfo *__restrict__ info,
                                                                 uint32_t *__restrict__ fallback) {
  __shared__ uint8_t s_win[2][H64];
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x;
  const ZsCJobDev cj = cjobs[blockIdx.x];
  if (!cj.ok) return;
  if (t == 0) s_bad = 0;
  const ZsJobDev jb = jobs[cj.job];
  const bool cont = (jb.flags & ZS_JF_CONT) != 0;  // as zs_link_kernel
  uint32_t wv = cont ? min(jb.hist, H64) : 0u;
  if (cont)
    for (uint32_t i = H64 - wv + t; i < H64; i += LINK_THREADS) s_win[0][i] = jb.out[(int64_t)i - (int64_t)H64];
  __syncthreads();
  int cur = 0;
  bool bad = false;
  uint4 v[L64_G];
  ZsLinkInfo li = info[cj.unit0];
  for (uint32_t j = 0; j < cj.nchain; j++) {
    link64_load(scratch, li, t, v);
    const ZsLinkInfo lin = j + 1 < cj.nchain ? info[cj.unit0 + j + 1] : li;
    const uint32_t n = li.n_out;
    uint8_t *W = s_win[cur];
    uint8_t *W2 = s_win[cur ^ 1];
    if (j != 0 || cont) {
      uint8_t *g = windows + (size_t)li.unit * H64;
      for (uint32_t i = t * 16; i < H64; i += LINK_THREADS * 16)
        *reinterpret_cast<uint4 *>(g + i) = *reinterpret_cast<const uint4 *>(W + i);
    }
    const uint32_t keep = n < H64 ? H64 - n : 0u;
    const uint32_t lowest = H64 - wv;
#pragma unroll
    for (int g = 0; g < L64_G; g++) {
      const uint32_t i0 = (uint32_t)g * (LINK_THREADS * 4) + t * 4;
      const uint32_t xs[4] = {v[g].x, v[g].y, v[g].z, v[g].w};
      uint32_t b[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t i = i0 + k, x = xs[k];
        if (i < keep) {
          b[k] = W[i + n];
        } else if (x < MARK_BASE) {
          b[k] = x;
        } else {
          const uint32_t wx = x - MARK_BASE;
          bad |= wx < lowest;
          b[k] = W[wx & (H64 - 1)];
        }
      }
      *reinterpret_cast<uint32_t *>(W2 + i0) = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
    }
    wv = min(H64, wv + n);
    cur ^= 1;
    li = lin;
    __syncthreads();
  }
  if (bad) s_bad = 1;
  __syncthreads();
  if (t == 0 && s_bad) {
    fallback[cj.job] = 1;
    cjobs[blockIdx.x].ok = 0;
  }
}

__global__ void __launch_bounds__(EMIT_THREADS) zs_emit64_kernel(const ZsJobDev *__restrict__ jobs, const ZsChunkDev *__restrict__ chunks,
                                                                 const uint16_t *__restrict__ scratch, const uint8_t *__restrict__ windows,
                                                                 uint32_t *__restrict__ fallback) {
  __shared__ uint8_t s_w[H64];
  const uint32_t c = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const ZsChunkDev ch = chunks[c];
  if (!ch.in_chain || fallback[ch.job]) return;
  const ZsJobDev jb = jobs[ch.job];
  const uint64_t hist = (jb.flags & ZS_JF_CONT) ? jb.hist : 0u;
  if (ch.ord != 0 || hist) {
    const uint8_t *g = windows + (size_t)c * H64;
    for (uint32_t i = t * 16; i < H64; i += EMIT_THREADS * 16)
      *reinterpret_cast<uint4 *>(s_w + i) = *reinterpret_cast<const uint4 *>(g + i);
    __syncthreads();
  }
  uint8_t *out = jb.out + ch.out_off;
  const uint32_t *e = reinterpret_cast<const uint32_t *>(scratch + ch.scratch);
  const uint32_t n = ch.n_out;
  const uint32_t lowest = H64 - (uint32_t)min<uint64_t>(H64, ch.out_off + hist);
  bool bad = false;
  for (uint32_t i = t; i < n; i += EMIT_THREADS) {
    const uint32_t v = e[i];
    out[i] = (uint8_t)(v < MARK_BASE ? v : s_w[(v - MARK_BASE) & (H64 - 1)]);
    bad |= v >= MARK_BASE && v - MARK_BASE < lowest;
  }
  if (__syncthreads_or(bad) && t == 0) fallback[ch.job] = 1;
}

// ---------------------------------------------------------------------------
// Link by parallel prefix, for batches of few long streams (one large file):
// the serial link resolves a stream's windows one chain member at a time,
// which for one stream of 1024 units is 1024 dependent steps.  Here each
// window W_j (the HN bytes before chain member j) is first a MAP over
// W_{j-1}: entry i is a literal byte, or MARK_BASE + w for byte w of W_{j-1}
//   M_j[i] = i < keep ? ref(i + n) : E_{j-1}[i + n - HN],
// n = member j-1's output, keep = HN - n (src/inffast.c window semantics, as
// zs_link_kernel).  Maps compose (A o B: literals stay, ref w -> B[w]), so
// a Hillis-Steele scan over the chain (ceil(log2 nchain) launches, each
// composing every map with the one 2^d members earlier) leaves every W_j in
// terms of the stream start: literals, or refs before it (never read by a
// valid stream; zs_emit_kernel reports any marker into them).  Entries are u16
// (std, markers < 256 + 32768) or u32 (deflate64).
// ---------------------------------------------------------------------------
#define PL_T 256
#define PL_E 16                      // entries per thread
#define PL_BLK (PL_T * PL_E)         // entries per workgroup

// chain member (job q, index j) of unit slot u of the group; false if unused
__device__ __forceinline__ bool pl_member(const ZsCJobDev *__restrict__ cjobs, uint32_t ncj, uint32_t u, uint32_t *q,
                                          uint32_t *j) {
  for (uint32_t k = 0; k < ncj; k++) {
    const ZsCJobDev &cj = cjobs[k];
    if (u >= cj.unit0 && u < cj.unit0 + cj.max_units) {
      *q = k;
      *j = u - cj.unit0;
      return cj.ok && *j < cj.nchain;
    }
  }
  return false;
}

template <uint32_t HN, typename T>
__global__ void __launch_bounds__(PL_T) zs_plink_init_kernel(const ZsCJobDev *__restrict__ cjobs, uint32_t ncj,
                                                             const uint16_t *__restrict__ scratch,
                                                             const ZsLinkInfo *__restrict__ info, T *__restrict__ A) {
  const uint32_t u = blockIdx.y;
  uint32_t q, j;
  if (!pl_member(cjobs, ncj, u, &q, &j) || j == 0) return;
  const ZsLinkInfo prev = info[cjobs[q].unit0 + j - 1];
  const T *E = reinterpret_cast<const T *>(scratch + prev.scratch);
  const uint32_t n = prev.n_out, keep = n < HN ? HN - n : 0u;
  T *out = A + (size_t)u * HN;
  const uint32_t i0 = blockIdx.x * PL_BLK + threadIdx.x;
#pragma unroll
  for (uint32_t k = 0; k < PL_E; k++) {
    const uint32_t i = i0 + k * PL_T;
    out[i] = i < keep ? (T)(MARK_BASE + i + n) : E[i + n - HN];
  }
}

template <uint32_t HN, typename T>
__global__ void __launch_bounds__(PL_T) zs_plink_step_kernel(const ZsCJobDev *__restrict__ cjobs, uint32_t ncj,
                                                             const T *__restrict__ A, T *__restrict__ B, uint32_t stride) {
  const uint32_t u = blockIdx.y;
  uint32_t q, j;
  if (!pl_member(cjobs, ncj, u, &q, &j) || j == 0) return;
  const T *a = A + (size_t)u * HN;
  T *b = B + (size_t)u * HN;
  const uint32_t i0 = blockIdx.x * PL_BLK + threadIdx.x;
  if (j <= stride) {  // already in terms of the stream start
#pragma unroll
    for (uint32_t k = 0; k < PL_E; k++) b[i0 + k * PL_T] = a[i0 + k * PL_T];
    return;
  }
  const T *e = A + (size_t)(u - stride) * HN;  // member j - stride
  T v[PL_E];
#pragma unroll
  for (uint32_t k = 0; k < PL_E; k++) v[k] = a[i0 + k * PL_T];
#pragma unroll
  for (uint32_t k = 0; k < PL_E; k++) {
    const uint32_t x = v[k];
    if (x >= MARK_BASE) v[k] = e[(x - MARK_BASE) & (HN - 1)];
  }
#pragma unroll
  for (uint32_t k = 0; k < PL_E; k++) b[i0 + k * PL_T] = v[k];
}

// windows[unit slot of member j] = W_j as bytes.  Refs before the stream
// start: 0 -- or, in a later piece of a long stream (ZS_JF_CONT), the earlier
// pieces' output before the piece, W_0 (member 0's map is the identity).
template <uint32_t HN, typename T>
__global__ void __launch_bounds__(PL_T) zs_plink_out_kernel(const ZsJobDev *__restrict__ jobs,
                                                            const ZsCJobDev *__restrict__ cjobs, uint32_t ncj,
                                                            const ZsLinkInfo *__restrict__ info, const T *__restrict__ A,
                                                            uint8_t *__restrict__ windows) {
  const uint32_t u = blockIdx.y;
  uint32_t q, j;
  if (!pl_member(cjobs, ncj, u, &q, &j)) return;
  const ZsJobDev jb = jobs[cjobs[q].job];
  const uint32_t hist = (jb.flags & ZS_JF_CONT) ? min(jb.hist, HN) : 0u;
  if (j == 0 && !hist) return;
  const uint32_t c = info[cjobs[q].unit0 + j].unit;
  const T *a = A + (size_t)u * HN;
  uint8_t *w = windows + (size_t)c * HN;
  const uint32_t i0 = blockIdx.x * PL_BLK + threadIdx.x;
#pragma unroll
  for (uint32_t k = 0; k < PL_E; k++) {
    const uint32_t i = i0 + k * PL_T;
    const uint32_t x = j ? (uint32_t)a[i] : MARK_BASE + i;
    uint8_t b = 0;
    if (x < MARK_BASE) {
      b = (uint8_t)x;
    } else {
      const uint32_t wx = (x - MARK_BASE) & (HN - 1);
      if (wx >= HN - hist) b = jb.out[(int64_t)wx - (int64_t)HN];
    }
    w[i] = b;
  }
}

// ---------------------------------------------------------------------------
// host launch helpers
// ---------------------------------------------------------------------------
extern "C" void zs_launch_fixed_tables(uint32_t *fixed, int d64, hipStream_t st) {
  hipLaunchKernelGGL(zs_fixed_tables_kernel, dim3(1), dim3(64), 0, st, fixed, d64);
}

extern "C" void zs_launch_parse(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, ZsChunkDev *d_chunks, uint32_t nchunks,
                                uint32_t *d_tokens, uint32_t *d_tables, const uint32_t *d_fixed, ZsTokPool pool, int d64,
                                int wave_units, hipStream_t st, int ctx);
extern "C" void zs_launch_expand(const ZsJobDev *d_jobs, ZsChunkDev *d_chunks, uint32_t nchunks, uint16_t *d_scratch,
                                 const uint32_t *d_tokens, ZsTokPool pool, uint32_t *d_fallback, int d64, hipStream_t st,
                                 int ctx);

// One group of chunked jobs, all raw/zlib/gzip (d64 = 0) or all deflate64
// (d64 = 1: 64 KiB history, so 64 KiB windows per unit slot).  ctx picks the
// host-side sort / split workspaces, so that two groups can run at once on two
// streams (zs_capi.cpp run_jobs); ev_found (optional) is recorded once the
// group's units are planned.
extern "C" void zs_launch_chunked(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, ZsSegDev *d_segs, uint32_t nseg,
                                  ZsCJobDev *d_cjobs, uint32_t ncjobs, ZsChunkDev *d_units, uint32_t nunit_slots,
                                  uint16_t *d_scratch, uint32_t *d_tokens, ZsTokPool pool, uint32_t *d_tables,
                                  const uint32_t *d_fixed, uint8_t *d_windows, void *d_linkinfo, ZsDecDev *d_decs,
                                  uint32_t *d_fallback, int d64, int wave_units, void *d_plink, uint32_t plink_levels,
                                  uint16_t *d_lmaps, uint32_t lsegs, hipStream_t st, hipEvent_t *ev, uint32_t *d_vlist,
                                  int ctx, hipEvent_t ev_found) {
  // ev (profiling, optional): [0] before find, [1] after find + plan, [2] after
  // parse + chain, [3] after expand, [4] after link, [5] after emit
  if (ev) (void)hipEventRecord(ev[0], st);
  // the finder's survivor lists (FQ_LIST words per segment) borrow the token
  // buffer (d_vlist: the group's own token regions, by default the buffer's
  // start): nothing reads or writes them before the parse (a segment is
  // 32 KiB of input, the token space >= 8 bytes per input byte), and a later
  // group on the same stream finds after this group's expand
  uint32_t *const vl = d_vlist ? d_vlist : d_tokens;
  const dim3 fgrid((nseg + FIND_WG - 1u) / FIND_WG), fblk(FIND_WG * WAVE);
  int ncu = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const dim3 vgrid(std::min<uint32_t>(nseg, (uint32_t)std::max(ncu, 1) * FV_WAVES_PER_CU));
  if (d64) {
    hipLaunchKernelGGL(zs_find_kernel<true>, fgrid, fblk, 0, st, d_jobs, d_heads, d_segs, vl, nseg);
    hipLaunchKernelGGL(zs_findval_kernel<true>, vgrid, dim3(WAVE), 0, st, d_jobs, d_segs, vl, nseg);
  } else {
    hipLaunchKernelGGL(zs_find_kernel<false>, fgrid, fblk, 0, st, d_jobs, d_heads, d_segs, vl, nseg);
    hipLaunchKernelGGL(zs_findval_kernel<false>, vgrid, dim3(WAVE), 0, st, d_jobs, d_segs, vl, nseg);
  }
  hipLaunchKernelGGL(zs_findsel_kernel, dim3((nseg + 255u) / 256u), dim3(256), 0, st, d_segs, vl, nseg);
  hipLaunchKernelGGL(zs_find_fixed_kernel, dim3(nseg), dim3(64), 0, st, d_jobs, d_heads, d_segs, nseg);
  hipLaunchKernelGGL(zs_plan_kernel, dim3(ncjobs), dim3(PLAN_T), 0, st, d_jobs, d_heads, d_segs, d_cjobs, d_units, pool);
  if (ev) (void)hipEventRecord(ev[1], st);
  if (ev_found) (void)hipEventRecord(ev_found, st);
  ZsLinkInfo *info = reinterpret_cast<ZsLinkInfo *>(d_linkinfo);
  zs_launch_parse(d_jobs, d_heads, d_units, nunit_slots, d_tokens, d_tables, d_fixed, pool, d64, wave_units, st, ctx);
  hipLaunchKernelGGL(zs_chain_kernel, dim3(ncjobs), dim3(LINK_THREADS), 0, st, d_jobs, d_heads, d_units, d_cjobs, info,
                     d_decs, d_fallback);
  if (ev) (void)hipEventRecord(ev[2], st);
  zs_launch_expand(d_jobs, d_units, nunit_slots, d_scratch, d_tokens, pool, d_fallback, d64, st, ctx);
  if (ev) (void)hipEventRecord(ev[3], st);
  if (d_plink) {  // few long streams: windows by parallel prefix over each chain
    const dim3 grid((d64 ? 65536u : HIST) / PL_BLK, nunit_slots);
    if (d64) {
      uint32_t *A = static_cast<uint32_t *>(d_plink), *B = A + (size_t)nunit_slots * 65536u;
      hipLaunchKernelGGL((zs_plink_init_kernel<65536u, uint32_t>), grid, dim3(PL_T), 0, st, d_cjobs, ncjobs, d_scratch,
                         info, A);
      for (uint32_t d = 0; d < plink_levels; d++) {
        hipLaunchKernelGGL((zs_plink_step_kernel<65536u, uint32_t>), grid, dim3(PL_T), 0, st, d_cjobs, ncjobs, A, B, 1u << d);
        uint32_t *t = A;
        A = B;
        B = t;
      }
      hipLaunchKernelGGL((zs_plink_out_kernel<65536u, uint32_t>), grid, dim3(PL_T), 0, st, d_jobs, d_cjobs, ncjobs, info,
                         A, d_windows);
    } else {
      uint16_t *A = static_cast<uint16_t *>(d_plink), *B = A + (size_t)nunit_slots * HIST;
      hipLaunchKernelGGL((zs_plink_init_kernel<HIST, uint16_t>), grid, dim3(PL_T), 0, st, d_cjobs, ncjobs, d_scratch,
                         info, A);
      for (uint32_t d = 0; d < plink_levels; d++) {
        hipLaunchKernelGGL((zs_plink_step_kernel<HIST, uint16_t>), grid, dim3(PL_T), 0, st, d_cjobs, ncjobs, A, B, 1u << d);
        uint16_t *t = A;
        A = B;
        B = t;
      }
      hipLaunchKernelGGL((zs_plink_out_kernel<HIST, uint16_t>), grid, dim3(PL_T), 0, st, d_jobs, d_cjobs, ncjobs, info, A,
                         d_windows);
    }
    if (ev) (void)hipEventRecord(ev[4], st);
    if (d64)
      hipLaunchKernelGGL(zs_emit64_kernel, dim3(nunit_slots), dim3(EMIT_THREADS), 0, st, d_jobs, d_units, d_scratch,
                         d_windows, d_fallback);
    else
      hipLaunchKernelGGL(zs_emit_kernel<HIST>, dim3(nunit_slots), dim3(EMIT_THREADS), 0, st, d_jobs, d_units, d_scratch,
                         d_windows, d_fallback);
  } else if (d64) {
    hipLaunchKernelGGL(zs_link64_kernel, dim3(ncjobs), dim3(LINK_THREADS), 0, st, d_jobs, d_cjobs, d_scratch, d_windows,
                       info, d_fallback);
    if (ev) (void)hipEventRecord(ev[4], st);
    hipLaunchKernelGGL(zs_emit64_kernel, dim3(nunit_slots), dim3(EMIT_THREADS), 0, st, d_jobs, d_units, d_scratch,
                       d_windows, d_fallback);
  } else if (d_lmaps && lsegs > 1) {  // segmented link: segment maps, joined, then the segments' byte windows
    hipLaunchKernelGGL(zs_linkseg_kernel, dim3(ncjobs * lsegs), dim3(LINK_THREADS), 0, st, d_jobs, d_cjobs, lsegs, d_scratch,
                       d_lmaps, info);
    hipLaunchKernelGGL(zs_linkseg_join_kernel, dim3(ncjobs), dim3(LINK_THREADS), 0, st, d_cjobs, lsegs, d_lmaps);
    hipLaunchKernelGGL(zs_link_kernel<HIST>, dim3(ncjobs * lsegs), dim3(LINK_THREADS), 0, st, d_jobs, d_cjobs, d_scratch,
                       d_windows, info, d_fallback, lsegs, (const uint16_t *)d_lmaps, (const ZsChunkDev *)d_units);
    if (ev) (void)hipEventRecord(ev[4], st);
    hipLaunchKernelGGL(zs_emit_kernel<HIST>, dim3(nunit_slots), dim3(EMIT_THREADS), 0, st, d_jobs, d_units, d_scratch,
                       d_windows, d_fallback);
  } else {
    hipLaunchKernelGGL(zs_link_kernel<HIST>, dim3(ncjobs), dim3(LINK_THREADS), 0, st, d_jobs, d_cjobs, d_scratch, d_windows,
                       info, d_fallback);
    if (ev) (void)hipEventRecord(ev[4], st);
    hipLaunchKernelGGL(zs_emit_kernel<HIST>, dim3(nunit_slots), dim3(EMIT_THREADS), 0, st, d_jobs, d_units, d_scratch,
                       d_windows, d_fallback);
  }
  if (ev) (void)hipEventRecord(ev[5], st);
}

// link counters of the profiling build (merged into zs_kprof_read's 48..63)
extern "C" int zs_kprof_read_ck(uint64_t *out16, int reset) {
#if KP_ON
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_kprof_ck), 16 * sizeof(uint64_t)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_kprof_ck), z, sizeof z) != hipSuccess) return -1;
  }
  return 16;
#else
  (void)out16;
  (void)reset;
  return 0;
#endif
}
