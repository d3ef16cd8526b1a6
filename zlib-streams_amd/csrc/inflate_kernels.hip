// inflate_kernels.hip -- MI355X (gfx950) inflate kernels.
//
// Hot path of the reference: the Huffman decode + window copy loop of
// src/inffast.c:100-287 and the symbol states of src/inflate.c:1037-1193, the
// block/table states of src/inflate.c:834-1033, and the table builder of
// src/inftrees.c:33-321 (incl. the deflate64 variant, windowBits == -16).
//
// Design (MI355X-first, not a translation):
//   * one 64-lane wave decodes one stream (or one chunk of one stream); the
//     decoder state is wave-uniform, so control flow never diverges;
//   * the compressed bitstream is staged through a 4 KiB LDS ring filled by
//     coalesced 16 B/lane loads (1 KiB per wave instruction), one piece ahead;
//   * the history window (32 KiB, or 64 KiB for deflate64) lives in LDS as a
//     ring; match copies are done by up to 64 lanes at once;
//   * output leaves the ring in 1 KiB pieces, 16 B per lane (dwordx4 stores);
//   * Huffman tables are rebuilt per block in LDS, with the canonical sort and
//     the root-table fill spread over the lanes (ballot ranks), and zlib's
//     sub-table layout kept exactly so the deflate64 ENOUGH-1 rule
//     (src/inftrees.c:211-212) rejects the same codes.
//
// Result semantics: one job == one inflate(strm, Z_FINISH) call over the whole
// input (ret, msg, total_in, total_out, adler identical to the reference).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zs_common.h"
// the stream / wave decoders keep the table builder as a call (round 6: inlined
// into them, one handle 252 -> 200 MiB/s and the perf harness's decompress
// 685 -> 411 MiB/s; the block-parallel path's kernels inline it)
#define BUILD_TABLE_ATTR __attribute__((noinline))
#include "zs_device.h"
#include "zs_check.h"

#include "zs_kprof.h"

#if KP_ON
__device__ unsigned long long g_kprof_w[32];  // KP_W_* - 64
#define KPW_ADD(i, v)                                                          \
  do {                                                                         \
    if (lane_id() == 0) atomicAdd(&g_kprof_w[(i) - 64], (unsigned long long)(v)); \
  } while (0)
#define KPW0_ADD(i, v)                                                          \
  do {                                                                          \
    if (threadIdx.x == 0) atomicAdd(&g_kprof_w[(i) - 64], (unsigned long long)(v)); \
  } while (0)
#else
#define KPW_ADD(i, v) ((void)0)
#define KPW0_ADD(i, v) ((void)0)
#endif

#define IN_RING_WORDS 1024   // 4 KiB compressed-input ring
#define PIECE_WORDS 256      // 1 KiB per fill (64 lanes x 16 B)
#define FLUSH_BYTES 1024     // output flush granule (64 lanes x 16 B)

// ---------------------------------------------------------------------------
// Header stage: zlib / gzip wrapper parse (src/inflate.c:629-833), one thread
// per job.  Byte-exact total_in on header errors and truncation.
// ---------------------------------------------------------------------------
__device__ uint32_t crc32_bytes(uint32_t crc, const uint8_t *p, uint64_t n) {
  crc = ~crc;
  for (uint64_t i = 0; i < n; i++) {
    crc ^= p[i];
#pragma unroll
    for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
  }
  return ~crc;
}

__global__ void zs_header_kernel(const ZsJobDev *__restrict__ jobs, ZsHeadDev *__restrict__ heads, uint32_t njobs) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  ZsJobDev jb = jobs[j];
  ZsHeadDev h;
  h.code = ZD_END;  // "continue to deflate data"
  h.msg = ZM_NONE;
  h.is_gzip = -1;
  h.ret = 0;
  h.start_byte = 0;
  h.total_in = 0;
  h.adler = 0;
  h.wbits = jb.wbits;
  const uint8_t *in = jb.in;
  const uint64_t n = jb.in_len;
  if (jb.wrap == ZW_RAW) {
    heads[j] = h;
    return;
  }
  uint32_t adler_reset = (uint32_t)(jb.wrap & 1);  // inflateResetKeep: strm->adler = wrap & 1
  h.adler = adler_reset;
  auto trunc = [&]() {
    h.code = ZD_SKIP;
    h.msg = ZM_NONE;
    h.total_in = n;
    h.ret = ZS_BUF_ERROR;
  };
  auto fail = [&](int msg, uint64_t consumed) {
    h.code = ZD_SKIP;
    h.msg = msg;
    h.total_in = consumed;
    h.ret = ZS_DATA_ERROR;
  };
  if (n < 2) {
    trunc();
    heads[j] = h;
    return;
  }
  uint32_t b0 = in[0], b1 = in[1];
  if ((jb.wrap & 2) && b0 == 0x1f && b1 == 0x8b) {
    uint64_t p = 2;
    uint32_t crc = crc32_bytes(0, in, 2);
    if (n < p + 2) { trunc(); heads[j] = h; return; }
    uint32_t flags = in[p] | (in[p + 1] << 8);
    if ((flags & 0xff) != 8) { fail(ZM_METHOD, p + 2); heads[j] = h; return; }
    if (flags & 0xe000) { fail(ZM_FLAGS, p + 2); heads[j] = h; return; }
    const bool hc = (flags & 0x0200) != 0;
    if (hc) crc = crc32_bytes(crc, in + p, 2);
    p += 2;
    if (n < p + 4) { trunc(); heads[j] = h; return; }  // MTIME
    if (hc) crc = crc32_bytes(crc, in + p, 4);
    p += 4;
    if (n < p + 2) { trunc(); heads[j] = h; return; }  // XFL, OS
    if (hc) crc = crc32_bytes(crc, in + p, 2);
    p += 2;
    if (flags & 0x0400) {
      if (n < p + 2) { trunc(); heads[j] = h; return; }
      uint32_t xlen = in[p] | (in[p + 1] << 8);
      if (hc) crc = crc32_bytes(crc, in + p, 2);
      p += 2;
      if (n < p + xlen) { trunc(); heads[j] = h; return; }
      if (hc) crc = crc32_bytes(crc, in + p, xlen);
      p += xlen;
    }
    for (int f = 0; f < 2; f++) {
      if (flags & (f == 0 ? 0x0800 : 0x1000)) {
        uint64_t q = p;
        while (q < n && in[q] != 0) q++;
        if (q >= n) { trunc(); heads[j] = h; return; }
        if (hc) crc = crc32_bytes(crc, in + p, q + 1 - p);
        p = q + 1;
      }
    }
    if (hc) {
      if (n < p + 2) { trunc(); heads[j] = h; return; }
      uint32_t want = in[p] | (in[p + 1] << 8);
      if (want != (crc & 0xffff)) { fail(ZM_HCRC, p + 2); heads[j] = h; return; }
      p += 2;
    }
    h.adler = 0;
    h.is_gzip = 1;
    if (h.wbits == 0) h.wbits = 15;  // src/inflate.c HEAD: gzip with windowBits 0 uses 15
    h.start_byte = p;
    heads[j] = h;
    return;
  }
  if (!(jb.wrap & 1) || (((b0 << 8) + b1) % 31) != 0) { fail(ZM_HEADER_CHECK, 2); heads[j] = h; return; }
  if ((b0 & 15) != 8) { fail(ZM_METHOD, 2); heads[j] = h; return; }
  uint32_t wlen = (b0 >> 4) + 8;
  uint32_t wb = jb.wbits == 0 ? wlen : (uint32_t)jb.wbits;
  if (wlen > 15 || wlen > wb) { fail(ZM_WINDOW, 2); heads[j] = h; return; }
  h.adler = 1;
  if (b1 & 0x20) {  // FDICT: DICTID then Z_NEED_DICT (src/inflate.c:817-828)
    if (n < 6) { trunc(); heads[j] = h; return; }
    h.code = ZD_NEED_DICT;
    h.adler = ((uint32_t)in[2] << 24) | ((uint32_t)in[3] << 16) | ((uint32_t)in[4] << 8) | in[5];
    h.total_in = 0;  // Z_NEED_DICT returns before inf_leave: totals untouched
    heads[j] = h;
    return;
  }
  h.is_gzip = 0;
  h.wbits = wb;
  h.start_byte = 2;
  heads[j] = h;
}

// ---------------------------------------------------------------------------
// The wave-uniform deflate decoder.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Workgroup-wide symbol window (the stream kernel: one handle call per
// 1 024-thread workgroup).  A call of the handle ABI decodes one slice (<= 32
// KiB in, <= 64 KiB out): one or two blocks, so there is no block parallelism
// to use, and one wave's fast_window (512 bits, <= 64 symbols) left the call
// at one wave's serial pace.  Here all 16 waves decode one window of up to
// WW_BITS = 8 192 bits (~900 symbols): every thread decodes a complete symbol
// at 8 bit offsets; pointer doubling over the jump table q -> q + bits(q)
// (10 rounds, workgroup barriers) gives the chain's first 1 024 symbol
// starts; symbol k's data moves to thread k through an on-chain mark; a
// workgroup scan of the output lengths admits the longest prefix that is
// plain (complete in the input, fits the output, distance within the history,
// not end-of-block / invalid -- as fast_window); the bytes expand 4 096 per
// step into the history ring (sources before the step read the ring, sources
// inside it resolve by pointer jumping).  Wave 0 runs the exact state machine
// (Inflater) and posts a window to the other waves, which wait at a barrier
// in between; everything a window does not take stays on the exact serial
// path, so results and stop points are the serial decoder's.
// ---------------------------------------------------------------------------
#define WW_T 1024u                 // threads of the stream kernel
#define WW_OFFS 8u                 // bit offsets per thread
#define WW_BITS (WW_T * WW_OFFS)   // 8 192-bit window
#define WW_JN (WW_BITS + 64u)      // jump-table entries (a symbol is <= 48 bits)
#define WW_SKIP 32u                // J5: 32-symbol jumps
#define WW_EB 8u                   // bytes expanded per thread and step
#define WW_STEP (WW_EB * WW_T)     // bytes expanded per step
#define WW_TCAP 16384u             // bytes per window (the ring keeps the unflushed tail)
#define WW_MIN_ROOM 512u           // output room below which the serial loop runs
#define WW_RUN 1u
#define WW_EXIT 2u
#define WW_COPY 3u                 // a stored block's bytes into the ring, by all WW_T threads
#define WW_COPY_MIN 4096u          // stored bytes below which wave 0 copies alone

struct WideLDS {
  // command (wave 0 -> all waves)
  uint32_t op, P, W, limit_bits, pos, cap, whave, lmask, dmask;
  uint32_t lt_off, dt_off;     // the code tables: byte offsets in the kernel's StreamLDS
  // results and reductions
  uint32_t n, cnt_min, carry;
  uint32_t open[2];            // expansion rounds alternate: one is set while the other is cleared
  // admitted prefix: first inadmissible thread n << 32 | its chain offset << 16 |
  // its output start (= the bytes admitted), by one 64-bit LDS min
  __attribute__((aligned(8))) unsigned long long nkey;
  uint32_t save, save_pos;     // end of the call: the history ring goes to the handle's state
  __attribute__((aligned(8))) unsigned long long cp_src;  // WW_COPY: the stored bytes' address (W bytes to ring position pos)
  uint32_t tab_in, tab_out;    // cached dynamic tables (ZsStreamDev::tab_bits) loaded / to save
  uint32_t wtot[WW_T / 64];
  uint32_t sk[WW_T / WW_SKIP];   // chain start of symbols 32 m
  uint32_t symL[WW_T], symD[WW_T];
  __attribute__((aligned(16))) uint8_t nb[WW_JN];  // symbol bits at each offset (0: no plain symbol starts there)
  __attribute__((aligned(16))) uint16_t ja[WW_JN];  // J0 (one symbol) -- kept
  __attribute__((aligned(16))) uint16_t jb[WW_JN];  // J1 .. J5, ping-pong with jc
  __attribute__((aligned(16))) uint16_t jc[WW_JN];
};
// expansion marks (u16) + entries (u32) of one step alias the three jump tables
static_assert(sizeof(uint16_t) * WW_JN * 3 >= WW_STEP * 6, "expansion marks + entries alias the jump tables");
static_assert(ZS_STREAM_TAB_WORDS == TABLE_ENTRIES, "ZsStreamDev::tab holds one table set");

// All LDS of one stream-kernel workgroup in one object, so every wave reaches
// it through the same LDS addresses (ds_* instructions, not flat ones)
template <bool D64>
struct StreamLDS {
  static constexpr uint32_t RING = D64 ? 65536u : 32768u;
  __attribute__((aligned(16))) uint8_t ring[RING];
  __attribute__((aligned(16))) uint32_t in[IN_RING_WORDS];
  uint32_t tab[TABLE_ENTRIES];
  uint32_t ftab[544];
  uint16_t lens[320];
  __attribute__((aligned(16))) uint16_t sorted[320];
  uint32_t scr[32];
  WideLDS wide;
  // the symbol decoded at each window offset (standard deflate: 1 | literal << 1,
  // or length << 1 | distance << 10), so the chain's k-th symbol moves to thread k
  // with one read (deflate64's lengths and distances do not fit: marks there)
  __attribute__((aligned(16))) uint32_t osym[D64 ? 4u : WW_BITS];
};

__device__ __forceinline__ uint32_t ww_scan_sum(uint32_t x) {  // inclusive, wave64
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}
__device__ __forceinline__ uint32_t ww_scan_max(uint32_t v) {  // inclusive, wave64
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}
// workgroup scan (sum or max) of one value per thread: inclusive, and the
// exclusive value (the inclusive one of thread t - 1; 0 for thread 0)
template <bool MAX>
__device__ __forceinline__ uint32_t ww_scan(WideLDS &w, uint32_t v, uint32_t *excl) {
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t inc = MAX ? ww_scan_max(v) : ww_scan_sum(v);
  const uint32_t up = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane ? lane - 1u : 0u) << 2), (int)inc);
  if (lane == 63) w.wtot[wv] = inc;
  __syncthreads();
  uint32_t pre = 0;
  for (uint32_t k = 0; k < wv; k++) pre = MAX ? max(pre, w.wtot[k]) : pre + w.wtot[k];
  // no trailing barrier: every caller passes one before its next scan writes wtot
  const uint32_t own = lane ? up : 0u;
  *excl = MAX ? max(pre, own) : pre + own;
  return MAX ? max(pre, inc) : pre + inc;
}

// index of the first thread whose flag is set (WW_T if none) into *dst (a
// word set to WW_T beforehand): one LDS atomic per wave
__device__ __forceinline__ void ww_first(uint32_t *dst, bool flag) {
  const uint64_t m = __ballot(flag);
  if (m && (threadIdx.x & 63u) == 0) atomicMin(dst, (threadIdx.x & ~63u) + (uint32_t)__builtin_ctzll(m));
}

__device__ __forceinline__ uint64_t ww_bits_at(const uint32_t *inring, uint32_t q) {
  const uint32_t wq = q >> 5, sh = q & 31u;
  const uint32_t a = inring[wq & (IN_RING_WORDS - 1)];
  const uint32_t b = inring[(wq + 1) & (IN_RING_WORDS - 1)];
  const uint32_t c = inring[(wq + 2) & (IN_RING_WORDS - 1)];
  uint64_t h = ((((uint64_t)b) << 32) | a) >> sh;
  if (sh) h |= (uint64_t)c << (64u - sh);
  return h;
}

// One complete symbol at bit q (as fast_window's stage 1): returns its bits
// (0: not a plain symbol), the length (0x80000000 | literal for a literal)
// and the distance.
template <bool D64>
__device__ __forceinline__ uint32_t ww_decode_bits(const WideLDS &w, const uint32_t *lt, const uint32_t *dt,
                                                   const uint64_t hh, uint32_t q, uint32_t &lv, uint32_t &dv) {
  uint32_t e = lt[(uint32_t)hh & w.lmask];
  uint32_t used = e_bits(e);
  {
    const uint32_t op0 = e_op(e);
    if (op0 != 0 && (op0 & 0xf0u) == 0) {
      const uint32_t e2 = lt[e_val(e) + (((uint32_t)(hh >> used)) & ((1u << op0) - 1))];
      used += e_bits(e2);
      e = e2;
    }
  }
  const uint32_t op = e_op(e);
  dv = 0;
  if (op == 0) {
    lv = 0x80000000u | e_val(e);
    return q + used > w.limit_bits ? 0u : used;
  }
  if (op & 96u) {  // end of block / invalid code: not plain
    lv = 0;
    return 0;
  }
  const uint32_t xb = op & (D64 ? 31u : 15u);
  lv = e_val(e) + ((uint32_t)(hh >> used) & ((1u << xb) - 1u));
  const uint32_t sb = used + xb;
  const uint64_t hd = hh >> sb;
  uint32_t d = dt[(uint32_t)hd & w.dmask];
  uint32_t dused = e_bits(d);
  {
    const uint32_t dop0 = e_op(d);
    if ((dop0 & 0xf0u) == 0) {
      const uint32_t d2 = dt[e_val(d) + (((uint32_t)(hd >> dused)) & ((1u << dop0) - 1))];
      dused += e_bits(d2);
      d = d2;
    }
  }
  const uint32_t dop = e_op(d);
  if (dop & 64u) return 0;  // invalid distance code
  const uint32_t dx = dop & 15u;
  dv = e_val(d) + ((uint32_t)(hd >> dused) & ((1u << dx) - 1u));
  const uint32_t nb = sb + dused + dx;
  return q + nb > w.limit_bits || nb > 63u ? 0u : nb;
}

// a stored block's W bytes from cp_src into the ring at pos, run by all WW_T
// threads (wave 0 posted the command; it flushes them afterwards).  A thread
// takes 16 bytes at a time as five aligned dword loads funnel-shifted by the
// source's misalignment (the loads reach <= 3 bytes before the piece -- the
// block's LEN / NLEN -- and 4 after it, inside the block but for the last
// pieces, which take byte loads); the ring takes bytes (any output alignment).
template <bool D64>
__device__ void ww_copy(StreamLDS<D64> &Ls) {
  constexpr uint32_t RMASK = (D64 ? 65536u : 32768u) - 1u;
  WideLDS &w = Ls.wide;
  uint8_t *ring = Ls.ring;
  const uint8_t *src = reinterpret_cast<const uint8_t *>((uintptr_t)w.cp_src);
  const uint32_t m = w.W, pos = w.pos;
  const uint32_t sh = (uint32_t)((uintptr_t)src & 3u);
  const uint32_t *a = reinterpret_cast<const uint32_t *>((uintptr_t)src & ~(uintptr_t)3);
  for (uint32_t i = 16u * threadIdx.x; i < m; i += 16u * WW_T) {
    uint32_t d[4];
    if (i + 20u <= m) {
      uint32_t x[5];
#pragma unroll
      for (int q = 0; q < 5; q++) x[q] = a[(i >> 2) + q];
#pragma unroll
      for (int q = 0; q < 4; q++) d[q] = __builtin_amdgcn_alignbyte(x[q + 1], x[q], sh);
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) d[q] = 0;
#pragma unroll
      for (uint32_t q = 0; q < 16; q++)
        if (i + q < m) d[q >> 2] |= (uint32_t)src[i + q] << (8u * (q & 3u));
    }
#pragma unroll
    for (uint32_t q = 0; q < 16; q++)
      if (i + q < m) ring[(pos + i + q) & RMASK] = (uint8_t)(d[q >> 2] >> (8u * (q & 3u)));
  }
  __syncthreads();  // the ring holds the bytes before wave 0 flushes them
}

// the window, run by all WW_T threads (wave 0 posted the command)
template <bool D64>
__device__ void ww_run(StreamLDS<D64> &Ls) {
  constexpr uint32_t RMASK = (D64 ? 65536u : 32768u) - 1u;
  WideLDS &w = Ls.wide;
  uint8_t *ring = Ls.ring;
  const uint32_t *inring = Ls.in;
  const uint32_t *lt = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(&Ls) + w.lt_off);
  const uint32_t *dt = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(&Ls) + w.dt_off);
  const uint32_t t = threadIdx.x;
  const uint32_t P = w.P, W = w.W;
  [[maybe_unused]] const uint64_t kt0 = KP_NOW();
  // 1. a complete symbol at every offset of the window: thread t the 8
  //    consecutive offsets 8t .. 8t + 7, whose bits one 128-bit read covers
  uint32_t lv[WW_OFFS], dv[WW_OFFS];
  uint32_t cur[WW_OFFS];  // the thread's own J0 .. J4 entries, offsets 8t .. 8t + 7
  static_assert(WW_OFFS == 8, "8 consecutive offsets per thread");
  {
    const uint32_t q0 = WW_OFFS * t, b0 = P + q0, wq = b0 >> 5, sh = b0 & 31u;
    const uint32_t a = inring[wq & (IN_RING_WORDS - 1)], b = inring[(wq + 1) & (IN_RING_WORDS - 1)];
    const uint32_t c = inring[(wq + 2) & (IN_RING_WORDS - 1)], d = inring[(wq + 3) & (IN_RING_WORDS - 1)];
    const uint64_t lo = ((uint64_t)b << 32) | a, hi = ((uint64_t)d << 32) | c;
    uint32_t nbw[2] = {0, 0}, jw[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < WW_OFFS; i++) {
      const uint32_t q = q0 + i, x = sh + i;  // x <= 38
      const uint64_t hh = (lo >> x) | (x ? hi << (64u - x) : 0ull);
      uint32_t nb = 0;
      lv[i] = dv[i] = 0;
      if (q < W) nb = ww_decode_bits<D64>(w, lt, dt, hh, P + q, lv[i], dv[i]);
      nbw[i >> 2] |= nb << (8u * (i & 3u));
      jw[i >> 1] |= (q + nb) << (16u * (i & 1u));
      cur[i] = q + nb;
    }
    *reinterpret_cast<uint2 *>(&w.nb[q0]) = make_uint2(nbw[0], nbw[1]);
    *reinterpret_cast<uint4 *>(&w.ja[q0]) = make_uint4(jw[0], jw[1], jw[2], jw[3]);
    if constexpr (!D64) {
      uint32_t o[WW_OFFS];
#pragma unroll
      for (uint32_t i = 0; i < WW_OFFS; i++)
        o[i] = (lv[i] & 0x80000000u) ? (1u | ((lv[i] & 0xffu) << 1)) : ((lv[i] << 1) | (dv[i] << 10));
      *reinterpret_cast<uint4 *>(&Ls.osym[q0]) = make_uint4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<uint4 *>(&Ls.osym[q0 + 4]) = make_uint4(o[4], o[5], o[6], o[7]);
    }
  }
  if (t < WW_JN - WW_BITS) {
    w.nb[WW_BITS + t] = 0;
    w.ja[WW_BITS + t] = (uint16_t)(WW_BITS + t);
  }
  if (t == 0) {
    w.cnt_min = WW_T;
    w.nkey = ~0ull;
  }
  // 2. the chain from the window start: J5 = 32 symbols per jump (five
  //    compositions of J0), a serial walk of J5 for every 32nd symbol, then
  //    each thread walks J0 from its group's start (<= 31 steps)
  [[maybe_unused]] const uint64_t kt1 = KP_NOW();
  {
    // J1 .. J4 ping-pong jb / jc (J3 ends in jb, J4 in jc); J5 is composed in
    // place over J4 (all reads, a barrier, then the writes), so J3 survives:
    // each thread then reaches its symbol from its 32-group's start in <= 3
    // J3 hops and <= 7 J0 hops instead of <= 31 J0 hops
    // the thread's own entries stay in registers (cur), so a round is 8 gathers
    // and one 16-byte store
    const uint16_t *src = w.ja;
    uint16_t *dst = w.jb;
    const uint32_t q0 = WW_OFFS * t;
#pragma unroll 1
    for (uint32_t k = 0; k < 4; k++) {
      __syncthreads();
#pragma unroll
      for (uint32_t i = 0; i < WW_OFFS; i++) cur[i] = src[cur[i]];
      *reinterpret_cast<uint4 *>(&dst[q0]) =
          make_uint4(cur[0] | cur[1] << 16, cur[2] | cur[3] << 16, cur[4] | cur[5] << 16, cur[6] | cur[7] << 16);
      if (t < WW_JN - WW_BITS) dst[WW_BITS + t] = (uint16_t)(WW_BITS + t);
      src = dst;
      dst = dst == w.jb ? w.jc : w.jb;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < WW_OFFS; i++) cur[i] = w.jc[cur[i]];
    __syncthreads();
    *reinterpret_cast<uint4 *>(&w.jc[q0]) =
        make_uint4(cur[0] | cur[1] << 16, cur[2] | cur[3] << 16, cur[4] | cur[5] << 16, cur[6] | cur[7] << 16);
    __syncthreads();
    KPW0_ADD(KP_W_CYC_COMPOSE, KP_NOW() - kt1);
    if (t == 0) {
      uint32_t x = 0;
      for (uint32_t m = 0; m < WW_T / WW_SKIP; m++) {
        w.sk[m] = x;
        x = w.jc[x];
      }
    }
    __syncthreads();
  }
  uint32_t s = w.sk[t / WW_SKIP];
  for (uint32_t r = (t % WW_SKIP) >> 3; r; r--) s = w.jb[s];
  for (uint32_t r = t & 7u; r; r--) s = w.ja[s];
  KPW0_ADD(KP_W_CYC_WALK, KP_NOW() - kt1);  // compose + walks (thread 0 walks the J5 chain)
  // 3. the chain's symbols: inside the window and plain
  const uint32_t snb = s < WW_BITS ? w.nb[s] : 0u;
  ww_first(&w.cnt_min, !(s < W && snb != 0));
  uint32_t cnt, L = 0, D = 0;
  if constexpr (!D64) {  // thread t reads its symbol (offset s) directly
    if (s < W && snb != 0) {
      const uint32_t o = Ls.osym[s];
      L = (o & 1u) ? (0x80000000u | (o >> 1)) : ((o >> 1) & 511u);
      D = (o & 1u) ? 0u : (o >> 10);
    }
    __syncthreads();
    cnt = w.cnt_min;
    if (t < cnt) {
      w.symL[t] = L;
      w.symD[t] = D;
    } else {
      L = D = 0;
    }
  } else {  // symbol k's data moves to thread k through an on-chain mark
    uint16_t *mark = w.jc;  // J5 is done with (J3 in jb may still be read by other threads' walks)
#pragma unroll
    for (uint32_t i = 0; i < WW_OFFS; i++) mark[t + i * WW_T] = 0;
    __syncthreads();
    cnt = w.cnt_min;
    if (t < cnt) mark[s] = (uint16_t)(t + 1u);
    __syncthreads();
    {
      const uint4 mk = *reinterpret_cast<const uint4 *>(&mark[WW_OFFS * t]);
      const uint32_t mw[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
      for (uint32_t i = 0; i < WW_OFFS; i++) {
        const uint32_t m = (mw[i >> 1] >> (16u * (i & 1u))) & 0xffffu;
        if (m) {
          w.symL[m - 1u] = lv[i];
          w.symD[m - 1u] = dv[i];
        }
      }
    }
    __syncthreads();
    if (t < cnt) {
      L = w.symL[t];
      D = w.symD[t];
    }
  }
  // 4. admissible prefix: fits the output (and WW_TCAP), distance within history
  const bool act = t < cnt;
  const bool lit = (L & 0x80000000u) != 0;
  const uint32_t olen = act ? (lit ? 1u : L) : 0u;
  uint32_t ost;
  // the first expansion step's marks (they alias J0, whose walks ended before the
  // last barrier); the scan's barrier orders these stores before the marks
  reinterpret_cast<uint4 *>(w.ja)[t] = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t incl = ww_scan<false>(w, olen, &ost);
  const uint32_t room = min(w.cap - w.pos, WW_TCAP);
  {
    // each wave posts its first inadmissible thread with that thread's chain
    // offset and output start (the admitted bytes when it is the first of all);
    // the last wave posts "none" (thread WW_T, the end of its last symbol)
    const uint64_t m = __ballot(!(act && incl <= room && (lit || D <= w.pos + ost + w.whave)));
    const uint32_t lane = t & 63u;
    unsigned long long key = ~0ull;
    if (m) {
      const int f = __builtin_ctzll(m);
      const uint32_t sf = (uint32_t)__builtin_amdgcn_readlane((int)s, f);
      const uint32_t of = (uint32_t)__builtin_amdgcn_readlane((int)min(ost, 0xffffu), f);
      key = ((unsigned long long)((t & ~63u) + (uint32_t)f) << 32) | (sf << 16) | of;
    } else if (t >= WW_T - 64u) {
      const uint32_t el = (uint32_t)__builtin_amdgcn_readlane((int)(s + snb), 63);
      const uint32_t il = (uint32_t)__builtin_amdgcn_readlane((int)min(incl, 0xffffu), 63);
      key = ((unsigned long long)WW_T << 32) | (el << 16) | il;
    }
    if (lane == 0 && key != ~0ull) atomicMin(&w.nkey, key);
  }
  if (t == 0) w.carry = 0;
  __syncthreads();
  const unsigned long long nk = w.nkey;
  const uint32_t n = (uint32_t)(nk >> 32), T = (uint32_t)nk & 0xffffu;
  [[maybe_unused]] const uint64_t kt2 = KP_NOW();
  KPW0_ADD(KP_W_CYC_DECODE, kt1 - kt0);
  KPW0_ADD(KP_W_CYC_CHAIN, kt2 - kt1);
  // 5. expansion, WW_STEP bytes per step, WW_EB consecutive per thread
  const uint32_t base = w.pos;
  uint16_t *marks = w.ja;                                        // WW_STEP u16
  uint32_t *ent = reinterpret_cast<uint32_t *>(w.ja + WW_STEP);  // WW_STEP u32 (into jb / jc)
  for (uint32_t b0 = 0; b0 < T; b0 += WW_STEP) {
    if (b0) {
      reinterpret_cast<uint4 *>(marks)[t] = make_uint4(0u, 0u, 0u, 0u);
      __syncthreads();
    }
    // round flags: each round ORs into open[r & 1] before its one barrier, reads
    // it after, and clears the other (read last round, before this barrier;
    // next set after the barrier the next round passes first)
    if (t == 0) {
      w.open[0] = 0;
      w.open[1] = 0;
    }
    if (t < n && ost >= b0 && ost < b0 + WW_STEP) marks[ost - b0] = (uint16_t)(t + 1u);
    __syncthreads();
    const uint4 mk = reinterpret_cast<const uint4 *>(marks)[t];
    uint32_t mm[WW_EB] = {mk.x & 0xffffu, mk.x >> 16, mk.y & 0xffffu, mk.y >> 16,
                          mk.z & 0xffffu, mk.z >> 16, mk.w & 0xffffu, mk.w >> 16};
#pragma unroll
    for (uint32_t r = 1; r < WW_EB; r++) mm[r] = max(mm[r], mm[r - 1]);
    const uint32_t carry = w.carry;
    // symbol of each byte: the last mark at or before it; the thread's bytes
    // before its own first mark continue the symbol open at the end of thread
    // t - 1, or of the previous step
    uint32_t pin;
    (void)ww_scan<true>(w, mm[WW_EB - 1], &pin);
    const uint32_t pv = max(pin, carry + 1u);
    uint32_t e[WW_EB];
    bool open = false;
#pragma unroll
    for (uint32_t r = 0; r < WW_EB; r++) {
      const uint32_t si = max(pv, mm[r]) - 1u;
      if (r == WW_EB - 1 && t == WW_T - 1u) w.carry = si;
      const uint32_t Ls = w.symL[si], Ds = w.symD[si];
      const uint32_t j = b0 + WW_EB * t + r;
      const int32_t sp = (int32_t)j - (int32_t)Ds;  // relative to `base`
      const uint32_t rv = ring[(base + (uint32_t)sp) & RMASK];
      e[r] = (Ls & 0x80000000u) ? (0x100u | (Ls & 0xffu))
                                : (sp >= (int32_t)b0 ? (((uint32_t)sp - b0) << 16) : (0x100u | rv));
      open = open || (j < T && !(e[r] & 0x100u));
    }
    reinterpret_cast<uint4 *>(ent)[2u * t] = make_uint4(e[0], e[1], e[2], e[3]);
    reinterpret_cast<uint4 *>(ent)[2u * t + 1u] = make_uint4(e[4], e[5], e[6], e[7]);
    if (__ballot(open) && (t & 63u) == 0) atomicOr(&w.open[0], 1u);
    __syncthreads();
    uint32_t rp = 0;
    while (w.open[rp]) {
      if (t == 0) w.open[rp ^ 1u] = 0;
      rp ^= 1u;
      KPW0_ADD(KP_W_JUMPS, 1);
      uint32_t g[WW_EB];
#pragma unroll
      for (uint32_t r = 0; r < WW_EB; r++) g[r] = ent[(e[r] & 0x100u) ? 0u : (e[r] >> 16)];
      open = false;
#pragma unroll
      for (uint32_t r = 0; r < WW_EB; r++) {
        if (!(e[r] & 0x100u)) e[r] = (g[r] & 0x100u) ? g[r] : (g[r] & 0xffff0000u);
        open = open || (b0 + WW_EB * t + r < T && !(e[r] & 0x100u));
      }
      __syncthreads();
      reinterpret_cast<uint4 *>(ent)[2u * t] = make_uint4(e[0], e[1], e[2], e[3]);
      reinterpret_cast<uint4 *>(ent)[2u * t + 1u] = make_uint4(e[4], e[5], e[6], e[7]);
      if (__ballot(open) && (t & 63u) == 0) atomicOr(&w.open[rp], 1u);
      __syncthreads();
    }
#pragma unroll
    for (uint32_t r = 0; r < WW_EB; r++) {
      const uint32_t j = b0 + WW_EB * t + r;
      if (j < T) ring[(base + j) & RMASK] = (uint8_t)e[r];
    }
    __syncthreads();
  }
  KPW0_ADD(KP_W_BATCHES, (T + WW_STEP - 1) / WW_STEP);
  KPW0_ADD(KP_W_CYC_EXPAND, KP_NOW() - kt2);
}

template <bool D64, bool WIDE = false>
struct Inflater {
  static constexpr uint32_t RING = D64 ? 65536u : 32768u;
  static constexpr uint32_t RMASK = RING - 1;

  uint8_t *ring;       // LDS history ring
  uint32_t *inring;    // LDS compressed-input ring
  uint32_t *tab;       // LDS dynamic tables
  uint32_t tab_bits = 0;  // tab holds built dynamic tables: lbits | dbits << 8 | 1 << 16
  uint32_t *ftab;      // LDS fixed tables (built on first use)
  uint16_t *lens;      // LDS code lengths
  uint16_t *sorted;    // LDS sort scratch
  uint32_t *scratch16; // LDS 32 words

  // input
  const uint8_t *abase;  // 16 B aligned base of the job input
  uint32_t limit_bits;   // (misalign + in_len) * 8
  uint32_t end_byte;     // misalign + in_len
  uint32_t wi;           // next 32-bit word to pull into hold
  uint32_t committed;    // pieces [committed-4, committed) are in the LDS ring
  uint4 pending;         // piece `committed`, in flight in registers
  uint64_t hold;
  uint32_t nbits;

  // output
  uint8_t *out;
  uint32_t cap, pos, flushed;
  uint32_t whave;  // bytes of history before output position 0
  bool fixed_ready;

  __device__ uint4 load_piece(uint32_t k) {
    uint32_t lane = lane_id();
    uint32_t b = k * (PIECE_WORDS * 4) + lane * 16;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (b < end_byte) {
      v = *reinterpret_cast<const uint4 *>(abase + b);
      if (b + 16 > end_byte) {  // zero the bytes past the end of the input
        uint32_t keep = end_byte - b;
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
          int kb = (int)keep - q * 4;
          uint32_t m = kb >= 4 ? 0xffffffffu : (kb <= 0 ? 0u : ((1u << (8 * kb)) - 1u));
          w[q] &= m;
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    return v;
  }
  __device__ void store_piece(uint32_t k, uint4 v) {
    uint32_t lane = lane_id();
    *reinterpret_cast<uint4 *>(&inring[(k & 3) * PIECE_WORDS + lane * 4]) = v;
  }
  // position the reader at absolute bit `bit` (relative to abase)
  __device__ void seek(uint32_t bit) {
    uint32_t w = bit >> 5;
    uint32_t k0 = w / PIECE_WORDS;
    __builtin_amdgcn_wave_barrier();
    store_piece(k0, load_piece(k0));
    store_piece(k0 + 1, load_piece(k0 + 1));
    store_piece(k0 + 2, load_piece(k0 + 2));
    committed = k0 + 3;
    pending = load_piece(committed);
    __builtin_amdgcn_wave_barrier();
    wi = w;
    hold = 0;
    nbits = 0;
    refill();
    uint32_t skip = bit & 31;
    hold >>= skip;
    nbits -= skip;
  }
  __device__ __forceinline__ void refill() {
    if (nbits < 32) {
      uint32_t w = inring[wi & (IN_RING_WORDS - 1)];
      hold |= (uint64_t)w << nbits;
      nbits += 32;
      wi++;
      if (wi + 16 >= committed * PIECE_WORDS) {
        __builtin_amdgcn_wave_barrier();
        store_piece(committed, pending);
        committed++;
        pending = load_piece(committed);
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  __device__ __forceinline__ uint32_t bitpos() const { return wi * 32u - nbits; }
  __device__ __forceinline__ void drop(uint32_t n) {
    hold >>= n;
    nbits -= n;
  }
  __device__ __forceinline__ bool short_of(uint32_t need) const { return bitpos() + need > limit_bits; }

  __device__ void flush_piece() {
    uint32_t lane = lane_id();
    uint4 v = *reinterpret_cast<const uint4 *>(&ring[(flushed + lane * 16) & RMASK]);
    if (__builtin_expect((reinterpret_cast<uintptr_t>(out) & 15u) == 0, 1)) {
      *reinterpret_cast<uint4 *>(out + flushed + lane * 16) = v;
    } else {  // a later piece of a long stream starts at any output byte
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; k++) out[flushed + lane * 16 + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
    flushed += FLUSH_BYTES;
  }
  __device__ __forceinline__ void maybe_flush() {
    while (pos - flushed >= FLUSH_BYTES) flush_piece();
  }
  __device__ void flush_tail() {
    uint32_t lane = lane_id();
    uint32_t rem = pos - flushed;
    for (uint32_t k = lane; k < rem; k += WAVE) out[flushed + k] = ring[(flushed + k) & RMASK];
    flushed = pos;
  }

  __device__ __forceinline__ void put_literal(uint32_t v) {
    ring[pos & RMASK] = (uint8_t)v;
    pos++;
    if (pos - flushed >= FLUSH_BYTES) flush_piece();
  }

  // copy n bytes (n <= len, room already checked) from `dist` back
  __device__ void copy_match(uint32_t n, uint32_t dist) {
    uint32_t lane = lane_id();
    if (dist >= WAVE) {
      // every batch reads bytes at least 64 back: all already final
      while (n) {
        uint32_t cnt = min(n, (uint32_t)WAVE);
        uint8_t v = 0;
        if (lane < cnt) v = ring[(pos + lane - dist) & RMASK];
        __builtin_amdgcn_wave_barrier();
        if (lane < cnt) ring[(pos + lane) & RMASK] = v;
        __builtin_amdgcn_wave_barrier();
        pos += cnt;
        n -= cnt;
        maybe_flush();
      }
    } else {
      // period P = dist * floor(64 / dist): batches of P lanes; the first batch
      // reads the source period, later ones read P bytes back.
      uint32_t per = (uint32_t)(64u / dist) * dist;
      uint32_t q = (uint32_t)((float)lane * __builtin_amdgcn_rcpf((float)dist) + 1e-3f);
      if (q * dist > lane) q--;
      if ((q + 1) * dist <= lane) q++;
      uint32_t lm = lane - q * dist;  // lane % dist
      bool firstb = true;
      while (n) {
        uint32_t cnt = min(n, per);
        uint8_t v = 0;
        if (lane < cnt) v = firstb ? ring[(pos - dist + lm) & RMASK] : ring[(pos + lane - per) & RMASK];
        __builtin_amdgcn_wave_barrier();
        if (lane < cnt) ring[(pos + lane) & RMASK] = v;
        __builtin_amdgcn_wave_barrier();
        pos += cnt;
        n -= cnt;
        firstb = false;
        maybe_flush();
      }
    }
  }

  // stored block copy of n bytes from input byte `src` (relative to abase)
  __device__ void copy_stored(uint32_t src, uint32_t n) {
    uint32_t lane = lane_id();
    uint32_t b = 0;
    if constexpr (WIDE) {
      // the stream kernel: the whole workgroup copies (its other waves idle
      // through a stored block otherwise: a 32 KiB stored call spent ~25 K of
      // its ~41 K wave-0 cycles here), 16 KiB at a time so that the ring's
      // unflushed bytes never wrap onto themselves
      if (wide != nullptr && src >= 4u) {
        while (n - b >= WW_COPY_MIN) {
          const uint32_t m = min(n - b, 16384u);
          WideLDS &w = wide->wide;
          if (lane == 0) {
            w.op = WW_COPY;
            w.W = m;
            w.pos = pos;
            w.cp_src = (unsigned long long)(uintptr_t)(abase + src + b);
          }
          __syncthreads();  // the other waves wait here for a command
          ww_copy<D64>(*wide);
          pos += m;
          b += m;
          maybe_flush();
        }
      }
    }
    // 4 KiB steps: a lane takes four 16-byte pieces, each as five aligned
    // dword loads funnel-shifted by the (uniform) source misalignment -- 20
    // loads in flight per lane, one memory latency per 4 KiB (the 1 KiB steps
    // of byte loads below paid one per KiB: a 32 KiB stored call of the handle
    // ABI spent ~32 us on its workgroup).  The loads reach at most 3 bytes
    // before the step's bytes (the block's LEN / NLEN) and 4 after (inside the
    // block while b + 4 KiB + 4 <= n).
    if (!WIDE && src >= 4u) {  // (the stream kernel's wave 0 took the bulk to its workgroup above)
      const uint32_t sh = src & 3u;
      for (; b + 4096u + 4u <= n; b += 4096u) {
        uint32_t d[4][4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t s0 = src + b + (uint32_t)j * 1024u + lane * 16u;
          const uint32_t *wp = reinterpret_cast<const uint32_t *>(abase + (s0 & ~3u));
          uint32_t x[5];
#pragma unroll
          for (int q = 0; q < 5; q++) x[q] = wp[q];
#pragma unroll
          for (int q = 0; q < 4; q++) d[j][q] = __builtin_amdgcn_alignbyte(x[q + 1], x[q], sh);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t o = pos + (uint32_t)j * 1024u + lane * 16u;
          if ((pos & 3u) == 0) {  // whole dwords (RING is a multiple of 4: none straddles the wrap)
#pragma unroll
            for (int q = 0; q < 4; q++) *reinterpret_cast<uint32_t *>(&ring[(o + 4u * q) & RMASK]) = d[j][q];
          } else {
#pragma unroll
            for (int q = 0; q < 16; q++) ring[(o + q) & RMASK] = (uint8_t)(d[j][q >> 2] >> (8 * (q & 3)));
          }
        }
        __builtin_amdgcn_wave_barrier();
        pos += 4096u;
        maybe_flush();
      }
    }
    // 1 KiB steps, 16 bytes per lane: the 16 byte loads of a lane are issued
    // together (one memory latency per KiB instead of one per 64 bytes)
    for (; b + 1024u <= n; b += 1024u) {
      const uint8_t *sp = abase + src + b + lane * 16u;
      uint8_t v[16];
#pragma unroll
      for (int q = 0; q < 16; q++) v[q] = sp[q];
      const uint32_t o = pos + lane * 16u;
#pragma unroll
      for (int q = 0; q < 16; q++) ring[(o + q) & RMASK] = v[q];
      __builtin_amdgcn_wave_barrier();
      pos += 1024u;
      maybe_flush();
    }
    for (; b < n; b += WAVE) {
      uint32_t k = b + lane;
      if (k < n) ring[(pos + lane) & RMASK] = abase[src + k];
      __builtin_amdgcn_wave_barrier();
      uint32_t adv = min(n - b, (uint32_t)WAVE);
      pos += adv;
      maybe_flush();
    }
  }

  __device__ void build_fixed() {
    // src/inflate.c:260-298 lengths: 0-143 -> 8, 144-255 -> 9, 256-279 -> 7, 280-287 -> 8; 32 distance codes of 5
    uint32_t lane = lane_id();
    for (uint32_t s = lane; s < 288; s += WAVE) lens[s] = s < 144 ? 8 : (s < 256 ? 9 : (s < 280 ? 7 : 8));
    __builtin_amdgcn_wave_barrier();
    uint32_t r = 9;
    build_table(T_LENS, lens, 288, ftab, &r, sorted, scratch16, D64);
    for (uint32_t s = lane; s < 32; s += WAVE) lens[s] = 5;
    __builtin_amdgcn_wave_barrier();
    r = 5;
    build_table(T_DISTS, lens, 32, ftab + 512, &r, sorted, scratch16, D64);
    fixed_ready = true;
  }

  uint32_t stop_bits;  // end bit of the last decoded element (errors / FULL / END)

  // Resume bookkeeping (ZsStreamDev): the state a later call continues from.
  // r_bit is the restart bit of the element in progress: a block header
  // restarts at its first bit, a symbol at its first bit (zlib keeps the
  // partial header / length / distance in its state instead; both resume to
  // the same bits and output).
  uint32_t r_mode, r_bit, r_len, r_dist, r_btype, r_nlen, r_ndist;
  bool blast;  // BFINAL of the current block
  // ZS_JF_PART (a piece of a longer stream): stop with ZD_STOP at the first
  // block boundary at or past bit stop_after or output byte out_stop
  uint32_t stop_after = 0xffffffffu, out_stop = 0xffffffffu;

  // stored bytes [src, src + slen) (src/inflate.c:885-904 COPY); -1 = complete
  __device__ int stored_copy(uint32_t src, uint32_t slen) {
    uint32_t avail = end_byte - src;
    uint32_t room = cap - pos;
    uint32_t m = min(slen, min(avail, room));
    copy_stored(src, m);
    if (m < slen) {
      r_mode = ZSM_STORED;
      r_len = slen - m;
      r_bit = (src + m) * 8;
      if (m == avail) return ZD_TRUNC;  // input exhausted first (or at the same time)
      stop_bits = (src + m) * 8;
      return ZD_FULL;
    }
    seek((src + slen) * 8);
    return -1;
  }

  // dynamic tables from lens[0, nlen + ndist) (src/inflate.c:1010-1032)
  __device__ int dyn_tables(uint32_t nlen, uint32_t ndist, const uint32_t **lt, const uint32_t **dt, uint32_t *lbits,
                            uint32_t *dbits) {
    *lbits = 9;
    if (build_table(T_LENS, lens, nlen, tab, lbits, sorted, scratch16, D64)) return ZD_ERROR | (ZM_LITLEN_SET << 8);
    // distance table goes right after the literal/length table; its size
    // is bounded by 852 entries (ENOUGH_LENS)
    *dbits = 6;
    if (build_table(T_DISTS, lens + nlen, ndist, tab + 852, dbits, sorted, scratch16, D64))
      return ZD_ERROR | (ZM_DIST_SET << 8);
    *lt = tab;
    *dt = tab + 852;
    tab_bits = *lbits | (*dbits << 8) | (1u << 16);
    return -1;
  }

  // Block header (src/inflate.c:834-1033).  -1: symbols follow with *lt/*dt;
  // -2: a stored block was copied whole; otherwise a ZD_* code.
  __device__ int block_header(const uint32_t **lt, const uint32_t **dt, uint32_t *lbits, uint32_t *dbits) {
    uint32_t lane = lane_id();
    r_mode = ZSM_TYPE;
    r_bit = bitpos();
    refill();
    if (short_of(3)) return ZD_TRUNC;
    blast = (hold & 1) != 0;
    uint32_t type = (uint32_t)(hold >> 1) & 3u;
    drop(3);
    if (type == 0) {
      uint32_t pad = bitpos() & 7u;
      if (pad) drop(8 - pad);
      refill();
      if (short_of(32)) return ZD_TRUNC;
      uint32_t v = (uint32_t)hold;
      if ((v & 0xffffu) != ((v >> 16) ^ 0xffffu)) {
        stop_bits = bitpos() + 32;
        return ZD_ERROR | (ZM_STORED_LEN << 8);
      }
      drop(32);
      int rc = stored_copy(bitpos() >> 3, v & 0xffffu);
      return rc < 0 ? -2 : rc;
    }
    if (type == 1) {
      if (!fixed_ready) build_fixed();
      *lt = ftab;
      *dt = ftab + 512;
      *lbits = 9;
      *dbits = 5;
      r_btype = 1;
      return -1;
    }
    if (type != 2) {
      stop_bits = bitpos();
      return ZD_ERROR | (ZM_BLOCK_TYPE << 8);
    }
    // ---- dynamic header (src/inflate.c:905-1033) ----
    refill();
    if (short_of(14)) return ZD_TRUNC;
    uint32_t nlen = (uint32_t)(hold & 31) + 257;
    uint32_t ndist = (uint32_t)((hold >> 5) & 31) + 1;
    uint32_t ncode = (uint32_t)((hold >> 10) & 15) + 4;
    drop(14);
    if (nlen > 286 || (!D64 && ndist > 30)) {
      stop_bits = bitpos();
      return ZD_ERROR | (ZM_TOO_MANY << 8);
    }
    // code-length code lengths (src/inflate.c:923-934)
    for (uint32_t i = 0; i < ncode; i++) {
      refill();
      if (short_of(3)) return ZD_TRUNC;
      if (lane == 0) lens[c_clorder[i]] = (uint16_t)(hold & 7u);
      drop(3);
    }
    if (lane >= ncode && lane < 19) lens[c_clorder[lane]] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t cbits = 7;
    if (build_table(T_CODES, lens, 19, tab, &cbits, sorted, scratch16, D64)) {
      stop_bits = bitpos();
      return ZD_ERROR | (ZM_CODE_LENGTHS << 8);
    }
    uint32_t total = nlen + ndist;
    uint32_t have = 0;
    uint32_t cmask = (1u << cbits) - 1;
    while (have < total) {
      refill();
      uint32_t e = tab[(uint32_t)hold & cmask];
      uint32_t eb = e_bits(e), ev = e_val(e);
      if (short_of(eb)) return ZD_TRUNC;
      if (ev < 16) {
        drop(eb);
        if (lane == 0) lens[have] = (uint16_t)ev;
        have++;
        continue;
      }
      uint32_t xb = ev == 16 ? 2 : (ev == 17 ? 3 : 7);
      if (short_of(eb + xb)) return ZD_TRUNC;
      drop(eb);
      if (ev == 16 && have == 0) {
        stop_bits = bitpos() + 2;
        return ZD_ERROR | (ZM_REPEAT << 8);
      }
      uint32_t rep = (ev == 16 ? 3 : (ev == 17 ? 3 : 11)) + ((uint32_t)hold & ((1u << xb) - 1));
      drop(xb);
      if (have + rep > total) {
        stop_bits = bitpos();
        return ZD_ERROR | (ZM_REPEAT << 8);
      }
      __builtin_amdgcn_wave_barrier();
      uint32_t fillv = ev == 16 ? uni(lens[have - 1]) : 0u;
      if (lane < rep) lens[have + lane] = (uint16_t)fillv;  // rep <= 138 > 64: loop
      if (lane + 64 < rep) lens[have + lane + 64] = (uint16_t)fillv;
      if (lane + 128 < rep) lens[have + lane + 128] = (uint16_t)fillv;
      __builtin_amdgcn_wave_barrier();
      have += rep;
    }
    __builtin_amdgcn_wave_barrier();
    if (uni(lens[256]) == 0) {
      stop_bits = bitpos();
      return ZD_ERROR | (ZM_MISSING_EOB << 8);
    }
    int rc = dyn_tables(nlen, ndist, lt, dt, lbits, dbits);
    if (rc >= 0) {
      stop_bits = bitpos();
      return rc;
    }
    r_btype = 2;
    r_nlen = nlen;
    r_ndist = ndist;
    return -1;
  }

  // ---- wave-parallel symbol window ----------------------------------------
  // The serial loop pays several dependent LDS round trips per symbol.  Here
  // the 64 lanes decode a complete symbol (literal/length code, extra bits,
  // distance code, extra bits) at EVERY bit offset of a 512-bit window, 8
  // offsets per lane, all independent; the true symbol chain is then followed
  // through register reads (readlane of packed lengths) and the chain's
  // symbols are expanded 64 output bytes at a time, in-batch copy sources
  // resolved by pointer jumping.  Only symbols with nothing exceptional are
  // taken (complete inside the input, fitting the output, legal distance,
  // not end-of-block / invalid): everything else stays on the exact serial
  // path, so results and stop points are unchanged.
  static constexpr uint32_t FW_OFFS = 8;
  static constexpr uint32_t FW_BITS = FW_OFFS * WAVE;
  static constexpr uint32_t FW_JN = FW_BITS + WAVE;  // jump-table entries (offsets past the window loop on themselves)
  uint16_t *jmp;  // LDS: 2 x FW_JN jump tables, reused as 256 u32 expansion entries

  __device__ __forceinline__ uint64_t bits_at(uint32_t q) const {
    const uint32_t w = q >> 5, sh = q & 31u;
    const uint32_t a = inring[w & (IN_RING_WORDS - 1)];
    const uint32_t b = inring[(w + 1) & (IN_RING_WORDS - 1)];
    const uint32_t c = inring[(w + 2) & (IN_RING_WORDS - 1)];
    uint64_t h = ((((uint64_t)b) << 32) | a) >> sh;
    if (sh) h |= (uint64_t)c << (64u - sh);
    return h;
  }
  // words [.., w_end) resident in the LDS input ring
  __device__ void ensure_words(uint32_t w_end) {
    while (committed * PIECE_WORDS < w_end) {
      __builtin_amdgcn_wave_barrier();
      store_piece(committed, pending);
      committed++;
      pending = load_piece(committed);
      __builtin_amdgcn_wave_barrier();
    }
  }
  // bit reader at absolute bit `bit` (its word is in the ring)
  __device__ void reseat(uint32_t bit) {
    wi = bit >> 5;
    hold = (uint64_t)inring[wi & (IN_RING_WORDS - 1)] >> (bit & 31u);
    nbits = 32u - (bit & 31u);
    wi++;
  }
  __device__ __forceinline__ static uint32_t scan_sum(uint32_t x) {  // inclusive, wave64
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return x;
  }
  __device__ __forceinline__ static uint32_t scan_max(uint32_t v) {  // inclusive, wave64
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
  }
  __device__ __forceinline__ static uint32_t perm(uint32_t from_lane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(from_lane << 2), (int)v);
  }

  // Returns the symbols applied (0: the caller decodes the next one serially).
  __device__ uint32_t fast_window(const uint32_t *lt, const uint32_t *dt, uint32_t lmask, uint32_t dmask) {
    const uint32_t lane = lane_id();
    const uint32_t P = bitpos();
    if (P + FW_BITS + 64u > limit_bits || pos == cap) return 0;
    [[maybe_unused]] const uint64_t kt0 = KP_NOW();
    ensure_words(((P + FW_BITS + 64u) >> 5) + 3u);
    // 1. a complete symbol at every offset P + lane + 64 i; straight-line
    //    stages (input bits, root, sub-table, distance root, distance
    //    sub-table) so each stage issues its 8 LDS loads back to back
    uint32_t nbp0 = 0, nbp1 = 0;  // total bits per slot, 8 bits each (0 = stop here)
    uint32_t lv[FW_OFFS], dv[FW_OFFS];
    uint64_t hh[FW_OFFS];
    uint32_t ee[FW_OFFS], e2[FW_OFFS], used[FW_OFFS];
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) hh[i] = bits_at(P + lane + i * WAVE);
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) ee[i] = lt[(uint32_t)hh[i] & lmask];
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) {
      const uint32_t op = e_op(ee[i]);
      used[i] = e_bits(ee[i]);
      const bool sub = op != 0 && (op & 0xf0u) == 0;
      e2[i] = lt[sub ? e_val(ee[i]) + (((uint32_t)(hh[i] >> used[i])) & ((1u << op) - 1)) : 0u];
    }
    uint64_t hd[FW_OFFS];
    uint32_t sb[FW_OFFS], de[FW_OFFS];
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) {
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
      de[i] = dt[(uint32_t)hd[i] & dmask];
    }
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) {
      const uint32_t dop0 = e_op(de[i]);
      const uint32_t du0 = e_bits(de[i]);
      const bool dsub = (dop0 & 0xf0u) == 0;
      e2[i] = dt[dsub ? e_val(de[i]) + (((uint32_t)(hd[i] >> du0)) & ((1u << dop0) - 1)) : 0u];
    }
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) {
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
      if (op == 0) {
        nb = used[i];
      } else if ((op & 96u) == 0 && (dop & 64u) == 0) {
        nb = sb[i] + dused + dx;
        dv[i] = e_val(d) + ((uint32_t)(hd[i] >> dused) & ((1u << dx) - 1u));
      }
      if (op == 0 || nb == 0) dv[i] = 0;
      const uint32_t q = P + lane + i * WAVE;
      if (q + nb > limit_bits) nb = 0;
      if (i < 4) nbp0 |= nb << (8u * i);
      else nbp1 |= nb << (8u * (i - 4u));
    }
    [[maybe_unused]] const uint64_t kt1 = KP_NOW();
    // 2. the chain from P by pointer doubling: J0(q) = q + bits(q) (q itself
    //    where no symbol may start, and past the window), J(k+1) = Jk o Jk;
    //    lane m ends with s_m, the start of the chain's m-th symbol
    //    (s_(2^k + i) = Jk(s_i)).
    uint16_t *ja = jmp, *jb = jmp + FW_JN;
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) {
      const uint32_t q = lane + i * WAVE;
      const uint32_t nb = ((i < 4 ? nbp0 : nbp1) >> (8u * (i & 3u))) & 0xffu;
      ja[q] = (uint16_t)(q + nb);
    }
    ja[FW_BITS + lane] = (uint16_t)(FW_BITS + lane);
    __builtin_amdgcn_wave_barrier();
    uint32_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < 6; k++) {
      const uint32_t half = 1u << k;
      const uint32_t t = perm(lane >= half ? lane - half : 0u, s);
      const uint32_t g = ja[t];
      if (lane >= half && lane < 2u * half) s = g;
      if (k < 5) {
#pragma unroll
        for (uint32_t i = 0; i < FW_OFFS + 1; i++) {
          const uint32_t q = lane + i * WAVE;
          jb[q] = ja[ja[q]];
        }
        __builtin_amdgcn_wave_barrier();
        uint16_t *tmp = ja;
        ja = jb;
        jb = tmp;
      }
    }
    // a chain symbol: inside the window and decodable (nbits != 0)
    const uint32_t xs = s < FW_BITS ? s : 0u;
    const uint32_t px0 = perm(xs & 63u, nbp0), px1 = perm(xs & 63u, nbp1);
    const uint32_t nbs = (((xs >> 6) < 4u ? px0 : px1) >> (8u * ((xs >> 6) & 3u))) & 0xffu;
    const uint64_t badc = __ballot(!(s < FW_BITS && nbs != 0));
    const uint32_t cnt = badc ? (uint32_t)__builtin_ctzll(badc) : WAVE;
    const uint32_t mypos = s;
    const uint32_t s63 = __builtin_amdgcn_readlane(s, WAVE - 1);
    const uint32_t nb63 = __builtin_amdgcn_readlane(nbs, WAVE - 1);
    const uint32_t cur = cnt < WAVE ? 0u : s63 + nb63;  // chain end when all 64 are symbols
    [[maybe_unused]] const uint64_t kt2 = KP_NOW();
    KPW_ADD(KP_W_WINDOWS, 1);
    KPW_ADD(KP_W_CYC_DECODE, kt1 - kt0);
    KPW_ADD(KP_W_CYC_CHAIN, kt2 - kt1);
    if (cnt == 0) {
      KPW_ADD(KP_W_EMPTY, 1);
      return 0;
    }
    // 3. symbol k -> lane k
    const uint32_t src = mypos & 63u, sl = mypos >> 6;
    uint32_t L = 0, D = 0;
#pragma unroll
    for (uint32_t i = 0; i < FW_OFFS; i++) {
      const uint32_t a = perm(src, lv[i]);
      const uint32_t b = perm(src, dv[i]);
      if (sl == i) {
        L = a;
        D = b;
      }
    }
    const bool act = lane < cnt;
    const bool lit = (L & 0x80000000u) != 0;
    const uint32_t olen = act ? (lit ? 1u : L) : 0u;
    const uint32_t incl = scan_sum(olen);
    const uint32_t ost = incl - olen;
    // admissible prefix: fits the output and the distance reaches written history
    const bool ok = act && incl <= cap - pos && (lit || D <= pos + ost + whave);
    const uint64_t badm = __ballot(!ok);
    const uint32_t n = badm ? (uint32_t)__builtin_ctzll(badm) : WAVE;
    if (n == 0) {
      KPW_ADD(KP_W_EMPTY, 1);
      return 0;
    }
    const uint32_t T = __builtin_amdgcn_readlane(incl, n - 1);
    const uint32_t endrel = n < WAVE ? __builtin_amdgcn_readlane(mypos, n) : cur;
    // 4. expand 256 output bytes per step, 4 consecutive per lane: symbol of
    //    each byte from start marks + a max-scan; copy sources before the step
    //    read the ring (final), sources inside it resolve by pointer jumping
    //    through an LDS entry array (0x100 | byte = resolved, else index << 16)
    const uint32_t base = pos;
    uint32_t carry = 0;
    uint16_t *marks = sorted;                            // table-build scratch, idle inside a block
    uint32_t *ent = reinterpret_cast<uint32_t *>(jmp);   // the jump tables are done with
    for (uint32_t b0 = 0; b0 < T; b0 += 4u * WAVE) {
      reinterpret_cast<uint2 *>(marks)[lane] = make_uint2(0u, 0u);
      __builtin_amdgcn_wave_barrier();
      if (lane < n && ost >= b0 && ost < b0 + 4u * WAVE) marks[ost - b0] = (uint16_t)(lane + 1u);
      __builtin_amdgcn_wave_barrier();
      const uint2 mk = reinterpret_cast<const uint2 *>(marks)[lane];
      uint32_t mm[4] = {mk.x & 0xffffu, mk.x >> 16, mk.y & 0xffffu, mk.y >> 16};
      mm[1] = max(mm[1], mm[0]);
      mm[2] = max(mm[2], mm[1]);
      mm[3] = max(mm[3], mm[2]);
      const uint32_t inc = scan_max(mm[3]);
      uint32_t prev = perm(lane ? lane - 1u : 0u, inc);
      prev = max(lane ? prev : 0u, carry + 1u);
      uint32_t e[4], Ls[4], Ds[4], rv[4];
      int32_t sp[4];
      bool open = false;
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        const uint32_t si = max(prev, mm[r]) - 1u;
        if (r == 3) carry = __builtin_amdgcn_readlane(si, WAVE - 1);
        Ls[r] = perm(si, L);
        Ds[r] = perm(si, D);
      }
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        sp[r] = (int32_t)(b0 + 4u * lane + r) - (int32_t)Ds[r];  // relative to `base`
        rv[r] = ring[(base + (uint32_t)sp[r]) & RMASK];
      }
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        const bool inb = sp[r] >= (int32_t)b0;
        e[r] = (Ls[r] & 0x80000000u) ? (0x100u | (Ls[r] & 0xffu))
                                     : (inb ? (((uint32_t)sp[r] - b0) << 16) : (0x100u | rv[r]));
        open = open || !(e[r] & 0x100u);
      }
      if (__ballot(open)) {
        reinterpret_cast<uint4 *>(ent)[lane] = make_uint4(e[0], e[1], e[2], e[3]);
        __builtin_amdgcn_wave_barrier();
        do {
          KPW_ADD(KP_W_JUMPS, 1);
          uint32_t g[4];
#pragma unroll
          for (uint32_t r = 0; r < 4; r++) g[r] = ent[(e[r] & 0x100u) ? 0u : (e[r] >> 16)];
          open = false;
#pragma unroll
          for (uint32_t r = 0; r < 4; r++) {
            if (!(e[r] & 0x100u)) e[r] = (g[r] & 0x100u) ? g[r] : (g[r] & 0xffff0000u);
            open = open || !(e[r] & 0x100u);
          }
          __builtin_amdgcn_wave_barrier();
          reinterpret_cast<uint4 *>(ent)[lane] = make_uint4(e[0], e[1], e[2], e[3]);
          __builtin_amdgcn_wave_barrier();
        } while (__ballot(open));
      }
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        const uint32_t j = b0 + 4u * lane + r;
        if (j < T) ring[(base + j) & RMASK] = (uint8_t)e[r];
      }
      __builtin_amdgcn_wave_barrier();
      pos = base + min(T, b0 + 4u * WAVE);
      maybe_flush();
    }
    reseat(P + endrel);
    [[maybe_unused]] const uint64_t kt3 = KP_NOW();
    KPW_ADD(KP_W_CYC_EXPAND, kt3 - kt2);
    KPW_ADD(KP_W_CYC_WINDOW, kt3 - kt0);
    KPW_ADD(KP_W_SYMS, n);
    KPW_ADD(KP_W_BYTES, T);
    KPW_ADD(KP_W_BATCHES, (T + WAVE - 1) / WAVE);
    return n;
  }

  // The workgroup-wide window (WIDE: the stream kernel, this wave is wave 0
  // of WW_T threads): post the window, take part in it, apply its prefix.
  StreamLDS<D64> *wide = nullptr;  // the workgroup's LDS (WIDE)
  __device__ uint32_t wide_window(const uint32_t *lt, const uint32_t *dt, uint32_t lmask, uint32_t dmask) {
    [[maybe_unused]] const uint64_t kq0 = KP_NOW();
    const uint32_t P = bitpos();
    // not worth a window: little output room, little input, or the next
    // symbol is not plain (end of block) -- the serial loop takes these
    if (cap - pos < WW_MIN_ROOM || P + 64u + 1024u > limit_bits) return 0;
    refill();
    {
      uint32_t e = lt[(uint32_t)hold & lmask];
      uint32_t op = e_op(e);
      if (op != 0 && (op & 0xf0u) == 0) op = e_op(lt[e_val(e) + (((uint32_t)(hold >> e_bits(e))) & ((1u << op) - 1))]);
      if (op & 96u) return 0;
    }
    const uint32_t W = min(WW_BITS, ((limit_bits - P - 64u) / 1024u) * 1024u);
    ensure_words(((P + W + 64u) >> 5) + 3u);
    WideLDS &w = wide->wide;
    const uint8_t *lb = reinterpret_cast<const uint8_t *>(wide);
    if (lane_id() == 0) {
      w.op = WW_RUN;
      w.P = P;
      w.W = W;
      w.limit_bits = limit_bits;
      w.pos = pos;
      w.cap = cap;
      w.whave = whave;
      w.lmask = lmask;
      w.dmask = dmask;
      w.lt_off = (uint32_t)(reinterpret_cast<const uint8_t *>(lt) - lb);
      w.dt_off = (uint32_t)(reinterpret_cast<const uint8_t *>(dt) - lb);
    }
    [[maybe_unused]] const uint64_t kw0 = KP_NOW();
    KPW_ADD(KP_W_CYC_PRE, kw0 - kq0);
    __syncthreads();  // the other waves wait here for a window
    ww_run<D64>(*wide);
    const unsigned long long nk = w.nkey;  // posted before the window's last barrier
    const uint32_t n = (uint32_t)(nk >> 32), T = (uint32_t)nk & 0xffffu, endrel = (uint32_t)(nk >> 16) & 0xffffu;
    [[maybe_unused]] const uint64_t kw1 = KP_NOW();
    KPW_ADD(KP_W_CYC_WINDOW, kw1 - kw0);
    KPW_ADD(KP_W_WINDOWS, 1);
    if (n == 0) {
      KPW_ADD(KP_W_EMPTY, 1);
      return 0;
    }
    pos += T;
    maybe_flush();
    reseat(P + endrel);
    KPW_ADD(KP_W_CYC_POST, KP_NOW() - kw1);
    KPW_ADD(KP_W_SYMS, n);
    KPW_ADD(KP_W_BYTES, T);
    return n;
  }

  // MATCH state (src/inflate.c:1142-1187): a decoded match, or the pending
  // rest of one in a resumed call; -1 = copied whole.  left == 0 is tested
  // before the distance, so a too-far distance met with a full output is
  // reported by the next call (whave then counts the earlier calls' output,
  // capped at the window size, as updatewindow keeps it).
  __device__ int finish_match(uint32_t len, uint32_t dist) {
    if (pos == cap) {
      r_mode = ZSM_MATCH;
      r_len = len;
      r_dist = dist;
      r_bit = stop_bits = bitpos();
      return ZD_FULL;
    }
    if (dist > pos + whave) {
      stop_bits = bitpos();
      r_mode = ZSM_BAD;
      return ZD_ERROR | (ZM_TOO_FAR << 8);
    }
    uint32_t n = min(len, cap - pos);
    copy_match(n, dist);
    if (n < len) {
      r_mode = ZSM_MATCH;
      r_len = len - n;
      r_dist = dist;
      r_bit = stop_bits = bitpos();
      return ZD_FULL;
    }
    return -1;
  }

  // ---- symbol loop (src/inffast.c:100-287 / src/inflate.c:1037-1193) ----
  // -1 at the end of the block, otherwise a ZD_* code
  __device__ int symbols(const uint32_t *lt, const uint32_t *dt, uint32_t lbits, uint32_t dbits) {
    r_mode = ZSM_SYMS;
    const uint32_t lmask = (1u << lbits) - 1, dmask = (1u << dbits) - 1;
    for (;;) {
      if constexpr (WIDE) {
        if (wide_window(lt, dt, lmask, dmask)) continue;
      } else {
        if (fast_window(lt, dt, lmask, dmask)) continue;
      }
      KPW_ADD(KP_W_SERIAL, 1);
      refill();
      r_bit = bitpos();
      uint32_t e = lt[(uint32_t)hold & lmask];
      uint32_t op = e_op(e);
      uint32_t used = e_bits(e);
      if (op != 0 && (op & 0xf0u) == 0) {  // second-level table
        uint32_t e2 = lt[e_val(e) + (((uint32_t)(hold >> used)) & ((1u << op) - 1))];
        used += e_bits(e2);
        e = e2;
        op = e_op(e);
      }
      if (short_of(used)) return ZD_TRUNC;
      drop(used);
      if (op == 0) {
        if (pos == cap) {
          r_mode = ZSM_LIT;
          r_len = e_val(e);
          r_bit = stop_bits = bitpos();
          return ZD_FULL;
        }
        put_literal(e_val(e));
        continue;
      }
      if (op & 32) return -1;  // end of block
      if (op & 64) {
        stop_bits = bitpos();
        return ZD_ERROR | (ZM_LITLEN_CODE << 8);
      }
      uint32_t len = e_val(e);
      uint32_t xb = op & (D64 ? 31u : 15u);
      if (xb) {
        if (short_of(xb)) return ZD_TRUNC;
        len += (uint32_t)hold & ((1u << xb) - 1);
        drop(xb);
      }
      refill();
      uint32_t d = dt[(uint32_t)hold & dmask];
      uint32_t dop = e_op(d);
      uint32_t dused = e_bits(d);
      if ((dop & 0xf0u) == 0) {
        uint32_t d2 = dt[e_val(d) + (((uint32_t)(hold >> dused)) & ((1u << dop) - 1))];
        dused += e_bits(d2);
        d = d2;
        dop = e_op(d);
      }
      if (short_of(dused)) return ZD_TRUNC;
      drop(dused);
      if (dop & 64) {
        stop_bits = bitpos();
        return ZD_ERROR | (ZM_DIST_CODE << 8);
      }
      uint32_t dist = e_val(d);
      uint32_t dx = dop & 15u;
      if (dx) {
        if (short_of(dx)) return ZD_TRUNC;
        dist += (uint32_t)hold & ((1u << dx) - 1);
        drop(dx);
      }
      int rc = finish_match(len, dist);
      if (rc >= 0) return rc;
    }
  }

  // Decode from the current bit position to the end of the final block, or
  // until the input or the output runs out.  `mode` is where a resumed call
  // starts (ZSM_TYPE for a whole stream).  Returns ZsDecCode | (ZsMsg << 8);
  // stop_bits says where it stopped and r_* where a next call resumes.
  __device__ int run(uint32_t mode) {
    const uint32_t *lt = ftab, *dt = ftab + 512;
    uint32_t lbits = 9, dbits = 5;
    bool in_block = false;
    int rc;
    if (mode == ZSM_STORED) {
      rc = stored_copy(bitpos() >> 3, r_len);
      if (rc >= 0) return rc;
    } else if (mode == ZSM_SYMS || mode == ZSM_LIT || mode == ZSM_MATCH) {
      if (r_btype == 1) {
        if (!fixed_ready) build_fixed();
      } else {
        if (tab_bits >> 16) {  // the tables a previous call built (zs_stream_kernel loaded them)
          lt = tab;
          dt = tab + 852;
          lbits = tab_bits & 0xffu;
          dbits = (tab_bits >> 8) & 0xffu;
        } else {
          dyn_tables(r_nlen, r_ndist, &lt, &dt, &lbits, &dbits);  // built once already: cannot fail
        }
      }
      if (mode == ZSM_LIT) {
        if (pos == cap) {
          stop_bits = bitpos();
          return ZD_FULL;
        }
        put_literal(r_len);
      } else if (mode == ZSM_MATCH) {
        rc = finish_match(r_len, r_dist);
        if (rc >= 0) return rc;
      }
      in_block = true;
    }
    for (bool first = true;; first = false) {
      if (!in_block) {
        if (blast) {
          stop_bits = bitpos();
          r_mode = ZSM_CHECK;
          r_bit = (stop_bits + 7u) & ~7u;
          return ZD_END;
        }
        if (!first && (bitpos() >= stop_after || pos >= out_stop)) {
          stop_bits = bitpos();
          return ZD_STOP;
        }
        [[maybe_unused]] const uint64_t kh0 = KP_NOW();
        rc = block_header(&lt, &dt, &lbits, &dbits);
        KPW_ADD(KP_W_CYC_TABLES, KP_NOW() - kh0);
        if (rc == -2) continue;
        if (rc >= 0) return rc;
      }
      in_block = false;
      rc = symbols(lt, dt, lbits, dbits);
      if (rc >= 0) return rc;
    }
  }
};

template <bool D64>
__global__ void __launch_bounds__(64) zs_decode_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                        const uint32_t *__restrict__ job_ids, ZsDecDev *__restrict__ decs,
                                                        const uint32_t *__restrict__ run_only) {
  constexpr uint32_t RING = D64 ? 65536u : 32768u;
  // run_only (optional, indexed by job): decode only flagged jobs -- the exact
  // serial decoder as the fallback of the speculative chunked path
  if (run_only && run_only[job_ids[blockIdx.x]] == 0) return;
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[RING];
  __shared__ __attribute__((aligned(16))) uint32_t s_in[IN_RING_WORDS];
  __shared__ uint32_t s_tab[TABLE_ENTRIES];
  __shared__ uint32_t s_ftab[544];
  __shared__ uint16_t s_lens[320];
  __shared__ __attribute__((aligned(16))) uint16_t s_sorted[320];
  __shared__ uint32_t s_scr[32];
  __shared__ __attribute__((aligned(16))) uint16_t s_jmp[2 * Inflater<D64>::FW_JN];

  const uint32_t j = job_ids[blockIdx.x];
  const ZsJobDev jb = jobs[j];
  const ZsHeadDev hd = heads[j];
  ZsDecDev res;
  res.code = ZD_SKIP;
  res.msg = ZM_NONE;
  res.end_bits = 0;
  res.total_out = 0;
  if (hd.code != ZD_END) {
    if (threadIdx.x == 0) decs[j] = res;
    return;
  }
  Inflater<D64> f;
  f.ring = s_ring;
  f.inring = s_in;
  f.tab = s_tab;
  f.ftab = s_ftab;
  f.lens = s_lens;
  f.sorted = s_sorted;
  f.scratch16 = s_scr;
  f.jmp = s_jmp;
  const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
  const uint32_t mis = (uint32_t)(ip & 15u);
  f.abase = reinterpret_cast<const uint8_t *>(ip - mis);
  f.end_byte = mis + (uint32_t)jb.in_len;
  f.limit_bits = f.end_byte * 8u;
  f.out = jb.out;
  f.cap = (uint32_t)jb.out_cap;
  f.pos = 0;
  f.flushed = 0;
  f.whave = 0;
  if (jb.flags & ZS_JF_CONT) {  // a later piece: the output before `out` is its history
    const uint32_t hv = min(jb.hist, RING);
    for (uint32_t i = threadIdx.x; i < hv; i += WAVE) s_ring[RING - hv + i] = jb.out[(int64_t)i - (int64_t)hv];
    __syncthreads();
    f.whave = hv;
  }
  if (jb.flags & ZS_JF_PART) {
    f.stop_after = mis * 8u + jb.stop_after;
    f.out_stop = (uint32_t)ZS_PART_OUT;
  }
  f.fixed_ready = false;
  f.blast = false;
  f.seek((mis + (uint32_t)hd.start_byte) * 8u + jb.sbit);
  f.stop_bits = 0;
  [[maybe_unused]] const uint64_t kt0 = KP_NOW();
  const int packed = f.run(ZSM_TYPE);
  KPW_ADD(KP_W_WAVES, 1);
  KPW_ADD(KP_W_CYC_TOTAL, KP_NOW() - kt0);
  const int code = packed & 0xff;
  f.flush_tail();
  res.code = code;
  res.msg = packed >> 8;
  res.end_bits = (code == ZD_TRUNC) ? (uint64_t)jb.in_len * 8u : (uint64_t)(f.stop_bits - mis * 8u);
  res.total_out = f.pos;
  if (threadIdx.x == 0) decs[j] = res;
}

template __global__ void zs_decode_kernel<false>(const ZsJobDev *, const ZsHeadDev *, const uint32_t *, ZsDecDev *,
                                                 const uint32_t *);
template __global__ void zs_decode_kernel<true>(const ZsJobDev *, const ZsHeadDev *, const uint32_t *, ZsDecDev *,
                                                const uint32_t *);

// ---------------------------------------------------------------------------
// Exact streaming inflate: one call of the handle / zlib ABI
// (src/wasm/wasm_stream_common.c:37-63 -> inflate(strm, flush)), resumed from
// the handle's device state.  The job holds the call buffer (bytes carried
// over from earlier calls + the new input) and the call's output buffer.
// ---------------------------------------------------------------------------
// wave 0 of zs_stream_kernel: one call
template <bool D64>
__device__ __forceinline__ void zs_stream_call(ZsStreamDev *__restrict__ st, const ZsJobDev *__restrict__ job,
                                               const ZsHeadDev *__restrict__ head, StreamLDS<D64> &L) {
  uint8_t *s_ring = L.ring;
  uint32_t *s_in = L.in;
  uint32_t *s_tab = L.tab;
  uint32_t *s_ftab = L.ftab;
  uint16_t *s_lens = L.lens;
  uint16_t *s_sorted = L.sorted;
  uint32_t *s_scr = L.scr;
  L.wide.save = 0;

  const uint32_t lane = lane_id();
  const ZsJobDev jb = *job;
  int32_t mode = st->mode;
  uint32_t rbit = st->rbit;
  int code = ZD_END, msg = ZM_NONE;
  uint32_t stop = rbit, produced = 0;
  if (mode == ZSM_HEAD) {
    const ZsHeadDev hd = *head;
    if (hd.code == ZD_SKIP) {
      if (hd.ret == ZS_BUF_ERROR) {
        code = ZD_TRUNC;
      } else {
        code = ZD_ERROR;
        msg = hd.msg;
        mode = ZSM_BAD;
        stop = (uint32_t)hd.total_in * 8u;
      }
    } else if (hd.code == ZD_NEED_DICT) {
      code = ZD_NEED_DICT;
      mode = ZSM_DICT;
      stop = 6u * 8u;
      if (lane == 0) st->check = hd.adler;
    } else {
      mode = ZSM_TYPE;
      rbit = (uint32_t)hd.start_byte * 8u;
      if (lane == 0) {
        st->is_gzip = hd.is_gzip;
        st->wbits = hd.wbits;
        st->ck_a = hd.is_gzip == 0 ? 1u : 0u;  // adler32(0, Z_NULL, 0) = 1 / CRC register 0
        st->ck_b = 0;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (mode >= ZSM_TYPE && mode <= ZSM_STORED) {
    Inflater<D64, true> f;
    f.wide = &L;
    f.ring = s_ring;
    f.inring = s_in;
    f.tab = s_tab;
    f.ftab = s_ftab;
    f.lens = s_lens;
    f.sorted = s_sorted;
    f.scratch16 = s_scr;
    const uintptr_t ip = reinterpret_cast<uintptr_t>(jb.in);
    const uint32_t mis = (uint32_t)(ip & 15u);
    f.abase = reinterpret_cast<const uint8_t *>(ip - mis);
    f.end_byte = mis + (uint32_t)jb.in_len;
    f.limit_bits = f.end_byte * 8u;
    f.out = jb.out;
    f.cap = (uint32_t)jb.out_cap;
    f.pos = 0;
    f.flushed = 0;
    const uint64_t total = st->total_out;
    const uint32_t wbits = st->wbits ? st->wbits : 15u;
    f.whave = (uint32_t)min<uint64_t>(total, 1ull << wbits);
    // history (window[WOFF + k] is ring position k - RING): loaded by the whole
    // workgroup before the call (zs_stream_kernel)
    f.fixed_ready = false;
    f.r_mode = (uint32_t)mode;
    f.r_bit = mis * 8u + rbit;
    f.r_len = st->len;
    f.r_dist = st->dist;
    f.r_btype = st->btype;
    f.r_nlen = st->nlen;
    f.r_ndist = st->ndist;
    f.blast = st->last != 0;
    f.tab_bits = L.wide.tab_in;  // tables loaded by the workgroup (zs_stream_kernel), or 0
    if (mode != ZSM_TYPE && mode != ZSM_STORED && f.r_btype == 2)
      for (uint32_t k = lane; k < f.r_nlen + f.r_ndist; k += WAVE) s_lens[k] = st->lens[k];
    __builtin_amdgcn_wave_barrier();
    f.seek(mis * 8u + rbit);
    f.stop_bits = 0;
    [[maybe_unused]] const uint64_t kc0 = KP_NOW();
    const int packed = f.run((uint32_t)mode);
    f.flush_tail();
    KPW_ADD(KP_W_WAVES, 1);
    KPW_ADD(KP_W_CYC_TOTAL, KP_NOW() - kc0);
    __builtin_amdgcn_wave_barrier();
    code = packed & 0xff;
    msg = packed >> 8;
    mode = code == ZD_ERROR ? (int32_t)ZSM_BAD : (int32_t)f.r_mode;
    stop = code == ZD_TRUNC ? (uint32_t)jb.in_len * 8u : f.stop_bits - mis * 8u;
    rbit = f.r_bit - mis * 8u;
    produced = f.pos;
    // window for the next call (the newest RING bytes, oldest first): saved
    // by the whole workgroup after the call (zs_stream_kernel)
    if (lane == 0) {
      L.wide.save = 1;
      L.wide.save_pos = f.pos;
    }
    const bool dyn = (mode == ZSM_SYMS || mode == ZSM_LIT || mode == ZSM_MATCH) && f.r_btype == 2;
    if (lane == 0) L.wide.tab_out = dyn ? f.tab_bits : 0u;  // saved with the window after the call
    if (dyn)
      for (uint32_t k = lane; k < f.r_nlen + f.r_ndist; k += WAVE) st->lens[k] = (uint8_t)s_lens[k];
    if (lane == 0) {
      st->len = f.r_len;
      st->dist = f.r_dist;
      st->btype = f.r_btype;
      st->nlen = f.r_nlen;
      st->ndist = f.r_ndist;
      st->last = (f.blast && f.r_mode != ZSM_TYPE) ? 1u : 0u;  // at a block header the previous block was not final
    }
  }
  if (lane == 0) {
    st->mode = mode;
    st->rbit = rbit;
    st->code = code;
    st->msg = msg;
    st->stop_bits = stop;
    st->produced = produced;
    st->acc_a = 0;
    st->acc_b = 0;
  }
}

// One call by the whole workgroup (head: the wrapper header parse, read only
// in HEAD mode): wave 0 runs the call's exact state machine, the other waves
// join its workgroup-wide symbol windows (WideLDS)
template <bool D64>
__device__ __forceinline__ void zs_stream_wg(ZsStreamDev *__restrict__ st, const ZsJobDev *__restrict__ job,
                                             const ZsHeadDev *__restrict__ head, StreamLDS<D64> &L) {
  constexpr uint32_t RING = StreamLDS<D64>::RING;
  constexpr uint32_t WOFF = 65536u - RING;
  const uint32_t t = threadIdx.x;
  {  // the handle's history window into the ring, by every wave (a resumed call)
    const int32_t mode0 = st->mode;
    if (mode0 >= ZSM_TYPE && mode0 <= ZSM_STORED && st->total_out)
      for (uint32_t k = t * 16u; k < RING; k += WW_T * 16u)
        *reinterpret_cast<uint4 *>(&L.ring[k]) = *reinterpret_cast<const uint4 *>(&st->window[WOFF + k]);
    // and the tables of a dynamic block in progress (built by an earlier call)
    const uint32_t tb = ((mode0 == ZSM_SYMS || mode0 == ZSM_LIT || mode0 == ZSM_MATCH) && st->btype == 2) ? st->tab_bits : 0u;
    if (tb >> 16)
      for (uint32_t k = t; k < TABLE_ENTRIES; k += WW_T) L.tab[k] = st->tab[k];
    if (t == 0) {
      L.wide.tab_in = tb;
      L.wide.tab_out = 0;
    }
  }
  __syncthreads();
  if (t >= WAVE) {
    for (;;) {
      __syncthreads();  // a window or a stored copy posted by wave 0, or the end of the call
      const uint32_t op = L.wide.op;
      if (op == WW_EXIT) break;
      if (op == WW_COPY) ww_copy<D64>(L);
      else ww_run<D64>(L);
    }
  } else {
    zs_stream_call<D64>(st, job, head, L);
    if (t == 0) L.wide.op = WW_EXIT;
    __syncthreads();
  }
  if (L.wide.save) {  // the newest RING bytes, oldest first, for the next call
    const uint32_t p0 = L.wide.save_pos;
    for (uint32_t k = 4u * t; k < RING; k += 4u * WW_T) {
      const uint32_t v = (uint32_t)L.ring[(p0 + k) & (RING - 1u)] | ((uint32_t)L.ring[(p0 + k + 1u) & (RING - 1u)] << 8) |
                         ((uint32_t)L.ring[(p0 + k + 2u) & (RING - 1u)] << 16) |
                         ((uint32_t)L.ring[(p0 + k + 3u) & (RING - 1u)] << 24);
      *reinterpret_cast<uint32_t *>(&st->window[WOFF + k]) = v;
    }
  }
  {  // the current dynamic block's tables for the next call
    const uint32_t tb = L.wide.tab_out;
    if (tb >> 16)
      for (uint32_t k = t; k < TABLE_ENTRIES; k += WW_T) st->tab[k] = L.tab[k];
    if (t == 0) st->tab_bits = tb;
  }
}

template <bool D64>
__global__ void __launch_bounds__(WW_T) zs_stream_kernel(ZsStreamDev *const *__restrict__ sts, const ZsJobDev *__restrict__ jobs,
                                                          const ZsHeadDev *__restrict__ heads) {
  // one workgroup per call of the batch (calls of different handles; see zs_launch_stream)
  __shared__ StreamLDS<D64> L;
  zs_stream_wg<D64>(sts[blockIdx.x], jobs + blockIdx.x, heads + blockIdx.x, L);
}

template __global__ void zs_stream_kernel<false>(ZsStreamDev *const *, const ZsJobDev *, const ZsHeadDev *);
template __global__ void zs_stream_kernel<true>(ZsStreamDev *const *, const ZsJobDev *, const ZsHeadDev *);

// A handle's device state after inflateInit / inflateReset (its first call sets
// it up: no copy or synchronisation of its own at init): zlib's mode for the
// wrapper, the window bits, everything else zero.
__device__ void stream_state_init(ZsStreamDev *st, const ZsJobDev &jb) {
  st->mode = jb.wrap == ZW_RAW ? ZSM_TYPE : ZSM_HEAD;
  st->rbit = st->last = st->btype = st->nlen = st->ndist = st->len = st->dist = 0;
  st->wbits = (uint32_t)jb.wbits;
  st->is_gzip = -1;
  st->total_out = 0;
  st->ck_a = st->ck_b = 0;
  st->code = st->msg = 0;
  st->stop_bits = st->produced = st->check = st->tab_bits = 0;
  st->acc_a = st->acc_b = 0;
}

// The calls' inputs from host-mapped staging into their device buffers, and
// the carried restart bit (a workgroup column per call; before the decode).
#define SIO_THREADS 256
__global__ void __launch_bounds__(SIO_THREADS) zs_stream_in_kernel(ZsStreamDev *const *__restrict__ sts,
                                                                   const ZsJobDev *__restrict__ jobs,
                                                                   const ZsStreamIo *__restrict__ io) {
  const ZsStreamIo c = io[blockIdx.y];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (c.fresh) stream_state_init(sts[blockIdx.y], jobs[blockIdx.y]);
    sts[blockIdx.y]->rbit = c.rbit;
  }
  if (!c.hin) return;
  const uint64_t n = jobs[blockIdx.y].in_len;
  uint8_t *dst = const_cast<uint8_t *>(jobs[blockIdx.y].in);
  const uint64_t nw = n / 16u;
  for (uint64_t k = (uint64_t)blockIdx.x * SIO_THREADS + threadIdx.x; k < nw; k += (uint64_t)gridDim.x * SIO_THREADS)
    reinterpret_cast<uint4 *>(dst)[k] = reinterpret_cast<const uint4 *>(c.hin)[k];
  if (blockIdx.x == 0 && threadIdx.x < (n & 15u)) dst[nw * 16u + threadIdx.x] = c.hin[nw * 16u + threadIdx.x];
}

// The call's output to its host-mapped staging, and its check contributions
// (zs_check.h accumulators); a workgroup per (piece, call).
#define SCHECK_THREADS 256
__global__ void __launch_bounds__(SCHECK_THREADS) zs_stream_check_kernel(ZsStreamDev *const *__restrict__ sts,
                                                                         const ZsJobDev *__restrict__ jobs,
                                                                         const ZsStreamIo *__restrict__ io) {
  ZsStreamDev *__restrict__ st = sts[blockIdx.y];
  const ZsJobDev *__restrict__ job = jobs + blockIdx.y;
  __shared__ uint32_t s_tab[4][256];
  __shared__ uint64_t s_red[16];
  const uint32_t t = threadIdx.x;
  const int gz = st->is_gzip;
  const uint64_t n = st->produced;
  if (n == 0 || st->mode == ZSM_HEAD) return;
  const uint8_t *p = job->out;
  const uint64_t piece = max<uint64_t>(4096u, ((n + gridDim.x - 1) / gridDim.x + 1023u) & ~1023ull);
  const uint64_t p0 = (uint64_t)blockIdx.x * piece;
  if (p0 >= n) return;
  const uint64_t plen = min(piece, n - p0);
  if (uint8_t *h = io[blockIdx.y].hout) {  // p0 is a multiple of 1024: 16-byte words
    const uint64_t nw = plen / 16u;
    for (uint64_t k = t; k < nw; k += SCHECK_THREADS)
      reinterpret_cast<uint4 *>(h + p0)[k] = reinterpret_cast<const uint4 *>(p + p0)[k];
    if (t < (plen & 15u)) h[p0 + nw * 16u + t] = p[p0 + nw * 16u + t];
  }
  if (gz < 0) return;
  const uint64_t per = ((plen + SCHECK_THREADS - 1) / SCHECK_THREADS + 3u) & ~3ull;
  const uint64_t lo = p0 + min(plen, per * t), hi = p0 + min(plen, per * (t + 1));
  if (gz == 1) {
    zs_crc_tables(s_tab);
    const uint32_t v = zs_block_xor(zs_crc_piece(p, lo, hi, n, s_tab), reinterpret_cast<uint32_t *>(s_red));
    if (t == 0 && v) atomicXor(reinterpret_cast<unsigned long long *>(&st->acc_a), (unsigned long long)v);
  } else {
    uint32_t A = 0, B = 0;
    if (hi > lo) zs_adler_piece(p, lo, hi, n, &A, &B);
    const uint64_t sa = zs_block_sum(A, s_red);
    const uint64_t sb = zs_block_sum(B, s_red);
    if (t == 0) {
      atomicAdd(reinterpret_cast<unsigned long long *>(&st->acc_a), (unsigned long long)sa);
      atomicAdd(reinterpret_cast<unsigned long long *>(&st->acc_b), (unsigned long long)sb);
    }
  }
}

// Running check, then the CHECK / LENGTH trailer states (src/inflate.c:1194-1232).
__device__ void stream_finish(ZsStreamDev &s, const ZsJobDev *__restrict__ job) {
  if (s.mode == ZSM_HEAD || s.mode == ZSM_DICT || s.code == ZD_NEED_DICT) return;
  const int gz = s.is_gzip;
  const uint64_t n = s.produced;
  if (n && gz == 1) {
    s.ck_a = zs_gf2_mul(zs_x8n(n), s.ck_a) ^ (uint32_t)s.acc_a;
  } else if (n && gz == 0) {
    const uint64_t a = s.ck_a, b = s.ck_b;
    s.ck_b = (uint32_t)((b + (n % ZS_ADLER_MOD) * a + s.acc_b % ZS_ADLER_MOD) % ZS_ADLER_MOD);
    s.ck_a = (uint32_t)((a + s.acc_a % ZS_ADLER_MOD) % ZS_ADLER_MOD);
  }
  s.total_out += n;
  uint32_t check = 0;
  if (gz == 1) check = ~(s.ck_a ^ zs_gf2_mul(zs_x8n(s.total_out), 0xffffffffu));
  else if (gz == 0) check = (s.ck_b << 16) | s.ck_a;
  if (gz >= 0) s.check = check;
  const uint8_t *in = job->in;
  const uint32_t len = (uint32_t)job->in_len;
  if (s.mode == ZSM_CHECK) {
    const uint32_t P = s.rbit >> 3;
    if (gz < 0) {
      s.mode = ZSM_DONE;
      s.code = ZD_END;
      s.stop_bits = s.rbit;
    } else if (P + 4 > len) {
      s.code = ZD_TRUNC;
      s.stop_bits = len * 8u;
    } else {
      uint32_t tr = (uint32_t)in[P] | ((uint32_t)in[P + 1] << 8) | ((uint32_t)in[P + 2] << 16) | ((uint32_t)in[P + 3] << 24);
      if (gz == 0) tr = (tr >> 24) | ((tr >> 8) & 0xff00u) | ((tr & 0xff00u) << 8) | (tr << 24);
      s.stop_bits = (P + 4) * 8u;
      s.rbit = (P + 4) * 8u;
      if (tr != check) {
        s.mode = ZSM_BAD;
        s.code = ZD_ERROR;
        s.msg = ZM_DATA_CHECK;
      } else if (gz == 1) {
        s.mode = ZSM_LENGTH;
      } else {
        s.mode = ZSM_DONE;
        s.code = ZD_END;
      }
    }
  }
  if (s.mode == ZSM_LENGTH) {
    const uint32_t P = s.rbit >> 3;
    if (P + 4 > len) {
      s.code = ZD_TRUNC;
      s.stop_bits = len * 8u;
    } else {
      const uint32_t isz = (uint32_t)in[P] | ((uint32_t)in[P + 1] << 8) | ((uint32_t)in[P + 2] << 16) | ((uint32_t)in[P + 3] << 24);
      s.stop_bits = (P + 4) * 8u;
      if (isz != (uint32_t)(s.total_out & 0xffffffffu)) {
        s.mode = ZSM_BAD;
        s.code = ZD_ERROR;
        s.msg = ZM_LENGTH_CHECK;
      } else {
        s.mode = ZSM_DONE;
        s.code = ZD_END;
      }
    }
  }
}

// The call's outcome, gathered for the host (one copy for the whole batch).
__global__ void zs_stream_finish_kernel(ZsStreamDev *const *__restrict__ sts, const ZsJobDev *__restrict__ jobs,
                                        ZsStreamRes *__restrict__ res) {
  if (threadIdx.x != 0) return;
  ZsStreamDev &s = *sts[blockIdx.x];
  stream_finish(s, jobs + blockIdx.x);
  ZsStreamRes r;
  r.mode = s.mode;
  r.rbit = s.rbit;
  r.code = s.code;
  r.msg = s.msg;
  r.stop_bits = s.stop_bits;
  r.produced = s.produced;
  r.check = s.check;
  r.is_gzip = s.is_gzip;
  res[blockIdx.x] = r;
}

// One batch of calls, one per handle (the library funnels concurrent calls of
// different handles into one launch): [wrapper headers] -> resumable decode
// (a workgroup per call) -> checks -> trailers -> outcome gather.
extern "C" void zs_launch_stream(int d64, int run_header, ZsStreamDev *const *d_sts, const ZsJobDev *d_jobs,
                                 ZsHeadDev *d_heads, const ZsStreamIo *io, uint32_t n, uint64_t max_in_len,
                                 uint64_t max_out_cap, ZsStreamRes *d_res, hipStream_t stream) {
  const uint32_t in_pieces = (uint32_t)std::min<uint64_t>(256, std::max<uint64_t>(1, (max_in_len + 16383) / 16384));
  hipLaunchKernelGGL(zs_stream_in_kernel, dim3(in_pieces, n), dim3(SIO_THREADS), 0, stream, d_sts, d_jobs, io);
  if (run_header) hipLaunchKernelGGL(zs_header_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_jobs, d_heads, n);
  if (d64)
    hipLaunchKernelGGL(zs_stream_kernel<true>, dim3(n), dim3(WW_T), 0, stream, d_sts, d_jobs, d_heads);
  else
    hipLaunchKernelGGL(zs_stream_kernel<false>, dim3(n), dim3(WW_T), 0, stream, d_sts, d_jobs, d_heads);
  const uint32_t pieces = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(1, (max_out_cap + 16383) / 16384));
  hipLaunchKernelGGL(zs_stream_check_kernel, dim3(pieces, n), dim3(SCHECK_THREADS), 0, stream, d_sts, d_jobs, io);
  hipLaunchKernelGGL(zs_stream_finish_kernel, dim3(n), dim3(64), 0, stream, d_sts, d_jobs, d_res);
}

// ---------------------------------------------------------------------------
// Persistent stream worker: a workgroup per mailbox (ZsMbox, host-coherent
// pinned memory) takes its handle's calls one at a time and completes each on
// its own -- input pull, the call (zs_stream_wg), output push and check, the
// trailer states, the outcome -- so a call returns when ITS workgroup is done,
// not when the slowest call of a launch is (the batch path: ~2x the mean call
// at 64 handles).  Wave 0 polls its mailbox with vector loads at system scope
// (never the scalar cache), sleeping between polls.  A workgroup leaves when
// no call was posted to any mailbox for idle_t ticks (s_memrealtime, 100 MHz),
// and then raises ctl[2] so that every other one leaves after its current
// call; also when the host sets ctl[0], or after its current call once the
// launch is older than life_t: the grid always drains; the host relaunches on
// demand.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pk_ld(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void pk_st(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool D64>
__global__ void __launch_bounds__(WW_T) zs_stream_pk_kernel(ZsMbox *__restrict__ mbs, const uint32_t *__restrict__ ctl,
                                                             uint32_t zero, uint64_t idle_t, uint64_t life_t) {
  __shared__ StreamLDS<D64> L;
  __shared__ __attribute__((aligned(16))) uint32_t s_mb[ZS_MBOX_CALL_WORDS];
  __shared__ uint32_t s_cmd, s_n, s_mode;
  __shared__ int32_t s_gz;
  __shared__ uint32_t s_tab[4][256];
  __shared__ uint64_t s_red[16];
  const uint32_t t = threadIdx.x, lane = t & 63u;
  // lane-dependent addresses (zero == 0): vector memory, never the scalar cache
  uint32_t *mbw = reinterpret_cast<uint32_t *>(mbs + blockIdx.x) + zero * t;
  const uint32_t *ctw = ctl + zero * t;
  uint32_t done = pk_ld(mbw + 1);  // seq_out: the last call of this mailbox already finished
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t tdone = t0;
  for (;;) {
    if (t < WAVE) {
      uint64_t last = __builtin_amdgcn_s_memrealtime();
      uint32_t post = pk_ld(ctw + 1), cmd = 0, nap = 1;
      for (;;) {
        // past its life (or told to stop) the launch leaves even with calls
        // posted -- they stay posted for the relaunch -- so every workgroup
        // goes within one call and no handle waits on the others' streams
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (now - t0 > life_t || pk_ld(ctw) != 0u || pk_ld(ctw + 2) != 0u) break;
        const uint32_t q = pk_ld(mbw);
        if (q != done) {
          cmd = q;
          break;
        }
        const uint32_t p2 = pk_ld(ctw + 1);
        if (p2 != post) {
          post = p2;
          last = now;
        }
        if (now - last > idle_t) {
          // leaving idle closes the whole launch: the other workgroups leave
          // after their current call, so a handle whose workgroup is gone
          // waits for one call at most, never for the launch's life (the host
          // relaunches once the grid has drained and clears ctl[2])
          pk_st(const_cast<uint32_t *>(ctw) + 2, 1u);
          break;
        }
        for (uint32_t k = 0; k < nap; k++) __builtin_amdgcn_s_sleep(32);
        nap = min(nap * 2u, 8u);  // (4, i.e. polls twice as often: the caller's wait per stored call 46 -> 60 us, measured and dropped)
      }
      if (cmd) {  // the call's fields after its seq_in (system-scope acquire)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        for (uint32_t k = lane; k < ZS_MBOX_CALL_WORDS; k += WAVE) s_mb[k] = pk_ld(mbw + 4u + k);
      }
      if (lane == 0) s_cmd = cmd;
    }
    __syncthreads();
    const uint32_t cmd = s_cmd;
    if (cmd == 0) break;
    const uint64_t tc0 = __builtin_amdgcn_s_memrealtime();
    ZsStreamDev *st = *reinterpret_cast<ZsStreamDev *const *>(&s_mb[0]);
    const ZsStreamIo io = *reinterpret_cast<const ZsStreamIo *>(&s_mb[4]);
    const ZsJobDev *job = reinterpret_cast<const ZsJobDev *>(&s_mb[12]);
    {  // input: host-mapped staging -> the job's device buffer; the carried restart bit
      const uint64_t n = job->in_len;
      uint8_t *dst = const_cast<uint8_t *>(job->in);
      if (io.hin) {  // four loads over the bus in flight per thread before their stores
        const uint64_t nw = n / 16u;
        const uint4 *hs = reinterpret_cast<const uint4 *>(io.hin);
        for (uint64_t k0 = t; k0 < nw; k0 += 4u * WW_T) {
          uint4 v[4];
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (k0 + j * WW_T < nw) v[j] = hs[k0 + j * WW_T];
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (k0 + j * WW_T < nw) reinterpret_cast<uint4 *>(dst)[k0 + j * WW_T] = v[j];
        }
        if (t < (n & 15u)) dst[nw * 16u + t] = io.hin[nw * 16u + t];
      }
      if (t == 0) {
        if (io.fresh) stream_state_init(st, *job);
        st->rbit = io.rbit;
      }
    }
    // the copies (stores complete at the barrier) before the call reads them:
    // an agent-scope acquire drops stale L1 lines (the handle's state from any
    // other workgroup, launch or batch kernel came in with the system-scope
    // acquire after seq_in, which also invalidates L2)
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    zs_stream_wg<D64>(st, job, nullptr, L);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (t == 0) {
      s_n = st->produced;
      s_mode = (uint32_t)st->mode;
      s_gz = st->is_gzip;
    }
    __syncthreads();
    const uint64_t n = s_n;
    if (n && s_mode != (uint32_t)ZSM_HEAD) {  // zs_stream_check_kernel for one call, one piece
      const uint8_t *p = job->out;
      if (uint8_t *h = io.hout) {  // (the same: the device loads of up to four stores over the bus first)
        const uint64_t nw = n / 16u;
        const uint4 *ps = reinterpret_cast<const uint4 *>(p);
        for (uint64_t k0 = t; k0 < nw; k0 += 4u * WW_T) {
          uint4 v[4];
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (k0 + j * WW_T < nw) v[j] = ps[k0 + j * WW_T];
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (k0 + j * WW_T < nw) reinterpret_cast<uint4 *>(h)[k0 + j * WW_T] = v[j];
        }
        if (t < (n & 15u)) h[nw * 16u + t] = p[nw * 16u + t];
      }
      const int gz = s_gz;
      const uint64_t per = ((n + WW_T - 1) / WW_T + 3u) & ~3ull;
      const uint64_t lo = min(n, per * t), hi = min(n, per * (t + 1));
      if (gz == 1) {
        zs_crc_tables(s_tab);
        const uint32_t v = zs_block_xor(zs_crc_piece(p, lo, hi, n, s_tab), reinterpret_cast<uint32_t *>(s_red));
        if (t == 0) st->acc_a = v;
      } else if (gz == 0) {
        uint32_t A = 0, B = 0;
        if (hi > lo) zs_adler_piece(p, lo, hi, n, &A, &B);
        const uint64_t sa = zs_block_sum(A, s_red);
        const uint64_t sb = zs_block_sum(B, s_red);
        if (t == 0) {
          st->acc_a = sa;
          st->acc_b = sb;
        }
      }
    }
    if (t == 0) {  // the trailer states and the outcome (zs_stream_finish_kernel)
      stream_finish(*st, job);
      const uint32_t r[8] = {(uint32_t)st->mode, st->rbit, (uint32_t)st->code, (uint32_t)st->msg,
                             st->stop_bits, (uint32_t)st->produced, st->check, (uint32_t)st->is_gzip};
#pragma unroll
      for (int k = 0; k < 8; k++) pk_st(mbw + 32u + k, r[k]);
      pk_st(mbw + 41u, (uint32_t)(tc0 - tdone));  // idle since the last call of this mailbox
    }
    // every wave's output words and state stores complete at the barrier; one
    // system-scope release writes the L2 back before seq_out
    __syncthreads();
    if (t == 0) {
      tdone = __builtin_amdgcn_s_memrealtime();
      pk_st(mbw + 40u, (uint32_t)(tdone - tc0));
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      pk_st(mbw + 1, cmd);
    }
    done = cmd;
  }
}

template __global__ void zs_stream_pk_kernel<false>(ZsMbox *, const uint32_t *, uint32_t, uint64_t, uint64_t);

extern "C" void zs_launch_stream_pk(ZsMbox *d_mb, uint32_t nw, const uint32_t *d_ctl, uint64_t idle_t, uint64_t life_t,
                                    hipStream_t stream) {
  hipLaunchKernelGGL(zs_stream_pk_kernel<false>, dim3(nw), dim3(WW_T), 0, stream, d_mb, d_ctl, 0u, idle_t, life_t);
}

// ---------------------------------------------------------------------------
// Checks: CRC-32 (gzip) / Adler-32 (zlib) over each job's output, segment
// parallel with an exact combine (UPDATE_CHECK, src/inflate.c:425-429).
// ---------------------------------------------------------------------------
// One workgroup per (job, piece): a piece of P = max(64 KiB, n / gridDim.y)
// bytes (4-byte multiple) adds its contribution to the job's accumulators
// (zs_check.h), so a 64 MiB output is checked by hundreds of workgroups.
#define CHECK_THREADS 256
__global__ void __launch_bounds__(CHECK_THREADS) zs_check_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                                                 const ZsDecDev *__restrict__ decs, uint64_t *__restrict__ checks) {
  __shared__ uint32_t s_tab[4][256];
  __shared__ ZsCkTabs s_ck;
  __shared__ uint64_t s_red[16];
  const uint32_t j = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const ZsHeadDev hd = heads[j];
  const ZsDecDev dc = decs[j];
  // raw streams are checked only on request (ZIP entries carry a CRC-32)
  const int kind = hd.is_gzip >= 0 ? hd.is_gzip : ((jobs[j].flags & ZS_JF_CRC32) ? 1 : -1);
  if (hd.code != ZD_END || kind < 0 || dc.code == ZD_SKIP) return;
  const uint8_t *p = jobs[j].out;
  const uint64_t n = dc.total_out;
  const uint64_t piece = max<uint64_t>(65536u, ((n + gridDim.y - 1) / gridDim.y + ZS_CK_STEP - 1) & ~(uint64_t)(ZS_CK_STEP - 1));
  const uint64_t p0 = (uint64_t)blockIdx.y * piece;
  if (p0 >= n) return;
  const uint64_t plen = min(piece, n - p0);
  if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0) {  // coalesced 4 KiB steps (zs_check.h)
    zs_ck_tables(s_ck);
    if (kind == 1) {
      const uint32_t v = zs_crc_block(p, p0, p0 + plen, n, s_ck, reinterpret_cast<uint32_t *>(s_red));
      if (t == 0 && v) atomicXor(reinterpret_cast<unsigned long long *>(&checks[2 * j]), (unsigned long long)v);
    } else {
      uint64_t sa, sb;
      zs_adler_block(p, p0, p0 + plen, n, s_red, &sa, &sb);
      if (t == 0) {
        atomicAdd(reinterpret_cast<unsigned long long *>(&checks[2 * j]), (unsigned long long)sa);
        atomicAdd(reinterpret_cast<unsigned long long *>(&checks[2 * j + 1]), (unsigned long long)sb);
      }
    }
    return;
  }
  const uint64_t per = ((plen + CHECK_THREADS - 1) / CHECK_THREADS + 3u) & ~3ull;
  const uint64_t lo = p0 + min(plen, per * t), hi = p0 + min(plen, per * (t + 1));
  if (kind == 1) {
    zs_crc_tables(s_tab);
    const uint32_t v = zs_block_xor(zs_crc_piece(p, lo, hi, n, s_tab), reinterpret_cast<uint32_t *>(s_red));
    if (t == 0 && v) atomicXor(reinterpret_cast<unsigned long long *>(&checks[2 * j]), (unsigned long long)v);
  } else {
    uint32_t A = 0, B = 0;
    if (hi > lo) zs_adler_piece(p, lo, hi, n, &A, &B);
    const uint64_t sa = zs_block_sum(A, s_red);
    const uint64_t sb = zs_block_sum(B, s_red);
    if (t == 0) {
      atomicAdd(reinterpret_cast<unsigned long long *>(&checks[2 * j]), (unsigned long long)sa);
      atomicAdd(reinterpret_cast<unsigned long long *>(&checks[2 * j + 1]), (unsigned long long)sb);
    }
  }
}

// ---------------------------------------------------------------------------
// Finalize: zlib's CHECK/LENGTH states and inf_leave totals
// (src/inflate.c:1194-1274).
// ---------------------------------------------------------------------------
__global__ void zs_finalize_kernel(const ZsJobDev *__restrict__ jobs, const ZsHeadDev *__restrict__ heads,
                                   const ZsDecDev *__restrict__ decs, const uint64_t *__restrict__ checks,
                                   ZsResultDev *__restrict__ res, uint32_t njobs) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  const ZsJobDev jb = jobs[j];
  const ZsHeadDev hd = heads[j];
  ZsResultDev r;
  r.pad = 0;
  r.msg = ZM_NONE;
  if (hd.code == ZD_SKIP) {
    r.ret = hd.ret;
    r.msg = hd.msg;
    r.total_in = hd.total_in;
    r.total_out = 0;
    r.adler = hd.adler;
    res[j] = r;
    return;
  }
  if (hd.code == ZD_NEED_DICT) {
    r.ret = ZS_NEED_DICT;
    r.total_in = 0;
    r.total_out = 0;
    r.adler = hd.adler;
    res[j] = r;
    return;
  }
  const ZsDecDev dc = decs[j];
  const bool raw = hd.is_gzip < 0;
  r.total_out = dc.total_out;
  r.adler = raw ? ((jb.flags & ZS_JF_CRC32) ? zs_crc_final((uint32_t)checks[2 * j], dc.total_out) : 0u)
                : hd.is_gzip == 1 ? zs_crc_final((uint32_t)checks[2 * j], dc.total_out)
                                  : zs_adler_final(checks[2 * j], checks[2 * j + 1], dc.total_out);
  // (an if-chain, not a switch: hipcc 7.2 dropped the msg copy of the default
  // arm of the equivalent switch for codes > ZD_FULL)
  const int code = dc.code;
  const uint64_t t = (dc.end_bits + 7) >> 3;  // bytes pulled (slow path) / not returned (fast path)
  r.msg = (code == ZD_END || code == ZD_TRUNC || code == ZD_FULL) ? (int32_t)ZM_NONE : dc.msg;
  r.ret = ZS_DATA_ERROR;
  r.total_in = t;
  if (code == ZD_TRUNC) {
    r.ret = ZS_BUF_ERROR;
    r.total_in = jb.in_len;
  } else if (code == ZD_FULL) {
    r.ret = ZS_BUF_ERROR;
  } else if (code == ZD_END) {
    if (raw) {
      r.ret = ZS_STREAM_END;
    } else if (t + 4 > jb.in_len) {  // CHECK: NEEDBITS(32) runs out of input
      r.ret = ZS_BUF_ERROR;
      r.total_in = jb.in_len;
    } else {
      const uint8_t *q = jb.in + t;
      uint32_t tr = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
      if (hd.is_gzip == 0) tr = (tr >> 24) | ((tr >> 8) & 0xff00u) | ((tr & 0xff00u) << 8) | (tr << 24);
      r.total_in = t + 4;
      if (tr != r.adler) {
        r.msg = ZM_DATA_CHECK;
      } else if (hd.is_gzip != 1) {
        r.ret = ZS_STREAM_END;
      } else if (t + 8 > jb.in_len) {  // LENGTH: NEEDBITS(32) runs out of input
        r.ret = ZS_BUF_ERROR;
        r.total_in = jb.in_len;
      } else {
        const uint32_t isz = (uint32_t)q[4] | ((uint32_t)q[5] << 8) | ((uint32_t)q[6] << 16) | ((uint32_t)q[7] << 24);
        r.total_in = t + 8;
        if (isz != (uint32_t)(dc.total_out & 0xffffffffu))
          r.msg = ZM_LENGTH_CHECK;
        else
          r.ret = ZS_STREAM_END;
      }
    }
  }
  res[j] = r;
}

// ---------------------------------------------------------------------------
// launch helpers (host side; every launch on `stream`, no host syncs)
// ---------------------------------------------------------------------------
extern "C" void zs_launch_header(const ZsJobDev *d_jobs, ZsHeadDev *d_heads, uint32_t njobs, hipStream_t stream) {
  const uint32_t tb = 64;
  hipLaunchKernelGGL(zs_header_kernel, dim3((njobs + tb - 1) / tb), dim3(tb), 0, stream, d_jobs, d_heads, njobs);
}

// serial (wave-per-stream) decode of the jobs listed in d_ids; run_only filters
extern "C" void zs_launch_decode(int d64, const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, const uint32_t *d_ids,
                                 uint32_t n, ZsDecDev *d_decs, const uint32_t *run_only, hipStream_t stream) {
  if (!n) return;
  if (d64)
    hipLaunchKernelGGL(zs_decode_kernel<true>, dim3(n), dim3(64), 0, stream, d_jobs, d_heads, d_ids, d_decs, run_only);
  else
    hipLaunchKernelGGL(zs_decode_kernel<false>, dim3(n), dim3(64), 0, stream, d_jobs, d_heads, d_ids, d_decs, run_only);
}

// max_out: the largest out_cap of the batch (sizes the piece grid)
extern "C" void zs_launch_finish(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, const ZsDecDev *d_decs,
                                 uint64_t *d_checks, ZsResultDev *d_res, uint32_t njobs, uint64_t max_out, hipStream_t stream) {
  const uint32_t tb = 64;
  const uint32_t pieces = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(1, (max_out + 262143) / 262144));
  (void)hipMemsetAsync(d_checks, 0, 2 * sizeof(uint64_t) * njobs, stream);
  hipLaunchKernelGGL(zs_check_kernel, dim3(njobs, pieces), dim3(CHECK_THREADS), 0, stream, d_jobs, d_heads, d_decs, d_checks);
  hipLaunchKernelGGL(zs_finalize_kernel, dim3((njobs + tb - 1) / tb), dim3(tb), 0, stream, d_jobs, d_heads, d_decs, d_checks,
                     d_res, njobs);
}

// serial-decoder counters of the profiling build (zs_kprof_read's 64..95)
extern "C" int zs_kprof_read_w(uint64_t *out32, int reset) {
#if KP_ON
  if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_kprof_w), 32 * sizeof(uint64_t)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_kprof_w), z, sizeof z) != hipSuccess) return -1;
  }
  return 32;
#else
  (void)out32;
  (void)reset;
  return 0;
#endif
}
