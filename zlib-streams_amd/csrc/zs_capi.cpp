// zs_capi.cpp -- host side of libzstreams_mi355x.so.
//
// Orchestrates the HIP kernels of inflate_kernels.hip behind three C-ABI
// surfaces (see include/zstreams_mi355x.h):
//   * zs_inflate_batch    -- many whole streams per launch sequence;
//   * the reference's handle ABI (src/wasm/*_stream_wasm.c, wasm_stream_common.c);
//   * the zlib inflate ABI (inflateInit2_/inflate/inflateEnd, src/inflate.c).
// The stream surfaces run every call as one exact, resumable inflate() on the
// GPU (zlib's per-call consumed / produced / ret, see "Stream surfaces").
// Every byte is produced by the GPU; a missing or failing device is a hard error.
#include <hip/hip_runtime.h>
#include <sys/prctl.h>
#include <zlib.h>

#include "zs_check.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zstreams_mi355x.h"
#include "zs_common.h"
#include "src_hash.h"  // build/src_hash.h (Makefile, srchash.py)

extern "C" void zs_launch_header(const ZsJobDev *d_jobs, ZsHeadDev *d_heads, uint32_t njobs, hipStream_t stream);
extern "C" void zs_launch_decode(int d64, const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, const uint32_t *d_ids,
                                 uint32_t n, ZsDecDev *d_decs, const uint32_t *run_only, hipStream_t stream);
extern "C" void zs_launch_finish(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, const ZsDecDev *d_decs,
                                 uint64_t *d_checks, ZsResultDev *d_res, uint32_t njobs, uint64_t max_out,
                                 hipStream_t stream);
extern "C" void zs_launch_stream(int d64, int run_header, ZsStreamDev *const *d_sts, const ZsJobDev *d_jobs,
                                 ZsHeadDev *d_heads, const ZsStreamIo *io, uint32_t n, uint64_t max_in_len,
                                 uint64_t max_out_cap, ZsStreamRes *d_res, hipStream_t stream);
extern "C" void zs_launch_stream_pk(ZsMbox *d_mb, uint32_t nw, const uint32_t *d_ctl, uint64_t idle_t, uint64_t life_t,
                                    hipStream_t stream);
extern "C" uint32_t zs_lane_resident_waves(void);
extern "C" void zs_launch_fixed_tables(uint32_t *fixed, int d64, hipStream_t st);
extern "C" void zs_launch_fixed_compact(uint32_t *fixed, hipStream_t st);
extern "C" void zs_launch_deflate(ZsDJobDev *d_jobs, uint32_t njobs, ZsDSegDev *d_segs, uint32_t nseg, uint16_t *d_dist16,
                                  uint8_t *d_len8, uint32_t *d_bm, uint32_t *d_aux, uint32_t *d_obuf, uint8_t *d_stage,
                                  uint16_t *d_lx16, int has_std, int has_d64, hipStream_t st, hipEvent_t *ev);
struct ZsZWorkDev {  // must match deflate_zlib.hip
  uint32_t job;
  uint32_t len;
  uint64_t start;
};
extern "C" int zs_launch_zdeflate(ZsDJobDev *d_jobs, uint32_t njobs, ZsDSegDev *d_segs, uint32_t nseg,
                                  const ZsZWorkDev *d_w1, uint32_t n1, const ZsZWorkDev *d_w1s, uint32_t n1s,
                                  const ZsZWorkDev *d_w2, uint32_t n2, const ZsZWorkDev *d_w3, uint32_t n3,
                                  uint16_t *d_prevd, uint32_t *d_ma, uint32_t *d_mb, uint32_t *d_bm, ZsZBlkDev *d_blks,
                                  uint32_t nblk_slots, const uint32_t *d_slot_job, uint32_t *d_aux, uint8_t *d_stage,
                                  uint32_t *d_flag, int has_slow, int has_fast, uint32_t max_regions, hipStream_t st,
                                  hipEvent_t *ev);
extern "C" void zs_launch_dz_trailer(ZsDJobDev *d_jobs, uint32_t njobs, uint8_t *d_stage, hipStream_t st);
extern "C" void zs_launch_stored_call(const uint8_t *d_src, const ZsPiece *d_pc, uint32_t np, uint64_t total,
                                      uint8_t *d_dst, uint64_t ck_lo, uint64_t ck_hi, uint32_t wrap, uint32_t *d_res,
                                      hipStream_t st);
extern "C" void zs_launch_chunked(const ZsJobDev *d_jobs, const ZsHeadDev *d_heads, ZsSegDev *d_segs, uint32_t nseg,
                                  ZsCJobDev *d_cjobs, uint32_t ncjobs, ZsChunkDev *d_units, uint32_t nunit_slots,
                                  uint16_t *d_scratch, uint32_t *d_tokens, ZsTokPool pool, uint32_t *d_tables,
                                  const uint32_t *d_fixed, uint8_t *d_windows, void *d_linkinfo, ZsDecDev *d_decs,
                                  uint32_t *d_fallback, int d64, int wave_units, void *d_plink, uint32_t plink_levels,
                                  uint16_t *d_lmaps, uint32_t lsegs, hipStream_t st, hipEvent_t *ev, uint32_t *d_vlist,
                                  int ctx, hipEvent_t ev_found);

namespace {

constexpr size_t TABLE_ENTRIES_HOST = 1448 + 724 + 176 + 192 + 16;  // must match TABLE_STRIDE (zs_device.h)
constexpr size_t FIXED_WORDS_HOST = 544 + 272;      // must match FIXED_WORDS (zs_device.h)
constexpr uint64_t MAX_RATIO = 1032;  // deflate's largest expansion: 258 bytes per 2 bits
// deflate64: code 285 carries 16 extra bits for up to 65538 bytes, so one 1-bit
// length code + 16 extra bits + a 1-bit distance code (18 bits) yield 65538 bytes
constexpr uint64_t MAX_RATIO_D64 = 65538ull * 8 / 18 + 1;

const char *const kMsgs[ZM_COUNT] = {
    nullptr,
    "incorrect header check",
    "unknown compression method",
    "invalid window size",
    "unknown header flags set",
    "header crc mismatch",
    "invalid block type",
    "invalid stored block lengths",
    "too many length or distance symbols",
    "invalid code lengths set",
    "invalid bit length repeat",
    "invalid code -- missing end-of-block",
    "invalid literal/lengths set",
    "invalid distances set",
    "invalid literal/length code",
    "invalid distance code",
    "invalid distance too far back",
    "incorrect data check",
    "incorrect length check",
};

thread_local std::string g_err;

void set_err(const std::string &s) { g_err = s; }

#define HIP_OK(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      set_err(std::string(#x) + ": " + hipGetErrorString(e_));                 \
      return ZS_ENODEV;                                                        \
    }                                                                          \
  } while (0)

// Device workspace, grown on demand and reused across calls.
struct Workspace {
  bool ready = false;
  int device = -1;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  size_t cap_jobs = 0;
  ZsJobDev *d_jobs = nullptr;
  ZsHeadDev *d_heads = nullptr;
  ZsDecDev *d_decs = nullptr;
  uint64_t *d_checks = nullptr;  // 2 per job: check accumulators (zs_check.h)
  ZsResultDev *d_res = nullptr;
  uint32_t *d_ids = nullptr;
  ZsJobDev *h_jobs = nullptr;     // pinned
  ZsResultDev *h_res = nullptr;   // pinned
  uint32_t *h_ids = nullptr;      // pinned
  size_t cap_in = 0, cap_out = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  uint32_t *d_fallback = nullptr;  // per job (cap_jobs)
  ZsCJobDev *d_cjobs = nullptr, *h_cjobs = nullptr;  // per job (cap_jobs)
  // chunked path: search segments and decode-unit slots
  size_t cap_segs = 0, cap_units = 0;
  ZsSegDev *d_segs = nullptr, *h_segs = nullptr;
  ZsChunkDev *d_chunks = nullptr, *h_chunks = nullptr;  // unit slots
  uint32_t *d_tables = nullptr;  // TABLE_STRIDE words per unit slot
  uint8_t *d_windows = nullptr;  // 32 KiB per unit slot (64 KiB for deflate64 units)
  size_t cap_windows = 0;
  uint8_t *d_lmaps = nullptr;  // segmented link: per chain LS_SEGS_MAX segment-end / start window maps (u16)
  size_t cap_lmaps = 0;
  uint64_t *d_linkinfo = nullptr;  // zs_link_kernel chain order: 16 B per unit slot
  uint8_t *d_plink = nullptr;      // parallel-prefix link maps (few long streams): 2 x slots x window entries
  size_t cap_plink = 0;
  size_t cap_scratch = 0;        // u16 entries (chain members at their output offsets)
  uint16_t *d_scratch = nullptr;
  size_t cap_tokens = 0;         // u32 parse tokens: primary regions + pool pages
  uint32_t *d_tokens = nullptr;
  uint32_t *d_ptab = nullptr;    // pool page table: ZS_TP_MAXPG per unit slot (cap_units)
  uint32_t *d_pool_next = nullptr;
  uint32_t *d_fixed = nullptr;
  // second chunked group (run_jobs): its stream, and the events that order it
  // against the launch stream (fork after the header kernel, group A's finder
  // done, join before the serial decoders)
  hipStream_t stream_b = nullptr;
  hipEvent_t ev_fork = nullptr, ev_found = nullptr, ev_join = nullptr;
  // timing (zs_profile): events on the launch stream
  bool prof = false;
  // boundaries: [0] batch start, [1] after header, [2] after find, [3] after
  // parse, [4] after expand, [5] after link, [6] after emit, [7] after the
  // serial decoders, [8] after finalize
  hipEvent_t ev[ZS_PROF_STAGES + 1] = {};
  double prof_stage[ZS_PROF_STAGES] = {};
  double prof_ms = 0.0, prof_batch_ms = 0.0;
  uint64_t prof_launches = 0;
  // last batch: chunked jobs, decode units planned, chunked jobs that fell back
  // to the serial decoder, serial jobs
  uint32_t stats[4] = {0, 0, 0, 0};
  // last launch's block-parallel path: parse mode / link levels of the std and
  // deflate64 groups, lane-parse resident waves, units per group, raw/zlib/gzip
  // groups run at once (zs_last_stats_ex)
  uint32_t path[8] = {UINT32_MAX, 0, UINT32_MAX, 0, 0, 0, 0, 0};
};

// chunked-path tuning (env: ZS_CHUNK_KB, ZS_NO_CHUNK, ZS_POOL_PER_KB)
uint32_t chunk_bytes() {
  static uint32_t v = [] {
    const char *e = std::getenv("ZS_CHUNK_KB");
    long kb = e ? std::atol(e) : 32;
    if (kb < 4) kb = 4;
    if (kb > 65536) kb = 65536;
    return (uint32_t)(kb * 1024);
  }();
  return v;
}
// Parse mode of a chunked group: a wave per unit when the group has few units
// for the GPU (about one per search segment), a lane per unit otherwise
// (env ZS_PARSE = lane | wave forces one; ZS_WAVE_SEGS moves the threshold).
// Link mode of a chunked group: the parallel-prefix link for a group of at
// most PLINK_JOBS streams with long chains (env ZS_PLINK = 0 disables it);
// returns the scan levels (0 = the serial per-stream link).
constexpr uint32_t PLINK_JOBS = 4;
uint32_t plink_levels(uint32_t njobs, uint32_t max_units, uint32_t flags) {
  static const bool off = [] {
    const char *e = std::getenv("ZS_PLINK");
    return e && e[0] == '0';
  }();
  if (off || (flags & ZS_F_LINK_SERIAL) || ZS_F_LINKSEG_GET(flags) || njobs == 0 || njobs > PLINK_JOBS ||
      max_units < 64)
    return 0;
  uint32_t lv = 0;
  while ((1u << lv) < max_units) lv++;
  return lv;
}
// Segmented link (zs_linkseg_kernel): a group of at most 64 streams on the
// serial link cuts each chain into segments so that about two workgroups per
// CU link; env ZS_LINKSEG = 0 (or ZS_F_LINK_SERIAL) keeps zs_link_kernel.
// (round 6: LS_TARGET_WG 512, 8 segments for 64 streams: C2 link 1.88 -> 1.77 ms)
constexpr uint32_t LS_SEGS_MAX_HOST = 8, LS_TARGET_WG = 512;
uint32_t link_segments(uint32_t njobs, uint32_t max_units, uint32_t flags) {
  // env ZS_LINKSEG: 0 = off, N = N segments per chain (at most LS_SEGS_MAX), unset = auto
  static const int force = [] {
    const char *e = std::getenv("ZS_LINKSEG");
    return (e && *e) ? atoi(e) : -1;
  }();
  if ((flags & ZS_F_LINK_SERIAL) || njobs == 0) return 1;
  const uint32_t fseg = ZS_F_LINKSEG_GET(flags);  // per call: forced segments (tests), any chain length
  if (fseg) return std::min<uint32_t>(LS_SEGS_MAX_HOST, fseg);
  if (force == 0 || njobs > 64 || max_units < 64) return 1;
  if (force > 0) return std::min<uint32_t>(LS_SEGS_MAX_HOST, (uint32_t)force);
  return std::min(LS_SEGS_MAX_HOST, std::max(1u, LS_TARGET_WG / njobs));
}
// 0 = lane per unit, 1 = wave per unit, 2 = the split parse (round 5: walk +
// sub-unit decode, the default where the lane parse was; env ZS_SPLIT=0 keeps
// the lane parse there).
int wave_units(size_t nseg, uint32_t flags) {
  if (flags & ZS_F_PARSE_SPLIT) return 2;
  if (flags & ZS_F_PARSE_LANE) return 0;
  if (flags & ZS_F_PARSE_WAVE) return 1;
  static const int force = [] {
    const char *e = std::getenv("ZS_PARSE");
    if (!e) return -1;
    return std::strcmp(e, "wave") == 0 ? 1 : (std::strcmp(e, "lane") == 0 ? 0 : (std::strcmp(e, "split") == 0 ? 2 : -1));
  }();
  static const size_t lim = [] {
    const char *e = std::getenv("ZS_WAVE_SEGS");
    return (size_t)(e ? std::atoll(e) : 12288);
  }();
  static const bool split = [] {
    const char *e = std::getenv("ZS_SPLIT");
    return !(e && e[0] == '0');
  }();
  if (force >= 0) return force;
  return nseg <= lim ? 1 : (split ? 2 : 0);
}
// Two chunked groups on two streams (run_jobs) for a raw/zlib/gzip group of
// at least 8 streams and TWO_GROUP_SEGS search segments (32 KiB of input
// each): env ZS_GROUPS=2.  Off by default -- measured (C2): 24.9-25.3 ms with
// two groups vs 22.0-22.3 with one, also with the walk at the highest wave
// priority; the groups' kernels squeeze each other's LDS (the walk keeps
// ~51 KiB per wave resident for its whole ~3.6 ms) and slow the walk's chain.
constexpr size_t TWO_GROUP_SEGS = 4096;
bool two_groups_enabled() {
  static const bool v = [] {
    const char *e = std::getenv("ZS_GROUPS");
    return e && e[0] == '2';
  }();
  return v;
}
bool chunking_enabled() {
  static bool v = [] {
    const char *e = std::getenv("ZS_NO_CHUNK");
    return !(e && e[0] == '1');
  }();
  return v;
}

std::mutex g_mu;
Workspace g_ws;

int ws_init() {
  if (g_ws.ready) return 0;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    set_err("no HIP device available (libzstreams_mi355x has no CPU path)");
    return ZS_ENODEV;
  }
  HIP_OK(hipGetDevice(&g_ws.device));
  HIP_OK(hipStreamCreateWithFlags(&g_ws.own_stream, hipStreamNonBlocking));
  if (!g_ws.stream) g_ws.stream = g_ws.own_stream;
  g_ws.ready = true;
  return 0;
}

template <typename T>
int grow_dev(T **p, size_t n) {
  if (*p) HIP_OK(hipFree(*p));
  *p = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(n, 1) * sizeof(T)));
  return 0;
}
template <typename T>
int grow_host(T **p, size_t n) {
  if (*p) HIP_OK(hipHostFree(*p));
  *p = nullptr;
  HIP_OK(hipHostMalloc(reinterpret_cast<void **>(p), std::max<size_t>(n, 1) * sizeof(T), hipHostMallocDefault));
  return 0;
}

int ws_reserve_jobs(size_t n) {
  if (n <= g_ws.cap_jobs) return 0;
  size_t c = std::max<size_t>(n, 2 * g_ws.cap_jobs);
  g_ws.cap_jobs = 0;
  int r;
  if ((r = grow_dev(&g_ws.d_jobs, c)) || (r = grow_dev(&g_ws.d_heads, c)) || (r = grow_dev(&g_ws.d_decs, c)) ||
      (r = grow_dev(&g_ws.d_checks, 2 * c)) || (r = grow_dev(&g_ws.d_res, c)) || (r = grow_dev(&g_ws.d_ids, 3 * c)) ||
      (r = grow_dev(&g_ws.d_fallback, c)) || (r = grow_dev(&g_ws.d_cjobs, c)) || (r = grow_host(&g_ws.h_cjobs, c)) ||
      (r = grow_host(&g_ws.h_jobs, c)) || (r = grow_host(&g_ws.h_res, c)) || (r = grow_host(&g_ws.h_ids, 3 * c)))
    return r;
  g_ws.cap_jobs = c;
  return 0;
}

// A failed allocation leaves the buffer null AND its capacity 0, so the next
// call allocates again instead of trusting a stale capacity.
int ws_reserve_chunks(size_t nseg, size_t nunits, size_t scratch_entries, size_t tokens, size_t window_bytes) {
  int r;
  if (window_bytes > g_ws.cap_windows) {
    size_t c = std::max(window_bytes, g_ws.cap_windows + g_ws.cap_windows / 2);
    g_ws.cap_windows = 0;
    if ((r = grow_dev(&g_ws.d_windows, c))) return r;
    g_ws.cap_windows = c;
  }
  if (nseg > g_ws.cap_segs) {
    size_t c = std::max(nseg, g_ws.cap_segs + g_ws.cap_segs / 2);
    g_ws.cap_segs = 0;
    if ((r = grow_dev(&g_ws.d_segs, c)) || (r = grow_host(&g_ws.h_segs, c))) return r;
    g_ws.cap_segs = c;
  }
  if (nunits > g_ws.cap_units) {
    size_t c = std::max(nunits, g_ws.cap_units + g_ws.cap_units / 2);
    g_ws.cap_units = 0;
    if ((r = grow_dev(&g_ws.d_chunks, c)) || (r = grow_host(&g_ws.h_chunks, c)) ||
        (r = grow_dev(&g_ws.d_tables, c * TABLE_ENTRIES_HOST)) ||
        (r = grow_dev(&g_ws.d_linkinfo, c * 2)) || (r = grow_dev(&g_ws.d_ptab, c * ZS_TP_MAXPG)))
      return r;
    g_ws.cap_units = c;
  }
  if (scratch_entries > g_ws.cap_scratch) {
    size_t c = std::max(scratch_entries, g_ws.cap_scratch + g_ws.cap_scratch / 4);
    g_ws.cap_scratch = 0;
    if ((r = grow_dev(&g_ws.d_scratch, c))) return r;
    g_ws.cap_scratch = c;
  }
  if (tokens > g_ws.cap_tokens) {
    size_t c = std::max(tokens, g_ws.cap_tokens + g_ws.cap_tokens / 4);
    g_ws.cap_tokens = 0;
    if ((r = grow_dev(&g_ws.d_tokens, c))) return r;
    g_ws.cap_tokens = c;
  }
  if (!g_ws.d_pool_next && (r = grow_dev(&g_ws.d_pool_next, 4))) return r;
  if (!g_ws.d_fixed) {  // fixed tables: the deflate set, then the deflate64 set
    if ((r = grow_dev(&g_ws.d_fixed, 2 * FIXED_WORDS_HOST))) return r;
    zs_launch_fixed_tables(g_ws.d_fixed, 0, g_ws.stream);
    zs_launch_fixed_compact(g_ws.d_fixed, g_ws.stream);
    zs_launch_fixed_tables(g_ws.d_fixed + FIXED_WORDS_HOST, 1, g_ws.stream);
    zs_launch_fixed_compact(g_ws.d_fixed + FIXED_WORDS_HOST, g_ws.stream);
  }
  return 0;
}

// pool tokens per KiB of chunked input (env ZS_POOL_PER_KB; 0 = default)
size_t pool_per_kb() {
  static size_t v = [] {
    const char *e = std::getenv("ZS_POOL_PER_KB");
    long x = e ? std::atol(e) : 0;
    return (size_t)(x < 0 ? 0 : x);
  }();
  return v;
}
// Pool tokens for a batch of in_sum compressed bytes.  Default: 32 per byte on
// top of the primary regions.  A symbol takes at least one bit, so a unit has at
// most 8 tokens per compressed byte; a spilling unit takes whole pages (the
// first one 64 Ki tokens), which for the shortest units (one block of 16 383
// one-bit symbols: 2 KiB) is 32 per byte.  So no stream outgrows it, however
// dense its symbols (Huffman-only or RLE over a small alphabet: ~5 per byte).
// Batches where that passes 4 Gi tokens (16 GiB, > 128 MiB compressed) get
// max(4 Gi, 2 per byte): there the pool is shared by many streams, and text
// averages < 0.4 tokens per byte past its primary region.
size_t pool_tokens(size_t in_sum) {
  if (pool_per_kb()) return in_sum / 1024 * pool_per_kb();
  const size_t dense = in_sum * 32, base = in_sum * 2, cap = (size_t)1 << 32;
  return std::max(base, std::min(dense, cap));
}

int ws_reserve_bytes(uint8_t **p, size_t *cap, size_t need) {
  if (need <= *cap) return 0;
  size_t c = std::max(need, *cap + *cap / 2);
  *cap = 0;
  int r = grow_dev(p, c);
  if (r) return r;
  *cap = c;
  return 0;
}

// windowBits rules of inflateReset2 (src/inflate.c:147-184).
bool parse_wbits(int wb, ZsJobDev *j) {
  int wrap;
  j->d64 = 0;
  if (wb < 0) {
    if (wb < -16) return false;
    wrap = 0;
    j->d64 = (wb == -16);
    wb = -wb;
  } else {
    wrap = (wb >> 4) + 5;
    if (wb < 48) wb &= 15;
  }
  if (wb && (wb < 8 || wb > (j->d64 ? 16 : 15))) return false;
  // wrap bits: 1 zlib, 2 gzip (4 = check, always set for wrapped streams)
  j->wrap = wrap == 0 ? ZW_RAW : ((wrap & 3) == 1 ? ZW_ZLIB : ((wrap & 3) == 2 ? ZW_GZIP : ZW_AUTO));
  j->wbits = wb;
  return true;
}

void fill_result(zs_result *r, int ret, const ZsResultDev *d) {
  std::memset(r, 0, sizeof *r);
  r->ret = ret;
  if (d) {
    r->total_in = d->total_in;
    r->total_out = d->total_out;
    r->adler = d->adler;
    r->msg = (d->msg > 0 && d->msg < ZM_COUNT) ? kMsgs[d->msg] : nullptr;
  }
}

// Limits of one launch (u32 bit and output positions inside the kernels); a
// stream past them decodes in pieces (run_pieces).
constexpr uint64_t ONE_IN_MAX = (1ull << 29) - 4096;
constexpr uint64_t ONE_OUT_MAX = 0xfff00000ull;
// compressed bytes per piece (env ZS_PIECE_KB, read per batch: tests set it
// to split small streams; a stream longer than it then decodes in pieces too)
uint64_t piece_bytes(bool *forced) {
  const char *e = std::getenv("ZS_PIECE_KB");
  const long kb = e ? std::atol(e) : 0;
  *forced = kb > 0;
  return kb > 0 ? std::max<uint64_t>(64, (uint64_t)kb) * 1024u : (256ull << 20);
}

int run_jobs(uint32_t nv, uint64_t max_out, uint32_t flags, ZsDecDev *dec_out, ZsHeadDev *head_out);
int run_pieces(const ZsJobDev &full, uint64_t piece, uint32_t flags, ZsResultDev *res, uint32_t stats[4]);

int batch_locked(const zs_job *jobs, uint32_t n, zs_result *results, uint32_t flags) {
  int r = ws_init();
  if (r) {
    for (uint32_t i = 0; i < n; i++) fill_result(&results[i], Z_STREAM_ERROR, nullptr);
    return r;
  }
  if ((r = ws_reserve_jobs(n))) return r;
  const bool dev = (flags & ZS_F_DEVICE) != 0;
  bool forced = false;
  const uint64_t piece = piece_bytes(&forced);
  // validate + lay out the staging arenas; streams past one launch's limits
  // (or, with ZS_PIECE_KB, longer than a piece) are decoded in pieces after
  // the batch
  constexpr uint32_t LONG = UINT32_MAX - 1;
  std::vector<uint32_t> slot(n, UINT32_MAX);
  std::vector<size_t> in_off(n, 0), out_off(n, 0);
  std::vector<ZsJobDev> longs(n);
  size_t in_total = 0, out_total = 0;
  uint64_t max_out = 0;
  uint32_t nv = 0;
  for (uint32_t i = 0; i < n; i++) {
    ZsJobDev jd{};
    const bool copy = jobs[i].mode == ZS_JOB_COPY;
    bool ok = (jobs[i].mode == ZS_JOB_INFLATE || copy) && parse_wbits(copy ? -15 : jobs[i].window_bits, &jd) &&
              (jobs[i].in || jobs[i].in_len == 0) && (jobs[i].out || jobs[i].out_cap == 0);
    if (dev && jobs[i].out && (reinterpret_cast<uintptr_t>(jobs[i].out) & 15u)) ok = false;
    if (!ok) {
      fill_result(&results[i], Z_STREAM_ERROR, nullptr);
      continue;
    }
    const bool is_long = !copy && (jobs[i].in_len > ONE_IN_MAX || jobs[i].out_cap > ONE_OUT_MAX ||
                                   (forced && jobs[i].in_len > piece));
    jd.flags = (copy ? ZS_JF_COPY | ZS_JF_CRC32 : 0) | ((flags & ZS_F_CRC32) && jd.wrap == ZW_RAW ? ZS_JF_CRC32 : 0);
    jd.in_len = jobs[i].in_len;
    jd.out_cap = jobs[i].out_cap;
    if (dev) {
      jd.in = static_cast<const uint8_t *>(jobs[i].in);
      jd.out = static_cast<uint8_t *>(jobs[i].out);
    } else {
      in_off[i] = in_total;
      in_total += (jobs[i].in_len + 15) & ~size_t(15);
      out_off[i] = out_total;
      out_total += (jobs[i].out_cap + 255) & ~size_t(255);
    }
    if (is_long) {
      slot[i] = LONG;
      longs[i] = jd;
      continue;
    }
    slot[i] = nv;
    max_out = std::max<uint64_t>(max_out, jd.out_cap);
    g_ws.h_jobs[nv] = jd;
    nv++;
  }
  hipStream_t st = g_ws.stream;
  if (!dev) {
    if ((r = ws_reserve_bytes(&g_ws.d_in, &g_ws.cap_in, in_total + 64))) return r;
    if ((r = ws_reserve_bytes(&g_ws.d_out, &g_ws.cap_out, out_total + 256))) return r;
    for (uint32_t i = 0; i < n; i++) {
      if (slot[i] == UINT32_MAX) continue;
      ZsJobDev &jd = slot[i] == LONG ? longs[i] : g_ws.h_jobs[slot[i]];
      jd.in = g_ws.d_in + in_off[i];
      jd.out = g_ws.d_out + out_off[i];
      if (jobs[i].in_len) HIP_OK(hipMemcpyAsync(g_ws.d_in + in_off[i], jobs[i].in, jobs[i].in_len, hipMemcpyHostToDevice, st));
    }
  }
  uint32_t stats[4] = {0, 0, 0, 0};
  if (nv) {
    if ((r = run_jobs(nv, max_out, flags, nullptr, nullptr))) return r;
    for (int k = 0; k < 4; k++) stats[k] += g_ws.stats[k];
    for (uint32_t i = 0; i < n; i++) {
      if (slot[i] == UINT32_MAX || slot[i] == LONG) continue;
      const ZsResultDev &d = g_ws.h_res[slot[i]];
      fill_result(&results[i], d.ret, &d);
      if (!dev && d.total_out)
        HIP_OK(hipMemcpyAsync(jobs[i].out, g_ws.d_out + out_off[i], d.total_out, hipMemcpyDeviceToHost, st));
    }
  }
  for (uint32_t i = 0; i < n; i++) {
    if (slot[i] != LONG) continue;
    ZsResultDev d{};
    if ((r = run_pieces(longs[i], piece, flags, &d, stats))) return r;
    fill_result(&results[i], d.ret, &d);
    if (!dev && d.total_out)
      HIP_OK(hipMemcpyAsync(jobs[i].out, g_ws.d_out + out_off[i], d.total_out, hipMemcpyDeviceToHost, st));
  }
  for (int k = 0; k < 4; k++) g_ws.stats[k] = stats[k];
  if (!dev) HIP_OK(hipStreamSynchronize(st));
  return 0;
}

// the second chunked group's stream and events, created once (0 = ready)
int ws_stream_b() {
  if (g_ws.stream_b) return 0;
  hipStream_t s = nullptr;
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
  for (int i = 0; i < 3 && ok; i++) ok = hipEventCreateWithFlags(&e[i], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    for (int i = 0; i < 3; i++)
      if (e[i]) (void)hipEventDestroy(e[i]);
    if (s) (void)hipStreamDestroy(s);
    (void)hipGetLastError();
    return -1;
  }
  g_ws.stream_b = s;
  g_ws.ev_fork = e[0];
  g_ws.ev_found = e[1];
  g_ws.ev_join = e[2];
  return 0;
}

// One launch over the prepared jobs g_ws.h_jobs[0, nv): routing, the chunked
// pipeline, the serial decoders, then (dec_out == nullptr) the checks and
// results into g_ws.h_res, or (pieces) each job's header and decode outcome
// into head_out / dec_out.
int run_jobs(uint32_t nv, uint64_t max_out, uint32_t flags, ZsDecDev *dec_out, ZsHeadDev *head_out) {
  hipStream_t st = g_ws.stream;
  // Route each job: raw/zlib/gzip streams with enough blocks -> speculative
  // chunked path (with the serial decoder as exact fallback); small ones and
  // deflate64 -> the wave-per-stream serial decoder.  Routing looks at the
  // compressed size (>= 4 search segments), or at >= 1 segment when the caller
  // allows >= 4 MiB of output (long-match streams); never at a ratio, since no
  // capacity on the chunked path depends on one.  Lists in h_ids:
  // [serial std | d64 | chunked].
  const uint32_t C = chunk_bytes();
  uint32_t n_std = 0, n_d64 = 0, n_cj = 0, n_cj64 = 0;
  size_t nseg = 0, nunit_slots = 0;
  // chunked jobs: the raw/zlib/gzip group first, then the deflate64 group
  std::vector<uint32_t> cj_list, cj64_list;
  std::vector<uint8_t> is_cj(nv, 0);
  for (uint32_t k = 0; k < nv; k++) {
    const ZsJobDev &jd = g_ws.h_jobs[k];
    const bool big = jd.in_len >= 4ull * C || (jd.in_len >= C && jd.out_cap >= (4ull << 20));
    if (chunking_enabled() && !(jd.flags & ZS_JF_COPY) && big) {
      (jd.d64 ? cj64_list : cj_list).push_back(k);
      is_cj[k] = 1;
    }
  }
  const uint32_t n_cj_std = (uint32_t)cj_list.size();
  cj_list.insert(cj_list.end(), cj64_list.begin(), cj64_list.end());
  std::vector<uint32_t> copies;  // ZIP stored entries: output = input
  for (uint32_t k = 0; k < nv; k++)
    if (g_ws.h_jobs[k].flags & ZS_JF_COPY) copies.push_back(k);
  // Plan the chunked jobs (segments, unit slots, token regions, entry ranges,
  // token pool, history windows) and upload them.  Any allocation failure here
  // only sends the jobs to the serial decoder.
  ZsTokPool pool{};
  size_t seg_std = 0, slots_std = 0;
  // Round 6: a large raw/zlib/gzip group runs as two groups on two streams
  // (A on the launch stream, B on stream_b once A's finder is done), so that
  // one group's boundary walk -- a serial chain per unit that keeps well under
  // one wave per SIMD busy -- overlaps the other group's finder, unit headers,
  // token decode, expand, link and emit.  n_a = raw/zlib/gzip jobs in group A
  // (n_cj_std: one group).
  uint32_t n_a = n_cj_std;
  size_t seg_a = 0, slots_a = 0;
  if (two_groups_enabled() && n_cj_std >= 8 && ws_stream_b() == 0) {
    size_t tot = 0;
    for (uint32_t q = 0; q < n_cj_std; q++) tot += (g_ws.h_jobs[cj_list[q]].in_len + C - 1) / C;
    if (tot >= TWO_GROUP_SEGS) {
      size_t acc = 0;
      for (uint32_t q = 0; q < n_cj_std; q++) {
        acc += (g_ws.h_jobs[cj_list[q]].in_len + C - 1) / C;
        if (2 * acc >= tot) {
          n_a = q + 1;
          break;
        }
      }
    }
  }
  if (!cj_list.empty()) {
    size_t slots = 0, toks = 0, ents = 0, in_sum = 0, win = 0;
    nseg = 0;
    for (uint32_t k : cj_list) nseg += (g_ws.h_jobs[k].in_len + C - 1) / C;
    int rr = ws_reserve_chunks(nseg, 0, 0, 0, 0);
    size_t si = 0;
    for (uint32_t q = 0; q < cj_list.size() && !rr; q++) {
      const uint32_t k = cj_list[q];
      const ZsJobDev &jd = g_ws.h_jobs[k];
      if (q == n_a && n_a < n_cj_std) {
        seg_a = si;
        slots_a = slots;
      }
      if (q == n_cj_std) {
        seg_std = si;
        slots_std = slots;
      }
      const uint32_t ns = (uint32_t)((jd.in_len + C - 1) / C);
      const uint32_t max_units = ns * SEG_SLOTS + 1;
      ZsCJobDev cj{};
      cj.job = k;
      // group-relative: group A from 0, group B from (seg_a, slots_a), deflate64 from (seg_std, slots_std)
      const size_t gseg = q >= n_cj_std ? seg_std : (q >= n_a ? seg_a : 0);
      const size_t gslot = q >= n_cj_std ? slots_std : (q >= n_a ? slots_a : 0);
      cj.first_seg = (uint32_t)(si - gseg);
      cj.nseg = ns;
      cj.unit0 = (uint32_t)(slots - gslot);
      cj.max_units = max_units;
      // primary token regions (zs_plan_kernel): per unit span x ZS_TOK_PER_BYTE
      // + slack, spans summing to at most the input plus a byte per unit
      cj.tok0 = toks;
      toks += ((jd.in_len + max_units) * ZS_TOK_PER_BYTE + (size_t)max_units * (ZS_TOK_SLACK + 32) + 63) & ~size_t(63);
      // entries: the verified chain's total never exceeds out_cap (else the
      // serial decoder answers); every member starts 8-entry aligned
      // (zs_chain_kernel), hence 8 entries of padding per possible unit
      cj.scratch0 = ents;
      // (a piece of a long stream cuts its chain at ZS_PART_OUT bytes)
      cj.scratch_n = std::min<uint64_t>(std::min<uint64_t>(jd.out_cap, (jd.d64 ? MAX_RATIO_D64 : MAX_RATIO) * jd.in_len + 64),
                                        (jd.flags & ZS_JF_PART) ? ZS_PART_OUT : ~0ull) +
                     8ull * max_units;
      cj.esz = jd.d64 ? 2u : 1u;  // deflate64: 17-bit entries, stored as u32
      ents += (cj.esz * (cj.scratch_n + 16) + 15) & ~size_t(15);
      in_sum += jd.in_len;
      win += (size_t)max_units * (jd.d64 ? 65536u : 32768u);
      g_ws.h_cjobs[q] = cj;
      for (uint32_t o = 0; o < ns; o++, si++) {
        ZsSegDev sg{};
        sg.job = k;
        sg.ord = o;
        sg.s_byte = o * C;
        sg.e_byte = (uint32_t)std::min<uint64_t>((uint64_t)(o + 1) * C, jd.in_len);
        sg.final_ok = o + 2 >= ns;  // the final block lies within the last segments
        g_ws.h_segs[si] = sg;
      }
      slots += max_units;
    }
    if (n_cj_std == cj_list.size()) {
      seg_std = si;
      slots_std = slots;
    }
    const size_t pool_pages = std::max<size_t>(64, (pool_tokens(in_sum) + ((size_t)1 << ZS_TP_LOG) - 1) >> ZS_TP_LOG);
    if (!rr) rr = ws_reserve_chunks(nseg, slots, ents + 16, toks + (pool_pages << ZS_TP_LOG), win);
    if (rr) {  // no room for the chunked path: every job decodes serially
      (void)hipGetLastError();  // the failed hipMalloc is tolerated: clear HIP's last error and ours
      g_err.clear();
      cj_list.clear();
      std::fill(is_cj.begin(), is_cj.end(), 0);
      nseg = 0;
    } else {
      n_cj = (uint32_t)cj_list.size();
      n_cj64 = n_cj - n_cj_std;
      nunit_slots = slots;
      pool.base = toks;
      pool.npages = (uint32_t)pool_pages;
      pool.next = g_ws.d_pool_next;
      pool.ptab = g_ws.d_ptab;
      HIP_OK(hipMemcpyAsync(g_ws.d_segs, g_ws.h_segs, nseg * sizeof(ZsSegDev), hipMemcpyHostToDevice, st));
      HIP_OK(hipMemcpyAsync(g_ws.d_cjobs, g_ws.h_cjobs, n_cj * sizeof(ZsCJobDev), hipMemcpyHostToDevice, st));
      HIP_OK(hipMemsetAsync(g_ws.d_pool_next, 0, sizeof(uint32_t), st));
    }
  }
  // serial lists: [std | d64 | chunked std | chunked d64] in h_ids
  for (uint32_t k = 0; k < nv; k++)
    if (!g_ws.h_jobs[k].d64 && !(g_ws.h_jobs[k].flags & ZS_JF_COPY) && !is_cj[k]) g_ws.h_ids[n_std++] = k;
  for (uint32_t k = 0; k < nv; k++)
    if (g_ws.h_jobs[k].d64 && !is_cj[k]) g_ws.h_ids[n_std + n_d64++] = k;
  for (uint32_t q = 0; q < n_cj; q++) g_ws.h_ids[n_std + n_d64 + q] = cj_list[q];
  HIP_OK(hipMemcpyAsync(g_ws.d_jobs, g_ws.h_jobs, nv * sizeof(ZsJobDev), hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(g_ws.d_ids, g_ws.h_ids, nv * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  hipEvent_t *ev = g_ws.prof ? g_ws.ev : nullptr;
  if (ev) HIP_OK(hipEventRecord(ev[0], st));
  zs_launch_header(g_ws.d_jobs, g_ws.d_heads, nv, st);
  const uint32_t n_cjs = n_cj - n_cj64;
  const uint32_t n_ga = std::min(n_a, n_cjs), n_gb = n_cjs - n_ga;  // the two raw/zlib/gzip groups (n_gb = 0: one)
  // parallel-prefix link buffers (groups of few long streams)
  uint32_t pl_std = 0, pl_d64 = 0, ls_std = 1, ls_b = 1;
  {
    uint32_t mu_std = 0, mu_d64 = 0, mu_a = 0, mu_b = 0;
    for (uint32_t q = 0; q < n_cj; q++) (q < n_cjs ? mu_std : mu_d64) = std::max((q < n_cjs ? mu_std : mu_d64), g_ws.h_cjobs[q].max_units);
    for (uint32_t q = 0; q < n_cjs; q++) (q < n_ga ? mu_a : mu_b) = std::max((q < n_ga ? mu_a : mu_b), g_ws.h_cjobs[q].max_units);
    pl_std = n_cjs && !n_gb ? plink_levels(n_cjs, mu_std, flags) : 0;
    ls_std = n_cjs && !pl_std ? link_segments(n_ga, mu_a, flags) : 1;
    ls_b = n_gb ? link_segments(n_gb, mu_b, flags) : 1;
    pl_d64 = n_cj64 ? plink_levels(n_cj64, mu_d64, flags) : 0;
    const size_t need = std::max<size_t>(pl_std ? 2 * slots_std * 32768u * 2u : 0,
                                         pl_d64 ? 2 * (nunit_slots - slots_std) * 65536u * 4u : 0);
    if (need && ws_reserve_bytes(&g_ws.d_plink, &g_ws.cap_plink, need)) {
      pl_std = pl_d64 = 0;  // serial link instead; the failed hipMalloc must not fail the batch
      (void)hipGetLastError();
      g_err.clear();
    }
    // segmented link: LS_SEGS_MAX segment-end maps (u16 per window byte) per chain of the group
    const size_t lneed = (ls_std > 1 || ls_b > 1) ? (size_t)n_cjs * LS_SEGS_MAX_HOST * 32768u * 2u : 0;
    if (lneed && ws_reserve_bytes(&g_ws.d_lmaps, &g_ws.cap_lmaps, lneed)) {
      ls_std = ls_b = 1;  // serial link instead
      (void)hipGetLastError();
      g_err.clear();
    }
  }
  const uint32_t wu_std = n_cjs ? (uint32_t)wave_units(seg_std, flags) : UINT32_MAX;
  const uint32_t wu_d64 = n_cj64 ? (uint32_t)wave_units(nseg - seg_std, flags) : UINT32_MAX;
  g_ws.path[0] = wu_std;
  g_ws.path[1] = pl_std ? pl_std : (ls_std > 1 ? 0x80000000u | ls_std : 0u);
  g_ws.path[2] = wu_d64;
  g_ws.path[3] = pl_d64;
  g_ws.path[7] = n_cjs ? (n_gb ? 2u : 1u) : 0u;
  if (n_cjs) {
    if (n_gb) {  // group B's stream starts after everything so far on the launch stream
      HIP_OK(hipEventRecord(g_ws.ev_fork, st));
      HIP_OK(hipStreamWaitEvent(g_ws.stream_b, g_ws.ev_fork, 0));
    }
    const size_t sa = n_gb ? seg_a : seg_std, ua = n_gb ? slots_a : slots_std;
    zs_launch_chunked(g_ws.d_jobs, g_ws.d_heads, g_ws.d_segs, (uint32_t)sa, g_ws.d_cjobs, n_ga, g_ws.d_chunks,
                      (uint32_t)ua, g_ws.d_scratch, g_ws.d_tokens, pool, g_ws.d_tables, g_ws.d_fixed,
                      g_ws.d_windows, g_ws.d_linkinfo, g_ws.d_decs, g_ws.d_fallback, 0, (int)wu_std,
                      pl_std ? g_ws.d_plink : nullptr, pl_std,
                      ls_std > 1 ? reinterpret_cast<uint16_t *>(g_ws.d_lmaps) : nullptr, ls_std, st,
                      ev ? ev + 1 : nullptr, nullptr, 0, n_gb ? g_ws.ev_found : nullptr);
    if (n_gb) {  // group B: its own slice of every per-unit array, its finder lists in its own token regions
      HIP_OK(hipStreamWaitEvent(g_ws.stream_b, g_ws.ev_found, 0));
      ZsTokPool pb = pool;
      pb.ptab = pool.ptab + slots_a * ZS_TP_MAXPG;
      zs_launch_chunked(g_ws.d_jobs, g_ws.d_heads, g_ws.d_segs + seg_a, (uint32_t)(seg_std - seg_a), g_ws.d_cjobs + n_ga,
                        n_gb, g_ws.d_chunks + slots_a, (uint32_t)(slots_std - slots_a), g_ws.d_scratch, g_ws.d_tokens, pb,
                        g_ws.d_tables + slots_a * TABLE_ENTRIES_HOST, g_ws.d_fixed, g_ws.d_windows + slots_a * 32768,
                        g_ws.d_linkinfo + slots_a * 2, g_ws.d_decs, g_ws.d_fallback, 0, (int)wu_std, nullptr, 0,
                        ls_b > 1 ? reinterpret_cast<uint16_t *>(g_ws.d_lmaps) + (size_t)n_ga * LS_SEGS_MAX_HOST * 32768u
                                 : nullptr,
                        ls_b, g_ws.stream_b, nullptr, g_ws.d_tokens + g_ws.h_cjobs[n_ga].tok0, 1, nullptr);
      HIP_OK(hipEventRecord(g_ws.ev_join, g_ws.stream_b));
    }
  }
  if (n_cj64) {  // the deflate64 group: its own slice of every per-unit array
    ZsTokPool p64 = pool;
    p64.ptab = pool.ptab + slots_std * ZS_TP_MAXPG;
    zs_launch_chunked(g_ws.d_jobs, g_ws.d_heads, g_ws.d_segs + seg_std, (uint32_t)(nseg - seg_std),
                      g_ws.d_cjobs + n_cjs, n_cj64, g_ws.d_chunks + slots_std, (uint32_t)(nunit_slots - slots_std),
                      g_ws.d_scratch, g_ws.d_tokens, p64, g_ws.d_tables + slots_std * TABLE_ENTRIES_HOST,
                      g_ws.d_fixed + FIXED_WORDS_HOST, g_ws.d_windows + slots_std * 32768, g_ws.d_linkinfo + slots_std * 2,
                      g_ws.d_decs, g_ws.d_fallback, 1, (int)wu_d64, pl_d64 ? g_ws.d_plink : nullptr,
                      pl_d64, nullptr, 1, st, (ev && !n_cjs) ? ev + 1 : nullptr, nullptr, 0, nullptr);
  }
  if (n_gb) HIP_OK(hipStreamWaitEvent(st, g_ws.ev_join, 0));  // group B done before its fallbacks and the results
  if (!n_cj && ev)
    for (int i = 1; i <= 6; i++) HIP_OK(hipEventRecord(ev[i], st));
  zs_launch_decode(0, g_ws.d_jobs, g_ws.d_heads, g_ws.d_ids, n_std, g_ws.d_decs, nullptr, st);
  zs_launch_decode(1, g_ws.d_jobs, g_ws.d_heads, g_ws.d_ids + n_std, n_d64, g_ws.d_decs, nullptr, st);
  if (n_cjs) zs_launch_decode(0, g_ws.d_jobs, g_ws.d_heads, g_ws.d_ids + n_std + n_d64, n_cjs, g_ws.d_decs, g_ws.d_fallback, st);
  if (n_cj64)
    zs_launch_decode(1, g_ws.d_jobs, g_ws.d_heads, g_ws.d_ids + n_std + n_d64 + n_cjs, n_cj64, g_ws.d_decs, g_ws.d_fallback, st);
  std::vector<ZsDecDev> copy_decs(copies.size());
  for (size_t q = 0; q < copies.size(); q++) {
    const ZsJobDev &jd = g_ws.h_jobs[copies[q]];
    const uint64_t m = std::min<uint64_t>(jd.in_len, jd.out_cap);
    if (m) HIP_OK(hipMemcpyAsync(jd.out, jd.in, m, hipMemcpyDeviceToDevice, st));
    copy_decs[q] = ZsDecDev{m == jd.in_len ? (int32_t)ZD_END : (int32_t)ZD_FULL, ZM_NONE, m * 8u, m};
    HIP_OK(hipMemcpyAsync(g_ws.d_decs + copies[q], &copy_decs[q], sizeof(ZsDecDev), hipMemcpyHostToDevice, st));
  }
  if (ev) HIP_OK(hipEventRecord(ev[7], st));
  if (!dec_out) zs_launch_finish(g_ws.d_jobs, g_ws.d_heads, g_ws.d_decs, g_ws.d_checks, g_ws.d_res, nv, max_out, st);
  if (ev) HIP_OK(hipEventRecord(ev[8], st));
  {
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) {
      set_err(std::string("kernel launch failed: ") + hipGetErrorString(le));
      return ZS_ENODEV;
    }
  }
  if (dec_out) {
    HIP_OK(hipMemcpyAsync(dec_out, g_ws.d_decs, nv * sizeof(ZsDecDev), hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(head_out, g_ws.d_heads, nv * sizeof(ZsHeadDev), hipMemcpyDeviceToHost, st));
  } else {
    HIP_OK(hipMemcpyAsync(g_ws.h_res, g_ws.d_res, nv * sizeof(ZsResultDev), hipMemcpyDeviceToHost, st));
  }
  // the chunked path's statistics ride along before the one synchronisation
  // (round 6: two blocking copies after it left the GPU idle between batches)
  uint32_t *const h_fb = g_ws.h_ids + nv;  // (pinned, 3 x cap_jobs; [0, nv) held the ids)
  if (n_cj) {
    HIP_OK(hipMemcpyAsync(h_fb, g_ws.d_fallback, nv * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(g_ws.h_cjobs, g_ws.d_cjobs, n_cj * sizeof(ZsCJobDev), hipMemcpyDeviceToHost, st));
  }
  HIP_OK(hipStreamSynchronize(st));
  if (ev) {
    float ms = 0.f, bms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, ev[1], ev[7]));
    HIP_OK(hipEventElapsedTime(&bms, ev[0], ev[8]));
    for (int i = 0; i < ZS_PROF_STAGES; i++) {
      float sm = 0.f;
      HIP_OK(hipEventElapsedTime(&sm, ev[i], ev[i + 1]));
      g_ws.prof_stage[i] += sm;
    }
    g_ws.prof_ms += ms;
    g_ws.prof_batch_ms += bms;
    g_ws.prof_launches++;
  }
  g_ws.path[4] = zs_lane_resident_waves();
  g_ws.path[5] = g_ws.path[6] = 0;
  g_ws.stats[0] = n_cj;
  g_ws.stats[1] = 0;
  g_ws.stats[2] = 0;
  g_ws.stats[3] = n_std + n_d64;
  if (n_cj) {
    for (uint32_t k : cj_list) g_ws.stats[2] += h_fb[k];
    for (uint32_t q = 0; q < n_cj; q++) g_ws.stats[1] += g_ws.h_cjobs[q].nunits;
    for (uint32_t q = 0; q < n_cj; q++) g_ws.path[q < n_cjs ? 5 : 6] += g_ws.h_cjobs[q].nunits;
    if (std::getenv("ZS_DEBUG_CHUNKS")) {
      uint32_t used = 0;
      HIP_OK(hipMemcpy(&used, g_ws.d_pool_next, sizeof used, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(g_ws.h_chunks, g_ws.d_chunks, nunit_slots * sizeof(ZsChunkDev), hipMemcpyDeviceToHost));
      size_t inch = 0, stopped = 0;
      for (size_t i = 0; i < nunit_slots; i++) {
        inch += g_ws.h_chunks[i].in_chain;
        stopped += (g_ws.h_chunks[i].code & 0xff) == ZD_STOP;
      }
      std::fprintf(stderr, "[zs] chunked jobs %u segments %zu units %u in_chain %zu stopped %zu fallback %u pool pages %u/%u\n",
                   n_cj, nseg, g_ws.stats[1], inch, stopped, g_ws.stats[2], used, pool.npages);
      const size_t show = std::getenv("ZS_DEBUG_CHUNKS")[0] == '2' ? nunit_slots : 8;
      for (size_t i = 0; i < nunit_slots && i < show; i++) {
        const ZsChunkDev &c = g_ws.h_chunks[i];
        std::fprintf(stderr, "  unit %zu ord %u start %u stop %u end %u code %d n_out %u ntok %u tcap %u chain %u\n", i,
                     c.ord, c.start_bit, c.stop_bit, c.end_bit, c.code, c.n_out, c.n_tok, c.tcap, c.in_chain);
      }
    }
  }
  return 0;
}

// A stream past one launch's limits, in pieces of `piece` compressed bytes:
// piece k is a one-job launch over the input from the bit where piece k-1
// stopped (ZS_JF_CONT: raw deflate at that block boundary, the output so far
// as history right before its own output), which stops at the last block
// boundary it verifies (ZS_JF_PART -> ZD_STOP, at most ZS_PART_OUT bytes) --
// the chunked path's cut chain, or the serial decoder's first boundary past a
// margin before the piece's end.  The last piece (the rest of the input)
// decodes to the end of the stream or to its error; the checks and the
// result then cover the whole stream (zs_finalize_kernel on the full job,
// with piece 0's header).  A piece that cannot reach a boundary (one deflate
// block longer than the piece) is retried twice as long.
int run_pieces(const ZsJobDev &full, uint64_t piece, uint32_t flags, ZsResultDev *res, uint32_t stats[4]) {
  hipStream_t st = g_ws.stream;
  const uint32_t HN = full.d64 ? 65536u : 32768u;
  ZsHeadDev head0{};
  ZsDecDev fin{};
  uint64_t bit = 0, total = 0;
  bool first = true;
  for (;;) {
    const uint64_t byte0 = bit >> 3, rem = full.in_len - byte0, ocap = full.out_cap - total;
    piece = std::min(piece, ONE_IN_MAX);
    const bool last = rem <= piece;
    ZsJobDev p = full;
    p.in = full.in + byte0;
    p.in_len = last ? rem : piece;
    p.out = full.out + total;
    p.out_cap = std::min(ocap, ONE_OUT_MAX);
    p.flags = 0;
    p.sbit = (uint32_t)(bit & 7u);
    if (!first) {
      p.wrap = ZW_RAW;
      p.flags |= ZS_JF_CONT;
      p.hist = (uint32_t)std::min<uint64_t>(total, HN);
    }
    const bool part = !last || ocap > ONE_OUT_MAX;
    if (part) {
      p.flags |= ZS_JF_PART;
      p.stop_after = (uint32_t)((p.in_len - std::min<uint64_t>(p.in_len / 2, 1u << 20)) * 8u);
    }
    g_ws.h_jobs[0] = p;
    ZsDecDev dec{};
    ZsHeadDev hd{};
    int r = run_jobs(1, p.out_cap, flags, &dec, &hd);
    if (r) return r;
    for (int k = 0; k < 4; k++) stats[k] += g_ws.stats[k];
    if (first) {
      head0 = hd;
      if (hd.code != ZD_END) {  // header error / need dictionary: answered by the header alone
        fin.code = ZD_SKIP;
        break;
      }
    }
    first = false;
    // no boundary within one launch's limits (a deflate block of > 512 MiB in
    // or > 4 GiB out): Z_STREAM_ERROR rather than a guess
    const bool stuck = (dec.code == ZD_STOP && dec.end_bits <= p.sbit) ||
                       (part && !last && dec.code == ZD_TRUNC && piece >= ONE_IN_MAX) ||
                       (part && dec.code == ZD_FULL && ocap > ONE_OUT_MAX);
    if (stuck) {
      set_err("a deflate block longer than one launch's limits (512 MiB in, 4 GiB out)");
      fin.code = ZD_SKIP;
      head0.code = ZD_SKIP;
      head0.ret = ZS_STREAM_ERROR;
      head0.total_in = byte0;
      head0.msg = ZM_NONE;
      break;
    }
    if (dec.code == ZD_STOP) {
      bit = byte0 * 8u + dec.end_bits;
      total += dec.total_out;
      continue;
    }
    if (part && !last && dec.code == ZD_TRUNC) {  // a block longer than the piece: retry it longer
      piece *= 2;
      continue;
    }
    fin = dec;
    fin.end_bits = byte0 * 8u + (dec.code == ZD_TRUNC ? p.in_len * 8u : dec.end_bits);
    fin.total_out = total + dec.total_out;
    break;
  }
  // the result of the whole stream
  ZsJobDev j = full;
  g_ws.h_jobs[0] = j;
  HIP_OK(hipMemcpyAsync(g_ws.d_jobs, g_ws.h_jobs, sizeof(ZsJobDev), hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(g_ws.d_heads, &head0, sizeof head0, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(g_ws.d_decs, &fin, sizeof fin, hipMemcpyHostToDevice, st));
  zs_launch_finish(g_ws.d_jobs, g_ws.d_heads, g_ws.d_decs, g_ws.d_checks, g_ws.d_res, 1, std::max<uint64_t>(fin.total_out, 1), st);
  HIP_OK(hipMemcpyAsync(res, g_ws.d_res, sizeof(ZsResultDev), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  return 0;
}

// ---------------------------------------------------------------------------
// Stream surfaces: every call is one exact inflate(strm, flush) on the GPU.
//
// A handle's decoder state (ZsStreamDev: mode, pending literal / match /
// stored bytes, current code lengths, the last 32 / 64 KiB of output, the
// running check) stays in device memory between calls.  zlib pulls input on
// demand (src/inflate.c:481-495, inffast.c:289-293): bytes it has pulled but
// not turned into output yet live in its bit buffer / partial state.  Here
// they are the host `carry` (at most a partial element: a symbol, a block
// header, a wrapper header or trailer, plus the partial byte of a FULL stop),
// put in front of the next call's new input.  So every call returns zlib's
// (consumed, produced, ret, msg, adler) -- SURVEY §8b Tier 2.
//
// A fresh stream offered >= ZS_STREAM_FAST_KB of input in one call (the
// zlib-ABI one-shot pattern) is first decoded by the batch pipeline (the
// chunk-parallel path for large standard streams); when that run ends the
// stream (STREAM_END or a data error) its result IS the call's result, as
// it is one inflate() over the same input and output space.  Otherwise the
// call runs on the resumable decoder.
// ---------------------------------------------------------------------------
constexpr size_t STREAM_SLICE = 64u << 20;  // input bytes per resumable launch (32-bit bit offsets)

struct StreamState {
  int inited = 0;
  int wbits = 0;
  ZsJobDev cfg{};               // wrap / d64 / wbits from parse_wbits
  int mode = ZSM_HEAD;          // host mirror of the device mode after the last call
  std::vector<uint8_t> carry;   // pulled, not yet consumed into output (see above)
  uint32_t carry_bit = 0;       // restart bit within carry[0]
  uint64_t total_in = 0, total_out = 0;
  const char *msg = nullptr;
  uint32_t adler = 0;
  ZsStreamDev *d_st = nullptr;
  // the handle's own call buffers and copy stream: calls of different handles
  // (different host threads) copy concurrently and share batch launches
  hipStream_t hs = nullptr;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  size_t cap_in = 0, cap_out = 0;
  uint8_t *h_in = nullptr, *h_out = nullptr;  // pinned staging (calls up to STAGE_MAX bytes)
  uint8_t *dh_in = nullptr, *dh_out = nullptr;  // their device views (host-mapped)
  size_t cap_hin = 0, cap_hout = 0;
  int fresh = 0;  // the device state is set up by the next call (ZsStreamIo::fresh)
  int pk_w = -1;  // the persistent worker's mailbox this handle holds (-1: none)
  uint64_t pk_last_ns = 0;  // its last call's time on the worker (the next wait sleeps most of it) ...
  uint64_t pk_last_in = 0;  // ... and that call's input bytes
};

constexpr size_t STAGE_MAX = 4u << 20;

// pinned staging buffer of >= need bytes (need <= STAGE_MAX), else nullptr.
// dp: the buffer's cached device view, dropped whenever the buffer is
// reallocated (a stale view would let a later mapped call write freed memory)
uint8_t *stage_buf(uint8_t **p, size_t *cap, size_t need, uint8_t **dp) {
  if (need > STAGE_MAX) return nullptr;
  if (need > *cap) {
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *dp = nullptr;
    *cap = 0;
    const size_t c = std::max<size_t>(need, 128u << 10);
    if (hipHostMalloc(reinterpret_cast<void **>(p), c, hipHostMallocDefault) != hipSuccess) {
      *p = nullptr;
      return nullptr;
    }
    *cap = c;
  }
  return *p;
}

// stage_buf plus the buffer's device view (kernels read / write it over the bus)
uint8_t *stage_mapped(uint8_t **p, size_t *cap, uint8_t **dp, size_t need) {
  uint8_t *h = stage_buf(p, cap, need, dp);
  if (!h) return nullptr;
  if (!*dp) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipGetLastError();
      *dp = nullptr;
      return nullptr;
    }
    *dp = static_cast<uint8_t *>(d);
  }
  return *dp ? h : nullptr;
}

template <typename T>
T *host_view(T *h) {  // device view of a pinned host array (nullptr if none)
  void *d = nullptr;
  if (!h || hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return static_cast<T *>(d);
}

size_t stream_fast_min() {
  static size_t v = [] {
    const char *e = std::getenv("ZS_STREAM_FAST_KB");
    return (size_t)(e ? std::atoll(e) : 1024) << 10;
  }();
  return v;
}

// ---------------------------------------------------------------------------
// Call batching.  A call's input is staged (host-mapped, or copied on its
// handle's stream), then the call joins the pending queue.  A caller that
// finds a free launch slot becomes that slot's leader: it takes every pending
// call (up to SQ_MAX) and runs them as ONE launch sequence on the slot's
// stream (zs_launch_stream: a workgroup per call), then waits for it outside
// the lock.  Up to SQ_SLOTS batches run at once (one per hardware queue).
// While a batch runs, a new one starts only once it holds a 1/SQ_SLOTS share
// of the active calls (pending + running): the calls that return from a
// batch gather into the next instead of each taking a slot alone.  A lone
// caller's batch is itself: no added latency.
// ---------------------------------------------------------------------------
constexpr size_t SQ_MAX = 2048;
constexpr int SQ_SLOTS = 32;  // most slots (ZS_STREAM_SLOTS); the default follows the process's hardware queues
constexpr long SQ_GAP_US = 40;   // deflate job gathering (DzQueue): quiet gap that ends it
constexpr long SQ_WAIT_US = 400; // deflate job gathering: longest wait

struct StreamCall {
  StreamState *s = nullptr;
  ZsJobDev jb{};
  ZsStreamIo io{};  // host-mapped staging of the call (or DMA: null), carried restart bit
  int run_header = 0;
  ZsStreamRes res{};
  int err = 0;
  std::string errmsg;
  bool taken = false;  // in a batch (its leader completes it)
  bool done = false;
};

struct SqSlot {  // one launch slot: its stream and the batch's call arrays
  hipStream_t st = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the batch's kernels (zs_stream_stats_ex)
  uint64_t last_kernel_ns = 0;
  size_t cap = 0;
  ZsJobDev *d_jobs = nullptr, *h_jobs = nullptr;
  ZsHeadDev *d_heads = nullptr;
  ZsStreamDev **d_sts = nullptr, **h_sts = nullptr;
  ZsStreamRes *d_res = nullptr, *h_res = nullptr;
  ZsStreamIo *h_io = nullptr;
  // device views of the pinned arrays: the kernels read the batch's jobs and
  // write its outcomes over the bus, no copies of their own
  ZsJobDev *v_jobs = nullptr;
  ZsStreamDev **v_sts = nullptr;
  ZsStreamIo *v_io = nullptr;
  ZsStreamRes *v_res = nullptr;
};

struct StreamQueue {
  std::mutex mu;
  std::condition_variable cv, arrive;
  std::vector<StreamCall *> pending;
  size_t last_n = 0;  // calls in the last batch
  SqSlot slot[SQ_SLOTS];
  bool busy[SQ_SLOTS] = {};
  size_t running = 0;  // calls in batches in flight
  uint64_t launches = 0, calls = 0;  // zs_stream_stats
  // zs_stream_stats_ex: launch sequences' wall time (sum over slots), the
  // leaders' gather waits, and the kernels' time (HIP events around the launch)
  uint64_t launch_ns = 0, gather_ns = 0, kernel_ns = 0;
} g_sq;

// a slot's leader only (busy[slot] set): one launch sequence per decoder variant
int sq_launch(SqSlot &q, std::vector<StreamCall *> &calls) {
  if (!q.st) HIP_OK(hipStreamCreateWithFlags(&q.st, hipStreamNonBlocking));
  if (!q.ev0) HIP_OK(hipEventCreate(&q.ev0));
  if (!q.ev1) HIP_OK(hipEventCreate(&q.ev1));
  const size_t n = calls.size();
  if (n > q.cap) {
    const size_t c = std::max<size_t>(n, 64);
    q.cap = 0;
    int r;
    if ((r = grow_dev(&q.d_jobs, c)) || (r = grow_host(&q.h_jobs, c)) || (r = grow_dev(&q.d_heads, c)) ||
        (r = grow_dev(&q.d_sts, c)) || (r = grow_host(&q.h_sts, c)) || (r = grow_dev(&q.d_res, c)) ||
        (r = grow_host(&q.h_res, c)) || (r = grow_host(&q.h_io, c)))
      return r;
    q.v_jobs = host_view(q.h_jobs);
    q.v_sts = host_view(q.h_sts);
    q.v_io = host_view(q.h_io);
    q.v_res = host_view(q.h_res);
    if (!q.v_io) {
      set_err("stream: pinned call array has no device view");
      return ZS_ENODEV;
    }
    q.cap = c;
  }
  std::vector<size_t> order;
  order.reserve(n);
  size_t nstd = 0;
  for (int d64 = 0; d64 < 2; d64++)
    for (size_t i = 0; i < n; i++)
      if ((calls[i]->s->cfg.d64 != 0) == (d64 != 0)) {
        order.push_back(i);
        nstd += d64 ? 0 : 1;
      }
  for (size_t k = 0; k < n; k++) {
    q.h_jobs[k] = calls[order[k]]->jb;
    q.h_sts[k] = calls[order[k]]->s->d_st;
    q.h_io[k] = calls[order[k]]->io;
  }
  const hipStream_t st = q.st;
  // jobs / states / outcomes: read and written by the kernels through the
  // pinned arrays' device views when the runtime gives them, else copied
  static const bool use_views = [] {  // env ZS_STREAM_VIEWS=0: copy the arrays instead (A/B)
    const char *e = std::getenv("ZS_STREAM_VIEWS");
    return !(e && e[0] == '0');
  }();
  const bool views = use_views && q.v_jobs && q.v_sts && q.v_res;
  ZsJobDev *jobs = views ? q.v_jobs : q.d_jobs;
  ZsStreamDev **sts = views ? q.v_sts : q.d_sts;
  ZsStreamRes *res = views ? q.v_res : q.d_res;
  if (!views) {
    HIP_OK(hipMemcpyAsync(q.d_jobs, q.h_jobs, n * sizeof(ZsJobDev), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(q.d_sts, q.h_sts, n * sizeof(ZsStreamDev *), hipMemcpyHostToDevice, st));
  }
  HIP_OK(hipEventRecord(q.ev0, st));
  for (int d64 = 0; d64 < 2; d64++) {
    const size_t k0 = d64 ? nstd : 0, k1 = d64 ? n : nstd;
    if (k1 == k0) continue;
    int run_header = 0;
    uint64_t max_out = 0, max_in = 0;
    for (size_t k = k0; k < k1; k++) {
      run_header |= calls[order[k]]->run_header;
      max_out = std::max<uint64_t>(max_out, q.h_jobs[k].out_cap);
      if (q.h_io[k].hin) max_in = std::max<uint64_t>(max_in, q.h_jobs[k].in_len);
    }
    zs_launch_stream(d64, run_header, sts + k0, jobs + k0, q.d_heads + k0, q.v_io + k0, (uint32_t)(k1 - k0), max_in,
                     max_out, res + k0, st);
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipEventRecord(q.ev1, st));
  if (!views) HIP_OK(hipMemcpyAsync(q.h_res, q.d_res, n * sizeof(ZsStreamRes), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  {
    float ms = 0.f;
    q.last_kernel_ns = hipEventElapsedTime(&ms, q.ev0, q.ev1) == hipSuccess ? (uint64_t)(ms * 1e6f) : 0u;
  }
  for (size_t k = 0; k < n; k++) calls[order[k]]->res = q.h_res[k];
  return 0;
}

int sq_slots() {  // env ZS_STREAM_SLOTS (1..SQ_SLOTS), else one per hardware queue (GPU_MAX_HW_QUEUES, HIP's default 4)
  static const int v = [] {
    const char *e = std::getenv("ZS_STREAM_SLOTS");
    const char *q = std::getenv("GPU_MAX_HW_QUEUES");
    const int k = e ? std::atoi(e) : (q ? std::atoi(q) : 4);
    return std::max(1, std::min(SQ_SLOTS, k));
  }();
  return v;
}

// env ZS_STREAM_GATHER_US: a new leader waits up to this long (while calls keep
// arriving, gaps below SQ_GAP_US) for as many calls as the last batch held
long sq_gather_us() {
  static const long v = [] {
    const char *e = std::getenv("ZS_STREAM_GATHER_US");
    return e ? std::max(0L, std::atol(e)) : 0L;
  }();
  return v;
}

int sq_submit(StreamCall *c) {
  const int slots = sq_slots();
  std::unique_lock<std::mutex> lk(g_sq.mu);
  g_sq.pending.push_back(c);
  g_sq.arrive.notify_one();
  for (;;) {
    if (c->done) break;
    int k = -1, nbusy = 0;
    for (int i = 0; i < slots; i++) nbusy += g_sq.busy[i] ? 1 : 0;
    const size_t share = (g_sq.pending.size() + g_sq.running + slots - 1) / slots;
    if (!c->taken && (nbusy == 0 || g_sq.pending.size() >= share))
      for (int i = 0; i < slots && k < 0; i++)
        if (!g_sq.busy[i]) k = i;
    if (k < 0) {  // our batch runs, or every slot does: wait for a completion
      g_sq.cv.wait(lk);
      continue;
    }
    g_sq.busy[k] = true;
    if (const long gw = sq_gather_us(); gw > 0 && g_sq.pending.size() < g_sq.last_n) {
      const auto g0 = std::chrono::steady_clock::now();
      const auto t_end = g0 + std::chrono::microseconds(gw);
      while (g_sq.pending.size() < g_sq.last_n) {
        const size_t had = g_sq.pending.size();
        const auto t = std::min(t_end, std::chrono::steady_clock::now() + std::chrono::microseconds(SQ_GAP_US));
        g_sq.arrive.wait_until(lk, t, [&] { return g_sq.pending.size() > had; });
        if (g_sq.pending.size() == had || std::chrono::steady_clock::now() >= t_end) break;
      }
      g_sq.gather_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - g0).count();
    }
    const size_t take = std::min(g_sq.pending.size(), SQ_MAX);
    g_sq.last_n = take;
    std::vector<StreamCall *> batch(g_sq.pending.begin(), g_sq.pending.begin() + take);
    g_sq.pending.erase(g_sq.pending.begin(), g_sq.pending.begin() + take);
    for (StreamCall *b : batch) b->taken = true;
    g_sq.running += batch.size();
    lk.unlock();
    const auto l0 = std::chrono::steady_clock::now();
    const int rc = sq_launch(g_sq.slot[k], batch);
    const uint64_t lns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - l0).count();
    const std::string msg = rc ? g_err : std::string();
    if (rc) (void)hipGetLastError();
    lk.lock();
    for (StreamCall *b : batch) {
      b->err = rc;
      b->errmsg = msg;
      b->done = true;
    }
    g_sq.busy[k] = false;
    g_sq.running -= batch.size();
    g_sq.launches++;
    g_sq.calls += batch.size();
    g_sq.launch_ns += lns;
    g_sq.kernel_ns += g_sq.slot[k].last_kernel_ns;
    g_sq.cv.notify_all();
  }
  if (c->err) set_err(c->errmsg);
  return c->err;
}

// ---------------------------------------------------------------------------
// Persistent stream worker (zs_stream_pk_kernel): one launch of PK_WGS
// workgroups, a mailbox each in host-coherent pinned memory.  A handle holds a
// mailbox from its first mapped, header-less call until it ends; each of its
// calls is posted there and returns when that workgroup finished it -- no
// launch, no batch, no wait for other handles' calls.  The launch leaves by
// itself after PK_IDLE_US without posts (or after its current call once PK_LIFE_MS old), and
// the next post relaunches it: a waiter that finds the launch ended with its
// call undone relaunches (only ever one launch; the call stays posted).
// Calls that need the wrapper header, DMA staging or deflate64, and handles
// beyond the mailboxes, take the batch path.  env ZS_STREAM_PK=0 disables it.
// ---------------------------------------------------------------------------
constexpr int PK_MAX = 256;
struct PkState {
  std::mutex mu;
  ZsMbox *h_mb = nullptr, *d_mb = nullptr;
  uint32_t *h_ctl = nullptr, *d_ctl = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;  // end of the current launch
  bool launched = false, broken = false;
  int nw = 0;
  std::vector<int> free_w;
  uint32_t seq[PK_MAX] = {};
  uint64_t launches = 0;
  std::atomic<uint64_t> calls{0}, busy_ns{0}, wait_ns{0};  // the calls' workgroup time; post to seen-done on the host
  std::atomic<uint64_t> idle_ns{0};  // the workgroups' wait for each call since their previous one
  std::atomic<int64_t> last_post{0};  // steady_clock ns of the last post (the launch outlives it by >= PK_IDLE)
  std::atomic<int64_t> launch_at{0};  // steady_clock ns of the current launch (its workgroups leave once PK_LIFE old)
} g_pk;
std::atomic<int> g_pk_on{-1};  // -1: from env ZS_STREAM_PK (default on)

bool pk_enabled() {
  int v = g_pk_on.load();
  if (v < 0) {
    const char *e = std::getenv("ZS_STREAM_PK");
    v = (e && e[0] == '0') ? 0 : 1;
    g_pk_on.store(v);
  }
  return v != 0;
}

void pk_atexit() {  // let the launch leave before the runtime tears down
  if (!g_pk.h_ctl) return;
  __atomic_store_n(&g_pk.h_ctl[0], 1u, __ATOMIC_SEQ_CST);
  if (g_pk.launched && g_pk.ev) (void)hipEventSynchronize(g_pk.ev);
}

int pk_init_locked() {
  if (g_pk.h_mb) return 0;
  if (g_pk.broken) return ZS_ENODEV;
  const char *e = std::getenv("ZS_PK_WGS");
  const int nw = std::max(1, std::min(PK_MAX, e ? std::atoi(e) : 64));
  void *h = nullptr;
  const size_t bytes = sizeof(ZsMbox) * (size_t)nw + ZS_PK_CTL_WORDS * sizeof(uint32_t);
  if (hipHostMalloc(&h, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    (void)hipGetLastError();
    g_pk.broken = true;
    return ZS_ENODEV;
  }
  std::memset(h, 0, bytes);
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || hipStreamCreateWithFlags(&g_pk.st, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&g_pk.ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipHostFree(h);
    g_pk.broken = true;
    return ZS_ENODEV;
  }
  g_pk.h_mb = static_cast<ZsMbox *>(h);
  g_pk.d_mb = static_cast<ZsMbox *>(d);
  g_pk.h_ctl = reinterpret_cast<uint32_t *>(g_pk.h_mb + nw);
  g_pk.d_ctl = reinterpret_cast<uint32_t *>(g_pk.d_mb + nw);
  g_pk.nw = nw;
  for (int w = nw - 1; w >= 0; w--) g_pk.free_w.push_back(w);
  std::atexit(pk_atexit);
  return 0;
}

bool pk_running_locked() {
  if (!g_pk.launched) return false;
  const hipError_t q = hipEventQuery(g_pk.ev);
  if (q == hipErrorNotReady) return true;
  (void)hipGetLastError();
  g_pk.launched = false;
  return false;
}

int64_t pk_idle_us() {
  static const int64_t v = [] {
    const char *e = std::getenv("ZS_PK_IDLE_US");
    return (int64_t)std::max(100LL, e ? std::atoll(e) : 2000LL);
  }();
  return v;
}

int64_t pk_life_ms() {
  static const int64_t v = [] {
    const char *e = std::getenv("ZS_PK_LIFE_MS");
    return (int64_t)std::max(1LL, e ? std::atoll(e) : 250LL);
  }();
  return v;
}

int64_t pk_now_ns() {
  return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Device buffers of ended streams that the pool did not take: hipFree
// synchronises the device, which with the persistent worker resident waits for
// the launch to end (up to ZS_PK_LIFE_MS).  stream_free defers them while a
// launch runs; they are freed before the next launch (the grid has drained).
std::vector<void *> g_defer_dev, g_defer_host;
void pk_defer_flush_locked() {
  for (void *p : g_defer_dev) (void)hipFree(p);
  for (void *p : g_defer_host) (void)hipHostFree(p);
  g_defer_dev.clear();
  g_defer_host.clear();
}

int pk_launch_locked() {
  const uint64_t idle_t = (uint64_t)pk_idle_us() * 100u;  // s_memrealtime ticks (100 MHz)
  const uint64_t life_t = (uint64_t)pk_life_ms() * 100000u;
  __atomic_store_n(&g_pk.h_ctl[2], 0u, __ATOMIC_SEQ_CST);  // the last launch's closing flag (it has drained)
  g_pk.launch_at.store(pk_now_ns());
  zs_launch_stream_pk(g_pk.d_mb, (uint32_t)g_pk.nw, g_pk.d_ctl, idle_t, life_t, g_pk.st);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(g_pk.ev, g_pk.st));
  g_pk.launched = true;
  g_pk.launches++;
  return 0;
}

// Relaunch the worker unless it runs (caller holds lk on g_pk.mu).  Device
// buffers deferred by stream_free are freed first -- the last launch has
// drained, so hipFree does not wait for it -- with the lock released, so that
// other handles' waiters do not queue behind the device-wide synchronisation;
// a launch another thread made meanwhile is taken as this one's.
int pk_relaunch(std::unique_lock<std::mutex> &lk) {
  if (pk_running_locked()) return 0;
  if (!g_defer_dev.empty() || !g_defer_host.empty()) {
    std::vector<void *> dv, hv;
    dv.swap(g_defer_dev);
    hv.swap(g_defer_host);
    lk.unlock();
    for (void *p : dv) (void)hipFree(p);
    for (void *p : hv) (void)hipHostFree(p);
    lk.lock();
    if (pk_running_locked()) return 0;
  }
  return pk_launch_locked();
}

void pk_detach(StreamState *s) {  // the handle's calls are all finished
  if (s->pk_w < 0) return;
  std::lock_guard<std::mutex> lk(g_pk.mu);
  g_pk.free_w.push_back(s->pk_w);
  s->pk_w = -1;
}

// the handle's mailbox (taken on first use), or -1: the batch path.  Once a
// launch has failed (g_pk.broken) a handle that still holds a mailbox gives it
// up, so its calls take the batch path like new handles' instead of retrying
// the launch on every call.
int pk_attach(StreamState *s) {
  if (s->pk_w >= 0) {
    if (!__atomic_load_n(&g_pk.broken, __ATOMIC_ACQUIRE)) return s->pk_w;
    pk_detach(s);
    return -1;
  }
  std::lock_guard<std::mutex> lk(g_pk.mu);
  if (pk_init_locked() || g_pk.broken || g_pk.free_w.empty()) return -1;
  s->pk_w = g_pk.free_w.back();
  g_pk.free_w.pop_back();
  return s->pk_w;
}

// A launch that fails after the call was posted: withdraw the call (seq_in
// back to the last finished one) and stop using the worker, so the mailbox
// never goes back to the free list with a call outstanding that a later
// launch would run against another handle's state.
int pk_fail_locked(ZsMbox *m, int w, int rc) {
  const uint32_t prev = __atomic_load_n(&m->seq_out, __ATOMIC_ACQUIRE);
  __atomic_store_n(&m->seq_in, prev, __ATOMIC_SEQ_CST);
  g_pk.seq[w] = prev;
  __atomic_store_n(&g_pk.broken, true, __ATOMIC_RELEASE);
  return rc;
}

int pk_submit(StreamCall *c, int w) {
  ZsMbox *m = g_pk.h_mb + w;
  m->st = c->s->d_st;
  m->io = c->io;
  m->job = c->jb;
  const uint32_t seq = ++g_pk.seq[w] ? g_pk.seq[w] : ++g_pk.seq[w];  // never 0 (the worker's "no call")
  __atomic_thread_fence(__ATOMIC_SEQ_CST);  // the call's fields before seq_in (also for write-combined mappings)
  __atomic_store_n(&m->seq_in, seq, __ATOMIC_SEQ_CST);
  __atomic_fetch_add(&g_pk.h_ctl[1], 1u, __ATOMIC_SEQ_CST);
  const int64_t t0 = pk_now_ns();
  // a post within half the idle time of the previous one finds the launch alive
  // (its workgroups saw that post and wait PK_IDLE after it); else look
  if (t0 - g_pk.last_post.exchange(t0) > pk_idle_us() * 500) {
    std::unique_lock<std::mutex> lk(g_pk.mu);
    if (int rc = pk_relaunch(lk)) return pk_fail_locked(m, w, rc);
  }
  // sleep through most of the expected call, then poll with short sleeps: many
  // handles' threads spinning would spend the host's CPU quota (a
  // cgroup-limited server throttles them for whole periods).  The expected
  // time is the handle's last call on the worker, scaled down when this call
  // has less input (a trailer or a 1 KiB call after a 4 MiB one finishes in
  // microseconds) but never up (a call that fills its output ends with input
  // left: scaling up by input overslept the JS schedule's calls, one handle
  // 254 -> 213 MiB/s), capped at 2 ms.  The waiting thread's timer slack drops
  // to 2 us for the wait, so the sleeps end on time, and is restored after it.
  const int prev_slack = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
  const bool slack = prev_slack >= 0 && prctl(PR_SET_TIMERSLACK, 2000UL, 0, 0, 0) == 0;
  const uint64_t last_in = std::max<uint64_t>(c->s->pk_last_in, 1);
  const uint64_t in_now = std::min<uint64_t>(std::max<uint64_t>(c->jb.in_len, 1), last_in);
  const int64_t expect = (int64_t)std::min<uint64_t>(c->s->pk_last_ns * in_now / last_in, 2000000u);
  if (expect > 80000) std::this_thread::sleep_for(std::chrono::nanoseconds(expect * 5 / 8));  // calls vary +-30%
  // the launch may have left (its life ended) before it saw the call: look
  // after three expected calls, then every 500 us -- and every 50 us once the
  // launch is past its life, when its workgroups leave after their current
  // calls and the posted calls wait for the relaunch (a waiter that looked only
  // on its own schedule left them waiting ~1 ms, tens under a kernel tracer)
  int64_t next_look = t0 + std::max<int64_t>(3 * expect, 500000);
  const int64_t life_ns = pk_life_ms() * 1000000;
  int64_t aged_look = t0 + 50000;
  for (;;) {
    if (__atomic_load_n(&m->seq_out, __ATOMIC_ACQUIRE) == seq) break;
    const int64_t now = pk_now_ns();
    const bool aged = now - g_pk.launch_at.load(std::memory_order_relaxed) > life_ns;
    if (now > next_look || (aged && now > aged_look)) {
      next_look = now + 500000;
      aged_look = now + 50000;
      std::unique_lock<std::mutex> lk(g_pk.mu);
      if (!pk_running_locked()) {
        if (__atomic_load_n(&m->seq_out, __ATOMIC_ACQUIRE) == seq) break;
        if (int rc = pk_relaunch(lk)) {
          if (slack) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)prev_slack, 0, 0, 0);
          return pk_fail_locked(m, w, rc);
        }
      }
    }
    std::this_thread::sleep_for(std::chrono::microseconds(now - t0 < 3 * std::max<int64_t>(expect, 100000) ? 6 : 25));
  }
  if (slack) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)prev_slack, 0, 0, 0);
  const uint64_t waited = (uint64_t)(pk_now_ns() - t0);
  const uint64_t busy = (uint64_t)__atomic_load_n(&m->busy, __ATOMIC_RELAXED) * 10u;
  // the next sleep follows the call's own time on the worker, not the wait: a
  // wait stretched by a relaunch would make every handle sleep long at once,
  // the worker would see no posts, leave idle, and the stretch would feed itself
  c->s->pk_last_ns = busy;
  c->s->pk_last_in = c->jb.in_len;
  ZsStreamRes r;
  std::memcpy(&r, (const void *)&m->res, sizeof(r));
  c->res = r;
  g_pk.calls.fetch_add(1);
  g_pk.busy_ns.fetch_add(busy);
  g_pk.wait_ns.fetch_add(waited);
  g_pk.idle_ns.fetch_add((uint64_t)__atomic_load_n(&m->idle, __ATOMIC_RELAXED) * 10u);
  return 0;
}

// Device / pinned resources of ended streams, kept for the next ones:
// hipMalloc, hipHostMalloc and stream creation cost up to milliseconds and
// serialise concurrent callers, and hipFree synchronises the device, so a
// server that opens and closes many streams reuses them instead.
struct StreamRes {
  ZsStreamDev *d_st;
  hipStream_t hs;
  uint8_t *d_in, *d_out, *h_in, *h_out, *dh_in, *dh_out;
  size_t cap_in, cap_out, cap_hin, cap_hout;
};
constexpr size_t STREAM_POOL_MAX = 1024;
constexpr size_t STREAM_POOL_BYTES = 64u << 20;  // larger buffers are freed, not kept
std::mutex g_pool_mu;
std::vector<StreamRes> g_pool;

void res_take(StreamState *s) {
  if (s->d_st) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (g_pool.empty()) return;
  const StreamRes r = g_pool.back();
  g_pool.pop_back();
  s->d_st = r.d_st;
  s->hs = r.hs;
  s->d_in = r.d_in;
  s->d_out = r.d_out;
  s->h_in = r.h_in;
  s->h_out = r.h_out;
  s->dh_in = r.dh_in;
  s->dh_out = r.dh_out;
  s->cap_in = r.cap_in;
  s->cap_out = r.cap_out;
  s->cap_hin = r.cap_hin;
  s->cap_hout = r.cap_hout;
}

bool res_give(StreamState *s) {  // true: s's resources went to the pool
  if (!s->d_st || !s->hs || s->cap_in + s->cap_out + s->cap_hin + s->cap_hout > STREAM_POOL_BYTES) return false;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (g_pool.size() >= STREAM_POOL_MAX) return false;
    g_pool.push_back({s->d_st, s->hs, s->d_in, s->d_out, s->h_in, s->h_out, s->dh_in, s->dh_out, s->cap_in, s->cap_out,
                      s->cap_hin, s->cap_hout});
  }
  s->d_st = nullptr;
  s->hs = nullptr;
  s->d_in = s->d_out = s->h_in = s->h_out = s->dh_in = s->dh_out = nullptr;
  s->cap_in = s->cap_out = s->cap_hin = s->cap_hout = 0;
  return true;
}

int stream_init(StreamState *s, int wbits) {
  ZsJobDev cfg{};
  if (!parse_wbits(wbits, &cfg)) return Z_STREAM_ERROR;
  res_take(s);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (ws_init()) return Z_STREAM_ERROR;
  }
  if (!s->hs) HIP_OK(hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking));
  if (!s->d_st && hipMalloc(&s->d_st, sizeof(ZsStreamDev)) != hipSuccess) {
    s->d_st = nullptr;
    set_err("stream: device state allocation failed");
    return Z_MEM_ERROR;
  }
  // the device state is set up by the first call (stream_state_init): no
  // copy or synchronisation here, which many handles opened at once serialise on
  const int mode0 = cfg.wrap == ZW_RAW ? ZSM_TYPE : ZSM_HEAD;
  StreamState keep = std::move(*s);
  *s = StreamState();
  s->d_st = keep.d_st;
  s->hs = keep.hs;
  s->d_in = keep.d_in;
  s->d_out = keep.d_out;
  s->cap_in = keep.cap_in;
  s->cap_out = keep.cap_out;
  s->h_in = keep.h_in;
  s->h_out = keep.h_out;
  s->cap_hin = keep.cap_hin;
  s->cap_hout = keep.cap_hout;
  s->dh_in = keep.dh_in;
  s->dh_out = keep.dh_out;
  s->pk_w = keep.pk_w;
  s->inited = 1;
  s->fresh = 1;
  s->wbits = wbits;
  s->cfg = cfg;
  s->mode = mode0;
  s->adler = (uint32_t)(cfg.wrap == ZW_RAW ? 0 : (cfg.wrap & 1));  // inflateResetKeep: strm->adler = wrap & 1
  return Z_OK;
}

void stream_free(StreamState *s) {
  pk_detach(s);
  if (s->hs) (void)hipStreamSynchronize(s->hs);
  if (res_give(s)) return;
  {
    std::lock_guard<std::mutex> lk(g_pk.mu);
    if (pk_running_locked()) {  // a free now would wait for the worker's launch to end: defer
      for (void *p : {(void *)s->d_st, (void *)s->d_in, (void *)s->d_out})
        if (p) g_defer_dev.push_back(p);
      for (void *p : {(void *)s->h_in, (void *)s->h_out})
        if (p) g_defer_host.push_back(p);
      s->d_st = nullptr;
      s->d_in = s->d_out = s->h_in = s->h_out = nullptr;
    } else {
      pk_defer_flush_locked();
    }
  }
  if (s->d_st) (void)hipFree(s->d_st);
  if (s->d_in) (void)hipFree(s->d_in);
  if (s->d_out) (void)hipFree(s->d_out);
  if (s->h_in) (void)hipHostFree(s->h_in);
  if (s->h_out) (void)hipHostFree(s->h_out);
  if (s->hs) (void)hipStreamDestroy(s->hs);
  s->h_in = s->h_out = nullptr;
  s->dh_in = s->dh_out = nullptr;
  s->cap_hin = s->cap_hout = 0;
  s->d_st = nullptr;
  s->d_in = s->d_out = nullptr;
  s->cap_in = s->cap_out = 0;
  s->hs = nullptr;
}

// Whole-stream attempt through the batch pipeline; true when it settled the call.
bool stream_fast(StreamState *s, const uint8_t *in, unsigned in_len, uint8_t *out, unsigned out_len, unsigned *consumed,
                 unsigned *produced, int *ret) {
  zs_job j{};
  j.in = in;
  j.in_len = in_len;
  j.out = out;
  j.out_cap = out_len;
  j.window_bits = s->wbits;
  zs_result r;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (batch_locked(&j, 1, &r, 0) || (r.ret != Z_STREAM_END && r.ret != Z_DATA_ERROR)) return false;
  }
  *consumed = (unsigned)r.total_in;
  *produced = (unsigned)r.total_out;
  *ret = r.ret;
  s->mode = r.ret == Z_STREAM_END ? ZSM_DONE : ZSM_BAD;
  s->msg = r.msg;
  if (s->cfg.wrap != ZW_RAW) s->adler = r.adler;
  // the device state is left behind: DONE / BAD never launch again
  return true;
}

// One zlib inflate(strm, flush) call.  *need_dict: Z_NEED_DICT returns before
// inf_leave, so total_in is not advanced (src/inflate.c:1325-1328).
int stream_call(StreamState *s, const uint8_t *in, unsigned in_len, uint8_t *out, unsigned out_len, int flush,
                unsigned *consumed, unsigned *produced) {
  *consumed = 0;
  *produced = 0;
  if (s->mode == ZSM_DONE) return Z_STREAM_END;
  if (s->mode == ZSM_BAD) return Z_DATA_ERROR;
  if (s->mode == ZSM_DICT) return Z_NEED_DICT;
  int fret;
  if (s->total_in == 0 && s->total_out == 0 && s->carry.empty() && in_len >= stream_fast_min() &&
      stream_fast(s, in, in_len, out, out_len, consumed, produced, &fret)) {
    s->total_in += *consumed;
    s->total_out += *produced;
    return fret;
  }
  const hipStream_t hs = s->hs;
  ZsStreamRes h{};
  size_t off = 0;
  uint64_t cons = 0, prod = 0;
  for (;;) {
    const size_t take = std::min<size_t>(in_len - off, STREAM_SLICE);
    const size_t clen = s->carry.size();
    const size_t blen = clen + take;
    if (ws_reserve_bytes(&s->d_in, &s->cap_in, std::max<size_t>(blen, 64)) ||
        ws_reserve_bytes(&s->d_out, &s->cap_out, std::max<size_t>((size_t)out_len - prod, 64))) {
      set_err("stream: device buffer allocation failed");
      return Z_MEM_ERROR;
    }
    // host-mapped staging both ways (the batch's kernels pull the input and
    // push the output: no copy or sync of the call's own), else DMA
    const size_t ocap = (size_t)out_len - prod;
    uint8_t *hmi = stage_mapped(&s->h_in, &s->cap_hin, &s->dh_in, std::max<size_t>(blen, 1));
    uint8_t *hmo = hmi ? stage_mapped(&s->h_out, &s->cap_hout, &s->dh_out, std::max<size_t>(ocap, 1)) : nullptr;
    const bool mapped = hmi && hmo;
    if (mapped) {
      if (clen) std::memcpy(hmi, s->carry.data(), clen);
      if (take) std::memcpy(hmi + clen, in + off, take);
    } else {
      if (uint8_t *hb = stage_buf(&s->h_in, &s->cap_hin, blen, &s->dh_in)) {  // one DMA from pinned staging
        if (clen) std::memcpy(hb, s->carry.data(), clen);
        if (take) std::memcpy(hb + clen, in + off, take);
        if (blen) HIP_OK(hipMemcpyAsync(s->d_in, hb, blen, hipMemcpyHostToDevice, hs));
      } else {
        if (clen) HIP_OK(hipMemcpyAsync(s->d_in, s->carry.data(), clen, hipMemcpyHostToDevice, hs));
        if (take) HIP_OK(hipMemcpyAsync(s->d_in + clen, in + off, take, hipMemcpyHostToDevice, hs));
      }
      HIP_OK(hipStreamSynchronize(hs));
    }
    StreamCall c;
    c.io.hin = mapped ? s->dh_in : nullptr;
    c.io.hout = mapped ? s->dh_out : nullptr;
    c.io.rbit = s->carry_bit;
    c.io.fresh = (uint32_t)s->fresh;
    c.s = s;
    c.jb = s->cfg;
    c.jb.in = s->d_in;
    c.jb.in_len = blen;
    c.jb.out = s->d_out;
    c.jb.out_cap = (uint64_t)out_len - prod;
    c.run_header = s->mode == ZSM_HEAD;
    const int pw = (mapped && !c.run_header && !s->cfg.d64 && pk_enabled()) ? pk_attach(s) : -1;
    if (int rc = pw >= 0 ? pk_submit(&c, pw) : sq_submit(&c)) return rc;
    s->fresh = 0;
    h = c.res;
    if (h.produced && mapped) {
      std::memcpy(out + prod, hmo, h.produced);
    } else if (h.produced) {
      uint8_t *hb = stage_buf(&s->h_out, &s->cap_hout, h.produced, &s->dh_out);
      HIP_OK(hipMemcpyAsync(hb ? hb : out + prod, s->d_out, h.produced, hipMemcpyDeviceToHost, hs));
      HIP_OK(hipStreamSynchronize(hs));
      if (hb) std::memcpy(out + prod, hb, h.produced);
    }
    prod += h.produced;
    s->mode = h.mode;
    if (h.is_gzip >= 0) s->adler = h.check;
    if (h.code == ZD_TRUNC) {
      // everything offered is pulled; keep the element in progress
      cons += take;
      const size_t rb = h.rbit >> 3;
      std::vector<uint8_t> nc;
      nc.reserve(blen - std::min(rb, blen));
      if (rb < clen) nc.insert(nc.end(), s->carry.begin() + rb, s->carry.end());
      const size_t from = rb > clen ? rb - clen : 0;
      nc.insert(nc.end(), in + off + from, in + off + take);
      s->carry.swap(nc);
      s->carry_bit = h.rbit & 7u;
      off += take;
      if (off < in_len && prod < out_len) continue;
      break;
    }
    const size_t pulled = (h.stop_bits + 7u) >> 3;
    cons += pulled > clen ? pulled - clen : 0;
    if (h.code == ZD_FULL) {
      // resume at rbit (== stop_bits): keep its partial byte
      const size_t rb = h.rbit >> 3;
      std::vector<uint8_t> nc;
      for (size_t k = rb; k < pulled; k++) nc.push_back(k < clen ? s->carry[k] : in[off + (k - clen)]);
      s->carry.swap(nc);
      s->carry_bit = h.rbit & 7u;
    } else {
      s->carry.clear();
      s->carry_bit = 0;
    }
    break;
  }
  *consumed = (unsigned)cons;
  *produced = (unsigned)prod;
  s->total_out += prod;
  if (h.code == ZD_NEED_DICT) {
    s->adler = h.check;
    return Z_NEED_DICT;
  }
  s->total_in += cons;
  if (h.code == ZD_ERROR) {
    s->msg = (h.msg > 0 && h.msg < ZM_COUNT) ? kMsgs[h.msg] : nullptr;
    return Z_DATA_ERROR;
  }
  if (s->mode == ZSM_DONE) return Z_STREAM_END;
  if ((cons == 0 && prod == 0) || flush == Z_FINISH) return Z_BUF_ERROR;
  return Z_OK;
}


struct Handle {
  z_stream strm;  // layout parity with the reference context (unused fields)
  StreamState st;
  unsigned last_consumed = 0;
};

uintptr_t handle_new() {
  Handle *h = new (std::nothrow) Handle();
  if (!h) return 0;
  std::memset(&h->strm, 0, sizeof h->strm);
  return reinterpret_cast<uintptr_t>(h);
}
int handle_init(uintptr_t hp, int wbits) {
  Handle *h = reinterpret_cast<Handle *>(hp);
  if (!h) return Z_STREAM_ERROR;
  return stream_init(&h->st, wbits);
}
int handle_process(uintptr_t hp, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush) {
  Handle *h = reinterpret_cast<Handle *>(hp);
  if (!h || !h->st.inited) return (int)((unsigned)(Z_STREAM_ERROR & 0xff) << 24);
  unsigned cons = 0, prod = 0;
  int ret = stream_call(&h->st, reinterpret_cast<const uint8_t *>(in_ptr), in_len, reinterpret_cast<uint8_t *>(out_ptr),
                        out_len, flush, &cons, &prod);
  h->last_consumed = cons;
  return (int)((prod & 0x00ffffffu) | ((unsigned)(ret & 0xff) << 24));
}
int handle_end(uintptr_t hp) {
  Handle *h = reinterpret_cast<Handle *>(hp);
  if (!h) return Z_STREAM_ERROR;
  stream_free(&h->st);
  delete h;
  return Z_OK;
}
unsigned handle_last_consumed(uintptr_t hp) {
  Handle *h = reinterpret_cast<Handle *>(hp);
  return h ? h->last_consumed : 0;
}


// ---------------------------------------------------------------------------
// GPU deflate (deflate_kernels.hip): batch of whole streams
// ---------------------------------------------------------------------------
constexpr uint64_t DZ_SEG_HOST = 65536;   // must match DZ_SEG
constexpr uint64_t DZ_OUTW_HOST = 18440;  // must match DZ_OUTW
constexpr uint64_t DZ_AUXW_HOST = 320 + 320 + 192 + 2400;  // must match DZ_AUXW

struct DzWorkspace {
  size_t cap_jobs = 0, cap_segs = 0, cap_tok = 0, cap_obuf = 0, cap_stage = 0, cap_in = 0;
  ZsDJobDev *d_jobs = nullptr, *h_jobs = nullptr;
  ZsDSegDev *d_segs = nullptr, *h_segs = nullptr;
  uint16_t *d_tok = nullptr;  // distance - 1 per position
  uint32_t *d_obuf = nullptr, *d_bm = nullptr, *d_aux = nullptr;
  uint8_t *d_len8 = nullptr;
  uint16_t *d_lx16 = nullptr;  // deflate64 merged-run lengths (batches with deflate64 jobs)
  size_t cap_bm = 0, cap_len8 = 0, cap_aux = 0, cap_lx16 = 0;
  uint8_t *d_stage = nullptr, *d_in = nullptr;
  hipEvent_t ev[5] = {};
  double stage_ms[4] = {};
  double ms = 0.0;
  uint64_t launches = 0;
};
DzWorkspace g_dz;

// zlib-identical deflate (deflate_zlib.hip): per position, per bitmap word,
// per work item, per block
constexpr uint64_t ZD_S1_HOST = 131072, ZD_S2_HOST = 8192, ZD_BLOCK_HOST = 16383, ZD_AUX_HOST = 352;
// jobs up to this size (stream segments, small buffers) take short prev items
constexpr uint64_t ZD_S1S_HOST = 8192, ZD_S2S_HOST = 2048, ZD_SMALL_JOB_HOST = 4ull << 20;
// search items of zs_zd_msearch_kernel.  ZS_ZD_MATCH (read per batch, for
// tests and A/B): unset = small jobs zs_zd_match_kernel, large ones
// zs_zd_msearch_kernel; "all" = every job zs_zd_match_kernel (every position,
// both budgets: the round-2 search); "demand" = every job
// zs_zd_msearch_kernel; "none" = no search kernel (every search on demand in
// the parse: zd_search_g, the fallback path)
constexpr uint64_t ZD_S3_HOST = 16384;
enum { ZD_M_AUTO = 0, ZD_M_ALL = 1, ZD_M_DEMAND = 2, ZD_M_NONE = 3 };
static int zd_match_mode() {
  const char *e = getenv("ZS_ZD_MATCH");
  if (!e) return ZD_M_AUTO;
  return !strcmp(e, "all") ? ZD_M_ALL : !strcmp(e, "demand") ? ZD_M_DEMAND : !strcmp(e, "none") ? ZD_M_NONE : ZD_M_AUTO;
}
constexpr uint32_t ZD_STATE_A_HOST = 2u << 1;  // deflate_slow state A (deflate_zlib.hip ZD_STATE_A)
struct ZdWorkspace {
  size_t cap_pos = 0, cap_bm = 0, cap_w1 = 0, cap_w1s = 0, cap_w2 = 0, cap_w3 = 0, cap_blk = 0;
  uint16_t *d_prevd = nullptr;
  uint32_t *d_ma = nullptr, *d_mb = nullptr, *d_bm = nullptr, *d_aux = nullptr, *d_slot_job = nullptr, *d_flag = nullptr;
  ZsZWorkDev *d_w1 = nullptr, *d_w1s = nullptr, *d_w2 = nullptr, *d_w3 = nullptr;
  ZsZBlkDev *d_blks = nullptr;
  hipEvent_t ev[4] = {};
};
ZdWorkspace g_zd;
uint64_t zd_bm_words(uint64_t L) { return (L + 32) / 32 + 1; }

// deflateInit2 windowBits as zlib 1.2.11 deflate.c checks them: 9..15 zlib,
// -9..-15 raw, 25..31 gzip; 8 only with the zlib wrapper, where it becomes 9
bool parse_dz_wbits(int wb, int *wrap, uint32_t *w) {
  int x = wb;
  if (x < 0) {
    *wrap = 0;
    x = -x;
  } else if (x > 15) {
    *wrap = 2;
    x -= 16;
  } else {
    *wrap = 1;
  }
  if (x < 8 || x > 15 || (x == 8 && *wrap != 1)) return false;
  *w = x == 8 ? 9u : (uint32_t)x;
  return true;
}

uint64_t dz_bound(uint64_t in_len, int wrap) {
  const uint64_t nseg = std::max<uint64_t>(1, (in_len + DZ_SEG_HOST - 1) / DZ_SEG_HOST);
  return in_len + in_len / 8 + nseg * 16 + 64 + (wrap == 2 ? 18 : 6);
}

template <typename T>
int dz_grow(T **p, size_t *cap, size_t need) {
  if (need <= *cap) return 0;
  const size_t c = std::max(need, *cap + *cap / 4);
  int r = grow_dev(p, c);
  if (r) return r;
  *cap = c;
  return 0;
}

// The zlib-identical jobs of the batch in g_dz.h_jobs[0..nv) (exact = 1): lay
// out their position arrays, bitmaps, work items and block slots, then run
// deflate_zlib.hip after the fast pipeline (whose check kernel computed their
// CRC-32 / Adler-32 pieces).
struct ZdHist {  // a deflate_fast job's insertion bits for its history [0, pstart)
  uint64_t word0;  // first word of the job's I bitmap
  const uint32_t *bits;
  size_t nwords;
};
struct ZdPlan {
  std::vector<ZsZWorkDev> w1, w1s, w2, w3;  // w1s: short prev items of small jobs (zs_zd_prev_small_kernel); w2 / w3: zs_zd_match_kernel / zs_zd_msearch_kernel items
  std::vector<uint32_t> slot_job;
  std::vector<ZdHist> hist;
  size_t pos = 0, bmw = 0;
  uint32_t nex = 0, nslow = 0, nfast = 0, max_regions = 0;  // max_regions: over the deflate_slow jobs
  int mmode = ZD_M_AUTO;
} g_zdp;

// before the jobs are uploaded: position arrays, bitmaps, block slots of the
// zlib-identical jobs
void zd_plan(uint32_t nv) {
  ZdPlan &P = g_zdp;
  P = ZdPlan();
  P.mmode = zd_match_mode();
  for (uint32_t k = 0; k < nv; k++) {
    ZsDJobDev &jd = g_dz.h_jobs[k];
    if (!jd.exact) continue;
    P.nex++;
    const uint64_t L = jd.in_len;
    jd.pos0 = P.pos;
    P.pos += (L + 64) & ~uint64_t(63);
    jd.bm0 = P.bmw;
    P.bmw += 6 * zd_bm_words(L) + 4;  // S, V, M, I, A, B
    if (jd.exact == ZD_FAST) {  // deflate_fast searches inside its own kernel
      P.nfast++;
    } else {
      P.nslow++;
      P.max_regions = std::max(P.max_regions, jd.nseg);
      const bool small = L <= ZD_SMALL_JOB_HOST;
      if (small)
        for (uint64_t a = 0; a < L; a += ZD_S1S_HOST) P.w1s.push_back({k, (uint32_t)std::min<uint64_t>(ZD_S1S_HOST, L - a), a});
      else
        for (uint64_t a = 0; a < L; a += ZD_S1_HOST) P.w1.push_back({k, (uint32_t)std::min<uint64_t>(ZD_S1_HOST, L - a), a});
      // large jobs: the demand-driven search (zs_zd_msearch_kernel); small
      // jobs (stream segments, where one call's latency is the rate) and
      // ZS_ZD_MATCH=all: every position in short items (zs_zd_match_kernel),
      // which spreads a small job over many workgroups
      if (P.mmode == ZD_M_NONE) {
        // no search items: the A / B bitmaps stay 0
      } else if (P.mmode == ZD_M_ALL || (small && P.mmode != ZD_M_DEMAND)) {
        const uint64_t s2 = small ? ZD_S2S_HOST : ZD_S2_HOST;
        for (uint64_t a = 0; a < L; a += s2) P.w2.push_back({k, (uint32_t)std::min<uint64_t>(s2, L - a), a});
      } else {
        for (uint64_t a = 0; a < L; a += ZD_S3_HOST) P.w3.push_back({k, (uint32_t)std::min<uint64_t>(ZD_S3_HOST, L - a), a});
      }
    }
    jd.zblk0 = (uint32_t)P.slot_job.size();
    jd.zblk_cap = (uint32_t)((L + ZD_BLOCK_HOST - 1) / ZD_BLOCK_HOST + 1);
    for (uint32_t b = 0; b < jd.zblk_cap; b++) P.slot_job.push_back(k);
  }
}

int zd_run(uint32_t nv, size_t nseg, hipStream_t st) {
  ZdPlan &P = g_zdp;
  std::vector<ZsZWorkDev> &w1 = P.w1, &w1s = P.w1s, &w2 = P.w2, &w3 = P.w3;
  std::vector<uint32_t> &slot_job = P.slot_job;
  const size_t pos = P.pos, bmw = P.bmw;
  const uint32_t nex = P.nex;
  if (!nex) return 0;
  int r;
  auto grow = [&](auto **p, size_t *cap, size_t need) -> int {
    if (need <= *cap) return 0;
    const size_t c = std::max(need, *cap + *cap / 4);
    *cap = 0;
    int rr = grow_dev(p, c);
    if (!rr) *cap = c;
    return rr;
  };
  size_t cpos = g_zd.cap_pos;
  if (pos + 64 > g_zd.cap_pos) {
    size_t dummy = 0;
    g_zd.cap_pos = 0;
    if ((r = grow(&g_zd.d_prevd, &dummy, pos + 64)) || (dummy = 0, r = grow(&g_zd.d_ma, &dummy, pos + 64)) ||
        (dummy = 0, r = grow(&g_zd.d_mb, &dummy, pos + 64)))
      return r;
    g_zd.cap_pos = pos + 64;
  }
  (void)cpos;
  if ((r = grow(&g_zd.d_bm, &g_zd.cap_bm, bmw + 16)) || (r = grow(&g_zd.d_w1, &g_zd.cap_w1, w1.size() + 1)) ||
      (r = grow(&g_zd.d_w1s, &g_zd.cap_w1s, w1s.size() + 1)) ||
      (r = grow(&g_zd.d_w2, &g_zd.cap_w2, w2.size() + 1)) || (r = grow(&g_zd.d_w3, &g_zd.cap_w3, w3.size() + 1)))
    return r;
  if (slot_job.size() > g_zd.cap_blk) {
    const size_t c = std::max(slot_job.size(), g_zd.cap_blk + g_zd.cap_blk / 4);
    g_zd.cap_blk = 0;
    if ((r = grow_dev(&g_zd.d_blks, c)) || (r = grow_dev(&g_zd.d_slot_job, c)) || (r = grow_dev(&g_zd.d_aux, c * ZD_AUX_HOST)))
      return r;
    g_zd.cap_blk = c;
  }
  if (!g_zd.d_flag && (r = grow_dev(&g_zd.d_flag, 4))) return r;
  // bitmaps start zeroed (the parse writes whole region words; a region's
  // tail word and the words past the input stay 0)
  HIP_OK(hipMemsetAsync(g_zd.d_bm, 0, (bmw + 16) * sizeof(uint32_t), st));
  for (const ZdHist &h : P.hist)
    if (h.nwords)
      HIP_OK(hipMemcpyAsync(g_zd.d_bm + h.word0, h.bits, h.nwords * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  if (!w1.empty()) HIP_OK(hipMemcpyAsync(g_zd.d_w1, w1.data(), w1.size() * sizeof(ZsZWorkDev), hipMemcpyHostToDevice, st));
  if (!w1s.empty())
    HIP_OK(hipMemcpyAsync(g_zd.d_w1s, w1s.data(), w1s.size() * sizeof(ZsZWorkDev), hipMemcpyHostToDevice, st));
  if (!w2.empty()) HIP_OK(hipMemcpyAsync(g_zd.d_w2, w2.data(), w2.size() * sizeof(ZsZWorkDev), hipMemcpyHostToDevice, st));
  if (!w3.empty()) HIP_OK(hipMemcpyAsync(g_zd.d_w3, w3.data(), w3.size() * sizeof(ZsZWorkDev), hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(g_zd.d_slot_job, slot_job.data(), slot_job.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  hipEvent_t *ev = nullptr;
  if (g_ws.prof) {
    if (!g_zd.ev[0])
      for (int i = 0; i < 4; i++) HIP_OK(hipEventCreate(&g_zd.ev[i]));
    ev = g_zd.ev;
  }
  if (zs_launch_zdeflate(g_dz.d_jobs, nv, g_dz.d_segs, (uint32_t)nseg, g_zd.d_w1, (uint32_t)w1.size(), g_zd.d_w1s,
                         (uint32_t)w1s.size(), g_zd.d_w2,
                         (uint32_t)w2.size(), g_zd.d_w3, (uint32_t)w3.size(), g_zd.d_prevd, g_zd.d_ma, g_zd.d_mb, g_zd.d_bm, g_zd.d_blks,
                         (uint32_t)slot_job.size(), g_zd.d_slot_job, g_zd.d_aux, g_dz.d_stage, g_zd.d_flag, P.nslow != 0,
                         P.nfast != 0, P.max_regions, st, ev)) {
    set_err("zlib-identical deflate: fix-up round failed");
    return ZS_ENODEV;
  }
  zs_launch_dz_trailer(g_dz.d_jobs, nv, g_dz.d_stage, st);
  if (ev) {
    HIP_OK(hipStreamSynchronize(st));
    float a = 0, b = 0, c = 0;
    HIP_OK(hipEventElapsedTime(&a, ev[0], ev[1]));
    HIP_OK(hipEventElapsedTime(&b, ev[1], ev[2]));
    HIP_OK(hipEventElapsedTime(&c, ev[2], ev[3]));
    g_dz.stage_ms[0] += a;
    g_dz.stage_ms[1] += b;
    g_dz.stage_ms[2] += c;
    g_dz.ms += a + b + c;
  }
  return 0;
}

// One deflate job as the kernels see it (the batch API's zs_djob + flags, or a
// segment of a stream surface).
struct DzSpec {
  const void *in = nullptr;
  uint64_t in_len = 0;
  void *out = nullptr;     // nullptr: keep the bytes in the staging area (stream segments copy them out)
  uint64_t out_cap = 0;
  int32_t window_bits = -15;
  int32_t level = 6;
  bool fast = false;       // ZS_F_DEFLATE_FAST
  uint32_t term = ZS_DT_FINAL, hdr = 1, trl = 1, bit0 = 0, pstate = ZD_STATE_A_HOST;
  uint64_t pstart = 0, skip = 0, abs0 = 0, ck0 = 0;
  // stream segments: zlib's pull-on-demand (ZsDJobDev lim_bytes / zb / rd0 / rtop)
  uint64_t lim_bytes = ~0ull, zb = 0, rd0 = ~0ull, rtop = ~0ull;
  // levels 1..3 (deflate_fast): which history positions [0, pstart) zlib had
  // inserted into its hash chains (bit q of word q / 32), and whether to
  // return the bits of the window before the next segment's entry
  const uint32_t *ins = nullptr;
  size_t ins_words = 0;
  bool want_ins = false;
  std::vector<uint32_t> ins_out;  // words [ins_w0, ...) of the job's insertion bits
  uint64_t ins_w0 = 0;
  // results
  int ret = Z_STREAM_ERROR;
  uint64_t total_out = 0, endbit = 0, stage = 0;
  uint32_t check = 0;
  uint64_t cut_pos = 0, cut_skip = 0, cut_open = 0;
  uint32_t cut_state = 0;
  bool early = false;  // deflate() returned after a block flush filled the output (the job ends as a cut)
  uint64_t rd_out = 0, zb_out = 0, next_top = 0;
};

int dz_run(DzSpec *sp, uint32_t n, bool dev) {
  int r = ws_init();
  if (r) return r;
  if (n > g_dz.cap_jobs) {
    const size_t c = std::max<size_t>(n, 2 * g_dz.cap_jobs);
    if ((r = grow_dev(&g_dz.d_jobs, c)) || (r = grow_host(&g_dz.h_jobs, c))) return r;
    g_dz.cap_jobs = c;
  }
  std::vector<uint32_t> slot(n, UINT32_MAX);
  std::vector<size_t> in_off(n, 0);
  size_t nseg = 0, stage_total = 0, in_total = 0;
  uint32_t nv = 0;
  for (uint32_t i = 0; i < n; i++) {
    DzSpec &s = sp[i];
    int wrap = 0;
    uint32_t w = 15;
    const int level = s.level == Z_DEFAULT_COMPRESSION ? 6 : s.level;
    // -16: raw deflate64 (64 KiB window, code 285 runs; a batch-API extension,
    // the reference has no deflate64 compressor)
    const bool d64 = s.window_bits == -16;
    if (d64) w = 16;
    // zlib's bytes: deflate_slow (levels 4..9) or deflate_fast (1..3); level 0
    // is deflate_stored's block grid on the throughput path
    const uint32_t exact = d64 || s.fast || level == 0 ? 0u : (level >= 4 ? ZD_SLOW : ZD_FAST);
    bool ok = (d64 || parse_dz_wbits(s.window_bits, &wrap, &w)) && level >= 0 && level <= 9 &&
              s.in_len < (1ull << 32) && (s.in || s.in_len == 0) && s.term <= ZS_DT_CUT && s.bit0 < 8 &&
              s.pstart <= s.in_len && s.ck0 <= s.in_len && (s.out || s.out_cap == 0);
    // history, a parse entry and a cut need the zlib-identical parse
    if (!exact && (s.pstart || s.skip || s.term == ZS_DT_CUT)) ok = false;
    if (!ok) {
      s.ret = Z_STREAM_ERROR;
      continue;
    }
    ZsDJobDev jd{};
    jd.in_len = s.in_len;
    jd.wrap = wrap;
    jd.level = level;
    jd.wbits = w;
    jd.exact = exact;
    jd.term = s.term;
    jd.hdr = s.hdr;
    jd.trl = s.trl;
    jd.bit0 = s.bit0;
    jd.pstart = s.pstart;
    jd.pstate = s.pstate;
    jd.skip = s.skip;
    jd.abs0 = s.abs0;
    jd.ck0 = s.ck0;
    jd.lim_bytes = s.lim_bytes;
    jd.zb = s.zb;
    jd.rd0 = s.rd0;
    jd.rtop = s.rtop;
    jd.seg0 = (uint32_t)nseg;
    jd.nseg = (uint32_t)std::max<uint64_t>(1, (jd.in_len + DZ_SEG_HOST - 1) / DZ_SEG_HOST);
    jd.stage = stage_total;
    stage_total += (dz_bound(jd.in_len, wrap) + 4095) & ~size_t(4095);
    nseg += jd.nseg;
    if (dev) {
      jd.in = static_cast<const uint8_t *>(s.in);
    } else {
      in_off[i] = in_total;
      in_total += (s.in_len + 15) & ~size_t(15);
    }
    slot[i] = nv;
    g_dz.h_jobs[nv++] = jd;
  }
  if (nv == 0) return 0;
  int has_std = 0, has_d64 = 0;
  for (uint32_t k = 0; k < nv; k++) (g_dz.h_jobs[k].wbits == 16 ? has_d64 : has_std) = 1;
  hipStream_t st = g_ws.stream;
  if (has_d64 && (r = dz_grow(&g_dz.d_lx16, &g_dz.cap_lx16, nseg * DZ_SEG_HOST))) return r;
  if (nseg > g_dz.cap_segs) {
    const size_t c = std::max(nseg, g_dz.cap_segs + g_dz.cap_segs / 2);
    if ((r = grow_dev(&g_dz.d_segs, c)) || (r = grow_host(&g_dz.h_segs, c))) return r;
    g_dz.cap_segs = c;
  }
  if ((r = dz_grow(&g_dz.d_tok, &g_dz.cap_tok, nseg * DZ_SEG_HOST)) ||
      (r = dz_grow(&g_dz.d_obuf, &g_dz.cap_obuf, nseg * DZ_OUTW_HOST)) ||
      (r = dz_grow(&g_dz.d_bm, &g_dz.cap_bm, nseg * (DZ_SEG_HOST / 32))) ||
      (r = dz_grow(&g_dz.d_len8, &g_dz.cap_len8, nseg * DZ_SEG_HOST)) ||
      (r = dz_grow(&g_dz.d_aux, &g_dz.cap_aux, nseg * DZ_AUXW_HOST)) ||
      (r = dz_grow(&g_dz.d_stage, &g_dz.cap_stage, stage_total)))
    return r;
  if (!dev) {
    if ((r = dz_grow(&g_dz.d_in, &g_dz.cap_in, in_total + 64))) return r;
    for (uint32_t i = 0; i < n; i++) {
      if (slot[i] == UINT32_MAX) continue;
      g_dz.h_jobs[slot[i]].in = g_dz.d_in + in_off[i];
      if (sp[i].in_len)
        HIP_OK(hipMemcpyAsync(g_dz.d_in + in_off[i], sp[i].in, sp[i].in_len, hipMemcpyHostToDevice, st));
    }
  }
  size_t si = 0;
  for (uint32_t k = 0; k < nv; k++) {
    const ZsDJobDev &jd = g_dz.h_jobs[k];
    for (uint32_t o = 0; o < jd.nseg; o++, si++) {
      ZsDSegDev sg{};
      sg.job = k;
      sg.last = o + 1 == jd.nseg && jd.term == ZS_DT_FINAL;
      sg.start = (uint64_t)o * DZ_SEG_HOST;
      sg.len = (uint32_t)std::min<uint64_t>(DZ_SEG_HOST, jd.in_len - std::min<uint64_t>(jd.in_len, sg.start));
      sg.tok = (uint64_t)si * DZ_SEG_HOST;
      sg.obuf = (uint64_t)si * DZ_OUTW_HOST * 4;
      g_dz.h_segs[si] = sg;
    }
  }
  HIP_OK(hipMemsetAsync(g_dz.d_stage, 0, stage_total, st));
  zd_plan(nv);
  for (uint32_t i = 0; i < n; i++) {
    if (slot[i] == UINT32_MAX) continue;
    const ZsDJobDev &jd = g_dz.h_jobs[slot[i]];
    if (jd.exact == ZD_FAST && jd.pstart && sp[i].ins)
      g_zdp.hist.push_back({jd.bm0 + 3 * zd_bm_words(jd.in_len), sp[i].ins,
                            std::min<size_t>(sp[i].ins_words, (size_t)((jd.pstart + 31) / 32))});
  }
  HIP_OK(hipMemcpyAsync(g_dz.d_jobs, g_dz.h_jobs, nv * sizeof(ZsDJobDev), hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(g_dz.d_segs, g_dz.h_segs, nseg * sizeof(ZsDSegDev), hipMemcpyHostToDevice, st));
  hipEvent_t *ev = nullptr;
  if (g_ws.prof) {
    if (!g_dz.ev[0])
      for (int i = 0; i < 5; i++) HIP_OK(hipEventCreate(&g_dz.ev[i]));
    ev = g_dz.ev;
  }
  zs_launch_deflate(g_dz.d_jobs, nv, g_dz.d_segs, (uint32_t)nseg, g_dz.d_tok, g_dz.d_len8, g_dz.d_bm, g_dz.d_aux, g_dz.d_obuf,
                    g_dz.d_stage, g_dz.d_lx16, has_std, has_d64, st, ev);
  if ((r = zd_run(nv, nseg, st))) return r;
  {
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) {
      set_err(std::string("kernel launch failed: ") + hipGetErrorString(le));
      return ZS_ENODEV;
    }
  }
  HIP_OK(hipMemcpyAsync(g_dz.h_jobs, g_dz.d_jobs, nv * sizeof(ZsDJobDev), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (ev) {
    float t = 0.f;
    HIP_OK(hipEventElapsedTime(&t, ev[0], ev[4]));
    g_dz.ms += t;
    for (int i = 0; i < 4; i++) {
      HIP_OK(hipEventElapsedTime(&t, ev[i], ev[i + 1]));
      g_dz.stage_ms[i] += t;
    }
    g_dz.launches++;
  }
  for (uint32_t i = 0; i < n; i++) {
    if (slot[i] == UINT32_MAX) continue;
    const ZsDJobDev &jd = g_dz.h_jobs[slot[i]];
    DzSpec &s = sp[i];
    s.total_out = jd.total_out;
    s.endbit = jd.endbit;
    s.stage = jd.stage;
    s.check = jd.check;
    s.cut_pos = jd.cut_pos;
    s.cut_state = jd.cut_state;
    s.cut_skip = jd.cut_skip;
    s.cut_open = jd.cut_open;
    s.early = jd.early != 0;
    s.rd_out = jd.rd_out;
    s.zb_out = jd.zb;
    s.next_top = jd.next_top;
    const uint64_t give = std::min<uint64_t>(jd.total_out, s.out_cap);
    if (give)
      HIP_OK(hipMemcpyAsync(s.out, g_dz.d_stage + jd.stage, give, dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
    s.ret = give == jd.total_out ? Z_STREAM_END : Z_OK;  // Z_OK: output space ran out (deflate(Z_FINISH) semantics)
    s.total_out = give;
    if (s.want_ins && jd.exact == ZD_FAST) {  // the insertion bits of the window before the next entry
      const uint64_t T = jd.term == ZS_DT_CUT ? jd.cut_pos : jd.in_len;
      const uint64_t a = T - std::min<uint64_t>(T, (uint64_t)1 << jd.wbits), w0 = a / 32, w1 = (T + 31) / 32;
      s.ins_w0 = w0;
      s.ins_out.assign((size_t)(w1 - w0), 0u);
      if (w1 > w0)
        HIP_OK(hipMemcpyAsync(s.ins_out.data(), g_zd.d_bm + jd.bm0 + 3 * zd_bm_words(jd.in_len) + w0,
                              (size_t)(w1 - w0) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    }
  }
  HIP_OK(hipStreamSynchronize(st));
  return 0;
}

int deflate_batch_locked(const zs_djob *jobs, uint32_t n, zs_result *results, uint32_t flags) {
  std::vector<DzSpec> sp(n);
  for (uint32_t i = 0; i < n; i++) {
    DzSpec &s = sp[i];
    s.in = jobs[i].in;
    s.in_len = jobs[i].in_len;
    s.out = jobs[i].out;
    s.out_cap = jobs[i].out_cap;
    s.window_bits = jobs[i].window_bits;
    s.level = jobs[i].level;
    s.fast = (flags & ZS_F_DEFLATE_FAST) != 0;
    s.term = (flags & ZS_F_DEFLATE_SYNC) ? ZS_DT_SYNC : ZS_DT_FINAL;
    s.trl = s.term == ZS_DT_FINAL;
  }
  const int r = dz_run(sp.data(), n, (flags & ZS_F_DEVICE) != 0);
  if (r) {
    for (uint32_t i = 0; i < n; i++) fill_result(&results[i], Z_STREAM_ERROR, nullptr);
    return r;
  }
  for (uint32_t i = 0; i < n; i++) {
    zs_result &res = results[i];
    std::memset(&res, 0, sizeof res);
    res.ret = sp[i].ret;
    if (res.ret == Z_STREAM_ERROR) continue;
    int wrap = 0;
    uint32_t w;
    parse_dz_wbits(jobs[i].window_bits, &wrap, &w);
    res.total_in = jobs[i].in_len;
    res.total_out = sp[i].total_out;
    res.adler = wrap ? sp[i].check : 1u;  // deflateResetKeep: adler32(0) for raw/zlib, crc32(0) for gzip
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Deflate stream surfaces (deflate_process, zlib deflate()): every call is
// zlib's deflate(strm, flush) -- the same bytes, produced by the same call.
//
// zlib's deflate_slow processes a loop top t only while the lookahead (input
// available past t) is >= MIN_LOOKAHEAD (262) unless the call flushes, and
// writes a block out as soon as its 16 383rd symbol is tallied.  A stream
// here is a sequence of GPU jobs over [history | unparsed input]: the last
// window of input before the parse position as history (zlib's window: its
// hash chains and match sources), the parse resuming in deflate_slow's exact
// state there, the symbols already sent skipped:
//   * Z_NO_FLUSH: a ZS_DT_CUT job sends exactly the blocks zlib completes with
//     the input so far, and names the next job's entry (an exact loop top and
//     state from the fix-up) -- no flush is ever injected;
//   * Z_SYNC_FLUSH / Z_FULL_FLUSH / Z_PARTIAL_FLUSH / Z_BLOCK: the job parses
//     to the end of the input as zlib does for a flush, ends its last block
//     non-final and writes the flush's terminator (empty stored block, empty
//     static block, nothing); the window carries over (Z_FULL_FLUSH restarts
//     it, as deflate.c's CLEAR_HASH + strstart = 0);
//   * Z_FINISH: the final block, then the trailer of the whole input (CRC-32 /
//     Adler-32 joined from the jobs' GPU checks).
// Bits past the last whole byte of a job wait for the next one (zlib keeps
// them in bi_buf).  The wrapper header is zlib's constant header, sent by the
// first call.  When a block flush fills the caller's output space, deflate()
// returns right there, having read only what fill_window had read (the GPU's
// read model, zs_zd_limit_kernel): the rest of the input is not consumed.
// Level 0 is zlib's deflate_stored call by call (ds_stored_call, below).
// Concurrent handles' jobs share launches.
// ---------------------------------------------------------------------------
constexpr uint32_t ZD_BLOCK_SYMS = 16383, ZD_LOOK_HOST = 262;

// a level-0 stream's call staging (ds_stored_call): pinned source / output and
// their device copies, its own HIP stream; kept across deflateReset-style inits
struct DsStage {
  hipStream_t hs = nullptr;
  uint8_t *h_src = nullptr, *h_dst = nullptr, *d_src = nullptr, *d_dst = nullptr;
  size_t cap_hsrc = 0, cap_hdst = 0, cap_dsrc = 0, cap_ddst = 0;
  DsStage() = default;
  DsStage(const DsStage &) = delete;
  DsStage &operator=(const DsStage &) = delete;
  DsStage &operator=(DsStage &&o) noexcept {
    std::swap(hs, o.hs);
    std::swap(h_src, o.h_src);
    std::swap(h_dst, o.h_dst);
    std::swap(d_src, o.d_src);
    std::swap(d_dst, o.d_dst);
    std::swap(cap_hsrc, o.cap_hsrc);
    std::swap(cap_hdst, o.cap_hdst);
    std::swap(cap_dsrc, o.cap_dsrc);
    std::swap(cap_ddst, o.cap_ddst);
    return *this;
  }
  ~DsStage() {
    if (hs) (void)hipStreamSynchronize(hs);
    if (h_src) (void)hipHostFree(h_src);
    if (h_dst) (void)hipHostFree(h_dst);
    if (d_src) (void)hipFree(d_src);
    if (d_dst) (void)hipFree(d_dst);
    if (hs) (void)hipStreamDestroy(hs);
  }
};

struct DStreamState {
  int inited = 0;
  int wbits = 15, level = 6, wrap = 0;
  uint32_t w = 15;             // window bits (zlib's wsize = 1 << w)
  bool exact = true;           // levels 1..9: zlib's bytes (deflate_fast 1..3, deflate_slow 4..9)
  std::vector<uint32_t> ins;   // levels 1..3: insertion bits of buf[0, hist) (zlib's hash chains)
  int status = 0;              // 0 no call yet, 1 busy, 2 finished (deflate.c INIT/BUSY/FINISH_STATE)
  int last_flush = -2;         // deflate.c s->last_flush (deflateResetKeep: -2)
  std::vector<uint8_t> buf;    // [history | unparsed input]
  size_t hist = 0;             // parse position in buf (bytes before it: history)
  uint64_t abs = 0;            // stream offset of buf[0] since the window last restarted
  uint32_t state = ZD_STATE_A_HOST;  // deflate_slow state at buf[hist]
  uint64_t skip = 0;           // symbols from buf[hist] already sent
  size_t ck_from = 0;          // buf[ck_from..) not yet in the running check
  size_t need = 16383 + 262;   // Z_NO_FLUSH: new bytes before a call can complete a block
  size_t fresh = 0;            // bytes added since the last job
  std::vector<uint8_t> out;    // output not yet served (from `served` on)
  size_t served = 0;
  uint64_t out_base = 0;       // stream offset of out[0]
  // the last flush job's terminator starts at stream offset `mark`: zlib
  // appends it in the call whose output reaches that byte, and a call with
  // the same flush after it ran out of space writes another (zlib.h: "avail_out
  // greater than six to avoid repeated flush markers")
  bool mark_valid = false;
  uint64_t mark = 0;
  uint8_t pend_byte = 0;       // bits of an unfinished last byte (zlib's bi_buf)
  uint32_t pend_bits = 0;
  uint32_t adler = 1;          // strm->adler: check of the input the jobs have covered
  uint64_t checked = 0;        // bytes in `adler`
  uint64_t total_in = 0;
  // level 0 (ds_stored_call): zlib's window positions strstart / block_start;
  // buf holds the window's bytes [block_start, strstart), read but not yet
  // framed; trl_done: the trailer is written (deflate.c negates s->wrap)
  size_t z_strstart = 0, z_block_start = 0;
  bool trl_done = false;
  // levels 1..9, zlib's reading (fill_window): its window start zb (stream
  // offset since the window restart) and, after a call that returned on a
  // full output, the loop top the next call resumes at (stream offset; NONE:
  // the next call fills at once)
  uint64_t zb = 0, rtop = UINT64_MAX;
  DsStage stage;
};

size_t dstream_run_min() {  // env ZS_DSTREAM_RUN_KB: Z_NO_FLUSH input gathered per job (default 0: every call)
  const char *e = std::getenv("ZS_DSTREAM_RUN_KB");
  return e ? (size_t)std::max<long long>(0, std::atoll(e)) << 10 : 0;
}

// checks of A || B from those of A and B (|B| = n2): CRC-32 by x^(8 n2) mod P
// (reflected), Adler-32 by a = a1 + a2 - 1, b = b1 + b2 + n2 (a1 - 1) mod 65521
uint32_t crc32_join(uint32_t c1, uint32_t c2, uint64_t n2) {
  uint32_t sq = 1u << 23, p = 1u << 31;  // x^8, and x^0
  for (uint64_t k = n2; k; k >>= 1) {
    if (k & 1) p = zs_gf2_mul(sq, p);
    sq = zs_gf2_mul(sq, sq);
  }
  return (c1 ? zs_gf2_mul(p, c1) : 0u) ^ c2;
}
uint32_t adler32_join(uint32_t x1, uint32_t x2, uint64_t n2) {
  const uint64_t M = 65521, a1 = x1 & 0xffffu, b1 = x1 >> 16, a2 = x2 & 0xffffu, b2 = x2 >> 16;
  const uint64_t a = (a1 + a2 + M - 1) % M;
  const uint64_t b = (b1 + b2 + (n2 % M) * ((a1 + M - 1) % M)) % M;
  return (uint32_t)(a | (b << 16));
}

void ds_put(DStreamState *s, const uint8_t *p, size_t n) {
  if (s->served == s->out.size()) {
    s->out_base += s->out.size();
    s->out.clear();
    s->served = 0;
  }
  s->out.insert(s->out.end(), p, p + n);
}

// zlib's wrapper header for (wrap, level), deflate.c (status INIT / GZIP)
void ds_header(DStreamState *s) {
  if (s->wrap == 2) {
    const uint8_t gz[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, (uint8_t)(s->level == 9 ? 2 : (s->level < 2 ? 4 : 0)), 3};
    ds_put(s, gz, 10);
  } else if (s->wrap == 1) {
    const uint32_t flevel = s->level < 2 ? 0u : (s->level < 6 ? 1u : (s->level == 6 ? 2u : 3u));
    uint32_t h = ((((s->w - 8u) << 4) | 8u) << 8) | (flevel << 6);
    h += 31u - (h % 31u);
    const uint8_t z[2] = {(uint8_t)(h >> 8), (uint8_t)h};
    ds_put(s, z, 2);
  }
}

// the job for the stream's next step: term as the call's flush asks
DzSpec ds_spec(const DStreamState *s, uint32_t term) {
  DzSpec j;
  j.in = s->buf.data();
  j.in_len = s->buf.size();
  j.window_bits = s->wbits;
  j.level = s->level;
  j.term = term;
  j.hdr = 0;
  j.trl = 0;
  j.bit0 = s->pend_bits;
  j.pstart = s->exact ? s->hist : 0;
  j.pstate = s->state;
  j.skip = s->skip;
  j.abs0 = s->abs;
  j.ck0 = s->ck_from;
  j.zb = s->zb;
  j.rtop = s->rtop == UINT64_MAX ? ~0ull : s->rtop - s->abs;
  if (s->exact && s->level <= 3) {
    j.ins = s->ins.data();
    j.ins_words = s->ins.size();
    j.want_ins = true;
  }
  return j;
}

// a finished job: its bytes into the output (the pending partial byte merged
// into its first byte, its own partial last byte kept back), the running
// check, and the next parse position (Z_FULL_FLUSH: full = true)
void ds_after(DStreamState *s, const DzSpec &j, const uint8_t *bytes, bool full) {
  const uint32_t term = j.term;
  uint64_t bits = j.endbit;  // blocks (and the pending bits) end here
  if (term == ZS_DT_PARTIAL) bits += 10;
  size_t nb = (size_t)j.total_out;
  std::vector<uint8_t> o(bytes, bytes + nb);
  if (s->pend_bits && !o.empty()) o[0] |= s->pend_byte;
  if (term == ZS_DT_PARTIAL || term == ZS_DT_BLOCK || term == ZS_DT_CUT) {
    const size_t whole = (size_t)(bits / 8);
    s->pend_bits = (uint32_t)(bits & 7u);
    s->pend_byte = s->pend_bits ? (uint8_t)(o[whole] & ((1u << s->pend_bits) - 1u)) : 0;
    o.resize(whole);
  } else {
    s->pend_bits = 0;
    s->pend_byte = 0;
  }
  const uint64_t n = s->buf.size() - s->ck_from;
  if (j.early) {
    // (ds_job checked what zlib read and cut buf there)
  } else if (s->wrap && n) {
    s->adler = s->checked == 0 ? j.check
                               : (s->wrap == 2 ? crc32_join(s->adler, j.check, n) : adler32_join(s->adler, j.check, n));
  }
  if (!j.early) s->checked += n;
  // zlib's reading: its window start after the call, and where it resumes
  s->zb = j.zb_out;
  s->rtop = j.early ? s->abs + j.next_top : UINT64_MAX;
  if (term == ZS_DT_FINAL && s->wrap) {  // the whole input's trailer
    const uint32_t c = s->adler, isz = (uint32_t)s->total_in;
    if (s->wrap == 2) {
      const uint8_t t8[8] = {(uint8_t)c, (uint8_t)(c >> 8), (uint8_t)(c >> 16), (uint8_t)(c >> 24),
                             (uint8_t)isz, (uint8_t)(isz >> 8), (uint8_t)(isz >> 16), (uint8_t)(isz >> 24)};
      o.insert(o.end(), t8, t8 + 8);
    } else {
      const uint8_t t4[4] = {(uint8_t)(c >> 24), (uint8_t)(c >> 16), (uint8_t)(c >> 8), (uint8_t)c};
      o.insert(o.end(), t4, t4 + 4);
    }
  }
  ds_put(s, nullptr, 0);
  s->mark_valid = term == ZS_DT_SYNC || term == ZS_DT_PARTIAL || term == ZS_DT_BLOCK;
  s->mark = s->out_base + s->out.size() + (size_t)(j.endbit / 8);  // the terminator's first byte
  ds_put(s, o.data(), o.size());
  // next parse position
  const size_t wsize = (size_t)1 << s->w;
  size_t T;
  if (term == ZS_DT_CUT) {
    T = (size_t)j.cut_pos;
    s->state = j.cut_state;
    s->skip = j.cut_skip;
    // new bytes before a call can complete the open block: each symbol it
    // still lacks starts at a distinct position past the last loop top zlib
    // processed, and needs the lookahead past it (after a call that returned on
    // a full output, zlib has read input it has not parsed: always a job)
    s->need = j.early ? 0 : (size_t)(ZD_BLOCK_SYMS - std::min<uint64_t>(ZD_BLOCK_SYMS, j.cut_open));
  } else {
    T = s->buf.size();
    s->state = ZD_STATE_A_HOST;
    s->skip = 0;
    s->need = ZD_BLOCK_SYMS + ZD_LOOK_HOST;
  }
  s->fresh = 0;
  s->ins.clear();
  if (full || !s->exact) {  // the window restarts (Z_FULL_FLUSH; level 0 always)
    s->buf.erase(s->buf.begin(), s->buf.begin() + (ptrdiff_t)T);
    s->hist = 0;
    s->abs = full ? 0 : s->abs + T;
    if (full) {  // deflate.c CLEAR_HASH, strstart = 0: the window starts over here
      s->zb = 0;
      s->rtop = UINT64_MAX;
    }
  } else {
    const size_t h = std::min(T, wsize);
    if (s->level <= 3) {  // deflate_fast: which window positions are in the hash chains
      s->ins.assign((h + 31) / 32, 0u);
      for (size_t i = 0; i < h; i++) {
        const uint64_t q = T - h + i, wi = q / 32 - j.ins_w0;
        if (wi < j.ins_out.size() && ((j.ins_out[(size_t)wi] >> (q & 31u)) & 1u)) s->ins[i / 32] |= 1u << (i & 31u);
      }
      // a flush leaves the last MIN_MATCH - 1 positions to the next fill_window
      // (deflate.c s->insert), which inserts them before any later search
      if (term != ZS_DT_CUT)
        for (size_t i = h - std::min<size_t>(h, 2); i < h; i++) s->ins[i / 32] |= 1u << (i & 31u);
    }
    s->buf.erase(s->buf.begin(), s->buf.begin() + (ptrdiff_t)(T - h));
    s->hist = h;
    s->abs += T - h;
  }
  s->ck_from = s->buf.size();  // every byte in buf is in the check now
}

// ---------------------------------------------------------------------------
// Deflate-call batching: a stream's job joins a queue; whichever caller finds
// no launch in flight runs every pending job (any handles, any flush) as ONE
// dz_run, so concurrent streams share launches (the pattern of sq_submit).
// ---------------------------------------------------------------------------
struct DzCall {
  DzSpec *spec = nullptr;
  int err = 0;
  std::string errmsg;
  bool done = false;
};
struct DzQueue {
  std::mutex mu;
  std::condition_variable cv, arrive;
  std::vector<DzCall *> pending;
  bool busy = false;
  size_t last_n = 0;
  uint64_t launches = 0, calls = 0;
} g_dq;

int dq_submit(DzCall *c) {
  std::unique_lock<std::mutex> lk(g_dq.mu);
  g_dq.pending.push_back(c);
  g_dq.arrive.notify_one();
  while (!c->done) {
    if (g_dq.busy) {
      g_dq.cv.wait(lk);
      continue;
    }
    g_dq.busy = true;
    if (g_dq.last_n > 1 && g_dq.pending.size() < g_dq.last_n) {  // gather the other active streams' next jobs
      const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(SQ_WAIT_US);
      for (;;) {
        const size_t had = g_dq.pending.size();
        const auto t = std::min(t_end, std::chrono::steady_clock::now() + std::chrono::microseconds(SQ_GAP_US));
        g_dq.arrive.wait_until(lk, t, [&] { return g_dq.pending.size() > had; });
        if (g_dq.pending.size() == had || g_dq.pending.size() >= g_dq.last_n || std::chrono::steady_clock::now() >= t_end)
          break;
      }
    }
    std::vector<DzCall *> batch(g_dq.pending.begin(), g_dq.pending.end());
    g_dq.pending.clear();
    g_dq.last_n = batch.size();
    lk.unlock();
    std::vector<DzSpec> specs(batch.size());
    for (size_t k = 0; k < batch.size(); k++) specs[k] = *batch[k]->spec;
    int rc;
    std::string msg;
    {
      std::lock_guard<std::mutex> g(g_mu);
      rc = dz_run(specs.data(), (uint32_t)specs.size(), false);
      if (rc) msg = g_err;
    }
    lk.lock();
    for (size_t k = 0; k < batch.size(); k++) {
      *batch[k]->spec = specs[k];
      batch[k]->err = rc;
      batch[k]->errmsg = msg;
      batch[k]->done = true;
    }
    g_dq.launches++;
    g_dq.calls += batch.size();
    g_dq.busy = false;
    g_dq.cv.notify_all();
  }
  if (c->err) set_err(c->errmsg);
  return c->err;
}

int ds_check_range(DStreamState *s, uint64_t lo, uint64_t hi);

// run the stream's next job (term) on the GPU and take its output.  rd0: buf
// offset where this call's input starts; room: output bytes of the job the
// call's output space takes.  When zlib's deflate() would have returned after
// a block flush filled that space (the job's `early`), it had read only up to
// rd_out: the rest of the call's input is given back (*dropped bytes).
int ds_job(DStreamState *s, uint32_t term, bool full, uint64_t rd0, uint64_t room, uint64_t *dropped) {
  *dropped = 0;
  DzSpec j = ds_spec(s, term);
  j.rd0 = rd0;
  j.lim_bytes = room;
  std::vector<uint8_t> bytes((size_t)dz_bound(s->buf.size(), s->wrap) + 64);
  j.out = bytes.data();
  j.out_cap = bytes.size();
  DzCall c;
  c.spec = &j;
  if (dq_submit(&c) || j.ret != Z_STREAM_END) return Z_STREAM_ERROR;
  if (j.early) {
    const uint64_t rd = std::min<uint64_t>(j.rd_out, s->buf.size());
    if (rd < s->ck_from || ds_check_range(s, s->ck_from, rd)) return Z_STREAM_ERROR;
    *dropped = s->buf.size() - rd;
    s->buf.resize((size_t)rd);
    s->total_in -= *dropped;
    s->fresh -= std::min<size_t>(s->fresh, *dropped);
    s->ck_from = (size_t)rd;
    j.term = ZS_DT_CUT;  // the job ends after its last flushed block
    full = false;
  }
  ds_after(s, j, bytes.data(), full);
  return Z_OK;
}

// zlib's reading during a Z_NO_FLUSH call that completes no block (no job):
// fill_window at the call's first loop top, then whenever the parse passes
// the read end - MIN_LOOKAHEAD, and a last attempt where the parse stops.
// Each slide is decided by where that loop top falls, known here only to
// within the longest gap between loop tops (258): false when that decides it
// either way (the call then runs a job, whose read model knows the loop tops).
bool ds_model_nojob(DStreamState *s, uint64_t rd, uint64_t end) {
  const uint64_t W = (uint64_t)1 << s->w, TH = 2 * W - ZD_LOOK_HOST;
  uint64_t zb = s->zb, lo = 0;
  auto decide = [&](uint64_t y) -> int { return y >= zb + TH ? 1 : (y + 258 < zb + TH ? 0 : -1); };
  if (s->rtop == UINT64_MAX) {
    rd = std::min(end, zb + 2 * W);
  } else {
    lo = s->rtop;
    if (rd - std::min(rd, s->rtop) < ZD_LOOK_HOST) {
      if (s->rtop >= zb + TH) zb += W;
      rd = std::min(end, zb + 2 * W);
    }
  }
  for (int guard = 0; guard < (1 << 20); guard++) {
    const uint64_t y = std::max(lo, rd >= ZD_LOOK_HOST - 1 ? rd - (ZD_LOOK_HOST - 1) : 0);
    const int d = decide(y);
    if (d < 0) return false;
    if (d) zb += W;
    if (rd >= end) break;
    rd = std::min(end, zb + 2 * W);
    lo = y + 1;
  }
  s->zb = zb;
  s->rtop = UINT64_MAX;
  return true;
}

size_t dstream_fast_max() {  // levels 0..3: input gathered per job (env ZS_DSTREAM_MAX_KB, default 64 MiB)
  const char *e = std::getenv("ZS_DSTREAM_MAX_KB");
  const long long kb = e ? std::atoll(e) : (64ll << 10);
  return (size_t)std::max<long long>(64, kb) << 10;
}

// ---------------------------------------------------------------------------
// Level 0: zlib's deflate() with deflate_stored (deflate.c, zlib 1.2.11), call
// by call.  Stored block lengths follow each call's avail_out and flush and
// zlib's window (strstart / block_start, slides of w_size): the host replays
// that arithmetic on positions only (StoredPlan: the call's output as stream
// byte ranges and header / marker bytes, in order) and the GPU writes the
// bytes and the check of the input the call reads (zs_stored_call_kernel).
// Output zlib leaves in its pending buffer waits in `out`, as for levels 1..9.
// ---------------------------------------------------------------------------
constexpr uint64_t ZS_MAX_STORED = 65535, ZS_PENDING_BUF = 65536;  // memLevel 8: lit_bufsize 16384 * 4

struct StoredPlan {
  struct Part {
    bool lit;      // header / marker bytes (lit[off, off + len)), else stream bytes at offset off
    uint64_t off;
    uint64_t len;
  };
  std::vector<Part> parts;
  std::vector<uint8_t> lit;
  uint64_t total = 0;
  void bytes(const uint8_t *p, size_t n) {
    parts.push_back({true, lit.size(), n});
    lit.insert(lit.end(), p, p + n);
    total += n;
  }
  void stream(uint64_t off, uint64_t n) {
    if (!n) return;
    parts.push_back({false, off, n});
    total += n;
  }
};

// _tr_stored_block's header (trees.c): 3 bits (last, type 00) after the pending
// bits, bi_windup, LEN, NLEN
void ds_stored_hdr(DStreamState *s, StoredPlan &P, uint32_t last, uint32_t len) {
  const uint32_t v = s->pend_byte | (last << s->pend_bits);
  uint8_t h[6];
  size_t n = 0;
  h[n++] = (uint8_t)v;
  if (s->pend_bits + 3 > 8) h[n++] = (uint8_t)(v >> 8);
  h[n++] = (uint8_t)len;
  h[n++] = (uint8_t)(len >> 8);
  h[n++] = (uint8_t)~len;
  h[n++] = (uint8_t)(~len >> 8);
  P.bytes(h, n);
  s->pend_bits = 0;
  s->pend_byte = 0;
}
// _tr_align (trees.c): an empty static block, 10 bits; whole bytes leave (bi_flush)
void ds_align(DStreamState *s, StoredPlan &P) {
  const uint32_t v = s->pend_byte | (2u << s->pend_bits), nb = s->pend_bits + 10;
  uint8_t h[3];
  const uint32_t whole = nb / 8;
  for (uint32_t k = 0; k < whole; k++) h[k] = (uint8_t)(v >> (8 * k));
  P.bytes(h, whole);
  s->pend_bits = nb % 8;
  s->pend_byte = (uint8_t)((v >> (8 * whole)) & ((1u << s->pend_bits) - 1u));
}

// deflate_stored (deflate.c): 0 need_more, 1 block_done, 2 finish_started, 3
// finish_done.  T0: stream offset of the call's input; *pos: input read so far;
// avail_out: caller space left; *pend: generated bytes not delivered yet.
int ds_stored_sim(DStreamState *s, StoredPlan &P, int flush, uint64_t T0, uint64_t in_len, uint64_t *pos,
                  uint64_t *avail_out, uint64_t *pend) {
  const uint64_t w_size = (uint64_t)1 << s->w, window_size = 2 * w_size;
  uint64_t &strstart = s->z_strstart, &block_start = s->z_block_start;
  auto avail_in = [&]() { return in_len - *pos; };
  auto flush_pending = [&]() {
    const uint64_t d = std::min(*pend, *avail_out);
    *pend -= d;
    *avail_out -= d;
  };
  // stream offset of window position i: the bytes before strstart are the last read
  auto wabs = [&](uint64_t i) { return T0 + *pos - strstart + i; };
  uint64_t min_block = std::min<uint64_t>(ZS_PENDING_BUF - 5, w_size);
  uint32_t last = 0;
  const uint64_t used0 = avail_in();
  do {
    uint64_t len = ZS_MAX_STORED;
    uint64_t have = (s->pend_bits + 42) >> 3;
    if (*avail_out < have) break;
    have = *avail_out - have;
    uint64_t left = strstart - block_start;
    if (len > left + avail_in()) len = left + avail_in();
    if (len > have) len = have;
    if (len < min_block && ((len == 0 && flush != Z_FINISH) || flush == Z_NO_FLUSH || len != left + avail_in())) break;
    last = flush == Z_FINISH && len == left + avail_in() ? 1u : 0u;
    const uint64_t g0 = P.total;
    ds_stored_hdr(s, P, last, (uint32_t)len);
    *pend += P.total - g0;
    flush_pending();  // the header fits: have >= its bytes
    if (left) {
      if (left > len) left = len;
      P.stream(wabs(block_start), left);
      *avail_out -= left;
      block_start += left;
      len -= left;
    }
    if (len) {  // read_buf straight to next_out
      P.stream(T0 + *pos, len);
      *avail_out -= len;
      *pos += len;
      // the window positions of bytes read this way are settled below
      strstart += len;
      block_start += len;
    }
  } while (last == 0);
  // undo the provisional strstart moves of the direct copies, then zlib's window update
  const uint64_t used = used0 - avail_in();
  strstart -= used;
  block_start -= used;
  if (used) {
    if (used >= w_size) {
      strstart = w_size;  // the window is the last w_size bytes read
    } else {
      if (window_size - strstart <= used) strstart -= w_size;  // slide
      strstart += used;
    }
    block_start = strstart;
  }
  if (last) return 3;
  if (flush != Z_NO_FLUSH && flush != Z_FINISH && avail_in() == 0 && strstart == block_start) return 1;
  // fill the window with the remaining input
  uint64_t have = window_size - strstart - 1;
  if (avail_in() > have && block_start >= w_size) {
    block_start -= w_size;
    strstart -= w_size;
    have += w_size;
  }
  if (have > avail_in()) have = avail_in();
  if (have) {
    *pos += have;
    strstart += have;
  }
  // a stored block from the window into the pending buffer
  have = (s->pend_bits + 42) >> 3;
  have = std::min<uint64_t>(ZS_PENDING_BUF - have, ZS_MAX_STORED);
  min_block = std::min<uint64_t>(have, w_size);
  const uint64_t left = strstart - block_start;
  if (left >= min_block ||
      ((left || flush == Z_FINISH) && flush != Z_NO_FLUSH && avail_in() == 0 && left <= have)) {
    const uint64_t len = std::min(left, have);
    last = flush == Z_FINISH && avail_in() == 0 && len == left ? 1u : 0u;
    const uint64_t g0 = P.total;
    ds_stored_hdr(s, P, last, (uint32_t)len);
    P.stream(wabs(block_start), len);
    *pend += P.total - g0;
    block_start += len;
    flush_pending();
  }
  return last ? 2 : 0;
}

template <typename T>
int ds_grow_pinned(T **p, size_t *cap, size_t need) {
  if (need <= *cap) return 0;
  const size_t c = std::max(need, *cap + *cap / 2);
  *cap = 0;
  int r = grow_host(p, c);
  if (!r) *cap = c;
  return r;
}

// run a plan on the GPU: the call's output bytes into `gen`, the check of
// in[0, n_in) into *check
int ds_stored_run(DStreamState *s, const StoredPlan &P, const uint8_t *in, uint64_t n_in, uint64_t T0,
                  std::vector<uint8_t> &gen, uint32_t *check) {
  DsStage &g = s->stage;
  if (!g.hs) HIP_OK(hipStreamCreateWithFlags(&g.hs, hipStreamNonBlocking));
  // carried window bytes: stream [C0, T0)
  const uint64_t C0 = T0 - s->buf.size();
  std::vector<ZsPiece> pc;
  pc.reserve(P.parts.size() + 4);
  const auto a16 = [](uint64_t x) { return (x + 15) & ~(uint64_t)15; };
  // staged source layout: [pieces | carried bytes | input | header bytes]
  size_t np = 0;
  for (const auto &q : P.parts) np += q.lit ? 1 : (q.off < T0 && q.off + q.len > T0 ? 2 : 1);
  const uint64_t o_car = a16(np * sizeof(ZsPiece)), o_in = a16(o_car + s->buf.size()), o_lit = a16(o_in + n_in);
  const uint64_t n_src = o_lit + P.lit.size();
  uint64_t dst = 0;
  for (const auto &q : P.parts) {
    if (q.lit) {
      pc.push_back({o_lit + q.off, dst, (uint32_t)q.len, 0});
    } else {
      uint64_t a = q.off, e = q.off + q.len;
      if (a < T0) {
        const uint64_t m = std::min(e, T0);
        pc.push_back({o_car + (a - C0), dst, (uint32_t)(m - a), 0});
        dst += m - a;
        a = m;
      }
      if (a < e) pc.push_back({o_in + (a - T0), dst, (uint32_t)(e - a), 0});
      dst += e - a;
      continue;
    }
    dst += q.len;
  }
  const uint64_t o_res = a16(P.total);
  int r;
  if ((r = ds_grow_pinned(&g.h_src, &g.cap_hsrc, n_src)) || (r = ds_grow_pinned(&g.h_dst, &g.cap_hdst, o_res + 16)) ||
      (r = ws_reserve_bytes(&g.d_src, &g.cap_dsrc, n_src)) || (r = ws_reserve_bytes(&g.d_dst, &g.cap_ddst, o_res + 16)))
    return r;
  std::memcpy(g.h_src, pc.data(), pc.size() * sizeof(ZsPiece));
  if (!s->buf.empty()) std::memcpy(g.h_src + o_car, s->buf.data(), s->buf.size());
  if (n_in) std::memcpy(g.h_src + o_in, in, n_in);
  if (!P.lit.empty()) std::memcpy(g.h_src + o_lit, P.lit.data(), P.lit.size());
  HIP_OK(hipMemcpyAsync(g.d_src, g.h_src, n_src, hipMemcpyHostToDevice, g.hs));
  zs_launch_stored_call(g.d_src, reinterpret_cast<const ZsPiece *>(g.d_src), (uint32_t)pc.size(), P.total, g.d_dst, o_in,
                        o_in + n_in, (uint32_t)s->wrap, reinterpret_cast<uint32_t *>(g.d_dst + o_res), g.hs);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(g.h_dst, g.d_dst, o_res + 16, hipMemcpyDeviceToHost, g.hs));
  HIP_OK(hipStreamSynchronize(g.hs));
  gen.assign(g.h_dst, g.h_dst + P.total);
  std::memcpy(check, g.h_dst + o_res, 4);
  return 0;
}

// strm->adler after a zlib-ABI deflate() call: zlib's read_buf updates it with
// every byte it reads, so the input this call appended but no GPU job has
// checked yet (buf[ck_from, end)) gets its check now (a check-only launch)
int ds_check_range(DStreamState *s, uint64_t lo, uint64_t hi) {
  const uint64_t n = hi - lo;
  if (!n || !s->wrap) {
    s->checked += n;
    return 0;
  }
  DsStage &g = s->stage;
  if (!g.hs) HIP_OK(hipStreamCreateWithFlags(&g.hs, hipStreamNonBlocking));
  int r;
  if ((r = ds_grow_pinned(&g.h_src, &g.cap_hsrc, n)) || (r = ds_grow_pinned(&g.h_dst, &g.cap_hdst, 16)) ||
      (r = ws_reserve_bytes(&g.d_src, &g.cap_dsrc, n)) || (r = ws_reserve_bytes(&g.d_dst, &g.cap_ddst, 16)))
    return r;
  std::memcpy(g.h_src, s->buf.data() + lo, n);
  HIP_OK(hipMemcpyAsync(g.d_src, g.h_src, n, hipMemcpyHostToDevice, g.hs));
  zs_launch_stored_call(g.d_src, nullptr, 0, 0, g.d_dst, 0, n, (uint32_t)s->wrap, reinterpret_cast<uint32_t *>(g.d_dst),
                        g.hs);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(g.h_dst, g.d_dst, 4, hipMemcpyDeviceToHost, g.hs));
  HIP_OK(hipStreamSynchronize(g.hs));
  uint32_t c;
  std::memcpy(&c, g.h_dst, 4);
  s->adler = s->wrap == 2 ? crc32_join(s->adler, c, n) : adler32_join(s->adler, c, n);
  s->checked += n;
  return 0;
}
int ds_check_rest(DStreamState *s) {
  const int r = ds_check_range(s, s->ck_from, s->buf.size());
  if (!r) s->ck_from = s->buf.size();
  return r;
}

// one deflate(strm, flush) call at level 0 (deflate.c deflate() around deflate_stored)
int ds_stored_call(DStreamState *s, const uint8_t *in, unsigned in_len, uint8_t *out, unsigned out_len, int flush,
                   unsigned *consumed, unsigned *produced) {
  *consumed = 0;
  *produced = 0;
  if (flush < 0 || flush > Z_BLOCK || (s->status == 2 && flush != Z_FINISH)) return Z_STREAM_ERROR;
  if (out_len == 0) return Z_BUF_ERROR;
  auto rank = [](int f) { return f * 2 - (f > 4 ? 9 : 0); };
  auto serve = [&]() {
    const size_t k = std::min<size_t>(s->out.size() - s->served, out_len - *produced);
    if (k) std::memcpy(out + *produced, s->out.data() + s->served, k);
    s->served += k;
    *produced += (unsigned)k;
  };
  const int old_flush = s->last_flush;
  s->last_flush = flush;
  if (s->served < s->out.size()) {  // flush as much pending output as possible
    serve();
    if (*produced == out_len) {
      s->last_flush = -1;
      return Z_OK;
    }
  } else if (in_len == 0 && rank(flush) <= rank(old_flush) && flush != Z_FINISH) {
    return Z_BUF_ERROR;
  }
  if (s->status == 2 && in_len != 0) return Z_BUF_ERROR;
  if (s->status == 0) {  // the header; compression starts with an empty pending buffer
    ds_header(s);
    s->status = 1;
    serve();
    if (s->served < s->out.size()) {
      s->last_flush = -1;
      return Z_OK;
    }
  }
  const uint64_t T0 = s->total_in;
  uint64_t avail_out = out_len - *produced, pend = 0, pos = 0;
  StoredPlan P;
  int ret = Z_OK;
  bool trailer = false, done = false;
  if (in_len || (flush != Z_NO_FLUSH && s->status != 2)) {
    const int bstate = ds_stored_sim(s, P, flush, T0, in_len, &pos, &avail_out, &pend);
    if (bstate >= 2) s->status = 2;
    if (bstate == 0 || bstate == 2) {
      if (avail_out == 0) s->last_flush = -1;
      done = true;
    } else if (bstate == 1) {
      const uint64_t g0 = P.total;
      if (flush == Z_PARTIAL_FLUSH) {
        ds_align(s, P);
      } else if (flush != Z_BLOCK) {
        ds_stored_hdr(s, P, 0, 0);
        if (flush == Z_FULL_FLUSH) s->z_strstart = s->z_block_start = 0;  // CLEAR_HASH, lookahead == 0
      }
      pend += P.total - g0;
      const uint64_t d = std::min(pend, avail_out);
      pend -= d;
      avail_out -= d;
      if (avail_out == 0) {
        s->last_flush = -1;
        done = true;
      }
    }
  }
  if (!done && flush == Z_FINISH) {
    if (s->wrap == 0 || s->trl_done) ret = Z_STREAM_END;
    else trailer = true;
  }
  // the GPU writes the plan's bytes and checks what the call read
  std::vector<uint8_t> gen;
  if (P.total || pos) {
    uint32_t c = 0;
    if (ds_stored_run(s, P, in, pos, T0, gen, &c)) return Z_STREAM_ERROR;
    if (pos && s->wrap) s->adler = s->wrap == 2 ? crc32_join(s->adler, c, pos) : adler32_join(s->adler, c, pos);
    s->checked += pos;
  }
  // the window's unframed bytes now: stream [strstart - block_start before the end of what was read)
  {
    const uint64_t T1 = T0 + pos, keep = s->z_strstart - s->z_block_start, C0 = T0 - s->buf.size();
    std::vector<uint8_t> nb(keep);
    for (uint64_t i = 0; i < keep; i++) {
      const uint64_t a = T1 - keep + i;
      nb[i] = a < T0 ? s->buf[a - C0] : in[a - T0];
    }
    s->buf.swap(nb);
  }
  s->total_in += pos;
  *consumed = (unsigned)pos;
  if (trailer) {  // deflate.c: the trailer into pending, then flush_pending
    const uint32_t c = s->adler, isz = (uint32_t)s->total_in;
    if (s->wrap == 2) {
      const uint8_t t8[8] = {(uint8_t)c, (uint8_t)(c >> 8), (uint8_t)(c >> 16), (uint8_t)(c >> 24),
                             (uint8_t)isz, (uint8_t)(isz >> 8), (uint8_t)(isz >> 16), (uint8_t)(isz >> 24)};
      gen.insert(gen.end(), t8, t8 + 8);
      pend += 8;
    } else {
      const uint8_t t4[4] = {(uint8_t)(c >> 24), (uint8_t)(c >> 16), (uint8_t)(c >> 8), (uint8_t)c};
      gen.insert(gen.end(), t4, t4 + 4);
      pend += 4;
    }
    pend -= std::min(pend, avail_out);
    s->trl_done = true;
    ret = pend ? Z_OK : Z_STREAM_END;
  }
  // delivered now: everything generated but the undelivered tail
  ds_put(s, gen.data(), gen.size());
  serve();
  return ret;
}

// One zlib deflate(strm, flush) call (deflate.c deflate(): argument checks,
// pending output first, Z_BUF_ERROR for a call that cannot progress -- the
// last_flush ranks --, the header at the first call, all input consumed).
int dstream_call(DStreamState *s, const uint8_t *in, unsigned in_len, uint8_t *out, unsigned out_len, int flush,
                 unsigned *consumed, unsigned *produced) {
  if (s->level == 0) return ds_stored_call(s, in, in_len, out, out_len, flush, consumed, produced);
  *consumed = 0;
  *produced = 0;
  if (flush < 0 || flush > Z_BLOCK || (s->status == 2 && flush != Z_FINISH)) return Z_STREAM_ERROR;
  if (out_len == 0) return Z_BUF_ERROR;
  auto rank = [](int f) { return f * 2 - (f > 4 ? 9 : 0); };
  auto serve = [&]() {
    const size_t k = std::min<size_t>(s->out.size() - s->served, out_len - *produced);
    if (k) std::memcpy(out + *produced, s->out.data() + s->served, k);
    s->served += k;
    *produced += (unsigned)k;
    return *produced == out_len;  // output space used up
  };
  const int old_flush = s->last_flush;
  s->last_flush = flush;
  const uint64_t served_start = s->out_base + s->served;
  const bool had_pending = s->served < s->out.size();
  if (had_pending) {
    if (serve()) {
      s->last_flush = -1;
      return Z_OK;
    }
  } else if (in_len == 0 && rank(flush) <= rank(old_flush) && flush != Z_FINISH) {
    return Z_BUF_ERROR;
  }
  if (s->status == 2 && in_len != 0) return Z_BUF_ERROR;
  if (s->status == 0) {  // the header; compression starts with an empty pending buffer (deflate.c)
    ds_header(s);
    s->status = 1;
    serve();
    if (s->served < s->out.size()) {
      s->last_flush = -1;
      return Z_OK;
    }
  }
  // a call that only delivers the rest of a flush whose terminator zlib
  // writes in this very call has nothing more to do
  const bool term_here = had_pending && !in_len && s->mark_valid && served_start <= s->mark;
  if (in_len || (flush != Z_NO_FLUSH && s->status != 2 && !term_here)) {
    const uint64_t rd0 = s->buf.size();  // zlib has read everything before this call's input
    if (in_len) {
      s->buf.insert(s->buf.end(), in, in + in_len);
      s->total_in += in_len;
      s->fresh += in_len;
      *consumed = in_len;
    }
    // output space left for the job's bytes (after the pending output and header)
    const uint64_t room = (uint64_t)(out_len - *produced) - (s->out.size() - s->served);
    int r = Z_OK;
    uint64_t dropped = 0;
    if (flush == Z_FINISH) {
      r = ds_job(s, ZS_DT_FINAL, false, rd0, room, &dropped);
      if (!r && s->rtop == UINT64_MAX) s->status = 2;  // else deflate_slow returned need_more: not finished
    } else if (flush != Z_NO_FLUSH) {
      r = ds_job(s, flush == Z_PARTIAL_FLUSH ? ZS_DT_PARTIAL : (flush == Z_BLOCK ? ZS_DT_BLOCK : ZS_DT_SYNC),
                 flush == Z_FULL_FLUSH, rd0, room, &dropped);
    } else if (s->exact) {
      if (s->fresh >= std::max(s->need, dstream_run_min()) ||
          !ds_model_nojob(s, s->abs + rd0, s->abs + rd0 + in_len))
        r = ds_job(s, ZS_DT_CUT, false, rd0, room, &dropped);
    } else if (s->buf.size() >= dstream_fast_max()) {
      r = ds_job(s, ZS_DT_BLOCK, false, rd0, room, &dropped);
    }
    if (r) return Z_STREAM_ERROR;
    *consumed = (unsigned)(in_len - dropped);
  }
  if (serve()) {
    s->last_flush = -1;
    return (s->status == 2 && s->served == s->out.size()) ? Z_STREAM_END : Z_OK;
  }
  if (flush != Z_FINISH) return Z_OK;
  return s->served == s->out.size() ? Z_STREAM_END : Z_OK;
}

struct DHandle {
  z_stream strm;  // layout parity with the reference context (unused fields)
  DStreamState st;
  unsigned last_consumed = 0;
};

uintptr_t dhandle_new() {
  DHandle *h = new (std::nothrow) DHandle();
  if (!h) return 0;
  std::memset(&h->strm, 0, sizeof h->strm);
  return reinterpret_cast<uintptr_t>(h);
}
// deflateInit2(level, Z_DEFLATED, wbits, 8, Z_DEFAULT_STRATEGY) state
int dstream_init(DStreamState *s, int level, int wbits) {
  int wrap;
  uint32_t w;
  if (level == Z_DEFAULT_COMPRESSION) level = 6;
  if (level < 0 || level > 9 || !parse_dz_wbits(wbits, &wrap, &w)) return Z_STREAM_ERROR;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (ws_init()) return Z_STREAM_ERROR;
  }
  DsStage keep;
  keep = std::move(s->stage);
  *s = DStreamState();
  s->stage = std::move(keep);
  s->inited = 1;
  s->level = level;
  s->wbits = wbits;
  s->wrap = wrap;
  s->w = w;
  s->exact = level >= 1;
  s->adler = wrap == 2 ? 0u : 1u;
  return Z_OK;
}
// src/wasm/deflate_stream_wasm.c:22-49: level < 0 -> Z_DEFAULT_COMPRESSION
int dhandle_init(uintptr_t hp, int level, int wbits) {
  DHandle *h = reinterpret_cast<DHandle *>(hp);
  if (!h) return Z_STREAM_ERROR;
  return dstream_init(&h->st, level < 0 ? Z_DEFAULT_COMPRESSION : level, wbits);
}
int dhandle_process(uintptr_t hp, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush) {
  DHandle *h = reinterpret_cast<DHandle *>(hp);
  if (!h) return Z_STREAM_ERROR;  // wasm_stream_common.c:41-43
  if (!h->st.inited) return (int)((unsigned)(Z_STREAM_ERROR & 0xff) << 24);
  unsigned cons = 0, prod = 0;
  const int ret = dstream_call(&h->st, reinterpret_cast<const uint8_t *>(in_ptr), in_len,
                               reinterpret_cast<uint8_t *>(out_ptr), out_len, flush, &cons, &prod);
  h->last_consumed = cons;
  return (int)((prod & 0x00ffffffu) | ((unsigned)(ret & 0xff) << 24));
}
// deflateEnd: Z_DATA_ERROR when the stream was left unfinished (deflate.c)
// (a raw stream starts in BUSY_STATE: deflateResetKeep)
int dstream_end_code(const DStreamState *s) {
  return s->inited && (s->status == 1 || (s->status == 0 && s->wrap == 0)) ? Z_DATA_ERROR : Z_OK;
}
}  // namespace

// ===========================================================================
// exported C-ABI
// ===========================================================================
extern "C" {

const char *zs_version(void) { return "zstreams-mi355x 0.5 (gfx950) src " ZS_SRC_HASH; }
const char *zs_source_hash(void) { return ZS_SRC_HASH; }
const char *zs_last_error(void) { return g_err.c_str(); }

int zs_set_stream(void *s) {
  std::lock_guard<std::mutex> lk(g_mu);
  int r = ws_init();
  if (r) return r;
  g_ws.stream = s ? static_cast<hipStream_t>(s) : g_ws.own_stream;
  return 0;
}

// Timing with HIP events on the launch stream: enable (1) / disable (0).
// zs_profile_read returns the accumulated milliseconds of the inflate pipeline
// (find .. serial decoders: everything between header parse and finalize), of
// whole batches (header .. finalize), and the number of batches;
// zs_profile_stages the per-kernel split (ZS_PROF_STAGES entries, order in the
// public header).
int zs_profile(int enable) {
  std::lock_guard<std::mutex> lk(g_mu);
  int r = ws_init();
  if (r) return r;
  if (!g_ws.ev[0])
    for (int i = 0; i <= ZS_PROF_STAGES; i++) HIP_OK(hipEventCreate(&g_ws.ev[i]));
  g_ws.prof = enable != 0;
  for (int i = 0; i < ZS_PROF_STAGES; i++) g_ws.prof_stage[i] = 0.0;
  g_ws.prof_ms = 0.0;
  g_ws.prof_batch_ms = 0.0;
  g_ws.prof_launches = 0;
  g_dz.ms = 0.0;
  for (double &x : g_dz.stage_ms) x = 0.0;
  g_dz.launches = 0;
  return 0;
}
int zs_profile_read(double *decode_ms, double *batch_ms, uint64_t *launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  *decode_ms = g_ws.prof_ms;
  *batch_ms = g_ws.prof_batch_ms;
  *launches = g_ws.prof_launches;
  return 0;
}

int zs_profile_stages(double *ms, uint32_t n) {
  std::lock_guard<std::mutex> lk(g_mu);
  const uint32_t k = n < ZS_PROF_STAGES ? n : ZS_PROF_STAGES;
  for (uint32_t i = 0; i < k; i++) ms[i] = g_ws.prof_stage[i];
  return (int)k;
}

int zs_stream_stats(uint64_t out[2]) {
  std::lock_guard<std::mutex> lk(g_sq.mu);
  out[0] = g_sq.launches;
  out[1] = g_sq.calls;
  return 0;
}

int zs_stream_stats_ex(uint64_t out[10]) {
  {
    std::lock_guard<std::mutex> lk(g_sq.mu);
    out[0] = g_sq.launches;
    out[1] = g_sq.calls;
    out[2] = g_sq.launch_ns;
    out[3] = g_sq.gather_ns;
    out[4] = g_sq.kernel_ns;
  }
  std::lock_guard<std::mutex> lk(g_pk.mu);
  out[5] = g_pk.launches;
  out[6] = g_pk.calls.load();
  out[7] = g_pk.busy_ns.load();
  out[8] = g_pk.wait_ns.load();
  out[9] = g_pk.idle_ns.load();
  return 0;
}

int zs_stream_persist(int on) {
  const int prev = pk_enabled() ? 1 : 0;
  if (on >= 0) g_pk_on.store(on ? 1 : 0);
  return prev;
}

int zs_last_stats(uint32_t out[4]) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (int i = 0; i < 4; i++) out[i] = g_ws.stats[i];
  return 0;
}

int zs_last_stats_ex(uint32_t *out, uint32_t n) {
  std::lock_guard<std::mutex> lk(g_mu);
  uint32_t v[12];
  for (int i = 0; i < 4; i++) v[i] = g_ws.stats[i];
  for (int i = 0; i < 8; i++) v[4 + i] = g_ws.path[i];
  const uint32_t k = n < 12 ? n : 12;
  for (uint32_t i = 0; i < k; i++) out[i] = v[i];
  return (int)k;
}

int zs_synchronize(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ws.ready) return 0;
  return hipStreamSynchronize(g_ws.stream) == hipSuccess ? 0 : ZS_ENODEV;
}

int zs_inflate_batch(const zs_job *jobs, uint32_t n, zs_result *results, uint32_t flags) {
  std::lock_guard<std::mutex> lk(g_mu);
  return batch_locked(jobs, n, results, flags);
}

// ---- reference handle ABI (src/wasm/inflate_stream_wasm.c, inflate9_stream_wasm.c) ----
uintptr_t inflate_new(void) { return handle_new(); }
int inflate_init(uintptr_t h) { return handle_init(h, 15); }
int inflate_init_raw(uintptr_t h) { return handle_init(h, -15); }
int inflate_init_gzip(uintptr_t h) { return handle_init(h, 15 + 16); }
int inflate_process(uintptr_t h, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush) {
  return handle_process(h, in_ptr, in_len, out_ptr, out_len, flush);
}
int inflate_end(uintptr_t h) { return handle_end(h); }
unsigned inflate_last_consumed(uintptr_t h) { return handle_last_consumed(h); }

uintptr_t inflate9_new(void) { return handle_new(); }
int inflate9_init_raw(uintptr_t h) { return handle_init(h, -16); }
int inflate9_init(uintptr_t h) { return inflate9_init_raw(h); }
int inflate9_process(uintptr_t h, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush) {
  return handle_process(h, in_ptr, in_len, out_ptr, out_len, flush);
}
int inflate9_end(uintptr_t h) { return handle_end(h); }
unsigned inflate9_last_consumed(uintptr_t h) { return handle_last_consumed(h); }

// ---- zlib inflate ABI (src/inflate.c:186 inflateInit2_, :597 inflate, :1277 inflateEnd) ----
int ZEXPORT inflateInit2_(z_streamp strm, int windowBits, const char *version, int stream_size) {
  if (version == Z_NULL || version[0] != '1' || stream_size != (int)sizeof(z_stream)) return Z_VERSION_ERROR;
  if (strm == Z_NULL) return Z_STREAM_ERROR;
  strm->msg = Z_NULL;
  ZsJobDev probe{};
  if (!parse_wbits(windowBits, &probe)) return Z_STREAM_ERROR;
  StreamState *s = new (std::nothrow) StreamState();
  if (!s) return Z_MEM_ERROR;
  const int r = stream_init(s, windowBits);
  if (r != Z_OK) stream_free(s);
  if (r != Z_OK) {
    delete s;
    return r;
  }
  strm->state = reinterpret_cast<struct internal_state *>(s);
  strm->total_in = strm->total_out = 0;
  if (probe.wrap != ZW_RAW) strm->adler = s->adler;
  return Z_OK;
}

int ZEXPORT inflateInit_(z_streamp strm, const char *version, int stream_size) {
  return inflateInit2_(strm, 15, version, stream_size);
}

int ZEXPORT inflate(z_streamp strm, int flush) {
  if (strm == Z_NULL || strm->state == Z_NULL || strm->next_out == Z_NULL ||
      (strm->next_in == Z_NULL && strm->avail_in != 0))
    return Z_STREAM_ERROR;
  StreamState *s = reinterpret_cast<StreamState *>(strm->state);
  unsigned cons = 0, prod = 0;
  int ret = stream_call(s, strm->next_in, strm->avail_in, strm->next_out, strm->avail_out, flush, &cons, &prod);
  strm->next_in += cons;
  strm->avail_in -= cons;
  if (ret != Z_NEED_DICT) strm->total_in += cons;  // Z_NEED_DICT returns before inf_leave
  strm->next_out += prod;
  strm->avail_out -= prod;
  strm->total_out += prod;
  if (s->msg) strm->msg = const_cast<char *>(s->msg);
  if (s->cfg.wrap != ZW_RAW) strm->adler = s->adler;
  return ret;
}

int ZEXPORT inflateEnd(z_streamp strm) {
  if (strm == Z_NULL || strm->state == Z_NULL) return Z_STREAM_ERROR;
  StreamState *s = reinterpret_cast<StreamState *>(strm->state);
  stream_free(s);
  delete s;
  strm->state = Z_NULL;
  return Z_OK;
}


// ---- deflate: batch, reference stream ABI, zlib ABI ----
int zs_deflate_batch(const zs_djob *jobs, uint32_t n, zs_result *results, uint32_t flags) {
  std::lock_guard<std::mutex> lk(g_mu);
  return deflate_batch_locked(jobs, n, results, flags);
}
uint64_t zs_deflate_bound(uint64_t in_len, int32_t window_bits) {
  int wrap = 0;
  uint32_t w = 15;
  if (!parse_dz_wbits(window_bits, &wrap, &w)) wrap = 2;
  return dz_bound(in_len, wrap);
}
int zs_profile_deflate(double *ms, uint32_t n) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (n > 0) ms[0] = g_dz.ms;
  for (uint32_t i = 1; i < n && i < 5; i++) ms[i] = g_dz.stage_ms[i - 1];
  if (n > 5) ms[5] = (double)g_dz.launches;
  return (int)std::min<uint32_t>(n, 6);
}

uintptr_t deflate_new(void) { return dhandle_new(); }
int deflate_init(uintptr_t h, int level) { return dhandle_init(h, level, 15); }
int deflate_init_raw(uintptr_t h, int level) { return dhandle_init(h, level, -15); }
int deflate_init_gzip(uintptr_t h, int level) { return dhandle_init(h, level, 15 + 16); }
int deflate_process(uintptr_t h, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush) {
  return dhandle_process(h, in_ptr, in_len, out_ptr, out_len, flush);
}
int deflate_end(uintptr_t h) {
  DHandle *d = reinterpret_cast<DHandle *>(h);
  if (!d) return Z_STREAM_ERROR;
  const int r = dstream_end_code(&d->st);
  delete d;
  return r;
}
unsigned deflate_last_consumed(uintptr_t h) {
  DHandle *d = reinterpret_cast<DHandle *>(h);
  return d ? d->last_consumed : 0;
}

// zlib deflate ABI (deflate.c deflateInit2_ / deflate / deflateEnd / deflateBound)
int ZEXPORT deflateInit2_(z_streamp strm, int level, int method, int windowBits, int memLevel, int strategy,
                          const char *version, int stream_size) {
  if (version == Z_NULL || version[0] != '1' || stream_size != (int)sizeof(z_stream)) return Z_VERSION_ERROR;
  if (strm == Z_NULL) return Z_STREAM_ERROR;
  strm->msg = Z_NULL;
  int wrap;
  uint32_t w;
  if (level == Z_DEFAULT_COMPRESSION) level = 6;
  if (method != Z_DEFLATED || memLevel < 1 || memLevel > 9 || level < 0 || level > 9 || strategy < 0 ||
      strategy > Z_FIXED || !parse_dz_wbits(windowBits, &wrap, &w))
    return Z_STREAM_ERROR;
  // memLevel (hash bits, lit_bufsize) and the strategies change zlib's bytes;
  // the GPU encoder implements memLevel 8 / Z_DEFAULT_STRATEGY -- the only
  // parameters the reference passes (src/wasm/deflate_stream_wasm.c:31-49) --
  // and refuses the rest rather than silently writing other bytes
  if (memLevel != 8 || strategy != Z_DEFAULT_STRATEGY) {
    set_err("deflateInit2_: only memLevel 8 and Z_DEFAULT_STRATEGY are implemented on the GPU");
    return Z_STREAM_ERROR;
  }
  DStreamState *s = new (std::nothrow) DStreamState();
  if (!s) return Z_MEM_ERROR;
  const int r = dstream_init(s, level, windowBits);
  if (r != Z_OK) {
    delete s;
    return r;
  }
  strm->state = reinterpret_cast<struct internal_state *>(s);
  strm->total_in = strm->total_out = 0;
  strm->adler = wrap == 2 ? 0u : 1u;
  return Z_OK;
}
int ZEXPORT deflateInit_(z_streamp strm, int level, const char *version, int stream_size) {
  return deflateInit2_(strm, level, Z_DEFLATED, 15, 8, Z_DEFAULT_STRATEGY, version, stream_size);
}
int ZEXPORT deflate(z_streamp strm, int flush) {
  if (strm == Z_NULL || strm->state == Z_NULL || strm->next_out == Z_NULL ||
      (strm->next_in == Z_NULL && strm->avail_in != 0) || flush < 0 || flush > Z_BLOCK)
    return Z_STREAM_ERROR;
  if (strm->avail_out == 0) return Z_BUF_ERROR;
  DStreamState *s = reinterpret_cast<DStreamState *>(strm->state);
  unsigned cons = 0, prod = 0;
  int ret = dstream_call(s, strm->next_in, strm->avail_in, strm->next_out, strm->avail_out, flush, &cons, &prod);
  if (ret >= Z_OK && s->level > 0 && ds_check_rest(s)) ret = Z_STREAM_ERROR;  // strm->adler covers every byte read
  strm->next_in += cons;
  strm->avail_in -= cons;
  strm->total_in += cons;
  strm->next_out += prod;
  strm->avail_out -= prod;
  strm->total_out += prod;
  if (s->checked) strm->adler = s->adler;  // the check of all input read so far (GPU)
  return ret;
}
int ZEXPORT deflateEnd(z_streamp strm) {
  if (strm == Z_NULL || strm->state == Z_NULL) return Z_STREAM_ERROR;
  DStreamState *s = reinterpret_cast<DStreamState *>(strm->state);
  const int r = dstream_end_code(s);
  delete s;
  strm->state = Z_NULL;
  return r;
}
uLong ZEXPORT deflateBound(z_streamp strm, uLong sourceLen) {
  int wrap = 1;
  uint32_t w = 15;
  if (strm && strm->state) parse_dz_wbits(reinterpret_cast<DStreamState *>(strm->state)->wbits, &wrap, &w);
  return (uLong)dz_bound(sourceLen, wrap);
}
}  // extern "C"
