/*
 * zstreams_mi355x.h -- C-ABI of libzstreams_mi355x.so, the MI355X inflate core.
 *
 * Three surfaces, all plain pointers and sizes:
 *
 *  1. The reference's handle-based stream ABI, symbol for symbol
 *     (reference export list: Makefile:288).  Handles are widened from the
 *     WASM `unsigned` to `uintptr_t` (a 64-bit process cannot round-trip a
 *     pointer through 32 bits).  Each entry replaces the function of the same
 *     name in the reference:
 *       inflate_new / inflate9_new         src/wasm/wasm_stream_common.c:7-18
 *       inflate_init                       src/wasm/inflate_stream_wasm.c:22-27
 *       inflate_init_raw                   src/wasm/inflate_stream_wasm.c:29-34
 *       inflate_init_gzip                  src/wasm/inflate_stream_wasm.c:36-45
 *       inflate9_init / inflate9_init_raw  src/wasm/inflate9_stream_wasm.c:15-22
 *       *_process                          src/wasm/wasm_stream_common.c:37-63
 *       *_last_consumed                    src/wasm/wasm_stream_common.c:30-35
 *       *_end                              src/wasm/wasm_stream_common.c:20-28
 *     process() returns (produced & 0x00ffffff) | ((ret & 0xff) << 24), the
 *     zlib code as a signed byte in the top 8 bits, exactly like the reference.
 *
 *  2. The zlib inflate ABI used by the reference's native harnesses
 *     (test/payload_decompress.c:124-178): inflateInit2_, inflateInit_,
 *     inflate, inflateEnd over the standard z_stream (sizeof 112 on x86-64).
 *     Declared by <zlib.h>; this library defines them.
 *
 *  3. A batch entry for many independent whole streams (new; no reference
 *     analog): zs_inflate_batch().  Each job has the semantics of ONE
 *     inflate(strm, Z_FINISH) call over the whole input into an out_cap-byte
 *     buffer after inflateInit2(strm, window_bits) (src/inflate.c:186, 597):
 *     same ret, msg, total_in, total_out and adler.
 *
 * Surfaces 1 and 2 are thread-safe across handles (a handle, like a z_stream,
 * belongs to one thread at a time): concurrent calls of different handles are
 * batched into shared GPU launches.
 *
 * All decoding runs on the GPU (HIP, gfx950).  There is no CPU fallback: if no
 * HIP device is usable every entry point fails with Z_STREAM_ERROR /
 * ZS_ENODEV and zs_last_error() says why.
 */
#ifndef ZSTREAMS_MI355X_H
#define ZSTREAMS_MI355X_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- 1. reference stream ABI (handles are uintptr_t, 0 = allocation failure) ---- */
uintptr_t inflate_new(void);
int inflate_init(uintptr_t h);
int inflate_init_raw(uintptr_t h);
int inflate_init_gzip(uintptr_t h);
int inflate_process(uintptr_t h, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush);
int inflate_end(uintptr_t h);
unsigned inflate_last_consumed(uintptr_t h);

uintptr_t deflate_new(void);
int deflate_init(uintptr_t h, int level);       /* src/wasm/deflate_stream_wasm.c:22-29 (level < 0 -> default) */
int deflate_init_raw(uintptr_t h, int level);   /* :31-39 */
int deflate_init_gzip(uintptr_t h, int level);  /* :41-49; deflate_process :51-55, _end :57-65, _last_consumed :67-69 */
int deflate_process(uintptr_t h, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush);
int deflate_end(uintptr_t h);
unsigned deflate_last_consumed(uintptr_t h);

uintptr_t inflate9_new(void);
int inflate9_init(uintptr_t h);
int inflate9_init_raw(uintptr_t h);
int inflate9_process(uintptr_t h, uintptr_t in_ptr, unsigned in_len, uintptr_t out_ptr, unsigned out_len, int flush);
int inflate9_end(uintptr_t h);
unsigned inflate9_last_consumed(uintptr_t h);

/* ---- 3. batch API ---- */
typedef struct zs_job {
  const void *in;      /* compressed bytes (host, or device with ZS_F_DEVICE) */
  uint64_t in_len;     /* any length: a stream past 2^29 - 4096 compressed bytes or 0xfff00000 of
                          out_cap decodes in 256 MiB pieces resumed at block boundaries (one deflate
                          block must fit one piece's limits, else Z_STREAM_ERROR) */
  void *out;           /* output buffer (host, or 16-byte aligned device memory) */
  uint64_t out_cap;    /* any size */
  int32_t window_bits; /* as inflateInit2: -8..-15 raw, -16 raw deflate64, 8..15 zlib, +16 gzip, +32 auto */
  int32_t mode;        /* ZS_JOB_INFLATE (0), or ZS_JOB_COPY: stored bytes (ZIP method 0), output = input */
} zs_job;
#define ZS_JOB_INFLATE 0
#define ZS_JOB_COPY 1

typedef struct zs_result {
  int32_t ret;         /* Z_STREAM_END, Z_DATA_ERROR, Z_BUF_ERROR, Z_NEED_DICT, Z_STREAM_ERROR */
  int32_t reserved;
  uint64_t total_in;
  uint64_t total_out;
  uint32_t adler;      /* strm->adler after the call (0 for raw streams) */
  uint32_t reserved2;
  const char *msg;     /* strm->msg (static string) or NULL */
} zs_result;

#define ZS_F_DEVICE 1u /* job in/out pointers are device (HBM) pointers: no staging copies */
#define ZS_F_CRC32 2u  /* raw and copy jobs: CRC-32 of the output in adler (ZIP entries; computed on the GPU) */
/* Parse mode of the block-parallel path (results are identical; speed differs).
   By default a batch with few decode units (<= 12288 search segments of 32 KiB
   compressed, env ZS_WAVE_SEGS) decodes each unit with a whole wave, a larger
   one with the split parse (below; env ZS_SPLIT=0: one lane per unit).  These
   force one mode (testing, tuning). */
#define ZS_F_PARSE_LANE 8u
#define ZS_F_PARSE_WAVE 16u
/* The split parse (default where the lane parse was): a boundary walk of each
   unit's first block records exact symbol checkpoints, then a wave decodes the
   block's sub-units in parallel.  This forces it for any batch size. */
#define ZS_F_PARSE_SPLIT 4096u
/* Link mode of the block-parallel path (results are identical): groups of at
   most 4 long streams use the parallel-prefix window link by default, larger
   groups the per-stream serial link (zs_link_kernel).  This forces the serial
   link (testing, tuning). */
#define ZS_F_LINK_SERIAL 32u
/* Force the segmented window link with n segments per chain (1 <= n <= 8; 1 is
   the serial link) for the raw/zlib/gzip group, whatever its size (testing,
   tuning; results are identical).  By default a group of 5..64 streams with
   chains of >= 64 units cuts each chain into min(8, 256 / streams) segments. */
#define ZS_F_LINKSEG(n) (((uint32_t)(n) & 15u) << 8)
#define ZS_F_LINKSEG_GET(flags) (((flags) >> 8) & 15u)

#define ZS_ENODEV (-100)
#define ZS_EFORMAT (-101) /* malformed container (zs_zip_scan) */
#define ZS_EINVAL (-102)  /* bad arguments */

/* ---- ZIP containers (new; generalises src/generator/create_deflate64.cpp:51-93,
 *      which reads the payload of the first local header) ---- */
typedef struct zs_zip_entry {
  uint64_t local_off;   /* local file header */
  uint64_t data_off;    /* compressed payload */
  uint64_t comp_size;
  uint64_t uncomp_size;
  uint64_t name_off;    /* file name bytes (central directory, or local header) */
  uint32_t name_len;
  uint32_t crc32;
  uint16_t method;      /* 0 stored, 8 deflate (windowBits -15), 9 deflate64 (-16) */
  uint16_t flags;
  uint32_t reserved;
} zs_zip_entry;

/* Lists the entries (central directory incl. ZIP64, else consecutive local
 * headers).  *n_out = entries in the archive; the first min(cap, n) are written.
 * Returns 0, ZS_EFORMAT or ZS_EINVAL.  Decode them with zs_inflate_batch
 * (ZS_F_CRC32; ZS_JOB_COPY for method 0) and compare adler with crc32. */
int zs_zip_scan(const void *zip, uint64_t len, zs_zip_entry *out, uint32_t cap, uint32_t *n_out);

int zs_inflate_batch(const zs_job *jobs, uint32_t n, zs_result *results, uint32_t flags);

/* ---- GPU deflate ---- */
typedef struct zs_djob {
  const void *in;      /* bytes to compress (host, or device with ZS_F_DEVICE) */
  uint64_t in_len;     /* < 2^32 */
  void *out;           /* compressed output (host, or device with ZS_F_DEVICE) */
  uint64_t out_cap;    /* zs_deflate_bound(in_len, window_bits) always suffices */
  int32_t window_bits; /* as deflateInit2: -9..-15 raw, 9..15 zlib, 25..31 gzip */
  int32_t level;       /* 0 stored, 1..9, or -1 (Z_DEFAULT_COMPRESSION = 6) */
} zs_djob;
/* Each job = deflateInit2(level, Z_DEFLATED, window_bits, 8, Z_DEFAULT_STRATEGY)
   + one deflate(Z_FINISH) over the whole input: ret Z_STREAM_END (Z_OK when
   out_cap was too small: total_out = out_cap bytes of the stream), total_in,
   total_out, adler (CRC-32 for gzip, Adler-32 for zlib, 1 for raw).
   Every level writes zlib's bytes: the same stream zlib 1.2.11 produces
   (the reference's deflate, src/wasm/deflate_stream_wasm.c:22-49 passes the
   level through; src/trees.c), byte for byte -- level 0 deflate_stored's
   65535-byte blocks, levels 1..3 deflate_fast (serial per stream: one wave
   per job, ~4-18 MiB/s per stream), levels 4..9 deflate_slow (data-parallel).
   window_bits -16 (deflate64) and ZS_F_DEFLATE_FAST write valid deflate that
   any inflater decodes to the input, with the GPU's own block structure (not
   zlib's bytes). */
#define ZS_F_DEFLATE_FAST 4u /* levels 1..9: the throughput path instead of zlib's bytes */
#define ZS_F_DEFLATE_SYNC 64u /* end each job as deflate(Z_SYNC_FLUSH) does at the end of its input: blocks
                                 not final, then an empty stored block (00 00 FF FF), no trailer; res.adler
                                 still holds the input's check (zlib/gzip) */
int zs_deflate_batch(const zs_djob *jobs, uint32_t n, zs_result *results, uint32_t flags);
uint64_t zs_deflate_bound(uint64_t in_len, int32_t window_bits);
/* accumulated deflate timing (zs_profile(1) enables): [0] whole pipeline ms,
   [1] match, [2] parse, [3] blocks + checks, [4] offsets + stitch + trailer,
   [5] batches.  zlib-identical jobs (levels 1..9): [1] chains + match search
   (levels 4..9), [2] parse + fix-up rounds (levels 1..3: the whole serial
   deflate_fast), [3] trees + bits, [4] trailer.  Returns the
   number of entries written. */
int zs_profile_deflate(double *ms, uint32_t n);
/* launch on this HIP stream (hipStream_t); NULL = the library's own stream */
int zs_set_stream(void *hip_stream);
int zs_synchronize(void);
/* kernel timing via HIP events on the launch stream (enable resets the sums) */
int zs_profile(int enable);
/* accumulated ms: inflate pipeline (find .. serial decode), whole batches; batch count */
int zs_profile_read(double *decode_ms, double *batch_ms, uint64_t *launches);
/* accumulated ms per stage, in this order: header, find, parse, expand, link,
   emit, serial decode, finalize.  Returns the number of entries written. */
#define ZS_PROF_STAGES 8
int zs_profile_stages(double *ms, uint32_t n);
/* in-kernel phase counters of the profiling build (libzstreams_mi355x_prof.so,
   `make prof`); the product library returns 0 (no counters).  reset != 0
   zeroes them after the read.  Returns the number of counters written. */
int zs_kprof_read(uint64_t *out, uint32_t n, int reset);
/* last batch: [jobs on the chunked path, decode units planned for them,
   chunked jobs whose chain did not verify (decoded by the serial decoder
   instead), jobs routed to the serial decoder] */
int zs_last_stats(uint32_t out[4]);
/* The same four counters, then the path the last batch's block-parallel groups
   took: [4] raw/zlib/gzip group parse mode (0 lane per unit, 1 wave per unit,
   UINT32_MAX no such group), [5] its link: 0 serial, 0x80000000 | S the
   segmented link with S segments per chain, else the parallel-prefix link's
   scan levels (< 32), [6] / [7] the same for the deflate64 group (which has no
   segmented link), [8] lane-parse waves
   resident at once (units dealt in groups of 64 x this), [9] decode units of the
   raw/zlib/gzip group, [10] of the deflate64 group.  Writes min(n, 11) entries
   and returns that count. */
int zs_last_stats_ex(uint32_t *out, uint32_t n);
/* stream-call batching since load: [launch sequences, calls they ran].  Calls of
   the handle / zlib ABIs made at the same time from different threads (one
   handle per thread) share one launch, a workgroup per call. */
int zs_stream_stats(uint64_t out[2]);
/* zs_stream_stats plus timing (ns, cumulative): out[0] launches, out[1] calls
 * (batch path), out[2] wall time of the launch sequences (submit to
 * synchronised, summed over slots), out[3] time leaders waited to gather calls
 * (ZS_STREAM_GATHER_US), out[4] the batches' kernel time (HIP events around
 * each launch sequence); the persistent worker: out[5] its launches, out[6] the
 * calls it ran, out[7] their workgroup time (pickup to done), out[8] their
 * host wait (post to seen done), out[9] the workgroups' idle time before each
 * call (since their previous one). */
int zs_stream_stats_ex(uint64_t out[10]);

/* Persistent stream worker on (1) / off (0) for later calls; -1 only reads.
 * Returns the previous setting.  Default: on (env ZS_STREAM_PK=0: off).  With
 * it on, a handle's mapped calls after the wrapper header run on a long-lived
 * workgroup of their own and return as soon as that call is done. */
int zs_stream_persist(int on);
const char *zs_version(void);
/* SHA-256 of the sources the library was built from (csrc + this header +
   the hipcc version; csrc/srchash.py), hex.  Ties measurements such as the
   bench's PMC traffic to sources rather than to one binary. */
const char *zs_source_hash(void);
const char *zs_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
