// zs_common.h -- layouts shared by the HIP kernels and the host orchestration.
//
// One "job" = one complete compressed stream handed to the GPU, with the
// semantics of a single zlib inflate(strm, Z_FINISH) call over the whole input
// into an out_cap-byte buffer (reference: src/inflate.c:597-1275 driven as in
// test/payload_decompress.c:148-178 with the whole payload in one buffer).
#pragma once
#include <stddef.h>
#include <stdint.h>

// zlib return codes (zlib.h; reference callers decode them in
// src/wasm/api/zlib-streams.js:89-95)
#define ZS_OK 0
#define ZS_STREAM_END 1
#define ZS_NEED_DICT 2
#define ZS_STREAM_ERROR (-2)
#define ZS_DATA_ERROR (-3)
#define ZS_MEM_ERROR (-4)
#define ZS_BUF_ERROR (-5)
#define ZS_VERSION_ERROR (-6)

// strm->msg strings of the reference (src/inflate.c:652-1223, inffast.c:158-283).
enum ZsMsg {
  ZM_NONE = 0,
  ZM_HEADER_CHECK,      // "incorrect header check"
  ZM_METHOD,            // "unknown compression method"
  ZM_WINDOW,            // "invalid window size"
  ZM_FLAGS,             // "unknown header flags set"
  ZM_HCRC,              // "header crc mismatch"
  ZM_BLOCK_TYPE,        // "invalid block type"
  ZM_STORED_LEN,        // "invalid stored block lengths"
  ZM_TOO_MANY,          // "too many length or distance symbols"
  ZM_CODE_LENGTHS,      // "invalid code lengths set"
  ZM_REPEAT,            // "invalid bit length repeat"
  ZM_MISSING_EOB,       // "invalid code -- missing end-of-block"
  ZM_LITLEN_SET,        // "invalid literal/lengths set"
  ZM_DIST_SET,          // "invalid distances set"
  ZM_LITLEN_CODE,       // "invalid literal/length code"
  ZM_DIST_CODE,         // "invalid distance code"
  ZM_TOO_FAR,           // "invalid distance too far back"
  ZM_DATA_CHECK,        // "incorrect data check"
  ZM_LENGTH_CHECK,      // "incorrect length check"
  ZM_COUNT
};

// Wrapper kinds, derived from windowBits exactly as inflateReset2 does
// (src/inflate.c:147-184).
enum ZsWrap { ZW_RAW = 0, ZW_ZLIB = 1, ZW_GZIP = 2, ZW_AUTO = 3 };

// Per-job device descriptor (filled by the host).
struct ZsJobDev {
  const uint8_t *in;   // device pointer to compressed bytes
  uint8_t *out;        // device pointer, 16-byte aligned
  uint64_t in_len;
  uint64_t out_cap;
  int32_t wrap;        // ZsWrap allowed by windowBits (0 raw, 1 zlib, 2 gzip, 3 auto)
  int32_t d64;         // 1 => raw deflate64 (windowBits == -16)
  int32_t wbits;       // window bits after the reset rules (8..16, or 0 = from header)
  int32_t flags;       // ZS_JF_*
  // pieces of a stream too long for one launch (zs_capi.cpp run_pieces):
  uint32_t sbit;       // ZS_JF_CONT: bits of input byte 0 already consumed (0..7)
  uint32_t hist;       // ZS_JF_CONT: output bytes before `out` that are history (the earlier pieces')
  uint32_t stop_after; // ZS_JF_PART, serial decoder: stop at the first block boundary at or past this bit
  uint32_t pad_;
};
#define ZS_JF_CRC32 1  // raw stream: CRC-32 of the output into the result's adler (ZIP entries)
#define ZS_JF_COPY 2   // stored bytes: output = input (ZIP method 0), checked like a raw stream
#define ZS_JF_CONT 4   // raw deflate resuming at a block boundary (bit sbit), with hist bytes of history
#define ZS_JF_PART 8   // the input is a piece of a longer stream: stop at a block boundary (ZD_STOP)
// ZS_JF_PART output budget: the chunked path cuts its chain, the serial
// decoder stops at a block boundary, once a piece has produced this much
#define ZS_PART_OUT (1ull << 30)

// Decoder outcome codes (device -> finalize).
enum ZsDecCode {
  ZD_END = 0,        // final block decoded; end_bits = bits consumed through it
  ZD_TRUNC = 1,      // input ran out (zlib NEEDBITS/PULLBYTE would return)
  ZD_FULL = 2,       // output buffer full before an output-producing symbol
  ZD_ERROR = 3,      // data error; msg set; end_bits = bits pulled
  ZD_NEED_DICT = 4,  // zlib header asked for a preset dictionary
  ZD_SKIP = 5        // header stage already produced the final result
};

// Header stage result.
struct ZsHeadDev {
  int32_t code;        // ZD_* (ZD_SKIP when the header itself failed / truncated)
  int32_t msg;
  int32_t is_gzip;     // 1 gzip trailer (CRC-32 + ISIZE), 0 zlib (Adler-32), -1 raw
  int32_t ret;         // zlib return code when code == ZD_SKIP
  uint64_t start_byte; // first byte of deflate data
  uint64_t total_in;   // valid when code == ZD_SKIP / ZD_NEED_DICT
  uint32_t adler;      // valid when code == ZD_SKIP / ZD_NEED_DICT
  uint32_t wbits;      // window bits in force after the header (zlib: CINFO when windowBits was 0)
};

// Deflate decode result.
struct ZsDecDev {
  int32_t code;
  int32_t msg;
  uint64_t end_bits;   // relative to the job's input byte 0
  uint64_t total_out;
};

// ---------------------------------------------------------------------------
// Speculative chunking of large raw/zlib/gzip streams.
// A stream's deflate data is cut into fixed-size search SEGMENTS; the block
// finder (zs_find_kernel) records up to SEG_SLOTS dynamic-block starts per
// segment, and zs_plan_kernel turns the stream start plus every recorded start
// into an ordered list of decode UNITS (ZsChunkDev), each decoding from its
// start to the first block end at or past the next unit's start.  Unit outputs
// are u16 entries where values >= 256 name bytes of the unknown 32 KiB history
// before the unit (markers).  zs_link_kernel follows the chain (a unit's end
// must be the start of a later unit; starts that are not true block
// boundaries are skipped), resolves the history windows in order, and
// zs_emit_kernel writes the final bytes.  A stream whose chain breaks goes to
// the exact serial decoder, so results never depend on the speculation.
// ---------------------------------------------------------------------------
#define ZS_NONE 0xffffffffu
#define ZD_STOP 6     // unit decode reached its stop bit at a block boundary
#define SEG_SLOTS 4   // block starts recorded per search segment

struct ZsSegDev {
  uint32_t job;        // job index
  uint32_t ord;        // ordinal of the segment within its job
  uint32_t s_byte;     // search range [s_byte, e_byte) of the job input
  uint32_t e_byte;
  uint32_t ncand;      // block starts found (<= SEG_SLOTS), ascending
  uint32_t cand[SEG_SLOTS];  // bit offsets from the 4-byte-aligned input base
  uint32_t final_ok;   // 1: BFINAL = 1 starts count too (the stream's last segments)
  uint32_t nfixed;     // fixed-block starts in cand[] (zs_find_fixed_kernel, only when ncand == 0)
  uint32_t pad;
};

struct ZsChunkDev {    // one decode unit
  uint32_t job;        // job index
  uint32_t ord;        // 0 = the stream's first unit (no history before it)
  uint32_t first;      // first unit of this job
  uint32_t nunits;     // units of this job
  uint32_t start_bit;  // decode start (bits from the 4-byte-aligned input base)
  uint32_t stop_bit;   // next unit's start (ZS_NONE: decode to the final block)
  uint32_t end_bit;    // where decoding stopped
  int32_t code;        // ZD_* | (ZsMsg << 8)
  uint32_t n_out;      // u16 entries produced
  uint32_t cap;        // output entry limit (the job's out_cap, clamped)
  uint64_t scratch;    // entry offset of this unit's u16 entries (zs_chain_kernel: job base + out_off)
  uint32_t chain_next; // next unit in the verified chain (ZS_NONE at the end)
  uint32_t in_chain;   // 1 = member of the verified chain of a non-fallback job
  uint64_t out_off;    // output byte offset (verified chain members)
  uint32_t n_tok;      // tokens produced by the parse pass
  uint32_t tcap;       // tokens in the primary region; later tokens go to pool pages
  uint64_t tok;        // offset of this unit's primary token region (u32 units)
  uint32_t hdr_bit;    // bit after the first block's header (when prebuilt)
  uint32_t hdr_info;   // bit 0: first header prebuilt by zs_unit_header_kernel;
                       // bit 1: its BFINAL; bits 8-11 / 12-15: lit/len and distance root bits
};

// Parse-pass tokens (u32), consumed by the expand pass:
//   hi16 == 0          literal, byte in bits 0-7 (stored-block bytes included)
//   hi16 in [3, 258]   match: length = hi16, distance = lo16 + 1
// A unit's token i lives in its primary region (i < tcap) or in page k of
// its page table, page k holding 2^k pool units of 2^ZS_TP_LOG tokens
// (geometric, so ZS_TP_MAXPG pages cover any unit), pages being taken on
// demand from a pool shared by the batch (ZsTokPool).  No token count is
// ever guessed from a compression ratio: a unit runs out of room only when
// the pool does.
#define ZS_TP_LOG 16                 // tokens per pool unit: 64 Ki
#define ZS_TP_MAXPG 16               // pages per unit (page k = 2^k pool units)
#define ZS_TOK_PER_BYTE 1            // primary region: tokens per byte of the unit's compressed span
#define ZS_TOK_SLACK 4096            // ... plus this many
struct ZsTokPool {
  uint64_t base;       // token offset of pool unit 1 (page ids = first pool unit, 1-based; 0 = none)
  uint32_t npages;     // pool units (2^ZS_TP_LOG tokens each)
  uint32_t pad;
  uint32_t *next;      // device counter: pages taken
  uint32_t *ptab;      // ZS_TP_MAXPG page ids per unit slot (zeroed by zs_plan_kernel)
};

struct ZsCJobDev {     // a job on the chunked path
  uint32_t job;        // job index
  uint32_t first_seg;  // first search segment
  uint32_t nseg;
  uint32_t unit0;      // first unit slot reserved for this job (host)
  uint32_t max_units;  // unit slots reserved (nseg * SEG_SLOTS + 1)
  uint32_t nunits;     // units planned (zs_plan_kernel)
  uint64_t tok0;       // first token of the job's primary regions (host)
  uint64_t scratch0;   // first u16 entry of the job's entry range (host)
  uint64_t scratch_n;  // entries reserved: min(out_cap, bound) -- the chain's total never exceeds it
  uint32_t nchain;     // units in the verified chain (zs_chain_kernel)
  uint32_t ok;         // chain verified (zs_chain_kernel); cleared again by zs_link_kernel on a bad window
  uint32_t esz;        // u16 slots per entry: 1, or 2 for deflate64 (17-bit entries stored as u32)
  uint32_t pad;
};
// ---------------------------------------------------------------------------
// GPU deflate (deflate_kernels.hip): one job = one whole stream compressed as
// with deflateInit2(level, Z_DEFLATED, window_bits) + deflate(Z_FINISH).
// ---------------------------------------------------------------------------
struct ZsDJobDev {
  const uint8_t *in;
  uint64_t in_len;
  int32_t wrap;        // 0 raw, 1 zlib, 2 gzip
  int32_t level;       // 0 stored, 1..9
  uint32_t seg0;       // first segment
  uint32_t nseg;       // segments (>= 1)
  uint64_t stage;      // byte offset of the job's 4 KiB-aligned staging area
  uint64_t total_out;  // compressed bytes (zs_dz_offsets_kernel)
  uint32_t check;      // CRC-32 (gzip) / Adler-32 (zlib) of the input
  uint32_t wbits;      // window bits 9..15 (match distances <= 2^wbits; zlib CINFO = wbits - 8)
  uint64_t ck_a;       // check accumulators (zs_check.h): CRC XOR / Adler sum A (zeroed by the host)
  uint64_t ck_b;       // Adler weighted sum B
  // zlib-identical mode (deflate_zlib.hip): exact = ZD_SLOW (levels 4..9,
  // deflate_slow) or ZD_FAST (levels 1..3, deflate_fast); 0: the throughput path
  uint32_t exact;
  uint32_t nzblk;      // blocks (zs_zd_blocks_kernel)
  uint64_t pos0;       // first entry of the job's position arrays
  uint64_t bm0;        // first word of the job's bitmaps
  uint32_t zblk0;      // first block slot
  uint32_t zblk_cap;   // block slots reserved: ceil(in_len / 16383) + 1
  // How the job's bits end (ZS_DT_*) and what else it writes.  A one-shot
  // job is hdr = 1, trl = 1, ZS_DT_FINAL from pstart = 0 in state A.  A stream
  // segment (deflate() of the stream surfaces) starts where the previous one
  // stopped: bit0 bits already pending in its first byte, bytes before pstart
  // as history (zlib's window), deflate_slow's state pstate at pstart, the
  // first `skip` symbols from pstart already sent in earlier blocks.
  uint32_t term;       // ZS_DT_FINAL / _SYNC / _PARTIAL / _BLOCK / _CUT
  uint32_t hdr;        // write the wrapper header first
  uint32_t trl;        // ZS_DT_FINAL: write the trailer (check of in[ck0, in_len))
  uint32_t bit0;       // 0..7 bits of the first byte belong to earlier output
  uint32_t pstate;     // deflate_slow state at pstart (deflate_zlib.hip encoding)
  uint32_t cut_state;  // ZS_DT_CUT (out): state at cut_pos
  uint64_t pstart;     // first loop top of the parse (zlib-identical jobs)
  uint64_t skip;       // symbols from pstart that earlier jobs already emitted
  uint64_t abs0;       // stream offset of in[0] since zlib's window last restarted (window slides)
  uint64_t ck0;        // the check covers in[ck0, in_len)
  uint64_t endbit;     // (out) bits of the job's blocks, bit0 and header included, before the terminator
  uint64_t cut_pos;    // ZS_DT_CUT (out): where the next segment's parse starts (job offset)
  uint64_t cut_skip;   // ZS_DT_CUT (out): ... and the symbols from there already emitted
  uint64_t cut_open;   // ZS_DT_CUT (out): symbols of the unsent block zlib has already tallied
  // zlib's pull-on-demand (zs_zd_limit_kernel): deflate() returns right after
  // the block flush that fills the caller's output space, having read only
  // what fill_window had read by then (deflate.c deflate_slow / deflate_fast,
  // FLUSH_BLOCK; fill_window reads to window_size after sliding by w_size once
  // strstart >= w_size + MAX_DIST)
  uint64_t lim_bytes;  // (in) job output bytes the call's output space takes (UINT64_MAX: no limit)
  uint64_t zb;         // (in / out) stream offset (since the window restart) of zlib's window start
  uint64_t rd0;        // (in) job offset up to which zlib has read before this call
  uint64_t rtop;       // (in) the call's first loop top when zlib may fill there (job offset), else UINT64_MAX:
                       //      it resumes where its last fill attempt already took place, and reads at once
  uint64_t rd_out;     // (out) job offset up to which zlib has read when the call returns
  uint64_t next_top;   // (out, early) the loop top the next call resumes at (job offset)
  uint64_t fstop;      // (deflate_fast CUT jobs) the loop top zs_zd_fast_kernel stopped at
  uint32_t early;      // (out) 1: the call returns after block early_k - 1, its output space full
  uint32_t early_k;
  uint32_t nzblk0;     // blocks before the cut (zs_zd_cut_kernel)
  uint32_t pad2;
};
#define ZD_SLOW 1u
#define ZD_FAST 2u
// Level-0 stream calls (zs_stored_call_kernel): one copy piece of the call's
// output -- `len` bytes from the staged source at `src` to output offset `dst`
// (pieces are contiguous in dst order)
struct ZsPiece {
  uint64_t src, dst;
  uint32_t len, pad;
};
// ZsDJobDev::term -- the end of a job's bits, as zlib's deflate() ends a call:
#define ZS_DT_FINAL 0u    // Z_FINISH: last block BFINAL = 1 (an empty one if needed), trailer
#define ZS_DT_SYNC 1u     // Z_SYNC_FLUSH / Z_FULL_FLUSH: blocks not final, empty stored block 00 00 FF FF
#define ZS_DT_PARTIAL 2u  // Z_PARTIAL_FLUSH: blocks not final, then an empty static block (_tr_align, 10 bits)
#define ZS_DT_BLOCK 3u    // Z_BLOCK: blocks not final, nothing after (not byte aligned)
#define ZS_DT_CUT 4u      // Z_NO_FLUSH: only the blocks zlib completes with this input (the stream goes on)
#ifdef __HIP__
// bytes of a job whose blocks end at bit `endbit`: the terminator, then the
// trailer (a ZS_DT_PARTIAL / _BLOCK / _CUT job's last byte is partial: the
// next segment of the stream continues it)
__device__ __forceinline__ uint64_t zs_dz_total_bytes(const ZsDJobDev &jb, uint64_t endbit) {
  switch (jb.term) {
    case ZS_DT_SYNC: return (endbit + 3 + 7) / 8 + 4;  // 000, pad, 00 00 FF FF
    case ZS_DT_PARTIAL: return (endbit + 10 + 7) / 8;
    case ZS_DT_BLOCK:
    case ZS_DT_CUT: return (endbit + 7) / 8;
    default: return (endbit + 7) / 8 + (jb.trl ? (jb.wrap == 2 ? 8u : (jb.wrap == 1 ? 4u : 0u)) : 0u);
  }
}
#endif

// zlib-identical mode (deflate_zlib.hip, levels 4..9): per job, position
// arrays at pos0 (previous same-hash distance u16, the two longest-match
// tables u32), bitmaps at bm0 (token starts S, match-table variant V, walk
// state-A marks M; one u32 word per 32 positions each), and blocks of 16383
// symbols at zblk0 (ZsZBlkDev), as zlib's deflate_slow + trees.c make them.
struct ZsZBlkDev {
  uint32_t job;
  uint32_t last;       // BFINAL
  uint64_t first;      // first input byte covered (== end for an empty block)
  uint64_t end;        // one past the last byte covered
  uint32_t nsym;       // symbols (<= 16383)
  uint32_t type;       // 0 stored, 1 fixed, 2 dynamic (zs_zd_tree_kernel)
  uint32_t stored_ok;  // the block's bytes still in zlib's window (_tr_flush_block's buf != NULL)
  uint32_t hbits;      // dynamic: tree header bits after the 3 block-type bits
  uint64_t bits;       // bits after the 3 block-type bits (stored: bytes * 8 + 32, alignment added at layout)
  uint64_t bitoff;     // bit offset of the block in the job's stream (zs_zd_layout_kernel)
  uint64_t top;        // loop top of the deflate_slow iteration that flushes it
  uint32_t lmax, dmax, blmax, pad;
};

struct ZsDSegDev {
  uint32_t job;
  uint32_t last;       // 1: the job's last segment (BFINAL)
  uint64_t start;      // input byte offset
  uint32_t len;        // input bytes (<= 64 KiB)
  uint32_t ntok;       // tokens (parse)
  uint64_t tok;        // offset of the segment's match/token region (u32 units)
  uint64_t obuf;       // byte offset of the segment's block buffer
  uint64_t bitoff;     // bit offset of the block in the job's stream
  uint32_t nbits;      // block bits
  uint32_t ck_a;       // CRC-32 of the segment, or Adler sum a
  uint32_t ck_b;       // Adler weighted sum b (to the segment end)
  // zlib-identical mode: the segment is a 64 KiB parse region; its exit is
  // the first loop top past it and deflate_slow's state there
  uint32_t nsym;       // token starts in the region
  uint32_t zs0;        // exit state of the region's own parse (entry = its start, state A)
  uint64_t zx0;        // ... and its position
  uint64_t zx[2];      // current exit (double-buffered across fix-up rounds)
  uint32_t zs[2];
  uint64_t zfix;       // tokens rewritten by fix-ups up to this position
  uint64_t sym0;       // symbols before the region (zs_zd_blocks_kernel)
};

// ---------------------------------------------------------------------------
// Exact streaming inflate (the reference's per-call contract, SURVEY §8b
// Tier 2): one handle's decoder state lives in device memory between calls,
// so each inflate(strm, flush) call of the handle / zlib ABI is one resumable
// decode on the GPU with zlib's pull-on-demand accounting.  The modes name
// the states of src/inflate.c (inflate.h:21-54) where a call can return.
// ---------------------------------------------------------------------------
enum ZsStreamMode {
  ZSM_HEAD = 0,    // wrapper header not complete yet (re-parsed from byte 0 of the carry)
  ZSM_TYPE = 1,    // at a block header (TYPE..CODELENS restart here)
  ZSM_SYMS = 2,    // inside a fixed/dynamic block at a symbol (LEN..DISTEXT restart here)
  ZSM_LIT = 3,     // LIT with left == 0: literal `len` pending
  ZSM_MATCH = 4,   // MATCH with left == 0: `len` bytes at `dist` pending
  ZSM_STORED = 5,  // COPY: `len` stored bytes pending
  ZSM_CHECK = 6,   // trailer CHECK (byte aligned)
  ZSM_LENGTH = 7,  // gzip trailer LENGTH
  ZSM_DONE = 8,
  ZSM_BAD = 9,
  ZSM_DICT = 10    // zlib FDICT: Z_NEED_DICT on every call
};

#define ZS_STREAM_TAB_WORDS 1448u  // TABLE_ENTRIES (zs_device.h)
struct ZsStreamDev {
  // resume point, in and out of every call; bit offsets relative to the
  // call buffer (the host rebases them onto the bytes it carries over)
  int32_t mode;        // ZsStreamMode
  uint32_t rbit;       // restart bit
  uint32_t last;       // BFINAL of the current block
  uint32_t btype;      // 1 fixed, 2 dynamic (SYMS / LIT / MATCH)
  uint32_t nlen, ndist;
  uint32_t len, dist;  // LIT literal; MATCH remaining length + distance; STORED remaining bytes
  uint32_t wbits;      // window bits (0: from the zlib header)
  int32_t is_gzip;     // -1 raw, 0 zlib, 1 gzip (set by the header)
  uint64_t total_out;  // bytes produced by earlier calls
  uint32_t ck_a, ck_b; // running check: CRC-32 register f(0, out) (zs_check.h) / Adler a, b
  // outcome of the last call
  int32_t code;        // ZD_END / ZD_TRUNC / ZD_FULL / ZD_ERROR / ZD_NEED_DICT
  int32_t msg;         // ZsMsg
  uint32_t stop_bits;  // bits pulled (FULL / END / ERROR / trailer): zlib total_in = ceil(/8)
  uint32_t produced;   // bytes written this call
  uint32_t check;      // strm->adler after the call
  uint32_t tab_bits;   // tab holds the current dynamic block's tables: lbits | dbits << 8 | 1 << 16 (0: rebuild)
  uint64_t acc_a, acc_b;  // check accumulators of this call's output
  uint8_t lens[320];   // code lengths of the current dynamic block
  __attribute__((aligned(16))) uint8_t window[65536];  // last 64 KiB (32 KiB used unless deflate64) of output, oldest first
  __attribute__((aligned(16))) uint32_t tab[ZS_STREAM_TAB_WORDS];  // built tables (TABLE_ENTRIES), see tab_bits
};

// Host side of one stream call (zs_capi.cpp sq_launch): with host-mapped
// pinned staging the call needs no copy of its own -- the batch's first kernel
// pulls every input into its device buffer and the check kernel pushes every
// output out.  Null pointers: the host copied by DMA (calls above the staging size).
struct ZsStreamIo {
  const uint8_t *hin;  // host-mapped input, in_len bytes -> the job's in
  uint8_t *hout;       // host-mapped output: the call's produced bytes <- the job's out
  uint32_t rbit;       // restart bit within input byte 0 (the carried partial byte)
  uint32_t fresh;      // 1: the handle's first call since init / reset -- the device state is set up first
};

// Outcome of one stream call (device -> host, gathered per batch).
struct ZsStreamRes {
  int32_t mode;
  uint32_t rbit;
  int32_t code;
  int32_t msg;
  uint32_t stop_bits;
  uint32_t produced;
  uint32_t check;
  int32_t is_gzip;
};

// Mailbox of one workgroup of the persistent stream worker (zs_stream_pk_kernel),
// in host-coherent pinned memory: the host writes the call (st, io, job), then
// seq_in; the workgroup runs it and writes res, then seq_out = seq_in.
struct ZsMbox {
  uint32_t seq_in;   // host -> device, written last
  uint32_t seq_out;  // device -> host, written last
  uint32_t pad0[2];
  ZsStreamDev *st;   // words 4..5: the call (ZS_MBOX_CALL_WORDS from word 4)
  uint64_t pad1;
  ZsStreamIo io;     // words 8..13
  uint64_t pad2;
  ZsJobDev job;      // words 16..31
  ZsStreamRes res;   // words 32..39
  uint32_t busy;     // word 40: the call's s_memrealtime ticks (100 MHz) from pickup to done
  uint32_t idle;     // word 41: ticks the workgroup waited for this call since its previous one
  uint32_t pad3[22];
};
#define ZS_MBOX_CALL_WORDS 28u  // st .. job (words 4..31)
static_assert(sizeof(ZsMbox) == 256, "one mailbox per 256 bytes");
static_assert(offsetof(ZsMbox, io) == 32 && offsetof(ZsMbox, job) == 64 && offsetof(ZsMbox, res) == 128, "mailbox layout");
// persistent worker control words (host-coherent): [0] stop, [1] posts (any mailbox)
#define ZS_PK_CTL_WORDS 16u

// Final per-job result (device -> host), zlib z_stream fields after the call.
struct ZsResultDev {
  int32_t ret;
  int32_t msg;
  uint64_t total_in;
  uint64_t total_out;
  uint32_t adler;
  int32_t pad;
};
