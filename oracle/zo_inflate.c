/*
 * zo_inflate.c -- CPU ORACLE.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker for the MI355X inflate path.  It is a
 * clean-room C restatement of the reference's resumable inflate state machine
 * (gildas-lormeau/zlib-streams, a deflate64-patched zlib 1.3.1.1 inflate):
 *
 *   - src/inflate.c:597-1275   inflate() state machine, wrappers, checks,
 *                              inf_leave accounting (1253-1274)
 *   - src/inflate.c:147-224    inflateReset2 / inflateInit2_ windowBits rules
 *                              (deflate64 when windowBits == -16, 156-161)
 *   - src/inflate.c:260-298    fixed tables (per mode)
 *   - src/inflate.c:375-419    updatewindow()
 *   - src/inffast.c:50-304     fast loop, including its byte accounting
 *                              (2-byte refills, unused-byte return 289-303)
 *   - src/inftrees.c:33-321    canonical Huffman -> 2-level table builder,
 *                              deflate64 base/extra tables (73-87), empty-code
 *                              reject (131-132), ENOUGH-1 limits (211-212)
 *
 * CRC-32 and Adler-32 live in the absent zlib submodule (src/zlib, madler/zlib
 * "1.3.1.1" per src/inftrees.c:13); they are restated here from their
 * published definitions (reflected CRC-32, poly 0xEDB88320; Adler-32 mod
 * 65521), not linked from any zlib.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (zlib-streams_amd/) never links it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#include "zo_inflate.h"

/* ------------------------------------------------------------------------ */
/* checks                                                                    */
/* ------------------------------------------------------------------------ */

static uint32_t crc_tab[256];
static int crc_ready = 0;

static void crc_init(void) {
  for (uint32_t n = 0; n < 256; n++) {
    uint32_t c = n;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
    crc_tab[n] = c;
  }
  crc_ready = 1;
}

uint32_t zo_crc32(uint32_t crc, const uint8_t *p, size_t n) {
  if (!crc_ready) crc_init();
  crc = ~crc;
  while (n--) crc = crc_tab[(crc ^ *p++) & 0xff] ^ (crc >> 8);
  return ~crc;
}

uint32_t zo_adler32(uint32_t adler, const uint8_t *p, size_t n) {
  uint32_t a = adler & 0xffff, b = adler >> 16;
  while (n) {
    size_t k = n < 5552 ? n : 5552; /* largest run without 32-bit overflow */
    n -= k;
    while (k--) { a += *p++; b += a; }
    a %= 65521u;
    b %= 65521u;
  }
  return (b << 16) | a;
}

/* ------------------------------------------------------------------------ */
/* table builder  (restates src/inftrees.c:33-321)                          */
/* ------------------------------------------------------------------------ */

enum { T_CODES = 0, T_LENS = 1, T_DISTS = 2 };

/* Length / distance base and extra-bit columns.  The op byte of an entry is
   16+extra (deflate) or 128+extra (deflate64); 64 = invalid, 96 = end of
   block (src/inftrees.h:31-38). */
static const uint16_t len_base_std[31] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                          35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 0, 0};
static const uint16_t len_op_std[31] = {16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 18, 18, 18, 18,
                                        19, 19, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21, 16, 73, 200};
static const uint16_t dist_base_std[32] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                           257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145,
                                           8193, 12289, 16385, 24577, 0, 0};
static const uint16_t dist_op_std[32] = {16, 16, 16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 21, 21, 22, 22,
                                         23, 23, 24, 24, 25, 25, 26, 26, 27, 27, 28, 28, 29, 29, 64, 64};
/* deflate64: code 285 is base 3 with 16 extra bits; distance codes 30/31 */
static const uint16_t len_base_d64[31] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                          35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 3, 0, 0};
static const uint16_t len_op_d64[31] = {128, 128, 128, 128, 128, 128, 128, 128, 129, 129, 129, 129,
                                        130, 130, 130, 130, 131, 131, 131, 131, 132, 132, 132, 132,
                                        133, 133, 133, 133, 144, 73, 200};
static const uint16_t dist_base_d64[32] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                           257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145,
                                           8193, 12289, 16385, 24577, 32769, 49153};
static const uint16_t dist_op_d64[32] = {128, 128, 128, 128, 129, 129, 130, 130, 131, 131, 132, 132,
                                         133, 133, 134, 134, 135, 135, 136, 136, 137, 137, 138, 138,
                                         139, 139, 140, 140, 141, 141, 142, 142};

#define ZO_LIMIT_LENS 852u  /* src/inftrees.h:52 */
#define ZO_LIMIT_DISTS 592u /* src/inftrees.h:53 */
#define ZO_LIMIT_DISTS9 594u

/* Returns 0 ok, -1 bad code, 1 table space exceeded.  *tab advances by the
   entries used; *root is in/out (requested / actual root bits). */
static int build_table(int type, const uint16_t *lens, unsigned n, zo_code **tab,
                       unsigned *root_io, uint16_t *order, int d64) {
  uint16_t cnt[16], start[16];
  memset(cnt, 0, sizeof cnt);
  for (unsigned s = 0; s < n; s++) cnt[lens[s]]++;

  unsigned maxlen = 15;
  while (maxlen >= 1 && cnt[maxlen] == 0) maxlen--;
  unsigned root = *root_io;
  if (root > maxlen) root = maxlen;
  if (maxlen == 0) {
    /* no codes at all: deflate64 rejects (inftrees.c:131-132); deflate builds
       a 1-bit table of invalid markers so decoding reports the error */
    if (d64) return -1;
    zo_code bad = {64, 1, 0};
    (*tab)[0] = bad;
    (*tab)[1] = bad;
    *tab += 2;
    *root_io = 1;
    return 0;
  }
  unsigned minlen = 1;
  while (minlen < maxlen && cnt[minlen] == 0) minlen++;
  if (root < minlen) root = minlen;

  /* Kraft check: over-subscribed always bad; incomplete bad unless a single
     one-bit code in a LENS/DISTS table */
  int room = 1;
  for (unsigned l = 1; l <= 15; l++) {
    room = (room << 1) - cnt[l];
    if (room < 0) return -1;
  }
  if (room > 0 && (type == T_CODES || maxlen != 1)) return -1;

  start[1] = 0;
  for (unsigned l = 1; l < 15; l++) start[l + 1] = start[l] + cnt[l];
  for (unsigned s = 0; s < n; s++)
    if (lens[s]) order[start[lens[s]]++] = (uint16_t)s;

  const uint16_t *base = NULL, *ops = NULL;
  unsigned first_coded = 0; /* symbols >= this use base/ops; 20 => none */
  if (type == T_CODES) {
    first_coded = 20;
  } else if (type == T_LENS) {
    base = d64 ? len_base_d64 : len_base_std;
    ops = d64 ? len_op_d64 : len_op_std;
    first_coded = 257;
  } else {
    base = d64 ? dist_base_d64 : dist_base_std;
    ops = d64 ? dist_op_d64 : dist_op_std;
    first_coded = 0;
  }
  unsigned lim_lens = d64 ? ZO_LIMIT_LENS - 1 : ZO_LIMIT_LENS;
  unsigned lim_dists = d64 ? ZO_LIMIT_DISTS9 - 1 : ZO_LIMIT_DISTS;

  zo_code *tbl = *tab;    /* root of this table set */
  zo_code *sub = tbl;     /* table currently being filled */
  unsigned cur = root;    /* index bits of current table */
  unsigned shift = 0;     /* code bits consumed by the root (0 while in root) */
  unsigned used = 1u << root;
  unsigned rmask = used - 1;
  unsigned open_low = ~0u; /* root index owning the current sub-table */
  unsigned code = 0;       /* bit-reversed canonical code */
  unsigned len = minlen;
  unsigned sym = 0;
  unsigned stride_prev = 0;

  if ((type == T_LENS && used > lim_lens) || (type == T_DISTS && used > lim_dists)) return 1;

  for (;;) {
    zo_code e;
    unsigned s = order[sym];
    e.bits = (uint8_t)(len - shift);
    if (s + 1u < first_coded) {
      e.op = 0;
      e.val = (uint16_t)s;
    } else if (s >= first_coded) {
      e.op = (uint8_t)ops[s - first_coded];
      e.val = base[s - first_coded];
    } else {
      e.op = 32 + 64; /* end of block */
      e.val = 0;
    }
    /* replicate over all indices whose low (len-shift) bits equal code>>shift */
    unsigned step = 1u << (len - shift);
    unsigned span = 1u << cur;
    stride_prev = span;
    for (unsigned k = span; k != 0;) {
      k -= step;
      sub[(code >> shift) + k] = e;
    }
    /* advance the reversed code: add one at the top bit of a len-bit code */
    unsigned bit = 1u << (len - 1);
    while (code & bit) bit >>= 1;
    code = bit ? ((code & (bit - 1)) + bit) : 0;

    sym++;
    if (--cnt[len] == 0) {
      if (len == maxlen) break;
      len = lens[order[sym]];
    }
    if (len > root && (code & rmask) != open_low) {
      if (shift == 0) shift = root;
      sub += stride_prev;
      /* size the sub-table: grow while the remaining codes need more room */
      cur = len - shift;
      int need = 1 << cur;
      while (cur + shift < maxlen) {
        need -= cnt[cur + shift];
        if (need <= 0) break;
        cur++;
        need <<= 1;
      }
      used += 1u << cur;
      if ((type == T_LENS && used > lim_lens) || (type == T_DISTS && used > lim_dists)) return 1;
      open_low = code & rmask;
      tbl[open_low].op = (uint8_t)cur;
      tbl[open_low].bits = (uint8_t)root;
      tbl[open_low].val = (uint16_t)(sub - tbl);
    }
  }
  if (code != 0) { /* incomplete single-code table: one invalid slot left */
    zo_code bad;
    bad.op = 64;
    bad.bits = (uint8_t)(len - shift);
    bad.val = 0;
    sub[code] = bad;
  }
  *tab += used;
  *root_io = root;
  return 0;
}

/* ------------------------------------------------------------------------ */
/* state                                                                     */
/* ------------------------------------------------------------------------ */

/* Mode order matters: inf_leave compares against CHECK and BAD exactly as
   src/inflate.c:1256-1257 does with the enum of src/inflate.h:21-54. */
enum {
  S_HEAD = 0, S_FLAGS, S_TIME, S_OS, S_EXLEN, S_EXTRA, S_NAME, S_COMMENT, S_HCRC,
  S_DICTID, S_DICT, S_TYPE, S_TYPEDO, S_STORED, S_COPY_, S_COPY, S_TABLE, S_LENLENS,
  S_CODELENS, S_LEN_, S_LEN, S_LENEXT, S_DIST, S_DISTEXT, S_MATCH, S_LIT, S_CHECK,
  S_LENGTH, S_DONE, S_BAD, S_MEM, S_SYNC
};

#define ZO_TABLE_SPACE (852 + 594)

typedef struct zo_state {
  int mode, last, wrap, flags, d64;
  uint32_t check;
  uint64_t total;
  unsigned wbits, wsize, whave, wnext;
  uint8_t *window;
  uint64_t hold;
  unsigned bits;
  unsigned length, offset, extra;
  const zo_code *lcode, *dcode;
  unsigned lbits, dbits;
  unsigned ncode, nlen, ndist, have;
  zo_code *next;
  uint16_t lens[320];
  uint16_t work[288];
  zo_code codes[ZO_TABLE_SPACE];
  int back;
  unsigned was;
} zo_state;

static zo_code fixed_set[2][544];
static const zo_code *fixed_l[2], *fixed_d[2];
static int fixed_done[2];

static void use_fixed(zo_state *st) {
  int m = st->d64;
  if (!fixed_done[m]) {
    uint16_t l[288], w[288];
    unsigned s = 0, rb;
    while (s < 144) l[s++] = 8;
    while (s < 256) l[s++] = 9;
    while (s < 280) l[s++] = 7;
    while (s < 288) l[s++] = 8;
    zo_code *nx = fixed_set[m];
    fixed_l[m] = nx;
    rb = 9;
    build_table(T_LENS, l, 288, &nx, &rb, w, m);
    for (s = 0; s < 32; s++) l[s] = 5;
    fixed_d[m] = nx;
    rb = 5;
    build_table(T_DISTS, l, 32, &nx, &rb, w, m);
    fixed_done[m] = 1;
  }
  st->lcode = fixed_l[m];
  st->lbits = 9;
  st->dcode = fixed_d[m];
  st->dbits = 5;
}

static int state_bad(zo_stream *z) {
  return z == NULL || z->st == NULL || z->st->mode < S_HEAD || z->st->mode > S_SYNC;
}

static void reset_keep(zo_stream *z) {
  zo_state *st = z->st;
  z->total_in = z->total_out = 0;
  st->total = 0;
  z->msg = NULL;
  if (st->wrap) z->adler = (uint32_t)(st->wrap & 1);
  st->mode = S_HEAD;
  st->last = 0;
  st->flags = -1;
  st->hold = 0;
  st->bits = 0;
  st->lcode = st->dcode = st->next = st->codes;
  st->back = -1;
}

int zo_inflate_init2(zo_stream *z, int wbits) {
  if (z == NULL) return ZO_STREAM_ERROR;
  z->msg = NULL;
  zo_state *st = (zo_state *)calloc(1, sizeof(zo_state));
  if (!st) return ZO_MEM_ERROR;
  z->st = st;
  st->window = NULL;
  st->mode = S_HEAD;
  int wrap;
  if (wbits < 0) {
    if (wbits < -16) goto bad;
    wrap = 0;
    st->d64 = (wbits == -16);
    wbits = -wbits;
  } else {
    wrap = (wbits >> 4) + 5;
    st->d64 = 0;
    if (wbits < 48) wbits &= 15;
  }
  if (wbits && (wbits < 8 || wbits > (st->d64 ? 16 : 15))) goto bad;
  st->wrap = wrap;
  st->wbits = (unsigned)wbits;
  st->wsize = st->whave = st->wnext = 0;
  reset_keep(z);
  return ZO_OK;
bad:
  free(st);
  z->st = NULL;
  return ZO_STREAM_ERROR;
}

int zo_inflate_end(zo_stream *z) {
  if (state_bad(z)) return ZO_STREAM_ERROR;
  free(z->st->window);
  free(z->st);
  z->st = NULL;
  return ZO_OK;
}

/* keep the last wsize bytes of output in the circular window
   (src/inflate.c:375-419) */
static int window_keep(zo_stream *z, const uint8_t *end, unsigned n) {
  zo_state *st = z->st;
  if (!st->window) {
    st->window = (uint8_t *)malloc(1u << st->wbits);
    if (!st->window) return 1;
  }
  if (st->wsize == 0) {
    st->wsize = 1u << st->wbits;
    st->wnext = st->whave = 0;
  }
  if (n >= st->wsize) {
    memcpy(st->window, end - st->wsize, st->wsize);
    st->wnext = 0;
    st->whave = st->wsize;
    return 0;
  }
  unsigned room = st->wsize - st->wnext;
  if (room > n) room = n;
  memcpy(st->window + st->wnext, end - n, room);
  n -= room;
  if (n) {
    memcpy(st->window, end - n, n);
    st->wnext = n;
    st->whave = st->wsize;
  } else {
    st->wnext += room;
    if (st->wnext == st->wsize) st->wnext = 0;
    if (st->whave < st->wsize) st->whave += room;
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* fast loop (restates src/inffast.c:50-304, same byte accounting)          */
/* ------------------------------------------------------------------------ */

static void fast_loop(zo_stream *z, unsigned start_out) {
  zo_state *st = z->st;
  const uint8_t *in = z->next_in;
  const uint8_t *in_stop = in + (z->avail_in - 5);
  uint8_t *out = z->next_out;
  uint8_t *out0 = out - (start_out - z->avail_out);
  uint8_t *out_stop = out + (z->avail_out - 257);
  unsigned wsize = st->wsize, whave = st->whave, wnext = st->wnext;
  const uint8_t *win = st->window;
  uint64_t hold = st->hold;
  unsigned bits = st->bits;
  const zo_code *lc = st->lcode, *dc = st->dcode;
  unsigned lm = (1u << st->lbits) - 1, dm = (1u << st->dbits) - 1;

  do {
    if (bits < 15) {
      hold += (uint64_t)(*in++) << bits; bits += 8;
      hold += (uint64_t)(*in++) << bits; bits += 8;
    }
    const zo_code *e = lc + (hold & lm);
    for (;;) {
      unsigned op = e->bits;
      hold >>= op;
      bits -= op;
      op = e->op;
      if (op == 0) {
        *out++ = (uint8_t)e->val;
        break;
      }
      if (op & 16) {
        unsigned len = e->val;
        op &= 15;
        if (op) {
          if (bits < op) { hold += (uint64_t)(*in++) << bits; bits += 8; }
          len += (unsigned)hold & ((1u << op) - 1);
          hold >>= op;
          bits -= op;
        }
        if (bits < 15) {
          hold += (uint64_t)(*in++) << bits; bits += 8;
          hold += (uint64_t)(*in++) << bits; bits += 8;
        }
        const zo_code *d = dc + (hold & dm);
        for (;;) {
          unsigned dop = d->bits;
          hold >>= dop;
          bits -= dop;
          dop = d->op;
          if (dop & 16) {
            unsigned dist = d->val;
            dop &= 15;
            if (bits < dop) {
              hold += (uint64_t)(*in++) << bits; bits += 8;
              if (bits < dop) { hold += (uint64_t)(*in++) << bits; bits += 8; }
            }
            dist += (unsigned)hold & ((1u << dop) - 1);
            hold >>= dop;
            bits -= dop;
            unsigned have_out = (unsigned)(out - out0);
            if (dist > have_out) {
              unsigned back = dist - have_out; /* bytes needed from window */
              if (back > whave) {
                z->msg = "invalid distance too far back";
                st->mode = S_BAD;
                goto leave;
              }
              /* position of the first window byte in the circular buffer */
              unsigned pos = (wnext >= back) ? wnext - back : wsize + wnext - back;
              while (len && back) {
                *out++ = win[pos];
                pos = (pos + 1 == wsize) ? 0 : pos + 1;
                back--;
                len--;
              }
            }
            const uint8_t *from = out - dist;
            while (len--) *out++ = *from++;
            goto next_sym;
          } else if ((dop & 64) == 0) {
            d = dc + d->val + (hold & ((1u << dop) - 1));
            continue;
          } else {
            z->msg = "invalid distance code";
            st->mode = S_BAD;
            goto leave;
          }
        }
      } else if ((op & 64) == 0) {
        e = lc + e->val + (hold & ((1u << op) - 1));
        continue;
      } else if (op & 32) {
        st->mode = S_TYPE;
        goto leave;
      } else {
        z->msg = "invalid literal/length code";
        st->mode = S_BAD;
        goto leave;
      }
    }
  next_sym:;
  } while (in < in_stop && out < out_stop);
leave:;
  /* give back whole unused bytes (src/inffast.c:289-293) */
  unsigned spare = bits >> 3;
  in -= spare;
  bits -= spare << 3;
  hold &= (1ull << bits) - 1;
  z->next_in = in;
  z->next_out = out;
  z->avail_in = (unsigned)(in < in_stop ? 5 + (in_stop - in) : 5 - (in - in_stop));
  z->avail_out = (unsigned)(out < out_stop ? 257 + (out_stop - out) : 257 - (out - out_stop));
  st->hold = hold;
  st->bits = bits;
}

/* ------------------------------------------------------------------------ */
/* state machine (restates src/inflate.c:597-1275)                           */
/* ------------------------------------------------------------------------ */

static const uint8_t cl_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

#define PULL()                                         \
  do {                                                 \
    if (have == 0) goto leave;                         \
    have--;                                            \
    hold += (uint64_t)(*next++) << bits;               \
    bits += 8;                                         \
  } while (0)
#define NEED(n)                                        \
  do {                                                 \
    while (bits < (unsigned)(n)) PULL();               \
  } while (0)
#define PEEK(n) ((unsigned)hold & ((1u << (n)) - 1))
#define SKIP(n)                                        \
  do {                                                 \
    hold >>= (n);                                      \
    bits -= (unsigned)(n);                             \
  } while (0)
#define CLEAR()                                        \
  do {                                                 \
    hold = 0;                                          \
    bits = 0;                                          \
  } while (0)
#define ALIGN()                                        \
  do {                                                 \
    hold >>= bits & 7;                                 \
    bits -= bits & 7;                                  \
  } while (0)
#define FAIL(m)                                        \
  do {                                                 \
    z->msg = (m);                                      \
    st->mode = S_BAD;                                  \
  } while (0)
#define CHECK_UPDATE(chk, p, n) (st->flags ? zo_crc32((chk), (p), (n)) : zo_adler32((chk), (p), (n)))

static void crc_word(uint32_t *c, uint64_t w, int nbytes) {
  uint8_t b[4];
  for (int i = 0; i < nbytes; i++) b[i] = (uint8_t)(w >> (8 * i));
  *c = zo_crc32(*c, b, (size_t)nbytes);
}

int zo_inflate(zo_stream *z, int flush) {
  if (state_bad(z) || z->next_out == NULL || (z->next_in == NULL && z->avail_in != 0))
    return ZO_STREAM_ERROR;
  zo_state *st = z->st;
  if (st->mode == S_TYPE) st->mode = S_TYPEDO;

  uint8_t *put = z->next_out;
  unsigned left = z->avail_out;
  const uint8_t *next = z->next_in;
  unsigned have = z->avail_in;
  uint64_t hold = st->hold;
  unsigned bits = st->bits;
  unsigned in0 = have, out0 = left;
  int ret = ZO_OK;
  zo_code here, parent;
  unsigned n;

  for (;;) {
    switch (st->mode) {
      case S_HEAD:
        if (st->wrap == 0) {
          st->mode = S_TYPEDO;
          break;
        }
        NEED(16);
        if ((st->wrap & 2) && hold == 0x8b1f) { /* gzip magic */
          if (st->wbits == 0) st->wbits = 15;
          st->check = 0;
          crc_word(&st->check, hold, 2);
          CLEAR();
          st->mode = S_FLAGS;
          break;
        }
        if (!(st->wrap & 1) || ((PEEK(8) << 8) + (unsigned)(hold >> 8)) % 31) {
          FAIL("incorrect header check");
          break;
        }
        if (PEEK(4) != 8) {
          FAIL("unknown compression method");
          break;
        }
        SKIP(4);
        n = PEEK(4) + 8;
        if (st->wbits == 0) st->wbits = n;
        if (n > 15 || n > st->wbits) {
          FAIL("invalid window size");
          break;
        }
        st->flags = 0;
        z->adler = st->check = 1;
        st->mode = (hold & 0x200) ? S_DICTID : S_TYPE;
        CLEAR();
        break;
      case S_FLAGS:
        NEED(16);
        st->flags = (int)hold;
        if ((st->flags & 0xff) != 8) {
          FAIL("unknown compression method");
          break;
        }
        if (st->flags & 0xe000) {
          FAIL("unknown header flags set");
          break;
        }
        if ((st->flags & 0x0200) && (st->wrap & 4)) crc_word(&st->check, hold, 2);
        CLEAR();
        st->mode = S_TIME;
        /* fallthrough */
      case S_TIME:
        NEED(32);
        if ((st->flags & 0x0200) && (st->wrap & 4)) crc_word(&st->check, hold, 4);
        CLEAR();
        st->mode = S_OS;
        /* fallthrough */
      case S_OS:
        NEED(16);
        if ((st->flags & 0x0200) && (st->wrap & 4)) crc_word(&st->check, hold, 2);
        CLEAR();
        st->mode = S_EXLEN;
        /* fallthrough */
      case S_EXLEN:
        if (st->flags & 0x0400) {
          NEED(16);
          st->length = (unsigned)hold;
          if ((st->flags & 0x0200) && (st->wrap & 4)) crc_word(&st->check, hold, 2);
          CLEAR();
        }
        st->mode = S_EXTRA;
        /* fallthrough */
      case S_EXTRA:
        if (st->flags & 0x0400) {
          n = st->length;
          if (n > have) n = have;
          if (n) {
            if ((st->flags & 0x0200) && (st->wrap & 4)) st->check = zo_crc32(st->check, next, n);
            have -= n;
            next += n;
            st->length -= n;
          }
          if (st->length) goto leave;
        }
        st->length = 0;
        st->mode = S_NAME;
        /* fallthrough */
      case S_NAME:
      case S_COMMENT: {
        for (;;) {
          int flag = (st->mode == S_NAME) ? 0x0800 : 0x1000;
          if (st->flags & flag) {
            if (have == 0) goto leave;
            unsigned k = 0, c;
            do {
              c = next[k++];
            } while (c && k < have);
            if ((st->flags & 0x0200) && (st->wrap & 4)) st->check = zo_crc32(st->check, next, k);
            have -= k;
            next += k;
            if (c) goto leave;
          }
          st->length = 0;
          if (st->mode == S_NAME) {
            st->mode = S_COMMENT;
            continue;
          }
          break;
        }
        st->mode = S_HCRC;
      }
        /* fallthrough */
      case S_HCRC:
        if (st->flags & 0x0200) {
          NEED(16);
          if ((st->wrap & 4) && hold != (st->check & 0xffff)) {
            FAIL("header crc mismatch");
            break;
          }
          CLEAR();
        }
        z->adler = st->check = 0;
        st->mode = S_TYPE;
        break;
      case S_DICTID:
        NEED(32);
        {
          uint32_t v = (uint32_t)hold;
          v = (v >> 24) | ((v >> 8) & 0xff00) | ((v & 0xff00) << 8) | (v << 24);
          z->adler = st->check = v;
        }
        CLEAR();
        st->mode = S_DICT;
        /* fallthrough */
      case S_DICT:
        /* no inflateSetDictionary in the reference ABI: always ask */
        z->next_out = put;
        z->avail_out = left;
        z->next_in = next;
        z->avail_in = have;
        st->hold = hold;
        st->bits = bits;
        return ZO_NEED_DICT;
      case S_TYPE:
        if (flush == ZO_BLOCK || flush == ZO_TREES) goto leave;
        /* fallthrough */
      case S_TYPEDO:
        if (st->last) {
          ALIGN();
          st->mode = S_CHECK;
          break;
        }
        NEED(3);
        st->last = (int)PEEK(1);
        SKIP(1);
        switch (PEEK(2)) {
          case 0:
            st->mode = S_STORED;
            break;
          case 1:
            use_fixed(st);
            st->mode = S_LEN_;
            if (flush == ZO_TREES) {
              SKIP(2);
              goto leave;
            }
            break;
          case 2:
            st->mode = S_TABLE;
            break;
          default:
            FAIL("invalid block type");
        }
        SKIP(2);
        break;
      case S_STORED:
        ALIGN();
        NEED(32);
        if ((hold & 0xffff) != ((hold >> 16) ^ 0xffff)) {
          FAIL("invalid stored block lengths");
          break;
        }
        st->length = (unsigned)hold & 0xffff;
        CLEAR();
        st->mode = S_COPY_;
        if (flush == ZO_TREES) goto leave;
        /* fallthrough */
      case S_COPY_:
        st->mode = S_COPY;
        /* fallthrough */
      case S_COPY:
        n = st->length;
        if (n) {
          if (n > have) n = have;
          if (n > left) n = left;
          if (n == 0) goto leave;
          memcpy(put, next, n);
          have -= n;
          next += n;
          left -= n;
          put += n;
          st->length -= n;
          break;
        }
        st->mode = S_TYPE;
        break;
      case S_TABLE:
        NEED(14);
        st->nlen = PEEK(5) + 257;
        SKIP(5);
        st->ndist = PEEK(5) + 1;
        SKIP(5);
        st->ncode = PEEK(4) + 4;
        SKIP(4);
        if (st->nlen > 286 || (!st->d64 && st->ndist > 30)) {
          FAIL("too many length or distance symbols");
          break;
        }
        st->have = 0;
        st->mode = S_LENLENS;
        /* fallthrough */
      case S_LENLENS:
        while (st->have < st->ncode) {
          NEED(3);
          st->lens[cl_order[st->have++]] = (uint16_t)PEEK(3);
          SKIP(3);
        }
        while (st->have < 19) st->lens[cl_order[st->have++]] = 0;
        st->next = st->codes;
        st->lcode = st->dcode = st->next;
        st->lbits = 7;
        if (build_table(T_CODES, st->lens, 19, &st->next, &st->lbits, st->work, st->d64)) {
          FAIL("invalid code lengths set");
          break;
        }
        st->have = 0;
        st->mode = S_CODELENS;
        /* fallthrough */
      case S_CODELENS:
        while (st->have < st->nlen + st->ndist) {
          for (;;) {
            here = st->lcode[PEEK(st->lbits)];
            if ((unsigned)here.bits <= bits) break;
            PULL();
          }
          if (here.val < 16) {
            SKIP(here.bits);
            st->lens[st->have++] = here.val;
          } else {
            unsigned rep, fillv;
            if (here.val == 16) {
              NEED(here.bits + 2);
              SKIP(here.bits);
              if (st->have == 0) {
                FAIL("invalid bit length repeat");
                break;
              }
              fillv = st->lens[st->have - 1];
              rep = 3 + PEEK(2);
              SKIP(2);
            } else if (here.val == 17) {
              NEED(here.bits + 3);
              SKIP(here.bits);
              fillv = 0;
              rep = 3 + PEEK(3);
              SKIP(3);
            } else {
              NEED(here.bits + 7);
              SKIP(here.bits);
              fillv = 0;
              rep = 11 + PEEK(7);
              SKIP(7);
            }
            if (st->have + rep > st->nlen + st->ndist) {
              FAIL("invalid bit length repeat");
              break;
            }
            while (rep--) st->lens[st->have++] = (uint16_t)fillv;
          }
        }
        if (st->mode == S_BAD) break;
        if (st->lens[256] == 0) {
          FAIL("invalid code -- missing end-of-block");
          break;
        }
        st->next = st->codes;
        st->lcode = st->next;
        st->lbits = 9;
        if (build_table(T_LENS, st->lens, st->nlen, &st->next, &st->lbits, st->work, st->d64)) {
          FAIL("invalid literal/lengths set");
          break;
        }
        st->dcode = st->next;
        st->dbits = 6;
        if (build_table(T_DISTS, st->lens + st->nlen, st->ndist, &st->next, &st->dbits, st->work,
                        st->d64)) {
          FAIL("invalid distances set");
          break;
        }
        st->mode = S_LEN_;
        if (flush == ZO_TREES) goto leave;
        /* fallthrough */
      case S_LEN_:
        st->mode = S_LEN;
        /* fallthrough */
      case S_LEN:
        if (!st->d64 && have >= 6 && left >= 258) {
          z->next_out = put;
          z->avail_out = left;
          z->next_in = next;
          z->avail_in = have;
          st->hold = hold;
          st->bits = bits;
          fast_loop(z, out0);
          put = z->next_out;
          left = z->avail_out;
          next = z->next_in;
          have = z->avail_in;
          hold = st->hold;
          bits = st->bits;
          if (st->mode == S_TYPE) st->back = -1;
          break;
        }
        st->back = 0;
        for (;;) {
          here = st->lcode[PEEK(st->lbits)];
          if ((unsigned)here.bits <= bits) break;
          PULL();
        }
        if (here.op && (here.op & 0xf0) == 0) {
          parent = here;
          for (;;) {
            here = st->lcode[parent.val + (PEEK(parent.bits + parent.op) >> parent.bits)];
            if ((unsigned)(parent.bits + here.bits) <= bits) break;
            PULL();
          }
          SKIP(parent.bits);
          st->back += parent.bits;
        }
        SKIP(here.bits);
        st->back += here.bits;
        st->length = here.val;
        if (here.op == 0) {
          st->mode = S_LIT;
          break;
        }
        if (here.op & 32) {
          st->back = -1;
          st->mode = S_TYPE;
          break;
        }
        if (here.op & 64) {
          FAIL("invalid literal/length code");
          break;
        }
        st->extra = here.op & (st->d64 ? 31u : 15u);
        st->mode = S_LENEXT;
        /* fallthrough */
      case S_LENEXT:
        if (st->extra) {
          NEED(st->extra);
          st->length += PEEK(st->extra);
          SKIP(st->extra);
          st->back += st->extra;
        }
        st->was = st->length;
        st->mode = S_DIST;
        /* fallthrough */
      case S_DIST:
        for (;;) {
          here = st->dcode[PEEK(st->dbits)];
          if ((unsigned)here.bits <= bits) break;
          PULL();
        }
        if ((here.op & 0xf0) == 0) {
          parent = here;
          for (;;) {
            here = st->dcode[parent.val + (PEEK(parent.bits + parent.op) >> parent.bits)];
            if ((unsigned)(parent.bits + here.bits) <= bits) break;
            PULL();
          }
          SKIP(parent.bits);
          st->back += parent.bits;
        }
        SKIP(here.bits);
        st->back += here.bits;
        if (here.op & 64) {
          FAIL("invalid distance code");
          break;
        }
        st->offset = here.val;
        st->extra = here.op & 15u;
        st->mode = S_DISTEXT;
        /* fallthrough */
      case S_DISTEXT:
        if (st->extra) {
          NEED(st->extra);
          st->offset += PEEK(st->extra);
          SKIP(st->extra);
          st->back += st->extra;
        }
        st->mode = S_MATCH;
        /* fallthrough */
      case S_MATCH: {
        if (left == 0) goto leave;
        unsigned produced = out0 - left;
        const uint8_t *src;
        if (st->offset > produced) { /* some bytes come from the window */
          n = st->offset - produced;
          if (n > st->whave) {
            FAIL("invalid distance too far back");
            break;
          }
          if (n > st->wnext) {
            n -= st->wnext;
            src = st->window + (st->wsize - n);
          } else {
            src = st->window + (st->wnext - n);
          }
          if (n > st->length) n = st->length;
        } else {
          src = put - st->offset;
          n = st->length;
        }
        if (n > left) n = left;
        left -= n;
        st->length -= n;
        do {
          *put++ = *src++;
        } while (--n);
        if (st->length == 0) st->mode = S_LEN;
        break;
      }
      case S_LIT:
        if (left == 0) goto leave;
        *put++ = (uint8_t)st->length;
        left--;
        st->mode = S_LEN;
        break;
      case S_CHECK:
        if (st->wrap) {
          NEED(32);
          n = out0 - left;
          z->total_out += n;
          st->total += n;
          if ((st->wrap & 4) && n) z->adler = st->check = CHECK_UPDATE(st->check, put - n, n);
          out0 = left;
          {
            uint32_t v = (uint32_t)hold;
            if (!st->flags) v = (v >> 24) | ((v >> 8) & 0xff00) | ((v & 0xff00) << 8) | (v << 24);
            if ((st->wrap & 4) && v != st->check) {
              FAIL("incorrect data check");
              break;
            }
          }
          CLEAR();
        }
        st->mode = S_LENGTH;
        /* fallthrough */
      case S_LENGTH:
        if (st->wrap && st->flags) {
          NEED(32);
          if ((st->wrap & 4) && hold != (st->total & 0xffffffffu)) {
            FAIL("incorrect length check");
            break;
          }
          CLEAR();
        }
        st->mode = S_DONE;
        /* fallthrough */
      case S_DONE:
        ret = ZO_STREAM_END;
        goto leave;
      case S_BAD:
        ret = ZO_DATA_ERROR;
        goto leave;
      case S_MEM:
        return ZO_MEM_ERROR;
      default:
        return ZO_STREAM_ERROR;
    }
  }

leave:
  z->next_out = put;
  z->avail_out = left;
  z->next_in = next;
  z->avail_in = have;
  st->hold = hold;
  st->bits = bits;
  if (st->wsize ||
      (out0 != z->avail_out && st->mode < S_BAD && (st->mode < S_CHECK || flush != ZO_FINISH))) {
    if (window_keep(z, z->next_out, out0 - z->avail_out)) {
      st->mode = S_MEM;
      return ZO_MEM_ERROR;
    }
  }
  in0 -= z->avail_in;
  out0 -= z->avail_out;
  z->total_in += in0;
  z->total_out += out0;
  st->total += out0;
  if ((st->wrap & 4) && out0) z->adler = st->check = CHECK_UPDATE(st->check, z->next_out - out0, out0);
  z->data_type = (int)st->bits + (st->last ? 64 : 0) + (st->mode == S_TYPE ? 128 : 0) +
                 (st->mode == S_LEN_ || st->mode == S_COPY_ ? 256 : 0);
  if (((in0 == 0 && out0 == 0) || flush == ZO_FINISH) && ret == ZO_OK) ret = ZO_BUF_ERROR;
  return ret;
}

/* ------------------------------------------------------------------------ */
/* convenience entry points for the tests (ctypes)                          */
/* ------------------------------------------------------------------------ */


static int snprintf_safe(char *dst, size_t cap, char tag, unsigned n, unsigned prod, int code,
                         unsigned cons) {
  int k = snprintf(dst, cap, "%c %u %d %d %u\n", tag, n, (int)prod, code, cons);
  return k < 0 ? 0 : (k >= (int)cap ? (int)cap - 1 : k);
}

size_t zo_stream_size(void) { return sizeof(zo_stream); }

/* One inflate(Z_FINISH) call over the whole input into out[0..cap).  This is
   the semantics the GPU batch API promises per job. */
int zo_oneshot(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t cap, int wbits,
               zo_result *res) {
  zo_stream z;
  memset(&z, 0, sizeof z);
  memset(res, 0, sizeof *res);
  int r = zo_inflate_init2(&z, wbits);
  if (r != ZO_OK) {
    res->ret = r;
    return r;
  }
  static uint8_t dummy;
  z.next_in = in_len ? in : NULL;
  z.avail_in = in_len;
  z.next_out = cap ? out : &dummy;
  z.avail_out = cap;
  r = zo_inflate(&z, ZO_FINISH);
  res->ret = r;
  res->msg = z.msg;
  res->total_in = z.total_in;
  res->total_out = z.total_out;
  res->adler = z.adler;
  res->data_type = z.data_type;
  zo_inflate_end(&z);
  return r;
}

/* The reference's JS/C-ABI call schedule (src/wasm/api/zlib-streams.js:64-156
   over src/wasm/wasm_stream_common.c:37-63): writes of `w` bytes, <=32 KiB
   process() slices with a 64 KiB output buffer, stop a write on consumed==0 or
   a negative code, then a Z_FINISH drain.  Emits one text line per call
   ("T n produced code consumed" / "F ...") into trace[], concatenates the
   produced bytes into out[], and returns the number of trace bytes. */
size_t zo_js_schedule(const uint8_t *in, size_t in_len, size_t w, int wbits, char *trace,
                      size_t trace_cap, uint8_t *out, size_t out_cap, size_t *out_len) {
  zo_stream z;
  memset(&z, 0, sizeof z);
  size_t tl = 0, ol = 0;
  *out_len = 0;
  if (zo_inflate_init2(&z, wbits) != ZO_OK) return 0;
  static uint8_t obuf[65536];
  uint8_t *ibuf = NULL;
  size_t ibuf_cap = 0;
  int failed = 0;
  for (size_t woff = 0; woff < in_len && !failed; woff += w) {
    size_t wl = in_len - woff < w ? in_len - woff : w;
    size_t off = 0;
    while (off < wl) {
      size_t nn = wl - off < 32768 ? wl - off : 32768;
      if (nn > ibuf_cap) {
        ibuf = (uint8_t *)realloc(ibuf, nn);
        ibuf_cap = nn;
      }
      memcpy(ibuf, in + woff + off, nn);
      z.next_in = ibuf;
      z.avail_in = (uint32_t)nn;
      z.next_out = obuf;
      z.avail_out = 65536;
      int r = zo_inflate(&z, ZO_NO_FLUSH);
      unsigned prod = 65536 - z.avail_out;
      unsigned cons = (unsigned)(nn - z.avail_in);
      int code = (int)(int8_t)(uint8_t)(r & 0xff);
      if (ol + prod <= out_cap) memcpy(out + ol, obuf, prod);
      ol += prod;
      if (tl + 64 < trace_cap) {
        int k = snprintf_safe(trace + tl, trace_cap - tl, 'T', (unsigned)nn, prod, code, cons);
        tl += (size_t)k;
      }
      if (code < 0) {
        failed = 1;
        break;
      }
      if (cons == 0) break;
      off += cons;
    }
  }
  if (!failed) {
    for (;;) {
      z.next_in = NULL;
      z.avail_in = 0;
      z.next_out = obuf;
      z.avail_out = 65536;
      int r = zo_inflate(&z, ZO_FINISH);
      unsigned prod = 65536 - z.avail_out;
      int code = (int)(int8_t)(uint8_t)(r & 0xff);
      if (ol + prod <= out_cap) memcpy(out + ol, obuf, prod);
      ol += prod;
      if (tl + 64 < trace_cap) tl += (size_t)snprintf_safe(trace + tl, trace_cap - tl, 'F', 0, prod, code, 0);
      if (code < 0) break;
      if (code == 1 || prod == 0) break;
    }
  }
  zo_inflate_end(&z);
  free(ibuf);
  *out_len = ol;
  if (tl < trace_cap) trace[tl] = 0;
  return tl;
}
