/*
 * dz_model.c -- CPU model of the GPU's zlib-identical deflate (levels 1..9),
 * test infrastructure only: it states the stage decomposition the HIP kernels
 * use and is checked byte-for-byte against host zlib (tests/test_dz_model.py),
 * so every stage's semantics are pinned before they run on the GPU.
 *
 * The reference compresses with zlib's deflate_slow + trees.c
 * (src/wasm/deflate_stream_wasm.c:31-49 -> deflateInit2(level, Z_DEFLATED,
 * -15|31, 8, Z_DEFAULT_STRATEGY); src/trees.c).  deflate_slow inserts EVERY
 * position into the hash chains (zlib deflate.c, deflate_slow's match-skip
 * loop), so the chain of position p is a pure function of the input: all
 * earlier positions q >= 1 with the same 15-bit hash of in[q..q+2].  That
 * makes the search data-parallel:
 *
 *   1. hash + previous same-hash position of every position;
 *   2. longest match of every position under the level's chain budget
 *      (max_chain, and max_chain >> 2 when prev_length >= good_length), the
 *      first candidate reaching nice_length ending the walk, ties to the
 *      earlier candidate (longest_match updates on strictly longer only);
 *   3. the lazy parse (deflate_slow's loop) replayed over those tables;
 *   4. blocks of 16383 symbols (trees.c _tr_tally, lit_bufsize - 1), each
 *      flushed as _tr_flush_block does: stored / static / dynamic by the
 *      same bit counts, trees built with the same heap order and
 *      overflow fix-up (trees.c build_tree / gen_bitlen / gen_codes).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* zlib deflate.c configuration_table rows 4..9: good, lazy, nice, chain */
static const uint16_t CFG[10][4] = {{0, 0, 0, 0},       {0, 0, 0, 0},         {0, 0, 0, 0},
                                    {0, 0, 0, 0},       {4, 4, 16, 16},       {8, 16, 32, 32},
                                    {8, 16, 128, 128},  {8, 32, 128, 256},    {32, 128, 258, 1024},
                                    {32, 258, 258, 4096}};

#define MINM 3
#define MAXM 258
#define HB 15
#define HMASK ((1u << HB) - 1u)
#define LOOKAHEAD_MIN (MAXM + MINM + 1)
#define TOO_FAR 4096
#define BLOCK_SYMS 16383 /* lit_bufsize - 1 for memLevel 8 */

/* ---- stage 1 ---------------------------------------------------------- */
static uint32_t hash3(const uint8_t *p) { return (((uint32_t)p[0] << 10) ^ ((uint32_t)p[1] << 5) ^ p[2]) & HMASK; }

/* prevd[p] = p - q for the latest q in [1, p) with hash(q) == hash(p), 0 when none */
static void stage_prev(const uint8_t *in, uint32_t L, uint32_t *prevd) {
  uint32_t *last = (uint32_t *)calloc(1u << HB, sizeof(uint32_t)); /* position + 1 */
  for (uint32_t p = 0; p + 2 < L; p++) {
    const uint32_t h = hash3(in + p);
    const uint32_t q = last[h];
    prevd[p] = (q > 1) ? p - (q - 1) : 0; /* position 0 is zlib's NIL */
    last[h] = p + 1;
  }
  free(last);
}

/* ---- stage 2 ---------------------------------------------------------- */
typedef struct {
  uint16_t len;  /* best length (0: no candidate) */
  uint16_t dist; /* distance of the first candidate reaching it */
} dz_match;

static void longest(const uint8_t *in, uint32_t L, const uint32_t *prevd, uint32_t p, uint32_t max_dist, uint32_t chain,
                    uint32_t nice, dz_match *out) {
  out->len = 0;
  out->dist = 0;
  if (p + MINM > L || !prevd[p] || prevd[p] > max_dist) return;
  const uint32_t look = L - p;
  const uint32_t cap = look < MAXM ? look : MAXM;
  const uint32_t nice_p = nice < look ? nice : look;
  uint32_t c = p - prevd[p], best = 0;
  for (uint32_t k = 0;;) {
    uint32_t n = 0;
    while (n < cap && in[c + n] == in[p + n]) n++;
    if (n > best) {
      best = n;
      out->len = (uint16_t)n;
      out->dist = (uint16_t)(p - c);
      if (n >= nice_p) break;
    }
    if (++k >= chain || !prevd[c]) break;
    const uint32_t nc = c - prevd[c];
    if (nc == 0 || p - nc >= max_dist) break; /* chain continues only while cur_match > strstart - MAX_DIST */
    c = nc;
  }
}

/* ---- stage 3 ---------------------------------------------------------- */
typedef struct {
  uint32_t lit_or_len; /* literal byte, or match length */
  uint32_t dist;       /* 0 for a literal */
  uint32_t pos;        /* first byte covered */
} dz_sym;

static uint32_t stage_parse(const uint8_t *in, uint32_t L, int level, const dz_match *ma, const dz_match *mb, dz_sym *syms,
                            int *end_lit) {
  const uint32_t good = CFG[level][0], lazy = CFG[level][1];
  uint32_t n = 0, p = 0, avail = 0, prev_len = MINM - 1, prev_dist = 0;
  while (p < L) {
    uint32_t mlen = MINM - 1, mdist = 0;
    if (prev_len < lazy) {
      const dz_match *m = prev_len >= good ? &mb[p] : &ma[p];
      if (m->len > prev_len) {
        mlen = m->len;
        mdist = m->dist;
      } else if (m->len) {
        mlen = prev_len; /* longest_match returns best_len = prev_length */
        mdist = 0;
      }
      if (mlen == MINM && mdist > TOO_FAR) mlen = MINM - 1;
    }
    if (prev_len >= MINM && mlen <= prev_len) {
      syms[n++] = (dz_sym){prev_len, prev_dist, p - 1};
      p = p - 1 + prev_len;
      avail = 0;
      prev_len = MINM - 1;
      continue;
    }
    if (avail) syms[n++] = (dz_sym){in[p - 1], 0, p - 1};
    avail = 1;
    prev_len = mlen;
    prev_dist = mdist;
    p++;
  }
  *end_lit = avail;  /* deflate_slow tallies the pending literal after its loop, ignoring bflush */
  if (avail) syms[n++] = (dz_sym){in[p - 1], 0, p - 1};
  return n;
}

/* ---- stage 4: trees.c, restated ---------------------------------------- */
static const uint8_t XL[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint8_t XD[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t XB[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
static const uint8_t BLORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static uint32_t len_code(uint32_t len) { /* 3..258 -> 0..28 */
  if (len == 258) return 28;
  uint32_t l = len - 3;
  if (l < 8) return l;
  uint32_t e = 31 - __builtin_clz(l) - 2; /* extra bits */
  return 4 * (e + 1) + ((l >> e) & 3);
}
static uint32_t len_base(uint32_t c) { return c == 28 ? 258 : c < 8 ? c + 3 : ((4u + (c & 3)) << (c / 4 - 1)) + 3; }
static uint32_t dist_code(uint32_t d) { /* 1..32768 -> 0..29 */
  uint32_t x = d - 1;
  if (x < 4) return x;
  uint32_t e = 31 - __builtin_clz(x) - 1;
  return 2 * (e + 1) + ((x >> e) & 1);
}
static uint32_t dist_base(uint32_t c) { return c < 4 ? c + 1 : ((2u + (c & 1)) << (c / 2 - 1)) + 1; }

#define HEAP_N 573
typedef struct {
  uint32_t freq[HEAP_N];
  uint16_t dad_len[HEAP_N]; /* parent while building, then code length (zlib shares the field) */
  uint16_t code[HEAP_N];
  uint8_t depth[HEAP_N];
  int heap[HEAP_N], heap_len, heap_max;
  uint16_t bl_count[16];
} dz_tree_ws;

typedef struct {
  uint64_t opt_len, static_len;
} dz_cost;

static int smaller(const dz_tree_ws *w, int n, int m) {
  return w->freq[n] < w->freq[m] || (w->freq[n] == w->freq[m] && w->depth[n] <= w->depth[m]);
}
static void sift(dz_tree_ws *w, int k) {
  const int v = w->heap[k];
  for (int j = k << 1; j <= w->heap_len; j <<= 1) {
    if (j < w->heap_len && smaller(w, w->heap[j + 1], w->heap[j])) j++;
    if (smaller(w, v, w->heap[j])) break;
    w->heap[k] = w->heap[j];
    k = j;
  }
  w->heap[k] = v;
}

/* Huffman code lengths for freq[0..elems), limited to maxlen, in zlib's
 * build_tree order; stat_len: static code lengths (NULL for the bit-length
 * tree); xb / xbase: extra bits of symbols >= xbase.  Returns max_code. */
static int build(dz_tree_ws *w, int elems, const uint8_t *stat_len, const uint8_t *xb, int xbase, int maxlen, dz_cost *cost) {
  int max_code = -1;
  w->heap_len = 0;
  w->heap_max = HEAP_N;
  for (int n = 0; n < elems; n++) {
    if (w->freq[n]) {
      w->heap[++w->heap_len] = max_code = n;
      w->depth[n] = 0;
    } else {
      w->dad_len[n] = 0;
    }
  }
  while (w->heap_len < 2) { /* at least two codes */
    const int node = w->heap[++w->heap_len] = max_code < 2 ? ++max_code : 0;
    w->freq[node] = 1;
    w->depth[node] = 0;
    cost->opt_len--;
    if (stat_len) cost->static_len -= stat_len[node];
  }
  for (int n = w->heap_len / 2; n >= 1; n--) sift(w, n);
  int node = elems;
  do {
    const int n = w->heap[1];
    w->heap[1] = w->heap[w->heap_len--];
    sift(w, 1);
    const int m = w->heap[1];
    w->heap[--w->heap_max] = n;
    w->heap[--w->heap_max] = m;
    w->freq[node] = w->freq[n] + w->freq[m];
    w->depth[node] = (uint8_t)((w->depth[n] >= w->depth[m] ? w->depth[n] : w->depth[m]) + 1);
    w->dad_len[n] = w->dad_len[m] = (uint16_t)node;
    w->heap[1] = node++;
    sift(w, 1);
  } while (w->heap_len >= 2);
  w->heap[--w->heap_max] = w->heap[1];
  /* lengths from the root down (gen_bitlen), overflow past maxlen repaired */
  memset(w->bl_count, 0, sizeof w->bl_count);
  w->dad_len[w->heap[w->heap_max]] = 0;
  int overflow = 0, h;
  for (h = w->heap_max + 1; h < HEAP_N; h++) {
    const int n = w->heap[h];
    int bits = w->dad_len[w->dad_len[n]] + 1;
    if (bits > maxlen) bits = maxlen, overflow++;
    w->dad_len[n] = (uint16_t)bits;
    if (n > max_code) continue;
    w->bl_count[bits]++;
    const int x = n >= xbase ? xb[n - xbase] : 0;
    cost->opt_len += (uint64_t)w->freq[n] * (uint64_t)(bits + x);
    if (stat_len) cost->static_len += (uint64_t)w->freq[n] * (uint64_t)(stat_len[n] + x);
  }
  if (overflow) {
    do {
      int bits = maxlen - 1;
      while (w->bl_count[bits] == 0) bits--;
      w->bl_count[bits]--;
      w->bl_count[bits + 1] += 2;
      w->bl_count[maxlen]--;
      overflow -= 2;
    } while (overflow > 0);
    for (int bits = maxlen; bits != 0; bits--) {
      int n = w->bl_count[bits];
      while (n != 0) {
        const int m = w->heap[--h];
        if (m > max_code) continue;
        if (w->dad_len[m] != bits) {
          cost->opt_len += ((uint64_t)bits - w->dad_len[m]) * w->freq[m];
          w->dad_len[m] = (uint16_t)bits;
        }
        n--;
      }
    }
  }
  /* canonical codes (gen_codes), bit-reversed for LSB-first output */
  uint16_t next[16];
  uint32_t code = 0;
  for (int b = 1; b <= 15; b++) next[b] = (uint16_t)(code = (code + w->bl_count[b - 1]) << 1);
  for (int n = 0; n <= max_code; n++) {
    const int len = w->dad_len[n];
    if (len) {
      uint32_t c = next[len]++, r = 0;
      for (int i = 0; i < len; i++, c >>= 1) r = (r << 1) | (c & 1);
      w->code[n] = (uint16_t)r;
    }
  }
  return max_code;
}

typedef struct {
  uint8_t *out;
  size_t cap, n;
  uint64_t acc;
  int nb;
} dz_bits;
static void put(dz_bits *b, uint32_t v, int n) {
  b->acc |= (uint64_t)v << b->nb;
  b->nb += n;
  while (b->nb >= 8) {
    if (b->n < b->cap) b->out[b->n] = (uint8_t)b->acc;
    b->n++;
    b->acc >>= 8;
    b->nb -= 8;
  }
}
static void align(dz_bits *b) {
  if (b->nb) put(b, 0, 8 - b->nb);
}

/* run-length coding of one code-length array (scan_tree / send_tree): mode 0
 * counts into bl->freq, mode 1 emits with bl's codes */
static void rle_lengths(const uint16_t *lens, int max_code, dz_tree_ws *bl, int mode, dz_bits *b) {
  int prevlen = -1, nextlen = lens[0], count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) max_count = 138, min_count = 3;
  for (int n = 0; n <= max_code; n++) {
    const int curlen = nextlen;
    nextlen = n + 1 <= max_code ? lens[n + 1] : 0xffff;
    if (++count < max_count && curlen == nextlen) continue;
    if (count < min_count) {
      if (mode == 0) bl->freq[curlen] += count;
      else
        do put(b, bl->code[curlen], bl->dad_len[curlen]); while (--count != 0);
    } else if (curlen != 0) {
      if (curlen != prevlen) {
        if (mode == 0) bl->freq[curlen]++;
        else put(b, bl->code[curlen], bl->dad_len[curlen]);
        count--;
      }
      if (mode == 0) bl->freq[16]++;
      else put(b, bl->code[16], bl->dad_len[16]), put(b, (uint32_t)count - 3, 2);
    } else if (count <= 10) {
      if (mode == 0) bl->freq[17]++;
      else put(b, bl->code[17], bl->dad_len[17]), put(b, (uint32_t)count - 3, 3);
    } else {
      if (mode == 0) bl->freq[18]++;
      else put(b, bl->code[18], bl->dad_len[18]), put(b, (uint32_t)count - 11, 7);
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) max_count = 138, min_count = 3;
    else if (curlen == nextlen) max_count = 6, min_count = 3;
    else max_count = 7, min_count = 4;
  }
}

static uint16_t STAT_L[288], STAT_D[30];
static uint16_t STAT_LC[288], STAT_DC[30];
static uint8_t STAT_L8[288], STAT_D8[30];
static void stat_init(void) {
  if (STAT_L[0]) return;
  uint16_t cnt[16] = {0}, next[16];
  for (int n = 0; n < 288; n++) {
    STAT_L[n] = n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8;
    STAT_L8[n] = (uint8_t)STAT_L[n];
    cnt[STAT_L[n]]++;
  }
  uint32_t code = 0;
  cnt[0] = 0;
  for (int b = 1; b <= 15; b++) next[b] = (uint16_t)(code = (code + cnt[b - 1]) << 1);
  for (int n = 0; n < 288; n++) {
    uint32_t c = next[STAT_L[n]]++, r = 0;
    for (int i = 0; i < STAT_L[n]; i++, c >>= 1) r = (r << 1) | (c & 1);
    STAT_LC[n] = (uint16_t)r;
  }
  for (int n = 0; n < 30; n++) {
    STAT_D[n] = 5;
    STAT_D8[n] = 5;
    uint32_t c = (uint32_t)n, r = 0;
    for (int i = 0; i < 5; i++, c >>= 1) r = (r << 1) | (c & 1);
    STAT_DC[n] = (uint16_t)r;
  }
}

static void emit_syms(dz_bits *b, const uint8_t *in, const dz_sym *s, uint32_t ns, const uint16_t *lc, const uint16_t *ll,
                      const uint16_t *dc, const uint16_t *dl) {
  (void)in;
  for (uint32_t i = 0; i < ns; i++) {
    if (!s[i].dist) {
      put(b, lc[s[i].lit_or_len], ll[s[i].lit_or_len]);
    } else {
      const uint32_t c = len_code(s[i].lit_or_len);
      put(b, lc[257 + c], ll[257 + c]);
      if (XL[c]) put(b, s[i].lit_or_len - len_base(c), XL[c]);
      const uint32_t d = dist_code(s[i].dist);
      put(b, dc[d], dl[d]);
      if (XD[d]) put(b, s[i].dist - dist_base(d), XD[d]);
    }
  }
  put(b, lc[256], ll[256]);
}

/* One block as _tr_flush_block chooses it.  stored_ok: the block's bytes
 * still in zlib's window (buf != NULL). */
static void flush_block(dz_bits *b, const uint8_t *in, const dz_sym *s, uint32_t ns, uint32_t first_byte, uint32_t nbytes,
                        int stored_ok, int last) {
  static dz_tree_ws lt, dt, bt;
  dz_cost cost = {0, 0};
  memset(lt.freq, 0, sizeof lt.freq);
  memset(dt.freq, 0, sizeof dt.freq);
  memset(bt.freq, 0, sizeof bt.freq);
  lt.freq[256] = 1;
  for (uint32_t i = 0; i < ns; i++) {
    if (!s[i].dist) lt.freq[s[i].lit_or_len]++;
    else {
      lt.freq[257 + len_code(s[i].lit_or_len)]++;
      dt.freq[dist_code(s[i].dist)]++;
    }
  }
  const int lmax = build(&lt, 286, STAT_L8, XL, 257, 15, &cost);
  const int dmax = build(&dt, 30, STAT_D8, XD, 0, 15, &cost);
  rle_lengths(lt.dad_len, lmax, &bt, 0, NULL);
  rle_lengths(dt.dad_len, dmax, &bt, 0, NULL);
  build(&bt, 19, NULL, XB, 0, 7, &cost);
  int blmax = 18;
  for (; blmax >= 3; blmax--)
    if (bt.dad_len[BLORD[blmax]] != 0) break;
  cost.opt_len += 3 * ((uint64_t)blmax + 1) + 5 + 5 + 4;
  uint64_t opt_b = (cost.opt_len + 3 + 7) >> 3, stat_b = (cost.static_len + 3 + 7) >> 3;
  if (stat_b <= opt_b) opt_b = stat_b;
  if ((uint64_t)nbytes + 4 <= opt_b && stored_ok) {
    put(b, (uint32_t)last, 3);
    align(b);
    put(b, nbytes & 0xffff, 16);
    put(b, ~nbytes & 0xffff, 16);
    for (uint32_t i = 0; i < nbytes; i++) put(b, in[first_byte + i], 8);
  } else if (stat_b == opt_b) {
    put(b, (1u << 1) + (uint32_t)last, 3);
    emit_syms(b, in, s, ns, STAT_LC, STAT_L, STAT_DC, STAT_D);
  } else {
    put(b, (2u << 1) + (uint32_t)last, 3);
    put(b, (uint32_t)lmax + 1 - 257, 5);
    put(b, (uint32_t)dmax + 1 - 1, 5);
    put(b, (uint32_t)blmax + 1 - 4, 4);
    for (int r = 0; r <= blmax; r++) put(b, bt.dad_len[BLORD[r]], 3);
    rle_lengths(lt.dad_len, lmax, &bt, 1, b);
    rle_lengths(dt.dad_len, dmax, &bt, 1, b);
    emit_syms(b, in, s, ns, lt.code, lt.dad_len, dt.code, dt.dad_len);
  }
  if (last) align(b);
}

/* zlib's window slides (fill_window) at a loop top t when the lookahead is
 * short and strstart >= wsize + MAX_DIST; returns the slides done by loop top t */
static uint32_t slides_at(uint32_t t, uint32_t L, uint32_t wsize, uint32_t max_dist) {
  uint32_t k = 0;
  for (;;) {
    const uint64_t base = (uint64_t)k * wsize;
    const uint64_t wend = base + 2ull * wsize < L ? base + 2ull * wsize : L;
    const uint64_t look = wend > t ? wend - t : 0;
    if (t >= base && look < LOOKAHEAD_MIN && t - base >= wsize + max_dist) k++;
    else return k;
  }
}

/* ---- levels 1..3: deflate_fast ------------------------------------------
 * zlib deflate.c configuration_table rows 1..3 (good, lazy = max_insert_length,
 * nice, chain).  deflate_fast searches at every loop top (prev_length stays
 * MIN_MATCH - 1, so the full chain budget always applies), takes any match of
 * >= MIN_MATCH (no TOO_FAR rule), and inserts a match's inner positions into
 * the hash chains only when its length is <= max_insert_length and >= 3 bytes
 * follow it.  So the chain of a position holds only the INSERTED earlier
 * positions of its hash: the search depends on every earlier parse decision,
 * and the model runs the loop serially, as the GPU kernel does (one wave per
 * stream, zs_zd_fast_kernel).  Iterating "matches under an assumed insertion
 * set -> parse -> the set it implies" to a fixed point is exact (the fixed
 * point is unique) but, measured on line text, fixes only ~1 K positions per
 * round: a wrong insertion history changes the parse for good
 * (tools/fast_resync_probe.c). */
static const uint16_t CFGF[4][4] = {{0, 0, 0, 0}, {4, 4, 8, 4}, {4, 5, 16, 8}, {4, 6, 32, 32}};

/* longest match at p over inserted positions only (ins: 1 per position) */
static void longest_ins(const uint8_t *in, uint32_t L, const uint32_t *prevd, const uint8_t *ins, uint32_t p,
                        uint32_t max_dist, uint32_t chain, uint32_t nice, dz_match *out) {
  out->len = 0;
  out->dist = 0;
  if (p + MINM > L) return;
  /* hash_head: the latest inserted same-hash position before p */
  uint32_t c = prevd[p] ? p - prevd[p] : 0;
  while (c && !ins[c] && p - c <= max_dist) c = prevd[c] ? c - prevd[c] : 0;
  if (!c || p - c > max_dist) return;
  const uint32_t look = L - p;
  const uint32_t cap = look < MAXM ? look : MAXM;
  const uint32_t nice_p = nice < look ? nice : look;
  uint32_t best = 0;
  for (uint32_t k = 0;;) {
    uint32_t n = 0;
    while (n < cap && in[c + n] == in[p + n]) n++;
    if (n > best) {
      best = n;
      out->len = (uint16_t)n;
      out->dist = (uint16_t)(p - c);
      if (n >= nice_p) break;
    }
    if (++k >= chain) break;
    uint32_t nc = prevd[c] ? c - prevd[c] : 0;
    while (nc && !ins[nc] && p - nc < max_dist) nc = prevd[nc] ? nc - prevd[nc] : 0;
    if (!nc || p - nc >= max_dist) break;
    c = nc;
  }
}

static size_t dz_blocks_out(const uint8_t *in, uint32_t L, int fast, uint32_t wbits, const dz_sym *syms, uint32_t ns,
                            int end_lit, uint8_t *out, size_t cap);
size_t dz_model_fast_serial(const uint8_t *in, uint32_t L, int level, int wbits, uint8_t *out, size_t cap);

/* Raw deflate of in[0..L) at `level` (1..9), window bits wbits (9..15):
 * returns the compressed size (bytes written up to cap). */
size_t dz_model_deflate(const uint8_t *in, uint32_t L, int level, int wbits, uint8_t *out, size_t cap) {
  stat_init();
  if (level < 1 || level > 9) return 0;
  if (level <= 3) return dz_model_fast_serial(in, L, level, wbits, out, cap);
  const uint32_t wsize = 1u << wbits, max_dist = wsize - LOOKAHEAD_MIN;
  uint32_t *prevd = (uint32_t *)calloc(L + 1, sizeof(uint32_t));
  dz_match *ma = (dz_match *)calloc(L + 1, sizeof(dz_match)), *mb = (dz_match *)calloc(L + 1, sizeof(dz_match));
  dz_sym *syms = (dz_sym *)malloc(((size_t)L + 1) * sizeof(dz_sym));
  stage_prev(in, L, prevd);
  const uint32_t chain = CFG[level][3], nice = CFG[level][2];
  for (uint32_t p = 0; p < L; p++) {
    longest(in, L, prevd, p, max_dist, chain, nice, &ma[p]);
    longest(in, L, prevd, p, max_dist, chain >> 2 ? chain >> 2 : 1, nice, &mb[p]);
  }
  int end_lit = 0;
  const uint32_t ns = stage_parse(in, L, level, ma, mb, syms, &end_lit);
  const size_t r = dz_blocks_out(in, L, 0, (uint32_t)wbits, syms, ns, end_lit, out, cap);
  free(prevd);
  free(ma);
  free(mb);
  free(syms);
  return r;
}

static size_t dz_blocks_out(const uint8_t *in, uint32_t L, int fast, uint32_t wbits, const dz_sym *syms, uint32_t ns,
                            int end_lit, uint8_t *out, size_t cap) {
  const uint32_t wsize = 1u << wbits, max_dist = wsize - LOOKAHEAD_MIN;
  dz_bits b = {out, cap, 0, 0, 0};
  /* blocks of BLOCK_SYMS symbols; the last one holds the rest -- or is empty
   * when a symbol of the main loop filled the previous block exactly */
  const uint32_t nfull = ns / BLOCK_SYMS;
  const int empty_last = ns % BLOCK_SYMS == 0 && !(ns && end_lit);
  const uint32_t nblocks = empty_last ? nfull + 1 : (ns + BLOCK_SYMS - 1) / BLOCK_SYMS;
  for (uint32_t k = 0; k < nblocks; k++) {
    const uint32_t s0 = k * BLOCK_SYMS;
    const uint32_t cnt = s0 >= ns ? 0 : (ns - s0 < BLOCK_SYMS ? ns - s0 : BLOCK_SYMS);
    const int last = k + 1 == nblocks;
    const dz_sym *e = cnt ? &syms[s0 + cnt - 1] : NULL;
    const uint32_t first = cnt ? syms[s0].pos : L;
    const uint32_t end = cnt ? e->pos + (e->dist ? e->lit_or_len : 1) : L;
    /* deflate_slow flushes in the iteration whose loop top followed the
     * block's last symbol's start (a literal at strstart-1, a match found at
     * strstart-1); deflate_fast in the symbol's own iteration; the final
     * block flushes after the loop (top = L) */
    const uint32_t top = last ? L : e->pos + (fast ? 0 : 1);
    const int stored_ok = (uint64_t)first >= (uint64_t)slides_at(top, L, wsize, max_dist) * wsize;
    flush_block(&b, in, syms + s0, cnt, first, end - first, stored_ok, last);
  }
  return b.n;
}

/* the serial deflate_fast (a hash chain walk per loop top, the insertion set
 * built as it goes), to pin the iterated form: returns the compressed size */
size_t dz_model_fast_serial(const uint8_t *in, uint32_t L, int level, int wbits, uint8_t *out, size_t cap) {
  stat_init();
  if (level < 1 || level > 3) return 0;
  const uint32_t wsize = 1u << wbits, max_dist = wsize - LOOKAHEAD_MIN;
  uint32_t *prevd = (uint32_t *)calloc(L + 1, sizeof(uint32_t));
  uint8_t *ins = (uint8_t *)calloc(L + 1, 1);
  dz_sym *syms = (dz_sym *)malloc(((size_t)L + 1) * sizeof(dz_sym));
  stage_prev(in, L, prevd);
  const uint32_t max_ins = CFGF[level][1], nice = CFGF[level][2], chain = CFGF[level][3];
  uint32_t n = 0, p = 0;
  while (p < L) {
    dz_match m;
    longest_ins(in, L, prevd, ins, p, max_dist, chain, nice, &m);
    if (p + MINM <= L) ins[p] = 1;
    if (m.len >= MINM) {
      syms[n++] = (dz_sym){m.len, m.dist, p};
      if (m.len <= max_ins && L - (p + m.len) >= MINM)
        for (uint32_t q = p + 1; q < p + m.len; q++) ins[q] = 1;
      p += m.len;
    } else {
      syms[n++] = (dz_sym){in[p], 0, p};
      p++;
    }
  }
  const size_t r = dz_blocks_out(in, L, 1, (uint32_t)wbits, syms, n, 0, out, cap);
  free(prevd);
  free(ins);
  free(syms);
  return r;
}
