/* js_perf.c -- the reference's stream perf workload (src/wasm/tests/
 * test_round_trip_stream_perf.js:23-185) as a native driver, for bench.py's
 * stream leg: a source buffer written in PACKET-byte writes through
 * CompressionStreamZlib('deflate-raw') (compress-only), the result written in
 * PACKET-byte writes through DecompressionStreamZlib (decompress-only), and
 * both chained (round trip: each compressed chunk the compressor enqueues is
 * written to the decompressor as it appears).  The per-write call schedule is
 * zlib-streams.js:64-156's: <= 32 KiB per *_process(flush 0), a 64 KiB output
 * buffer per call, advance by *_last_consumed, stop a write on 0; flush() calls
 * *_process(Z_FINISH) until code 1 or nothing produced.
 *
 * Two backends behind the same handle API:
 *   lib_path != NULL: the product library (dlopen'ed: deflate_new / _init_raw /
 *                     _process / _end / _last_consumed and the inflate_* set);
 *   lib_path == NULL: host zlib through a shim that is the reference's WASM glue
 *                     (src/wasm/wasm_stream_common.c:37-63, deflate_stream_wasm.c:
 *                     31-39, inflate_stream_wasm.c:29-34) compiled natively.
 *
 * Bench tooling only: not part of the product library. */
#include <dlfcn.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

typedef uintptr_t (*new_fn)(void);
typedef int (*dinit_fn)(uintptr_t, int);
typedef int (*iinit_fn)(uintptr_t);
typedef int (*proc_fn)(uintptr_t, uintptr_t, unsigned, uintptr_t, unsigned, int);
typedef int (*end_fn)(uintptr_t);
typedef unsigned (*cons_fn)(uintptr_t);

typedef struct {
  new_fn d_new, i_new;
  dinit_fn d_init;
  iinit_fn i_init;
  proc_fn d_proc, i_proc;
  end_fn d_end, i_end;
  cons_fn d_cons, i_cons;
} api_t;

/* ---- host zlib behind the reference's WASM glue ---- */
typedef struct {
  z_stream strm;
  unsigned last_consumed;
  unsigned char *inbuf;
  unsigned inbuf_sz;
} zctx;

static uintptr_t z_new(void) { return (uintptr_t)calloc(1, sizeof(zctx)); }
static int z_dinit(uintptr_t h, int level) {
  zctx *c = (zctx *)h;
  return deflateInit2(&c->strm, level < 0 ? Z_DEFAULT_COMPRESSION : level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
}
static int z_iinit(uintptr_t h) { return inflateInit2(&((zctx *)h)->strm, -15); }
static int z_proc(uintptr_t h, uintptr_t in, unsigned in_len, uintptr_t out, unsigned out_len, int flush, int dfl) {
  zctx *c = (zctx *)h;
  if (in_len > c->inbuf_sz) {
    unsigned char *nb = (unsigned char *)realloc(c->inbuf, in_len);
    if (!nb) return Z_MEM_ERROR;
    c->inbuf = nb;
    c->inbuf_sz = in_len;
  }
  if (in_len) memcpy(c->inbuf, (const void *)in, in_len);
  c->strm.next_in = c->inbuf;
  c->strm.avail_in = in_len;
  c->strm.next_out = (unsigned char *)out;
  c->strm.avail_out = out_len;
  const int ret = dfl ? deflate(&c->strm, flush) : inflate(&c->strm, flush);
  const int produced = (int)(out_len - c->strm.avail_out);
  c->last_consumed = in_len - c->strm.avail_in;
  return (produced & 0x00ffffff) | ((ret & 0xff) << 24);
}
static int z_dproc(uintptr_t h, uintptr_t in, unsigned n, uintptr_t out, unsigned m, int f) {
  return z_proc(h, in, n, out, m, f, 1);
}
static int z_iproc(uintptr_t h, uintptr_t in, unsigned n, uintptr_t out, unsigned m, int f) {
  return z_proc(h, in, n, out, m, f, 0);
}
static int z_end(uintptr_t h, int dfl) {
  zctx *c = (zctx *)h;
  const int r = dfl ? deflateEnd(&c->strm) : inflateEnd(&c->strm);
  free(c->inbuf);
  free(c);
  return r;
}
static int z_dend(uintptr_t h) { return z_end(h, 1); }
static int z_iend(uintptr_t h) { return z_end(h, 0); }
static unsigned z_cons(uintptr_t h) { return ((zctx *)h)->last_consumed; }

static int load_api(const char *lib_path, api_t *a) {
  if (!lib_path) {
    *a = (api_t){z_new, z_new, z_dinit, z_iinit, z_dproc, z_iproc, z_dend, z_iend, z_cons, z_cons};
    return 0;
  }
  void *lib = dlopen(lib_path, RTLD_NOW | RTLD_LOCAL);
  if (!lib) return -1;
  a->d_new = (new_fn)dlsym(lib, "deflate_new");
  a->i_new = (new_fn)dlsym(lib, "inflate_new");
  a->d_init = (dinit_fn)dlsym(lib, "deflate_init_raw");
  a->i_init = (iinit_fn)dlsym(lib, "inflate_init_raw");
  a->d_proc = (proc_fn)dlsym(lib, "deflate_process");
  a->i_proc = (proc_fn)dlsym(lib, "inflate_process");
  a->d_end = (end_fn)dlsym(lib, "deflate_end");
  a->i_end = (end_fn)dlsym(lib, "inflate_end");
  a->d_cons = (cons_fn)dlsym(lib, "deflate_last_consumed");
  a->i_cons = (cons_fn)dlsym(lib, "inflate_last_consumed");
  return (a->d_new && a->i_new && a->d_init && a->i_init && a->d_proc && a->i_proc && a->d_end && a->i_end &&
          a->d_cons && a->i_cons)
             ? 0
             : -1;
}

#define OUTB 65536u
#define SLICE 32768u

/* one TransformStream: a handle, its 64 KiB output buffer, and a sink for the
 * chunks it enqueues (the next stream's transform, or the result buffer) */
typedef struct ts ts_t;
struct ts {
  const api_t *a;
  int dfl;
  uintptr_t h;
  uint8_t out[OUTB];
  ts_t *next;     /* chained stream, or NULL: append to res */
  uint8_t *res;   /* result buffer */
  size_t res_len, res_cap;
  int err;
};

static int ts_enqueue(ts_t *t, const uint8_t *p, size_t n);

/* transform(chunk): zlib-streams.js:64-103 */
static int ts_transform(ts_t *t, const uint8_t *buf, size_t len) {
  proc_fn proc = t->dfl ? t->a->d_proc : t->a->i_proc;
  cons_fn cons = t->dfl ? t->a->d_cons : t->a->i_cons;
  size_t off = 0;
  while (off < len) {
    const unsigned k = (unsigned)(len - off < SLICE ? len - off : SLICE);
    const uint32_t r = (uint32_t)proc(t->h, (uintptr_t)(buf + off), k, (uintptr_t)t->out, OUTB, 0);
    const uint32_t prod = r & 0xffffffu;
    if (prod && ts_enqueue(t, t->out, prod)) return -1;
    if (!t->dfl) {
      const int code = (r >> 31) ? (int)(r >> 24) - 256 : (int)(r >> 24);
      if (code < 0) return t->err = code;
    }
    const unsigned c = cons(t->h);
    if (c == 0) break;
    off += c;
  }
  return 0;
}

/* flush(): zlib-streams.js:104-141 */
static int ts_flush(ts_t *t) {
  proc_fn proc = t->dfl ? t->a->d_proc : t->a->i_proc;
  for (;;) {
    const uint32_t r = (uint32_t)proc(t->h, 0, 0, (uintptr_t)t->out, OUTB, Z_FINISH);
    const uint32_t prod = r & 0xffffffu;
    const int code = (r >> 31) ? (int)(r >> 24) - 256 : (int)(r >> 24);
    if (!t->dfl && code < 0) return t->err = code;
    if (prod && ts_enqueue(t, t->out, prod)) return -1;
    if (code == 1 || prod == 0) break;
  }
  return 0;
}

static int ts_enqueue(ts_t *t, const uint8_t *p, size_t n) {
  if (t->next) return ts_transform(t->next, p, n);
  if (t->res_len + n > t->res_cap) return t->err = -100;
  memcpy(t->res + t->res_len, p, n);
  t->res_len += n;
  return 0;
}

static int ts_open(ts_t *t, const api_t *a, int dfl, int level) {
  memset(t, 0, sizeof(*t));
  t->a = a;
  t->dfl = dfl;
  t->h = dfl ? a->d_new() : a->i_new();
  if (!t->h) return -1;
  return dfl ? a->d_init(t->h, level) : a->i_init(t->h);
}

static int ts_close(ts_t *t) { return t->dfl ? t->a->d_end(t->h) : t->a->i_end(t->h); }

/* phase 0: compress src -> out; 1: decompress src -> out; 2: src -> compress ->
 * decompress -> out.  Writes of `packet` bytes.  Returns wall seconds of the
 * phase (writes + close), or a negative code; *out_len = bytes in out. */
double zs_js_perf(const char *lib_path, int phase, const uint8_t *src, size_t n, size_t packet, int level,
                  uint8_t *out, size_t out_cap, size_t *out_len) {
  api_t a;
  if (load_api(lib_path, &a)) return -1.0;
  ts_t *c = (ts_t *)malloc(sizeof(ts_t)), *d = (ts_t *)malloc(sizeof(ts_t));
  if (!c || !d) {
    free(c);
    free(d);
    return -2.0;
  }
  int rc = 0;
  ts_t *head;
  if (phase == 0) {
    rc |= ts_open(c, &a, 1, level);
    head = c;
    c->res = out;
    c->res_cap = out_cap;
  } else if (phase == 1) {
    rc |= ts_open(d, &a, 0, level);
    head = d;
    d->res = out;
    d->res_cap = out_cap;
  } else {
    rc |= ts_open(c, &a, 1, level);
    rc |= ts_open(d, &a, 0, level);
    c->next = d;
    head = c;
    d->res = out;
    d->res_cap = out_cap;
  }
  if (rc) {
    free(c);
    free(d);
    return -3.0;
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (size_t off = 0; off < n && !rc; off += packet)
    rc = ts_transform(head, src + off, n - off < packet ? n - off : packet);
  if (!rc) rc = ts_flush(head);
  if (!rc && phase == 2) rc = ts_flush(d);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  ts_t *last = phase == 0 ? c : d;
  *out_len = last->res_len;
  int e1 = ts_close(head);
  if (phase == 2) e1 |= ts_close(d);
  free(c);
  free(d);
  if (rc) return -10.0 + (rc < 0 ? rc : 0) * 1e-3;
  if (e1) return -4.0;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
