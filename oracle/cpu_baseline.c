/*
 * cpu_baseline.c -- CPU baseline timer for bench.py (test/bench infrastructure).
 *
 * Times host zlib inflate (libz, the upstream of the reference's vendored
 * src/inflate.c; SURVEY.md §6: within 3-9% of the reference build) and the
 * oracle port (zo_inflate.c) over whole streams: inflateInit2(wbits) + one
 * inflate(Z_FINISH) per stream, streams dealt round-robin to `nthreads`
 * pthreads.  Returns wall seconds; *total_out receives the bytes produced.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

#include "zo_inflate.h"

typedef struct {
  const uint8_t *const *comp;
  const size_t *comp_len;
  uint8_t *const *out;
  size_t out_cap;
  int n, nthreads, tid, wbits, use_oracle;
  uint64_t produced;
  int bad;
  int per_thread_out; /* 1: out[tid] is this thread's buffer for all its streams */
} task_t;

static void *run(void *arg) {
  task_t *t = (task_t *)arg;
  for (int i = t->tid; i < t->n; i += t->nthreads) {
    uint8_t *dst = t->per_thread_out ? t->out[t->tid] : t->out[i];
    if (t->use_oracle) {
      zo_result r;
      zo_oneshot(t->comp[i], (uint32_t)t->comp_len[i], dst, (uint32_t)t->out_cap, t->wbits, &r);
      t->produced += r.total_out;
      t->bad |= r.ret != 1;
    } else {
      z_stream z;
      memset(&z, 0, sizeof z);
      inflateInit2(&z, t->wbits);
      z.next_in = (Bytef *)t->comp[i];
      z.avail_in = (uInt)t->comp_len[i];
      z.next_out = dst;
      z.avail_out = (uInt)t->out_cap;
      int r = inflate(&z, Z_FINISH);
      t->produced += z.total_out;
      t->bad |= r != Z_STREAM_END;
      inflateEnd(&z);
    }
  }
  return NULL;
}

static double inflate_timed(const uint8_t *const *comp, const size_t *comp_len, uint8_t *const *out, size_t out_cap, int n,
                            int nthreads, int wbits, int use_oracle, int per_thread_out, uint64_t *total_out, int *bad) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  task_t *ts = (task_t *)calloc((size_t)nthreads, sizeof(task_t));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  /* warm any lazily built static tables before timing (single thread) */
  if (n > 0) {
    task_t w = {comp, comp_len, out, out_cap, 1, 1, 0, wbits, use_oracle, 0, 0, per_thread_out};
    run(&w);
  }
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int k = 0; k < nthreads; k++) {
    ts[k] = (task_t){comp, comp_len, out, out_cap, n, nthreads, k, wbits, use_oracle, 0, 0, per_thread_out};
    pthread_create(&th[k], NULL, run, &ts[k]);
  }
  uint64_t tot = 0;
  int anybad = 0;
  for (int k = 0; k < nthreads; k++) {
    pthread_join(th[k], NULL);
    tot += ts[k].produced;
    anybad |= ts[k].bad;
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  free(ts);
  free(th);
  *total_out = tot;
  *bad = anybad;
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

double zs_cpu_inflate(const uint8_t *const *comp, const size_t *comp_len, uint8_t *const *out, size_t out_cap, int n,
                      int nthreads, int wbits, int use_oracle, uint64_t *total_out, int *bad) {
  return inflate_timed(comp, comp_len, out, out_cap, n, nthreads, wbits, use_oracle, 0, total_out, bad);
}

/* all-core variant: n streams (a stream may repeat) dealt round-robin to
 * nthreads threads, thread k decoding every one of its streams into out[k] */
double zs_cpu_inflate_pt(const uint8_t *const *comp, const size_t *comp_len, uint8_t *const *out, size_t out_cap, int n,
                         int nthreads, int wbits, uint64_t *total_out, int *bad) {
  return inflate_timed(comp, comp_len, out, out_cap, n, nthreads, wbits, 0, 1, total_out, bad);
}

const char *zs_cpu_zlib_version(void) { return zlibVersion(); }

/* host zlib deflate (deflateInit2(level, Z_DEFLATED, wbits, 8,
 * Z_DEFAULT_STRATEGY) + one deflate(Z_FINISH) per buffer, byte-identical to the
 * reference's shipped deflate), buffers dealt round-robin to
 * `nthreads` pthreads.  Returns wall seconds; *total_in receives the bytes
 * consumed, comp_len[i] each output size. */
typedef struct {
  const uint8_t *const *raw;
  const size_t *raw_len;
  uint8_t *const *comp;
  size_t *comp_len;
  size_t comp_cap;
  int n, nthreads, tid, level, wbits;
  uint64_t consumed;
  int bad;
  int per_thread_out; /* 1: comp[tid] / comp_len[tid] serve all of this thread's buffers */
} dtask_t;

static void *drun(void *arg) {
  dtask_t *t = (dtask_t *)arg;
  for (int i = t->tid; i < t->n; i += t->nthreads) {
    z_stream z;
    memset(&z, 0, sizeof z);
    deflateInit2(&z, t->level, Z_DEFLATED, t->wbits, 8, Z_DEFAULT_STRATEGY);
    z.next_in = (Bytef *)t->raw[i];
    z.avail_in = (uInt)t->raw_len[i];
    const int o = t->per_thread_out ? t->tid : i;
    z.next_out = t->comp[o];
    z.avail_out = (uInt)t->comp_cap;
    int r = deflate(&z, Z_FINISH);
    t->consumed += z.total_in;
    t->comp_len[o] = z.total_out;
    t->bad |= r != Z_STREAM_END;
    deflateEnd(&z);
  }
  return NULL;
}

static double deflate_timed(const uint8_t *const *raw, const size_t *raw_len, uint8_t *const *comp, size_t *comp_len,
                            size_t comp_cap, int n, int nthreads, int level, int wbits, int per_thread_out,
                            uint64_t *total_in, int *bad) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  dtask_t *ts = (dtask_t *)calloc((size_t)nthreads, sizeof(dtask_t));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int k = 0; k < nthreads; k++) {
    ts[k] = (dtask_t){raw, raw_len, comp, comp_len, comp_cap, n, nthreads, k, level, wbits, 0, 0, per_thread_out};
    pthread_create(&th[k], NULL, drun, &ts[k]);
  }
  uint64_t tot = 0;
  int anybad = 0;
  for (int k = 0; k < nthreads; k++) {
    pthread_join(th[k], NULL);
    tot += ts[k].consumed;
    anybad |= ts[k].bad;
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  free(ts);
  free(th);
  *total_in = tot;
  *bad = anybad;
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

double zs_cpu_deflate(const uint8_t *const *raw, const size_t *raw_len, uint8_t *const *comp, size_t *comp_len,
                      size_t comp_cap, int n, int nthreads, int level, int wbits, uint64_t *total_in, int *bad) {
  return deflate_timed(raw, raw_len, comp, comp_len, comp_cap, n, nthreads, level, wbits, 0, total_in, bad);
}

/* all-core variant: thread k compresses every one of its buffers into comp[k] */
double zs_cpu_deflate_pt(const uint8_t *const *raw, const size_t *raw_len, uint8_t *const *comp, size_t *comp_len,
                         size_t comp_cap, int n, int nthreads, int level, int wbits, uint64_t *total_in, int *bad) {
  return deflate_timed(raw, raw_len, comp, comp_len, comp_cap, n, nthreads, level, wbits, 1, total_in, bad);
}

/* The reference's stream call schedule on host zlib (src/wasm/api/zlib-streams.js:64-136 over
 * wasm_stream_common.c:37-63): writes of `write_size` bytes, each fed in <= 32 KiB slices to
 * inflate(Z_NO_FLUSH) with a 64 KiB output buffer, advancing by the bytes consumed and stopping
 * a write on consumed == 0; then Z_FINISH drains.  Output lands consecutively in `out`.  Streams
 * dealt round-robin to `nthreads` threads (out[k] per thread).  Returns wall seconds. */
typedef struct {
  const uint8_t *const *comp;
  const size_t *comp_len;
  uint8_t *const *out;
  size_t out_cap, write_size;
  int n, nthreads, tid, wbits;
  uint64_t produced;
  int bad;
} stask_t;

static void *srun(void *arg) {
  stask_t *t = (stask_t *)arg;
  for (int i = t->tid; i < t->n; i += t->nthreads) {
    z_stream z;
    memset(&z, 0, sizeof z);
    inflateInit2(&z, t->wbits);
    uint8_t *dst = t->out[t->tid];
    size_t put = 0;
    int r = Z_OK;
    for (size_t w = 0; w < t->comp_len[i] && r >= 0 && r != Z_STREAM_END; w += t->write_size) {
      const size_t len = t->comp_len[i] - w < t->write_size ? t->comp_len[i] - w : t->write_size;
      size_t off = 0;
      while (off < len) {
        const size_t n = len - off < 32768 ? len - off : 32768;
        size_t room = t->out_cap - put < 65536 ? t->out_cap - put : 65536;
        z.next_in = (Bytef *)(t->comp[i] + w + off);
        z.avail_in = (uInt)n;
        z.next_out = dst + put;
        z.avail_out = (uInt)room;
        r = inflate(&z, Z_NO_FLUSH);
        const size_t consumed = n - z.avail_in;
        put += room - z.avail_out;
        if (r < 0 && r != Z_BUF_ERROR) break;
        if (consumed == 0) break;
        off += consumed;
      }
    }
    for (;;) {
      size_t room = t->out_cap - put < 65536 ? t->out_cap - put : 65536;
      z.next_in = NULL;
      z.avail_in = 0;
      z.next_out = dst + put;
      z.avail_out = (uInt)room;
      r = inflate(&z, Z_FINISH);
      const size_t got = room - z.avail_out;
      put += got;
      if (r < 0 || r == Z_STREAM_END || got == 0) break;
    }
    t->produced += put;
    t->bad |= r != Z_STREAM_END;
    inflateEnd(&z);
  }
  return NULL;
}

double zs_cpu_inflate_js(const uint8_t *const *comp, const size_t *comp_len, uint8_t *const *out, size_t out_cap, int n,
                         int nthreads, int wbits, size_t write_size, uint64_t *total_out, int *bad) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  stask_t *ts = (stask_t *)calloc((size_t)nthreads, sizeof(stask_t));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int k = 0; k < nthreads; k++) {
    ts[k] = (stask_t){comp, comp_len, out, out_cap, write_size, n, nthreads, k, wbits, 0, 0};
    pthread_create(&th[k], NULL, srun, &ts[k]);
  }
  uint64_t tot = 0;
  int anybad = 0;
  for (int k = 0; k < nthreads; k++) {
    pthread_join(th[k], NULL);
    tot += ts[k].produced;
    anybad |= ts[k].bad;
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  free(ts);
  free(th);
  *total_out = tot;
  *bad = anybad;
  return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
