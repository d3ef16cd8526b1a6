/* js_driver.c -- native host threads driving the handle ABI with the reference
 * JS call schedule (src/wasm/api/zlib-streams.js:64-136), for bench.py's
 * aggregate stream leg: 64 KiB writes, <= 32 KiB per inflate_process, a 64 KiB
 * output buffer per call, advance by inflate_last_consumed, stop a write on 0,
 * then Z_FINISH drains.  The library is dlopen'ed by path (the product .so), so
 * the same loop shape as oracle/cpu_baseline.c's host-zlib driver runs on
 * native threads instead of Python threads holding the GIL between calls.
 *
 * Bench tooling only: not part of the product library. */
#include <dlfcn.h>
#include <stdio.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef uintptr_t (*new_fn)(void);
typedef int (*init_fn)(uintptr_t);
typedef int (*proc_fn)(uintptr_t, uintptr_t, unsigned, uintptr_t, unsigned, int);
typedef int (*end_fn)(uintptr_t);
typedef unsigned (*cons_fn)(uintptr_t);

typedef struct {
  new_fn f_new;
  init_fn f_init;
  proc_fn f_proc;
  end_fn f_end;
  cons_fn f_cons;
} api_t;

typedef struct {
  const api_t *api;
  const uint8_t *comp;
  size_t comp_len, write_size, out_cap;
  uint8_t *out;
  uint64_t produced, calls;
  int code;
  double t_total, t_proc, t_init, t_end;  /* env ZS_JS_DRIVE_PROF: per-thread split (stderr) */
  double t_start;                         /* absolute start (ZS_JS_DRIVE_PROF=2: per-thread lines) */
} job_t;

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int unpack(uint32_t r, uint32_t *got) {
  *got = r & 0xffffffu;
  return (r >> 31) ? (int)(r >> 24) - 256 : (int)(r >> 24);
}

static void *run_job(void *arg) {
  job_t *j = (job_t *)arg;
  const api_t *a = j->api;
  const double ts = now_s();
  const uintptr_t h = a->f_new();
  a->f_init(h);
  const double ti = now_s();
  double tp = 0;
  size_t put = 0;
  int code = 0;
  uint64_t calls = 0;
  for (size_t w = 0; w < j->comp_len && code >= 0; w += j->write_size) {
    const size_t ln = j->comp_len - w < j->write_size ? j->comp_len - w : j->write_size;
    size_t off = 0;
    while (off < ln) {
      const size_t k = ln - off < 32768 ? ln - off : 32768;
      uint32_t got;
      const size_t room = j->out_cap - put < 65536 ? j->out_cap - put : 65536;
      const double tq = now_s();
      code = unpack((uint32_t)a->f_proc(h, (uintptr_t)(j->comp + w + off), (unsigned)k, (uintptr_t)(j->out + put),
                                        (unsigned)room, 0),
                    &got);
      tp += now_s() - tq;
      calls++;
      put += got;
      if (code < 0) break;
      const unsigned c = a->f_cons(h);
      if (c == 0) break;
      off += c;
    }
  }
  while (code >= 0) {
    uint32_t got;
    const size_t room = j->out_cap - put < 65536 ? j->out_cap - put : 65536;
    code = unpack((uint32_t)a->f_proc(h, 0, 0, (uintptr_t)(j->out + put), (unsigned)room, 4), &got);
    calls++;
    put += got;
    if (code == 1 || got == 0) break;
  }
  const double te0 = now_s();
  a->f_end(h);
  const double te1 = now_s();
  j->t_total = te1 - ts;
  j->t_start = ts;
  j->t_proc = tp;
  j->t_init = ti - ts;
  j->t_end = te1 - te0;
  j->produced = put;
  j->calls = calls;
  j->code = code;
  return NULL;
}

/* n streams, one native thread each; produced[k] / codes[k] per stream.
 * Returns wall seconds, or a negative value (-1: library/symbols, -2: threads). */
double zs_js_drive(const char *lib_path, const uint8_t *const *comp, const size_t *comp_len, uint8_t *const *out,
                   const size_t *out_cap, int n, size_t write_size, uint64_t *produced, int *codes,
                   uint64_t *total_calls) {
  void *lib = dlopen(lib_path, RTLD_NOW | RTLD_LOCAL);
  if (!lib) return -1.0;
  api_t a;
  a.f_new = (new_fn)dlsym(lib, "inflate_new");
  a.f_init = (init_fn)dlsym(lib, "inflate_init_raw");
  a.f_proc = (proc_fn)dlsym(lib, "inflate_process");
  a.f_end = (end_fn)dlsym(lib, "inflate_end");
  a.f_cons = (cons_fn)dlsym(lib, "inflate_last_consumed");
  if (!a.f_new || !a.f_init || !a.f_proc || !a.f_end || !a.f_cons) return -1.0;
  job_t *js = (job_t *)calloc((size_t)n, sizeof(job_t));
  pthread_t *th = (pthread_t *)calloc((size_t)n, sizeof(pthread_t));
  if (!js || !th) {
    free(js);
    free(th);
    return -2.0;
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  int started = 0;
  for (int k = 0; k < n; k++) {
    js[k] = (job_t){&a, comp[k], comp_len[k], write_size, out_cap[k], out[k], 0, 0, 0};
    if (pthread_create(&th[k], NULL, run_job, &js[k]) != 0) break;
    started++;
  }
  uint64_t calls = 0;
  for (int k = 0; k < started; k++) {
    pthread_join(th[k], NULL);
    produced[k] = js[k].produced;
    codes[k] = js[k].code;
    calls += js[k].calls;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  *total_calls = calls;
  if (getenv("ZS_JS_DRIVE_PROF") && started) {
    double tt = 0, tp = 0, ti = 0, te = 0, tmax = 0;
    for (int k = 0; k < started; k++) {
      tt += js[k].t_total;
      tp += js[k].t_proc;
      ti += js[k].t_init;
      te += js[k].t_end;
      tmax = js[k].t_total > tmax ? js[k].t_total : tmax;
    }
    fprintf(stderr, "js_drive %d threads: per thread avg total %.2f ms (max %.2f), in process() %.2f ms, init %.3f ms, end %.3f ms; %.1f us per call in process()\n",
            started, 1e3 * tt / started, 1e3 * tmax, 1e3 * tp / started, 1e3 * ti / started, 1e3 * te / started,
            1e6 * tp / (double)(calls ? calls : 1));
    if (atoi(getenv("ZS_JS_DRIVE_PROF")) >= 2) {
      const double t0s = (double)t0.tv_sec + 1e-9 * (double)t0.tv_nsec;
      for (int k = 0; k < started; k++)
        fprintf(stderr, "  thread %2d: start +%.2f ms, total %.2f ms, %llu calls, %.1f us per call\n", k,
                1e3 * (js[k].t_start - t0s), 1e3 * js[k].t_total, (unsigned long long)js[k].calls,
                1e6 * js[k].t_proc / (double)(js[k].calls ? js[k].calls : 1));
    }
  }
  free(js);
  free(th);
  return started < n ? -2.0 : (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
