/*
 * zs_corpus.c -- deterministic benchmark workload generator (test/bench
 * infrastructure, not product code).  SURVEY.md §8d configs:
 *   stream i, i % 64 < 32 : Zipf text, 5 000-word lowercase vocabulary
 *                           (lengths 2-10), weight 1/(rank+1), a newline every
 *                           10 000 words, splitmix64 seed 1000+i;
 *   stream i, i % 64 >= 32: "line-%08d\n" records starting at (i % 64) << 20.
 * Streams are compressed with host zlib deflateInit2(level, Z_DEFLATED, wbits,
 * memLevel 8, Z_DEFAULT_STRATEGY) -- byte-identical to the reference's shipped
 * deflate -- on a pthread pool.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

static uint64_t sm64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

#define NV 5000
static char vocab[NV][12];
static int vlen[NV];
static double cdf[NV];
static pthread_once_t once = PTHREAD_ONCE_INIT;

static void init_vocab(void) {
  uint64_t s = 12345;
  double tot = 0;
  for (int i = 0; i < NV; i++) {
    vlen[i] = 2 + (int)(sm64(&s) % 9);
    for (int k = 0; k < vlen[i]; k++) vocab[i][k] = (char)('a' + sm64(&s) % 26);
    tot += 1.0 / (i + 1.0);
  }
  double acc = 0;
  for (int i = 0; i < NV; i++) {
    acc += 1.0 / (i + 1.0) / tot;
    cdf[i] = acc;
  }
  cdf[NV - 1] = 1.0;
}

void zs_corpus_zipf(uint8_t *out, size_t n, uint64_t seed) {
  pthread_once(&once, init_vocab);
  uint64_t s = seed;
  size_t p = 0;
  uint64_t w = 0;
  while (p < n) {
    double u = (double)(sm64(&s) >> 11) * (1.0 / 9007199254740992.0);
    int lo = 0, hi = NV - 1;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (cdf[mid] < u) lo = mid + 1; else hi = mid;
    }
    for (int k = 0; k < vlen[lo] && p < n; k++) out[p++] = (uint8_t)vocab[lo][k];
    if (p < n) out[p++] = (++w % 10000 == 0) ? '\n' : ' ';
  }
}

void zs_corpus_lines(uint8_t *out, size_t n, uint64_t start) {
  size_t p = 0;
  char rec[16];
  for (uint64_t v = start; p < n; v++) {
    uint64_t x = v;
    memcpy(rec, "line-", 5);
    for (int k = 12; k >= 5; k--) { rec[k] = (char)('0' + x % 10); x /= 10; }
    rec[13] = '\n';
    for (int k = 0; k < 14 && p < n; k++) out[p++] = (uint8_t)rec[k];
  }
}

void zs_corpus_stream(uint8_t *out, size_t n, int i) {
  if (i % 64 < 32) zs_corpus_zipf(out, n, 1000u + (unsigned)i);
  else zs_corpus_lines(out, n, (uint64_t)(i % 64) << 20);
}

/* compress src[0..n) -> dst (cap bytes); returns compressed length or 0 */
size_t zs_corpus_deflate(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, int level, int wbits) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (deflateInit2(&z, level, Z_DEFLATED, wbits, 8, Z_DEFAULT_STRATEGY) != Z_OK) return 0;
  z.next_in = (Bytef *)src;
  z.next_out = dst;
  size_t done_in = 0;
  int r = Z_OK;
  while (r != Z_STREAM_END) {
    size_t chunk = n - done_in > (1u << 30) ? (1u << 30) : n - done_in;
    z.avail_in = (uInt)chunk;
    z.next_in = (Bytef *)src + done_in;
    size_t room = cap - z.total_out;
    z.avail_out = (uInt)(room > (1u << 30) ? (1u << 30) : room);
    int fl = (done_in + chunk == n) ? Z_FINISH : Z_NO_FLUSH;
    r = deflate(&z, fl);
    done_in += chunk - z.avail_in;
    if (r != Z_OK && r != Z_STREAM_END && r != Z_BUF_ERROR) { deflateEnd(&z); return 0; }
    if (z.avail_out == 0 && r != Z_STREAM_END && z.total_out >= cap) { deflateEnd(&z); return 0; }
  }
  size_t out = z.total_out;
  deflateEnd(&z);
  return out;
}

size_t zs_corpus_bound(size_t n) { return n + n / 1000 + (n >> 12) + 1024; }

typedef struct {
  int first, count, nthreads, level, wbits;
  size_t nbytes;
  uint8_t **raw, **comp;
  size_t *comp_len;
  int tid;
} job_t;

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (int k = j->tid; k < j->count; k += j->nthreads) {
    int i = j->first + k;
    zs_corpus_stream(j->raw[k], j->nbytes, i);
    if (j->comp) j->comp_len[k] = zs_corpus_deflate(j->raw[k], j->nbytes, j->comp[k], zs_corpus_bound(j->nbytes), j->level, j->wbits);
  }
  return NULL;
}

/* Generate streams first..first+count-1 (nbytes each) into raw[k] and, if
   comp != NULL, compress them into comp[k] (capacity zs_corpus_bound). */
int zs_corpus_batch(int first, int count, size_t nbytes, int level, int wbits, int nthreads, uint8_t **raw,
                    uint8_t **comp, size_t *comp_len) {
  if (nthreads < 1) nthreads = 1;
  pthread_t th[256];
  job_t jb[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; t++) {
    jb[t] = (job_t){first, count, nthreads, level, wbits, nbytes, raw, comp, comp_len, t};
    pthread_create(&th[t], NULL, worker, &jb[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
