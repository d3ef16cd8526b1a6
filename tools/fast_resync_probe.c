// fast_resync_probe.c -- does zlib's deflate_fast (levels 1..3), started
// mid-stream at a true loop top but with a wrong insertion history for the
// window before it (all positions inserted, or none), ever rejoin the true
// parse?  Prints, per start, how many loop-top decisions differ afterwards and
// the offset of the last difference.  Measured (4 MiB inputs): Zipf text
// rejoins within ~0.1-0.25 MiB; `line-%08d` text never does (13% of decisions
// differ to the end) -- which is why zs_zd_fast_kernel parses each stream
// serially instead of speculating per region.
//   gcc -O2 -o /tmp/resync tools/fast_resync_probe.c && /tmp/resync FILE LEVEL
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define MINM 3
#define MAXM 258
static const uint16_t CFGF[4][4] = {{0, 0, 0, 0}, {4, 4, 8, 4}, {4, 5, 16, 8}, {4, 6, 32, 32}};
static uint32_t hash3(const uint8_t *p) { return (((uint32_t)p[0] << 10) ^ ((uint32_t)p[1] << 5) ^ p[2]) & 0x7fff; }
static void walk(const uint8_t *in, uint32_t L, const uint32_t *prevd, const uint8_t *ins, uint32_t p, uint32_t max_dist,
                 uint32_t chain, uint32_t nice, uint32_t *len, uint32_t *dist) {
  *len = 0; *dist = 0;
  if (p + MINM > L) return;
  uint32_t c = prevd[p] ? p - prevd[p] : 0;
  while (c && !ins[c] && p - c <= max_dist) c = prevd[c] ? c - prevd[c] : 0;
  if (!c || p - c > max_dist) return;
  uint32_t look = L - p, cap = look < MAXM ? look : MAXM, nice_p = nice < look ? nice : look, best = 0;
  for (uint32_t k = 0;;) {
    uint32_t n = 0;
    while (n < cap && in[c + n] == in[p + n]) n++;
    if (n > best) { best = n; *len = n; *dist = p - c; if (n >= nice_p) break; }
    if (++k >= chain) break;
    uint32_t nc = prevd[c] ? c - prevd[c] : 0;
    while (nc && !ins[nc] && p - nc < max_dist) nc = prevd[nc] ? nc - prevd[nc] : 0;
    if (!nc || p - nc >= max_dist) break;
    c = nc;
  }
}
// run from p0 with ins[] preset; record decision at each loop top in dec[] (len<<16|dist, or 1 for literal), 0 = not loop top
static void run(const uint8_t *in, uint32_t L, int level, const uint32_t *prevd, uint8_t *ins, uint32_t p0, uint32_t *dec) {
  const uint32_t max_ins = CFGF[level][1], nice = CFGF[level][2], chain = CFGF[level][3], max_dist = 32768 - 262;
  uint32_t p = p0;
  while (p < L) {
    uint32_t len, dist;
    walk(in, L, prevd, ins, p, max_dist, chain, nice, &len, &dist);
    if (p + MINM <= L) ins[p] = 1;
    if (len >= MINM) {
      dec[p] = (len << 16) | dist;
      if (len <= max_ins && L - (p + len) >= MINM) for (uint32_t q = p + 1; q < p + len; q++) ins[q] = 1;
      p += len;
    } else { dec[p] = 1; p++; }
  }
}
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); uint32_t L = ftell(f); fseek(f, 0, SEEK_SET);
  uint8_t *in = malloc(L); if (fread(in, 1, L, f) != L) return 1; fclose(f);
  int level = atoi(argv[2]);
  uint32_t *prevd = calloc(L + 1, 4), *last = calloc(32768, 4);
  for (uint32_t p = 0; p + 2 < L; p++) { uint32_t h = hash3(in + p), q = last[h]; prevd[p] = q > 1 ? p - (q - 1) : 0; if (p - (q-1) > 32767) prevd[p] = 0; last[h] = p + 1; }
  uint8_t *ins = calloc(L + 1, 1), *ins2 = calloc(L + 1, 1);
  uint32_t *dec = calloc(L + 1, 4), *dec2 = calloc(L + 1, 4);
  run(in, L, level, prevd, ins, 0, dec);
  for (uint32_t s = 65536; s + 200000 < L; s += 131072) {
    // entry: the true loop top at or after s; history: all inserted / none inserted / true
    uint32_t t = s; while (!dec[t]) t++;
    for (int mode = 0; mode < 2; mode++) {
      memcpy(ins2, ins, L + 1);
      for (uint32_t q = t - 32768; q < t; q++) ins2[q] = mode == 0 ? (q + 3 <= L) : 0;
      for (uint32_t q = t; q <= L; q++) ins2[q] = 0;
      memset(dec2, 0, (L + 1) * 4);
      run(in, L, level, prevd, ins2, t, dec2);
      // last position where the decisions differ
      uint32_t lastdiff = 0, ndiff = 0;
      for (uint32_t q = t; q < L; q++) if (dec[q] != dec2[q]) { lastdiff = q; ndiff++; }
      printf("start %u mode %d: ndiff %u, last diff at +%u\n", t, mode, ndiff, lastdiff ? lastdiff - t : 0);
    }
  }
}
