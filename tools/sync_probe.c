// sync_probe: how far a deflate symbol walk started at an arbitrary bit offset
// inside a dynamic block runs before it lands on the block's true symbol path
// (Huffman self-synchronisation).  Measures the design question of a parallel
// boundary walk; host tool, no GPU.
//   usage: sync_probe RAW_DEFLATE_FILE [stride_bits]
// Output: per-block and overall histograms of the convergence distance (bits
// past the start offset), and the starts whose walk stopped (invalid code, end
// of block, > 4096 bits) before converging.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const uint8_t *in;
static size_t in_bits;

static uint32_t bit(size_t p) { return p < in_bits ? (in[p >> 3] >> (p & 7)) & 1u : 0u; }
static uint32_t bits(size_t p, int n) {
  uint32_t v = 0;
  for (int i = 0; i < n; i++) v |= bit(p + i) << i;
  return v;
}

typedef struct {
  int count[16];
  int sym[320];  // symbols by canonical order
  int maxlen;
} Huff;

static int huff_build(Huff *h, const uint8_t *len, int n) {
  memset(h, 0, sizeof *h);
  for (int i = 0; i < n; i++) h->count[len[i]]++;
  h->count[0] = 0;
  int offs[16] = {0};
  for (int l = 1; l < 16; l++) offs[l] = offs[l - 1] + h->count[l - 1];
  offs[0] = 0;
  int o[16];
  o[1] = 0;
  for (int l = 2; l < 16; l++) o[l] = o[l - 1] + h->count[l - 1];
  for (int i = 0; i < n; i++)
    if (len[i]) h->sym[o[len[i]]++] = i;
  for (int l = 15; l > 0; l--)
    if (h->count[l]) {
      h->maxlen = l;
      break;
    }
  return 0;
}
// canonical decode (puff-style); returns symbol or -1, *used = bits
static int huff_dec(const Huff *h, size_t p, int *used) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; l++) {
    code |= (int)bit(p + l - 1);
    int c = h->count[l];
    if (code - c < first) {
      *used = l;
      return h->sym[index + (code - first)];
    }
    index += c;
    first += c;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

static const int lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static int dext(int d) { return d < 4 ? 0 : d / 2 - 1; }

// one symbol at p: bits consumed, or -1 invalid, -2 end of block
static int step(const Huff *L, const Huff *D, size_t p) {
  int u;
  int s = huff_dec(L, p, &u);
  if (s < 0) return -1;
  if (s < 256) return u;
  if (s == 256) return -2;
  if (s > 285) return -1;
  int n = u + lext[s - 257];
  int du;
  int d = huff_dec(D, p + n, &du);
  if (d < 0 || d >= 30) return -1;
  return n + du + dext(d);
}

#define MAXD 4096
// Parallel-walk simulation of one block: n lanes, lane j walks from st_j
// (segment start s_j, or its predecessor's crossing after a restart), records
// its positions in [s_j, s_j + W), continues into [s_{j+1}, s_{j+1} + W)
// looking for a position of lane j + 1's path; rounds restart every lane that
// its predecessor did not merge with, until the chain from lane 0 reaches the
// last lane.  Reports rounds and the steps of the longest lane per round.
#define W 1024
static long rounds_hist[66], sim_blocks, sim_steps, sim_fallback, sim_serial_steps;
static int pos_in(const uint8_t *bm, size_t s, size_t q) { return q >= s && q < s + W && bm[q - s]; }
static void sim_block(const Huff *L, const Huff *D, size_t b0, size_t b1, long nsym) {
  size_t range = b1 - b0;
  size_t seg = range / 64 > W + 64 ? range / 64 : W + 64;
  int n = (int)(range / seg);
  if (n < 1) n = 1;
  static size_t st[64], sj[65], cr[64];
  static uint8_t bm[64][W];
  static int merged[64], stopped[64];
  for (int j = 0; j < n; j++) { sj[j] = b0 + j * seg; st[j] = sj[j]; }
  sj[n] = (size_t)-1;
  int todo_from = 0, r;
  long steps_total = 0;
  for (r = 1; r <= 64; r++) {
    long maxsteps = 0;
    for (int j = todo_from; j < n; j++) {  // phase A: own window
      memset(bm[j], 0, W);
      size_t p = st[j];
      long k = 0;
      stopped[j] = 0;
      while (p < sj[j] + W && p < b1) {
        bm[j][p - sj[j]] = 1;
        int u = step(L, D, p);
        if (u < 0) { stopped[j] = 1; break; }
        p += u; k++;
      }
      (void)k;
    }
    for (int j = todo_from; j < n; j++) {  // phase A + B steps, merge check with lane j + 1
      size_t p = st[j];
      long k = 0;
      merged[j] = 0;
      cr[j] = 0;
      while (j + 1 < n ? p < sj[j + 1] + W : p < b1) {
        if (j + 1 < n && p >= sj[j + 1]) {
          if (!cr[j]) cr[j] = p;
          if (pos_in(bm[j + 1], sj[j + 1], p)) { merged[j] = 1; break; }
        }
        int u = step(L, D, p);
        if (u < 0) break;
        p += u; k++;
      }
      if (k > maxsteps) maxsteps = k;
    }
    steps_total += maxsteps;
    // the chain from lane todo_from: first lane whose predecessor did not merge
    int J = todo_from + 1;
    while (J < n && merged[J - 1]) J++;
    if (J >= n) break;
    // restart every lane >= J whose predecessor did not merge, from the predecessor's crossing
    for (int j = J; j < n; j++)
      if (!merged[j - 1] && cr[j - 1]) st[j] = cr[j - 1];
    todo_from = J - 1 > 0 ? J - 1 : 0;
    todo_from = J;  // lanes < J are final; lane J - 1's merge with the restarted lane J is at its start
  }
  sim_blocks++;
  if (r > 64) { sim_fallback++; r = 64; }
  rounds_hist[r]++;
  sim_steps += steps_total;
  sim_serial_steps += nsym;
}
static long hist[MAXD / 64 + 2], hsyms[130], fails_stop, fails_far, starts;

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *buf = malloc(n);
  if (fread(buf, 1, n, f) != (size_t)n) return 2;
  fclose(f);
  in = buf;
  in_bits = (size_t)n * 8;
  int stride = argc > 2 ? atoi(argv[2]) : 97;
  size_t p = 0;
  int blocks = 0;
  uint8_t *truth = calloc(in_bits + 1, 1);
  while (p + 3 < in_bits && blocks < 400) {
    int final = bit(p), type = bits(p + 1, 2);
    p += 3;
    if (type != 2) break;
    int hlit = bits(p, 5) + 257, hdist = bits(p + 5, 5) + 1, hclen = bits(p + 10, 4) + 4;
    p += 14;
    static const int ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint8_t cl[19] = {0};
    for (int i = 0; i < hclen; i++, p += 3) cl[ord[i]] = bits(p, 3);
    Huff C;
    huff_build(&C, cl, 19);
    uint8_t lens[320] = {0};
    int k = 0;
    while (k < hlit + hdist) {
      int u;
      int s = huff_dec(&C, p, &u);
      p += u;
      if (s < 16) lens[k++] = s;
      else if (s == 16) {
        int r = 3 + bits(p, 2);
        p += 2;
        for (int i = 0; i < r; i++, k++) lens[k] = lens[k - 1];
      } else if (s == 17) {
        int r = 3 + bits(p, 3);
        p += 3;
        k += r;
      } else {
        int r = 11 + bits(p, 7);
        p += 7;
        k += r;
      }
    }
    Huff L, D;
    huff_build(&L, lens, hlit);
    huff_build(&D, lens + hlit, hdist);
    size_t b0 = p;
    long nsym = 0;
    for (;;) {
      truth[p] = 1;
      int u = step(&L, &D, p);
      if (u == -2) {
        int used;
        huff_dec(&L, p, &used);
        p += used;
        break;
      }
      if (u < 0) {
        fprintf(stderr, "bad stream\n");
        return 1;
      }
      p += u;
      nsym++;
    }
    size_t b1 = p;
    // speculative walks from offsets inside the block
    for (size_t s = b0 + 1; s + MAXD < b1; s += stride) {
      starts++;
      size_t q = s;
      long ns = 0;
      int ok = 0;
      while (q - s < MAXD) {
        if (truth[q]) {
          ok = 1;
          break;
        }
        int u = step(&L, &D, q);
        if (u < 0) break;
        q += u;
        ns++;
      }
      if (ok) {
        hist[(q - s) / 64]++;
        hsyms[ns < 128 ? ns : 128]++;
      } else if (q - s >= MAXD)
        fails_far++;
      else
        fails_stop++;
    }
    sim_block(&L, &D, b0, b1, nsym);
    blocks++;
    if (final) break;
    (void)nsym;
  }
  printf("blocks %d starts %ld fails_stop %ld fails_far %ld\n", blocks, starts, fails_stop, fails_far);
  printf("pwalk: blocks %ld fallback %ld  wave-steps %.1f per block vs serial %.1f\n", sim_blocks, sim_fallback,
         (double)sim_steps / sim_blocks, (double)sim_serial_steps / sim_blocks);
  for (int i = 0; i < 66; i++)
    if (rounds_hist[i]) printf("  rounds %2d: %ld\n", i, rounds_hist[i]);
  long cum = 0;
  for (int i = 0; i < MAXD / 64; i++) {
    cum += hist[i];
    if (hist[i]) printf("bits < %4d: %8ld  cum %.6f\n", (i + 1) * 64, hist[i], (double)cum / starts);
  }
  cum = 0;
  for (int i = 0; i <= 128; i++) {
    cum += hsyms[i];
    if (hsyms[i] && (i < 16 || i % 8 == 0)) printf("syms <= %3d: cum %.6f\n", i, (double)cum / starts);
  }
  return 0;
}
