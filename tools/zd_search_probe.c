/*
 * zd_search_probe.c (CPU, tools only) -- how many longest_match walks does the
 * zlib-bytes deflate (levels 4..9, deflate_slow) need, and where?
 *
 *   all      every position walked under the full chain budget (what
 *            zs_zd_match_kernel does today: one walk, the short budget's result
 *            snapshotted on the way)
 *   true     only the loop tops of deflate_slow's parse with prev_length <
 *            max_lazy, each under the budget it uses (zlib's own work)
 *   spec PL  the searches a demand-driven kernel makes: per 8 KiB item, pieces
 *            of PL positions walked from state A at their start, then re-walked
 *            from their predecessor's exit until the walks merge (rounds until
 *            no exit changes), every (position, budget) searched once
 *
 * Costs are chain candidates examined (the GPU kernel's steps).  Corpus: the
 * bench's C2 text (tests/tools/zs_corpus.c).
 *   gcc -O2 -o /tmp/zsp tools/zd_search_probe.c tests/tools/zs_corpus.c -lz -lpthread
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void zs_corpus_zipf(uint8_t *out, size_t n, uint64_t seed);
void zs_corpus_lines(uint8_t *out, size_t n, uint64_t start);

static const uint16_t CFG[10][4] = {{0, 0, 0, 0},      {0, 0, 0, 0},        {0, 0, 0, 0},
                                    {0, 0, 0, 0},      {4, 4, 16, 16},      {8, 16, 32, 32},
                                    {8, 16, 128, 128}, {8, 32, 128, 256},   {32, 128, 258, 1024},
                                    {32, 258, 258, 4096}};
#define MINM 3
#define MAXM 258
#define HMASK 0x7fffu
#define TOO_FAR 4096u
#define MAXD (32768u - 262u)

static const uint8_t *in;
static uint32_t L, *prevd;
static int level;

static uint32_t walk(uint32_t p, uint32_t chain, uint32_t *steps) {  // best | dist << 9
  *steps = 0;
  if (p + MINM > L || !prevd[p] || prevd[p] > MAXD) return 0;
  const uint32_t look = L - p, cap = look < MAXM ? look : MAXM, nice = CFG[level][2] < look ? CFG[level][2] : look;
  uint32_t c = p - prevd[p], best = 0, bd = 0;
  for (uint32_t k = 0;;) {
    uint32_t n = 0;
    while (n < cap && in[c + n] == in[p + n]) n++;
    (*steps)++;
    if (n > best) {
      best = n;
      bd = p - c;
      if (n >= nice) break;
    }
    if (++k >= chain || !prevd[c]) break;
    const uint32_t nc = c - prevd[c];
    if (nc == 0 || p - nc >= MAXD) break;
    c = nc;
  }
  return best | bd << 9;
}

// parse state: bit0 avail, 1-9 prev_len, 10 variant, 11.. prev_dist (deflate_zlib.hip's packing)
#define STATE_A (2u << 1)
static uint64_t cost;
static uint8_t *seen;  // bit0: variant a searched, bit1: b
static uint32_t *res[2];

static uint64_t cost_dup;  // steps of repeated searches (no cache on the GPU)
static int nocache, classes, helpers;
static uint64_t wl_hist[8], ws_hist[8];
static uint32_t search(uint32_t p, uint32_t var) {
  if (nocache && (seen[p] & (1u << var))) {
    uint32_t s;
    (void)walk(p, var ? CFG[level][3] >> 2 : CFG[level][3], &s);
    cost_dup += s;
  }
  if (!(seen[p] & (1u << var))) {
    uint32_t s;
    res[var][p] = walk(p, var ? CFG[level][3] >> 2 : CFG[level][3], &s);
    seen[p] |= 1u << var;
    cost += s;
  }
  return res[var][p];
}

static int approx;           // the walk's searches are approximate (helper prefix)
static uint64_t cost_approx;
static void step(uint32_t *p, uint32_t *st) {
  const uint32_t pl = (*st >> 1) & 511u, good = CFG[level][0], lazy = CFG[level][1];
  uint32_t mlen = 2, mdist = 0, mvar = 0;
  if (pl < lazy) {
    mvar = pl >= good;
    uint32_t m, sa;
    if (approx) {
      m = walk(*p, 4, &sa);
      cost_approx += sa;
    } else {
      m = search(*p, mvar);
    }
    const uint32_t ml = m & 511u;
    if (ml > pl) {
      mlen = ml;
      mdist = m >> 9;
    } else if (ml) {
      mlen = pl;
    }
    if (mlen == MINM && mdist > TOO_FAR) mlen = 2;
  }
  if (pl >= MINM && mlen <= pl) {
    *p = *p - 1 + pl;
    *st = STATE_A;
    return;
  }
  *st = 1u | (mlen << 1) | (mvar << 10) | (mdist << 11);
  *p += 1;
}

static void reset(void) {
  memset(seen, 0, L);
  cost = 0;
  cost_dup = 0;
  cost_approx = 0;
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) << 20 : 16u << 20;
  level = argc > 2 ? atoi(argv[2]) : 6;
  uint8_t *buf = malloc(n + 64);
  prevd = malloc(sizeof(uint32_t) * n);
  seen = malloc(n);
  res[0] = malloc(4u * n);
  res[1] = malloc(4u * n);
  uint32_t *last = malloc(4u << 15);
  for (int kind = 0; kind < 2; kind++) {
    if (kind == 0) zs_corpus_zipf(buf, n, 1);
    else zs_corpus_lines(buf, n, 0);
    in = buf;
    L = n;
    memset(last, 0, 4u << 15);
    for (uint32_t p = 0; p < L; p++) {
      if (p + 2 >= L) {
        prevd[p] = 0;
        continue;
      }
      const uint32_t h = (((uint32_t)in[p] << 10) ^ ((uint32_t)in[p + 1] << 5) ^ in[p + 2]) & HMASK, q = last[h];
      prevd[p] = q > 1 ? p - (q - 1) : 0;
      last[h] = p + 1;
    }
    // all
    uint64_t c_all = 0;
    for (uint32_t p = 0; p < L; p++) {
      uint32_t s;
      (void)walk(p, CFG[level][3], &s);
      c_all += s;
    }
    // true parse
    reset();
    uint64_t tops = 0;
    for (uint32_t p = 0, st = STATE_A; p < L;) {
      tops++;
      step(&p, &st);
    }
    uint64_t searched = 0;
    for (uint32_t p = 0; p < L; p++) searched += __builtin_popcount(seen[p]);
    const uint64_t c_true = cost;
    printf("%s L%d %u MiB: all %.3f steps/B | true: tops %.3f/B searches %.3f/B steps %.3f/B\n", kind ? "lines" : "zipf",
           level, n >> 20, (double)c_all / L, (double)tops / L, (double)searched / L, (double)c_true / L);
    static const uint32_t PLS[] = {8, 16, 32, 64};
    for (int pi = 0; pi < (getenv("SPEC") ? 4 : 0); pi++) {
      const uint32_t PL = PLS[pi], ITEM = 8192, np = ITEM / PL;
      reset();
      uint64_t rounds_tot = 0, items = 0, rounds_max = 0;
      uint32_t *xp = malloc(4 * np), *xs = malloc(4 * np), *sp = malloc(4 * np), *ss = malloc(4 * np);
      uint8_t *markA = calloc(ITEM + 512, 1);
      for (uint32_t i0 = 0; i0 < L; i0 += ITEM) {
        const uint32_t iend = i0 + ITEM < L ? i0 + ITEM : L;
        memset(markA, 0, ITEM + 512);
        for (uint32_t k = 0; k < np; k++) {
          const uint32_t a = i0 + k * PL, b = a + PL < iend ? a + PL : iend;
          uint32_t p = a, st = STATE_A;
          while (a < iend && p < b) {
            if (st == STATE_A) markA[p - i0] = 1;
            step(&p, &st);
          }
          sp[k] = xp[k] = a < iend ? p : a;
          ss[k] = xs[k] = st;
        }
        uint32_t r = 0;
        for (;;) {
          r++;
          int changed = 0;
          for (uint32_t k = 1; k < np; k++) {
            const uint32_t a = i0 + k * PL, b = a + PL < iend ? a + PL : iend;
            if (a >= iend) break;
            uint32_t q = xp[k - 1], qs = xs[k - 1];
            int merged = 0;
            while (q < b) {
              if (qs == STATE_A && markA[q - i0]) {
                merged = 1;
                break;
              }
              step(&q, &qs);
            }
            const uint32_t rp = merged ? sp[k] : q, rs = merged ? ss[k] : qs;
            if (rp != xp[k] || rs != xs[k]) {
              xp[k] = rp;
              xs[k] = rs;
              changed = 1;
            }
          }
          if (!changed) break;
        }
        rounds_tot += r;
        if (r > rounds_max) rounds_max = r;
        items++;
      }
      searched = 0;
      for (uint32_t p = 0; p < L; p++) searched += __builtin_popcount(seen[p]);
      printf("  spec PL=%2u: searches %.3f/B steps %.3f/B (%.2fx fewer than all), rounds avg %.2f max %lu\n", PL,
             (double)searched / L, (double)cost / L, (double)c_all / cost, (double)rounds_tot / items,
             (unsigned long)rounds_max);
      free(xp);
      free(xs);
      free(sp);
      free(ss);
      free(markA);
    }
    // merge-stop walks with a start queue: ITEM positions per workgroup of NL
    // lanes, a start every PL positions, a lane takes the next start when its
    // walk ends; a walk stops at a state-A position another walk already
    // claimed.  Event order by lane clock (chain steps).  eff = steps / (NL *
    // slowest lane), the share of lane time doing chain steps.
    static const uint32_t CF[][3] = {{16384, 512, 16}, {16384, 1024, 16}, {16384, 1024, 8}, {16384, 1024, 4}, {16384, 512, 8}};
    nocache = 1;
    static const uint32_t CF2[][3] = {{16384, 1024, 16}, {16384, 1024, 8}, {16384, 512, 16}};
    for (int ci = 0; ci < 1; ci++) {
      classes = getenv("CLASSES") ? atoi(getenv("CLASSES")) : 1;
      helpers = ci >= 3;
      const uint32_t ITEM = CF2[ci % 3][0], NL = CF2[ci % 3][1], PL = CF2[ci % 3][2];
      (void)CF;
      reset();
      uint64_t tmax_sum = 0, items = 0;
      uint8_t *claimA = calloc(ITEM + 1024, 1);
      uint64_t *clk = malloc(8 * NL);
      uint32_t *lp = malloc(4 * NL), *ls = malloc(4 * NL), *lact = malloc(4 * NL), *lap = calloc(NL, 4), *lstart = calloc(NL, 4);
      uint64_t *lclk0 = calloc(NL, 8);
      memset(wl_hist, 0, sizeof wl_hist);
      memset(ws_hist, 0, sizeof ws_hist);
      for (uint32_t i0 = 0; i0 < L; i0 += ITEM) {
        const uint32_t iend = i0 + ITEM < L ? i0 + ITEM : L;
        memset(claimA, 0, ITEM + 1024);
        uint32_t nexts = 0;
        const uint32_t nst = (iend - i0 + PL - 1) / PL;
        for (uint32_t l = 0; l < NL; l++) {
          clk[l] = 0;
          lact[l] = nexts < nst;
          if (lact[l]) {
            lp[l] = i0 + nexts * PL;
            lstart[l] = lp[l];
            lclk0[l] = 0;
            ls[l] = STATE_A;
            lap[l] = helpers && (nexts * PL) % 256u != 0;
            nexts++;
          }
        }
        for (;;) {
          int best = -1;
          for (uint32_t l = 0; l < NL; l++)
            if (lact[l] && (best < 0 || clk[l] < clk[best])) best = (int)l;
          if (best < 0) break;
          const uint32_t l = (uint32_t)best;
          int stop = lp[l] >= iend;
          if (!stop && lap[l] && ls[l] == STATE_A && lp[l] != i0 + ((lp[l] - i0) / PL) * PL) lap[l] = 0;  // in phase: exact from here
          if (!stop && lap[l]) {
            const uint64_t a0 = cost_approx;
            approx = 1;
            step(&lp[l], &ls[l]);
            approx = 0;
            clk[l] += (cost_approx - a0) + 1;
            continue;
          }
          if (!stop && ls[l] == STATE_A) {
            if (claimA[lp[l] - i0] & 1) stop = 1;
            else claimA[lp[l] - i0] |= 1;
          } else if (!stop && classes) {
            // canonical classes: a literal pending with no match (prev_len < 3)
            // walks on exactly as state A; a pending match is a function of the
            // search at q - 1 and its budget
            const uint32_t pl = (ls[l] >> 1) & 511u;
            const uint32_t cb = pl < 3 ? 1u : (ls[l] >> 10 & 1u) ? 4u : 2u;
            if (claimA[lp[l] - i0] & cb) stop = 1;
            else claimA[lp[l] - i0] |= cb;
          }
          if (!stop) {
            const uint64_t c0 = cost;
            const uint64_t d0 = cost_dup;
            step(&lp[l], &ls[l]);
            clk[l] += (cost - c0) + (cost_dup - d0) + 1;  // + the parse step itself
            continue;
          }
          {
            const uint32_t wlen = lp[l] - lstart[l];
            const uint64_t wst = clk[l] - lclk0[l];
            int b = 0;
            while (b < 7 && (16u << (2 * b)) <= wlen) b++;
            wl_hist[b]++;
            b = 0;
            while (b < 7 && (16u << (2 * b)) <= wst) b++;
            ws_hist[b]++;
          }
          if (nexts < nst) {
            lp[l] = i0 + nexts * PL;
            lstart[l] = lp[l];
            lclk0[l] = clk[l];
            ls[l] = STATE_A;
            lap[l] = helpers && (nexts * PL) % 256u != 0;
            nexts++;
          } else {
            lact[l] = 0;
          }
        }
        uint64_t tm = 0;
        for (uint32_t l = 0; l < NL; l++) tm = clk[l] > tm ? clk[l] : tm;
        tmax_sum += tm;
        items++;
      }
      searched = 0;
      for (uint32_t p = 0; p < L; p++) searched += __builtin_popcount(seen[p]);
      printf("  merge-stop%s%s item %u lanes %u PL %u: approx %.2f/B searches %.3f/B steps %.3f/B (+%.3f repeated), eff %.2f -> %.2f lane-steps/B (all: %.1f)\n",
             classes ? "(classes)" : "", helpers ? "(helpers)" : "", ITEM, NL, PL, (double)cost_approx / L, (double)searched / L, (double)cost / L, (double)cost_dup / L, (double)(cost + cost_dup + cost_approx) / ((double)tmax_sum * NL),
             (double)tmax_sum * NL / L, (double)c_all / L);
      free(claimA);
      free(clk);
      free(lp);
      free(ls);
      free(lact);
      free(lap);
      free(lstart);
      free(lclk0);
      printf("    walk positions <16,<64,<256,<1K,<4K,<16K,<64K,more:");
      for (int b = 0; b < 8; b++) printf(" %lu", (unsigned long)wl_hist[b]);
      printf("\n    walk steps same bins:");
      for (int b = 0; b < 8; b++) printf(" %lu", (unsigned long)ws_hist[b]);
      printf("\n");
    }
    // ring: one workgroup streams a span through an LDS ring of RING positions
    // (32 KiB window + ACT active); a start is taken only below the loaded
    // front, a walk waits while it would read past the front (q + 278), the
    // front moves by CH when every walk is at >= front - ACT + CH
    if (!getenv("NORING")) {
      static const uint32_t RC[][4] = {{1024, 16, 16384, 4096}, {1024, 16, 16384, 2048}, {1024, 16, 8192, 2048}, {512, 16, 16384, 4096}};
      for (int ri = 0; ri < 4; ri++) {
        const uint32_t NL = RC[ri][0], PL = RC[ri][1], ACT = RC[ri][2], CH = RC[ri][3], SPAN = 1u << 20;
        reset();
        classes = 1;
        helpers = 0;
        uint64_t tsum = 0, stalls = 0;
        uint8_t *claim = calloc(SPAN + 1024, 1);
        uint64_t *clk = malloc(8 * NL);
        uint32_t *lp = malloc(4 * NL), *ls = malloc(4 * NL), *lact = malloc(4 * NL);
        for (uint32_t i0 = 0; i0 < L; i0 += SPAN) {
          const uint32_t iend = i0 + SPAN < L ? i0 + SPAN : L;
          memset(claim, 0, SPAN + 1024);
          uint32_t nexts = 0, front = i0 + ACT;  // loaded [.., front)
          if (front > iend) front = iend;
          const uint32_t nst = (iend - i0 + PL - 1) / PL;
          uint64_t now = 0, front_t = 0;
          for (uint32_t l = 0; l < NL; l++) {
            clk[l] = 0;
            lact[l] = 0;
          }
          for (;;) {
            // pick the lane with the smallest clock among those that can act
            int best = -1;
            uint32_t minq = 0xffffffffu;
            int any = 0;
            for (uint32_t l = 0; l < NL; l++) {
              if (lact[l]) {
                any = 1;
                if (lp[l] < minq) minq = lp[l];
              }
            }
            // advance the front while the slowest walk allows it
            while (front < iend && ((!any && i0 + nexts * PL + 278 >= front) || (any && minq >= front - ACT + CH))) {
              front = front + CH < iend ? front + CH : iend;
              front_t = now;  // lanes waiting on the front resume no earlier than this
            }
            for (uint32_t l = 0; l < NL; l++) {
              int can;
              if (lact[l]) can = lp[l] >= iend || lp[l] + 278 < front || front == iend;
              else can = nexts < nst && i0 + nexts * PL + 278 < front + (front == iend ? 1000 : 0);
              if (can && (best < 0 || clk[l] < clk[best])) best = (int)l;
            }
            if (best < 0) {
              int waiting = 0;
              for (uint32_t l = 0; l < NL; l++) waiting |= lact[l];
              if (!waiting && nexts >= nst) break;
              // everyone blocked: the front must move (the slowest walk's clock passes)
              stalls++;
              if (front < iend) front = front + CH < iend ? front + CH : iend;
              front_t = now;
              continue;
            }
            const uint32_t l = (uint32_t)best;
            if (clk[l] < front_t) clk[l] = front_t;
            if (!lact[l]) {
              lp[l] = i0 + nexts * PL;
              ls[l] = STATE_A;
              nexts++;
              lact[l] = 1;
              if (clk[l] < now) clk[l] = now;
              continue;
            }
            now = clk[l] > now ? clk[l] : now;
            int stop = lp[l] >= iend;
            if (!stop) {
              const uint32_t pl = (ls[l] >> 1) & 511u;
              const uint32_t cb = ls[l] == STATE_A || pl < 3 ? 1u : (ls[l] >> 10 & 1u) ? 4u : 2u;
              if (claim[lp[l] - i0] & cb) stop = 1;
              else claim[lp[l] - i0] |= cb;
            }
            if (!stop) {
              const uint64_t c0 = cost, d0 = cost_dup;
              step(&lp[l], &ls[l]);
              clk[l] += (cost - c0) + (cost_dup - d0) + 1;
              continue;
            }
            lact[l] = 0;
          }
          uint64_t tm = 0;
          for (uint32_t l = 0; l < NL; l++) tm = clk[l] > tm ? clk[l] : tm;
          tsum += tm;
        }
        printf("  ring lanes %u PL %u active %u chunk %u (%lu forced): steps %.3f/B (+%.3f repeated), eff %.2f -> %.2f lane-steps/B\n", NL, PL,
               ACT, CH, (unsigned long)stalls, (double)cost / L, (double)cost_dup / L, (double)(cost + cost_dup) / ((double)tsum * NL),
               (double)tsum * NL / L);
        free(claim);
        free(clk);
        free(lp);
        free(ls);
        free(lact);
      }
    }
  }
  return 0;
}
