// zs_check.h -- piece-parallel CRC-32 / Adler-32 (device side).
//
// The check values of src/inflate.c UPDATE_CHECK (425-429) and deflate.c's
// read_buf, computed over any split of a buffer into pieces that are combined
// in any order:
//   CRC-32: with f(c, M) the table-driven register update from c (no final
//     xor), f(0, .) is GF(2)-linear, f(0, A|B) = f(0, A) * x^(8|B|) ^ f(0, B),
//     and crc32(M) = ~(f(0, M) ^ 0xffffffff * x^(8|M|)).  A piece [lo, hi) of
//     an n-byte buffer contributes f(0, piece) * x^(8(n - hi)); contributions
//     combine with XOR (atomicXor), so no piece waits for another.
//   Adler-32: a = 1 + sum x_i, b = n + sum x_i * (n - i) (mod 65521); a piece
//     contributes its two partial sums, combined with atomicAdd.
// x^(8k) mod P comes from a compile-time table of x^(8 * 2^j), one GF(2)
// multiply per set bit of k.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZS_CRC_POLY 0xEDB88320u
#define ZS_ADLER_MOD 65521u

// a(x) * b(x) mod P(x), reflected bit order (bit 31 = x^0); a != 0 or b == 0
__host__ __device__ constexpr uint32_t zs_gf2_mul(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  if (a == 0) return 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ ZS_CRC_POLY : b >> 1;
  }
  return p;
}

struct ZsX8Pow {
  uint32_t v[64];
};
__host__ __device__ constexpr ZsX8Pow zs_make_x8pow() {
  ZsX8Pow t{};
  uint32_t sq = 1u << 23;  // x^8
  for (int j = 0; j < 64; j++) {
    t.v[j] = sq;
    sq = zs_gf2_mul(sq, sq);
  }
  return t;
}
__constant__ constexpr ZsX8Pow zs_x8pow = zs_make_x8pow();

// x^(8k) mod P
__device__ __forceinline__ uint32_t zs_x8n(uint64_t k) {
  uint32_t p = 1u << 31;
  for (int j = 0; k; j++, k >>= 1)
    if (k & 1) p = zs_gf2_mul(zs_x8pow.v[j], p);
  return p;
}

// slice-by-4 tables in LDS; every thread of the block helps (blockDim >= 64)
__device__ __forceinline__ void zs_crc_tables(uint32_t (*T)[256]) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (ZS_CRC_POLY ^ (c >> 1)) : (c >> 1);
    T[0][i] = c;
  }
  __syncthreads();
  for (int s = 1; s < 4; s++) {
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) T[s][i] = (T[s - 1][i] >> 8) ^ T[0][T[s - 1][i] & 0xffu];
    __syncthreads();
  }
}

// f(0, p[lo, hi)): bytes up to 4-byte alignment, then aligned words
__device__ __forceinline__ uint32_t zs_crc_raw(const uint8_t *p, uint64_t lo, uint64_t hi, const uint32_t (*T)[256]) {
  uint32_t c = 0;
  uint64_t i = lo;
  while (i < hi && ((reinterpret_cast<uintptr_t>(p) + i) & 3u)) c = T[0][(c ^ p[i++]) & 0xffu] ^ (c >> 8);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(p + i);
  const uint64_t nw = (hi - i) >> 2;
  for (uint64_t k = 0; k < nw; k++) {
    c ^= w[k];
    c = T[3][c & 0xffu] ^ T[2][(c >> 8) & 0xffu] ^ T[1][(c >> 16) & 0xffu] ^ T[0][c >> 24];
  }
  i += nw << 2;
  while (i < hi) c = T[0][(c ^ p[i++]) & 0xffu] ^ (c >> 8);
  return c;
}

// piece contribution to the XOR accumulator of an n-byte buffer
__device__ __forceinline__ uint32_t zs_crc_piece(const uint8_t *p, uint64_t lo, uint64_t hi, uint64_t n,
                                                 const uint32_t (*T)[256]) {
  if (hi <= lo) return 0;
  const uint32_t f = zs_crc_raw(p, lo, hi, T);
  return n > hi ? zs_gf2_mul(zs_x8n(n - hi), f) : f;
}
// crc32 of the whole n-byte buffer from its XOR accumulator
__device__ __forceinline__ uint32_t zs_crc_final(uint32_t acc, uint64_t n) {
  return ~(acc ^ zs_gf2_mul(zs_x8n(n), 0xffffffffu));
}

// Adler-32 partial sums of p[lo, hi) in an n-byte buffer: A = sum x_i,
// B = sum x_i * (n - i), both mod 65521
__device__ __forceinline__ void zs_adler_piece(const uint8_t *p, uint64_t lo, uint64_t hi, uint64_t n, uint32_t *A,
                                               uint32_t *B) {
  uint64_t s1 = 0, s2 = 0, acc1 = 0, acc2 = 0;  // s2 = sum x_i * (i - lo) within a 4 KiB run
  uint64_t i = lo;
  while (i < hi) {
    const uint64_t e = min(hi, i + 4096);
    const uint64_t base = i;
    s1 = 0;
    s2 = 0;
    uint64_t k = i;
    while (k < e && ((reinterpret_cast<uintptr_t>(p) + k) & 3u)) {
      s1 += p[k];
      s2 += (k - base) * p[k];
      k++;
    }
    for (; k + 4 <= e; k += 4) {
      const uint32_t w = *reinterpret_cast<const uint32_t *>(p + k);
      const uint32_t b0 = w & 0xffu, b1 = (w >> 8) & 0xffu, b2 = (w >> 16) & 0xffu, b3 = w >> 24;
      const uint64_t o = k - base;
      s1 += b0 + b1 + b2 + b3;
      s2 += o * (b0 + b1 + b2 + b3) + b1 + 2u * b2 + 3u * b3;
    }
    for (; k < e; k++) {
      s1 += p[k];
      s2 += (k - base) * p[k];
    }
    // sum x_k (n - k) over the run = (n - base) * s1 - s2
    acc1 = (acc1 + s1) % ZS_ADLER_MOD;
    acc2 = (acc2 + ((n - base) % ZS_ADLER_MOD) * (s1 % ZS_ADLER_MOD) + ZS_ADLER_MOD - s2 % ZS_ADLER_MOD) % ZS_ADLER_MOD;
    i = e;
  }
  *A = (uint32_t)acc1;
  *B = (uint32_t)acc2;
}
__device__ __forceinline__ uint32_t zs_adler_final(uint64_t sumA, uint64_t sumB, uint64_t n) {
  const uint64_t a = (1u + sumA % ZS_ADLER_MOD) % ZS_ADLER_MOD;
  const uint64_t b = (n % ZS_ADLER_MOD + sumB % ZS_ADLER_MOD) % ZS_ADLER_MOD;
  return (uint32_t)((b << 16) | a);
}

// block-wide reductions (blockDim.x = 64 * k, k <= 16); s = 16-entry LDS scratch
__device__ __forceinline__ uint32_t zs_block_xor(uint32_t v, uint32_t *s) {
  for (int o = 32; o >= 1; o >>= 1) v ^= __shfl_xor(v, o);
  if ((threadIdx.x & 63u) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
  for (uint32_t w = 0; w < blockDim.x / 64u; w++) r ^= s[w];
  __syncthreads();
  return r;
}
__device__ __forceinline__ uint64_t zs_block_sum(uint64_t v, uint64_t *s) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63u) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t r = 0;
  for (uint32_t w = 0; w < blockDim.x / 64u; w++) r += s[w];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// Coalesced block checks (256 threads).  A block reads its range in 4 KiB
// steps, thread t the 16 bytes at 16 t of each step (one 4 KiB coalesced load
// per step for the block), so each thread sees 16 bytes, a 4080-byte gap,
// 16 bytes, ...  CRC-32: a thread's register c moves over the gap as
// c * x^(8 * 4080) (linear in c: 4 tables G), then takes the next 16 bytes
// (slice-by-16: 16 tables Tp); its register then stands at the end of its
// last 16 bytes and reaches the end of the step by x^(8 (4080 - 16 t)).
// Tables are XORs of a compile-time basis (a table of a linear map is fixed by
// its values at the 8 single-bit bytes).  Adler-32: per-thread byte and
// position-weighted sums, exact in u64, reduced mod 65521 once.
// ---------------------------------------------------------------------------
#define ZS_CK_T 256u
#define ZS_CK_STEP (ZS_CK_T * 16u)

__host__ __device__ constexpr uint32_t zs_crc_byte(uint32_t x) {  // f(0, one byte x)
  uint32_t c = x;
  for (int k = 0; k < 8; k++) c = (c & 1) ? (ZS_CRC_POLY ^ (c >> 1)) : (c >> 1);
  return c;
}
__host__ __device__ constexpr uint32_t zs_x8n_c(uint64_t k) {  // x^(8k) mod P, compile time
  const ZsX8Pow t = zs_make_x8pow();
  uint32_t p = 1u << 31;
  for (int j = 0; k; j++, k >>= 1)
    if (k & 1) p = zs_gf2_mul(t.v[j], p);
  return p;
}
struct ZsCkBasis {
  uint32_t tp[16][8];   // Tp[b][1 << k]: byte 1 << k at position b of 16, then 15 - b zero bytes
  uint32_t g[4][8];     // G[q][1 << k]: register byte q = 1 << k, then 4080 zero bytes
  uint32_t c[ZS_CK_T];  // x^(8 (4080 - 16 t))
};
__host__ __device__ constexpr ZsCkBasis zs_make_ck_basis() {
  ZsCkBasis B{};
  for (int b = 0; b < 16; b++) {
    const uint32_t sh = zs_x8n_c(15 - b);
    for (int k = 0; k < 8; k++) B.tp[b][k] = zs_gf2_mul(sh, zs_crc_byte(1u << k));
  }
  const uint32_t gap = zs_x8n_c(ZS_CK_STEP - 16);
  for (int q = 0; q < 4; q++)
    for (int k = 0; k < 8; k++) B.g[q][k] = zs_gf2_mul(gap, 1u << (8 * q + k));
  const uint32_t x128 = zs_x8n_c(16);
  uint32_t c = 1u << 31;  // t = 255: no shift
  for (int t = ZS_CK_T - 1; t >= 0; t--) {
    B.c[t] = c;
    c = zs_gf2_mul(x128, c);
  }
  return B;
}
__constant__ constexpr ZsCkBasis zs_ck_basis = zs_make_ck_basis();

struct ZsCkTabs {
  uint32_t tp[16][256];
  uint32_t g[4][256];
};
// every thread of the (256-thread) block builds entry threadIdx.x of the 20 tables
__device__ __forceinline__ void zs_ck_tables(ZsCkTabs &T) {
  const uint32_t x = threadIdx.x;
#pragma unroll
  for (int b = 0; b < 16; b++) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) v ^= ((x >> k) & 1u) ? zs_ck_basis.tp[b][k] : 0u;
    T.tp[b][x] = v;
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) v ^= ((x >> k) & 1u) ? zs_ck_basis.g[q][k] : 0u;
    T.g[q][x] = v;
  }
  __syncthreads();
}

// CRC-32 accumulator contribution of p[lo, hi) in an n-byte buffer (zs_crc_piece's
// meaning), for the whole block; p + lo 16-byte aligned; valid in thread 0
__device__ __forceinline__ uint32_t zs_crc_block(const uint8_t *p, uint64_t lo, uint64_t hi, uint64_t n,
                                                 const ZsCkTabs &T, uint32_t *s_red) {
  const uint32_t t = threadIdx.x;
  const uint64_t J = (hi - lo) / ZS_CK_STEP, E = lo + J * ZS_CK_STEP;
  const uint4 *q = reinterpret_cast<const uint4 *>(p + lo) + t;
  uint32_t c = 0;
  for (uint64_t j = 0; j < J; j++) {
    uint4 v = q[j * ZS_CK_T];
    v.x ^= T.g[0][c & 0xffu] ^ T.g[1][(c >> 8) & 0xffu] ^ T.g[2][(c >> 16) & 0xffu] ^ T.g[3][c >> 24];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 16; b++) r ^= T.tp[b][(w[b >> 2] >> (8 * (b & 3))) & 0xffu];
    c = r;
  }
  // the tail [E, hi), < 4 KiB: thread t's 16-byte slot ends 4080 - 16 t before
  // hi (the shift of the main part), its bytes before E skipped
  const uint64_t L = hi - E;
  const uint32_t d = ZS_CK_STEP - 16u * t;  // the slot's distance from hi
  uint32_t ct = 0;
  for (uint32_t k = 0; k < 16; k++)
    if (d - k <= L) ct = T.tp[15][(ct ^ p[hi - (d - k)]) & 0xffu] ^ (ct >> 8);
  const uint32_t a = zs_block_xor(zs_gf2_mul(zs_ck_basis.c[t], c), s_red);
  const uint32_t b = zs_block_xor(zs_gf2_mul(zs_ck_basis.c[t], ct), s_red);
  if (t != 0) return 0;
  uint32_t r = 0;
  if (a) r ^= zs_gf2_mul(zs_x8n(n - E), a);
  if (b) r ^= n > hi ? zs_gf2_mul(zs_x8n(n - hi), b) : b;
  return r;
}

// Adler-32 partial sums (zs_adler_piece's A, B) of p[lo, hi) for the whole
// block; p + lo 16-byte aligned; valid in thread 0
__device__ __forceinline__ void zs_adler_block(const uint8_t *p, uint64_t lo, uint64_t hi, uint64_t n, uint64_t *s_red,
                                               uint64_t *A, uint64_t *B) {
  const uint32_t t = threadIdx.x;
  const uint64_t J = (hi - lo) / ZS_CK_STEP, E = lo + J * ZS_CK_STEP;
  const uint4 *q = reinterpret_cast<const uint4 *>(p + lo) + t;
  uint64_t sa = 0, sw = 0;  // sum x, sum x * (i - lo - 16 t)
  for (uint64_t j = 0; j < J; j++) {
    const uint4 v = q[j * ZS_CK_T];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t bs = 0, bw = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t x = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
      bs += x;
      bw += x * (uint32_t)k;
    }
    sa += bs;
    sw += j * ZS_CK_STEP * bs + bw;
  }
  sw += (uint64_t)(16u * t) * sa;
  for (uint64_t i = E + 16u * t; i < hi && i < E + 16u * t + 16u; i++) {
    const uint32_t x = p[i];
    sa += x;
    sw += (i - lo) * x;
  }
  // sum x_i (n - i) = (n - lo) sum x_i - sum x_i (i - lo)
  const uint64_t am = sa % ZS_ADLER_MOD;
  const uint64_t bm = ((n - lo) % ZS_ADLER_MOD * am + ZS_ADLER_MOD - sw % ZS_ADLER_MOD) % ZS_ADLER_MOD;
  const uint64_t ra = zs_block_sum(am, s_red), rb = zs_block_sum(bm, s_red);
  *A = ra;
  *B = rb;
}

