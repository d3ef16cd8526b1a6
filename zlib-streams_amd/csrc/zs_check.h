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
