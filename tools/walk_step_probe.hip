// walk_step_probe.hip -- cycles per step of the split parse's boundary walk
// (lane_decode.hip zs_walk_kernel) on synthetic data, one wave per SIMD, to
// find where its ~1 100 cycles per step go.  Each lane walks its own random
// lane-interleaved u8 tables and a 32-word circular input ring in LDS.
//   mode 0: the walk step (3 ring reads, literal then distance lookup)
//   mode 1: the same, input bits from a register LFSR instead of the ring
//   mode 2: the same, table reads replaced by register arithmetic
//   mode 3: mode 0 with 2 waves per SIMD (half the LDS per block)
// build: hipcc --offload-arch=gfx950 -O3 tools/walk_step_probe.hip -o tools/walk_step_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define STEPS 8192
#define RW 32

template <int MODE, int LDSW>
__global__ void __launch_bounds__(64) probe(const uint32_t *init, uint64_t *cyc, uint32_t *sink) {
  // LDSW: dwords of table per lane (128 = 512 u8 entries)
  __shared__ uint32_t wl[LDSW][64];
  __shared__ uint32_t wd[32][64];
  __shared__ uint32_t ring[RW][64];
  const uint32_t lane = threadIdx.x;
  uint32_t x = init[blockIdx.x * 64 + lane] | 1u;
  for (int i = 0; i < LDSW; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    // entries: bits 0-3 = 4..11 bits consumed, bit 5 = has distance (1 in 4)
    uint32_t v = 0;
    for (int b = 0; b < 4; b++) v |= ((4u + ((x >> (8 * b)) & 7u)) | (((x >> (8 * b + 3)) & 3u) == 0 ? 0x20u : 0u)) << (8 * b);
    wl[i][lane] = v;
  }
  for (int i = 0; i < 32; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    uint32_t v = 0;
    for (int b = 0; b < 4; b++) v |= (5u + ((x >> (8 * b)) & 7u)) << (8 * b);
    wd[i][lane] = v;
  }
  for (int i = 0; i < RW; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    ring[i][lane] = x;
  }
  __syncthreads();
  const uint8_t *wlb = reinterpret_cast<const uint8_t *>(&wl[0][lane]);
  const uint8_t *wdb = reinterpret_cast<const uint8_t *>(&wd[0][lane]);
  uint32_t p = lane * 3u, acc = 0, lf = x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < STEPS; s++) {
    uint32_t bits, dbits;
    uint64_t A = 0, B = 0;
    const uint32_t wq = p >> 5, sh = p & 31u;
    if (MODE == 1) {
      lf ^= lf << 13; lf ^= lf >> 17; lf ^= lf << 5;
      A = ((uint64_t)lf << 32) | (lf ^ p);
      B = A ^ 0x5555;
    } else {
      const uint32_t x0 = ring[wq & (RW - 1)][lane], x1 = ring[(wq + 1) & (RW - 1)][lane],
                     x2 = ring[(wq + 2) & (RW - 1)][lane];
      A = ((uint64_t)x1 << 32) | x0;
      B = ((uint64_t)x2 << 32) | x1;
    }
    bits = (uint32_t)(A >> sh);
    uint32_t e;
    const uint32_t i1 = bits & 511u;
    if (MODE == 2) e = 4u + (i1 & 7u) + ((i1 & 0x18u) == 0 ? 0x20u : 0u);
    else e = wlb[((i1 >> 2) * 64u) * 4u + (i1 & 3u)];
    const uint32_t n = e & 15u;
    const uint32_t q = sh + n;
    dbits = (uint32_t)((q < 32u ? A : B) >> (q & 31u));
    const uint32_t i2 = dbits & 127u;
    uint32_t d;
    if (MODE == 2) d = 5u + (i2 & 7u);
    else d = wdb[((i2 >> 2) * 64u) * 4u + (i2 & 3u)];
    const uint32_t dn = (e & 0x20u) ? (d & 15u) : 0u;
    p += n + dn;
    acc += e + d;
    if (__builtin_expect(__ballot(p > 0xfffff000u) != 0, 0)) acc ^= p;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + lane] = acc + p;
}

int main() {
  const int nb = 1024;
  std::vector<uint32_t> h(nb * 64 * 2);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u) ^ 0x9e3779b9u;
  uint32_t *d, *ds;
  uint64_t *dc;
  hipMalloc(&d, h.size() * 4);
  hipMalloc(&dc, nb * 2 * 8);
  hipMalloc(&ds, nb * 2 * 64 * 4);
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  auto run = [&](auto kern, int blocks, const char *name) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, d, dc, ds);
    hipDeviceSynchronize();
    std::vector<uint64_t> c(blocks);
    hipMemcpy(c.data(), dc, blocks * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : c) s += (double)v;
    printf("%-52s %.1f cycles/step\n", name, s / blocks / STEPS);
  };
  for (int rep = 0; rep < 2; rep++) {
    run(probe<0, 128>, nb, "walk step, ring + u8 tables (1 wave/SIMD)");
    run(probe<1, 128>, nb, "walk step, bits from registers");
    run(probe<2, 128>, nb, "walk step, tables as arithmetic");
    run(probe<0, 32>, 2 * nb, "walk step, 2 waves/SIMD");
  }
  return 0;
}
