// lds_chain_probe.hip -- cycles per step of a dependent per-lane table walk
// at one wave per SIMD (the split parse's walk / the lane parse's step shape).
// Each lane walks its own random 512-entry u8 table: idx -> e = tab[idx];
// idx = f(idx, e) with the variants below; s_memtime around the loop.
//   mode 0: own table per lane (lane stride 512 B)
//   mode 1: every lane reads lane 0's table (broadcast / conflict pattern)
//   mode 2: own table, lane stride 516 B (bank-skewed)
//   mode 3: own table, plus a 64-bit shift chain per step (the walk's hold)
//   mode 4: two dependent table reads per step (literal then distance)
// build: hipcc --offload-arch=gfx950 -O3 tools/lds_chain_probe.hip -o tools/lds_chain_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define STEPS 4096

template <int MODE>
__global__ void __launch_bounds__(64) probe(const uint8_t *tabs, uint64_t *cyc, uint32_t *sink) {
  __shared__ uint8_t t[64 * 520];
  const uint32_t lane = threadIdx.x;
  const uint32_t stride = MODE == 2 ? 516u : 512u;
  for (uint32_t i = 0; i < 512; i++) t[lane * stride + i] = tabs[(blockIdx.x * 64 + lane) * 512 + i];
  __syncthreads();
  const uint8_t *my = &t[(MODE == 1 ? 0u : lane) * stride];
  uint32_t idx = lane * 7u;
  uint64_t hold = 0x123456789abcdefull ^ ((uint64_t)lane << 40);
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < STEPS; s++) {
    uint32_t e = my[idx & 511u];
    if (MODE == 3) {
      hold = (hold >> (e & 15u)) | ((uint64_t)e << 50);
      idx = (uint32_t)hold;
    } else if (MODE == 4) {
      const uint32_t n = e & 15u;
      const uint32_t d = my[((idx >> n) ^ e) & 511u];
      idx = idx * 5u + e + d;
    } else {
      idx = idx * 5u + e;
    }
    acc += e;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + lane] = acc + idx;
}

int main() {
  const int nb = 1024;  // one wave per SIMD on 256 CUs
  std::vector<uint8_t> h((size_t)nb * 64 * 512);
  uint32_t x = 12345;
  for (auto &v : h) {
    x = x * 1103515245u + 12345u;
    v = (uint8_t)(x >> 16);
  }
  uint8_t *d;
  uint64_t *dc;
  uint32_t *ds;
  hipMalloc(&d, h.size());
  hipMalloc(&dc, nb * 8);
  hipMalloc(&ds, nb * 64 * 4);
  hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
  auto run = [&](auto kern, const char *name) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(64), 0, 0, d, dc, ds);
    hipDeviceSynchronize();
    std::vector<uint64_t> c(nb);
    hipMemcpy(c.data(), dc, nb * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : c) s += (double)v;
    printf("%-40s %.1f cycles/step\n", name, s / nb / STEPS);
  };
  for (int rep = 0; rep < 2; rep++) {
    run(probe<0>, "own table (stride 512)");
    run(probe<1>, "lane 0's table for all");
    run(probe<2>, "own table (stride 516)");
    run(probe<3>, "own table + 64-bit shift chain");
    run(probe<4>, "own table, two dependent reads");
  }
  return 0;
}
