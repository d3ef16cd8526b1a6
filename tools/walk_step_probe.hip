// walk_step_probe.hip -- cycles per step of the split parse's boundary walk
// (lane_decode.hip zs_walk_kernel) on synthetic data, to separate the step's
// own latency from everything around it.  The layout is the kernel's: u8
// tables lane-interleaved (dword k of lane L at [k][L]), the input ring one
// row of 35 words per lane, 52 KiB of LDS per wave (three waves per CU).
//   mode 0: the kernel's step (ring read, literal entry, distance entry)
//   mode 1: the same without the exception bookkeeping
//   mode 2: the ring read and the literal lookup only (two LDS round trips)
//   mode 3: one dependent LDS read per step (the LDS latency)
//   mode 4: mode 0 with every lane at its own random ring slot (the kernel's units)
//   mode 5: mode 4 plus a 64-byte global load per lane every 9 steps (the refill prefetch)
// build: hipcc --offload-arch=gfx950 -O3 tools/walk_step_probe.hip -o tools/walk_step_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define STEPS 8192
#define RS 35
#define WAVE 64

struct ProbeLDS {
  uint32_t wl[128][WAVE];
  uint32_t wd[32][WAVE];
  uint32_t pad[9][WAVE];
  uint32_t ring[WAVE][RS];
};

__device__ __forceinline__ uint32_t byte_at(uint32_t base, uint32_t i, uint32_t nbits) {
  typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
  const uint32_t a = ((i & ((1u << nbits) - 4u)) << 6) | ((i & 3u) | base);
  return *(lds_cu8 *)(uintptr_t)a;
}

template <int MODE>
__global__ void __launch_bounds__(64) probe(const uint32_t *init, uint64_t *cyc, uint32_t *sink) {
  __shared__ ProbeLDS L;
  typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
  const uint32_t lane = threadIdx.x;
  uint32_t x = init[blockIdx.x * 64 + lane] | 1u;
  for (int i = 0; i < 128; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    uint32_t v = 0;  // entries: 4..11 bits, one in four with a distance
    for (int b = 0; b < 4; b++) v |= ((4u + ((x >> (8 * b)) & 7u)) | (((x >> (8 * b + 3)) & 3u) == 0 ? 0x20u : 0u)) << (8 * b);
    L.wl[i][lane] = v;
  }
  for (int i = 0; i < 32; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    uint32_t v = 0;
    for (int b = 0; b < 4; b++) v |= (5u + ((x >> (8 * b)) & 7u)) << (8 * b);
    L.wd[i][lane] = v;
  }
  for (int i = 0; i < RS; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    L.ring[lane][i] = x;
  }
  __syncthreads();
  uint32_t rra = (uint32_t)(uintptr_t)(lds_cu32 *)&L.ring[lane][0];
  uint32_t wla = (uint32_t)(uintptr_t)(lds_cu32 *)&L.wl[0][lane], wda = (uint32_t)(uintptr_t)(lds_cu32 *)&L.wd[0][lane];
  asm volatile("" : "+v"(rra), "+v"(wla), "+v"(wda));
  uint32_t p = (MODE >= 4) ? (x & 0x3ffu) : lane * 3u, ntok = 0, xp = 0, pstop = 0, tstop = 0, acc = 0;
  const uint4 *gsrc = reinterpret_cast<const uint4 *>(init) + (x & 0xfffu) * 4u;
  const uint32_t limit = 0xfffff000u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int st = 0; st < STEPS; st++) {
    if (MODE == 3) {
      lds_cu32 *r = (lds_cu32 *)(uintptr_t)(rra + 4u * (p & 31u));
      p = r[0];
      continue;
    }
    lds_cu32 *r = (lds_cu32 *)(uintptr_t)(rra + 4u * __builtin_amdgcn_ubfe(p, 5, 5));
    const uint32_t x0 = r[0], x1 = r[1], x2 = r[2];
    const uint32_t lo = __builtin_amdgcn_alignbit(x1, x0, p);
    const uint32_t hi = __builtin_amdgcn_alignbit(x2, x1, p);
    const uint32_t e = byte_at(wla, lo, 9);
    if (MODE == 2) {
      p += (e & 31u);
      continue;
    }
    const uint32_t n = e & 31u;
    const uint32_t d = byte_at(wda, __builtin_amdgcn_alignbit(hi, lo, n), 7);
    const uint32_t dd = (e & 0x20u) ? d : 0u;
    const uint32_t p0 = p;
    p += n + (dd & 31u);
    ntok++;
    if (MODE == 5 && (st % 9) == 0) {
      uint4 g = gsrc[(st * 64u) & 0xffffu];
      asm volatile("" : "+v"(g.x), "+v"(g.y), "+v"(g.z), "+v"(g.w));
      acc += g.x;  // consumed 9 steps later by the compiler's wait, as the kernel's prefetch
    }
    if (MODE == 0 || MODE >= 4) {
      const uint32_t xx = ((e | dd) & 0x40u) | (p > limit ? 1u : 0u);
      const bool first = xx && !xp;
      pstop = first ? p0 : pstop;
      tstop = first ? ntok - 1u : tstop;
      xp |= xx;
    } else {
      acc += e + d;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + lane] = acc + p + ntok + pstop + tstop + xp;
}

int main() {
  const int nb = 768;  // three per CU, like the walk
  std::vector<uint32_t> h(1u << 20);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u) ^ 0x9e3779b9u;
  uint32_t *d, *ds;
  uint64_t *dc;
  if (hipMalloc(&d, h.size() * 4 + (1u << 22)) || hipMalloc(&dc, nb * 8) || hipMalloc(&ds, nb * 64 * 4)) return 1;
  if (hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice)) return 1;
  auto run = [&](auto kern, const char *name) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(64), 0, 0, d, dc, ds);
    if (hipDeviceSynchronize()) return;
    std::vector<uint64_t> c(nb);
    if (hipMemcpy(c.data(), dc, nb * 8, hipMemcpyDeviceToHost)) return;
    double s = 0;
    for (auto v : c) s += (double)v;
    printf("%-60s %.1f cycles/step\n", name, s / nb / STEPS);
  };
  for (int rep = 0; rep < 2; rep++) {
    run(probe<0>, "kernel step (ring, literal, distance, exception state)");
    run(probe<1>, "same, no exception state");
    run(probe<2>, "ring + literal lookup only");
    run(probe<3>, "one dependent LDS read");
    run(probe<4>, "kernel step, random ring slots per lane");
    run(probe<5>, "kernel step, random slots + a global load per 9 steps");
  }
  return 0;
}
