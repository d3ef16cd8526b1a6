// zs_kprof.h -- optional in-kernel phase counters (build with -DZS_KPROF, i.e.
// `make prof` -> libzstreams_mi355x_prof.so).  Product builds compile every
// macro to nothing.  Counters are u64 sums over waves (cycles from s_memtime,
// event counts), read back with zs_kprof_read().
#pragma once
#include <stdint.h>

enum ZsKprof {
  // parse pass (zs_lane_kernel), per wave
  KP_P_WAVES = 0, KP_P_CYC_TOTAL, KP_P_CYC_COOP, KP_P_CYC_STEPS, KP_P_CYC_FLUSH, KP_P_GROUPS, KP_P_COOP,
  KP_P_LANE_STEPS, KP_P_WAVE_STEPS, KP_P_SLOW_LIT, KP_P_SLOW_DIST, KP_P_CYC_MAX, KP_P_CYC_INIT, KP_P_REFILLS,
  KP_P_BUSY, KP_P_CYC_BUSY,  // waves that decoded at least one group, and their cycles
  // expand pass (zs_expand_kernel), per workgroup (wave 0)
  KP_E_BLOCKS = 16, KP_E_CYC_TOTAL, KP_E_ROUNDS, KP_E_JUMP_ITERS, KP_E_CYC_JUMP, KP_E_BATCHES, KP_E_CYC_MAX,
  KP_E_CYC_INIT, KP_E_JUMP_ROUNDS,
  // deflate block kernel (deflate_kernels.hip; its own array, copied into 26..37), per workgroup
  KP_D_BLOCKS = 26, KP_D_CYC_TOTAL, KP_D_CYC_HIST, KP_D_CYC_BUILD, KP_D_CYC_HDR, KP_D_CYC_EMIT, KP_D_CYC_OUT,
  KP_D_CHUNKS,
  // parse step phases (s_memtime, wave-uniform): refill 1, literal/length
  // lookup (+ slow path), length extra + refill 2, distance lookup (+ slow
  // path), checks + token write
  KP_S_REFILL1 = 40, KP_S_LIT, KP_S_REFILL2, KP_S_DIST, KP_S_TAIL,
  // link (chunk_kernels.hip; its own counter array, copied into 48..63)
  KP_L_STREAMS = 48, KP_L_STEPS, KP_L_CYC_SUCC, KP_L_CYC_WALK, KP_L_CYC_WINWRITE, KP_L_CYC_RESOLVE,
  KP_L_CYC_BARRIER, KP_L_MARKERS, KP_L_CYC_TOTAL, KP_L_CYC_MAX,
  KP_COUNT = 64,
  // serial wave decoder (inflate_kernels.hip; its own array, read into 64..79)
  KP_W_WAVES = 64, KP_W_CYC_TOTAL, KP_W_WINDOWS, KP_W_EMPTY, KP_W_SYMS, KP_W_BYTES, KP_W_BATCHES, KP_W_JUMPS,
  KP_W_CYC_DECODE, KP_W_CYC_CHAIN, KP_W_CYC_EXPAND, KP_W_SERIAL, KP_W_CYC_WINDOW,
  // stream window sub-phases: jump-table compositions, chain walks, wave 0
  // before (post + refill) and after (flush + reseat) a window, table builds
  KP_W_CYC_COMPOSE, KP_W_CYC_WALK, KP_W_CYC_PRE, KP_W_CYC_POST, KP_W_CYC_TABLES, KP_W_STEPS, KP_W_REDOS,
  KP_TOTAL = 96
};

#ifdef ZS_KPROF
#define KP_ON 1
#define KP_NOW() ((uint64_t)__builtin_amdgcn_s_memtime())
#else
#define KP_ON 0
#define KP_NOW() ((uint64_t)0)
#endif
