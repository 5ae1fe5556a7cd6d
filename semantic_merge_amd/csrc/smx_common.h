// smx_common.h — shared device helpers for libsmx (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smx.h"

typedef uint64_t u64;
typedef uint32_t u32;
typedef int64_t i64;
typedef int32_t i32;
typedef uint16_t u16;
typedef uint8_t u8;

#define WAVE 64
#define BLOCK 256
#define NWAVES (BLOCK / WAVE)

// Device-side state of one smx_compose call (lives at the start of the workspace).
// Counters written by kernels; read by later kernels and (once) by the host.
struct ComposeMeta {
  u64 kcnt[SMX_N_KINDS];     // ops per precedence rank (stats kernel)
  u64 base[SMX_N_KINDS + 1]; // exclusive prefix of kcnt: T-order segment starts
  u64 nonmono[2];            // per side: 1 if timestamps decrease somewhere
  u64 n_move_none;           // moves with a None newAddress or newFile
  u64 f_fail;                // presorted windows exceed LDS capacity
  u64 bad_sym;               // sym >= n_sym seen
  u64 n_ren_side[2];         // renames per side
  u64 key_or[2][3];          // per side OR / AND of (ts, hi, lo): constant radix digits
  u64 key_and[2][3];
  u64 n_cand;                // DivergentRename candidate starts
  u64 n_conf;                // conflicts (real)
  u64 pad[8];
};

__device__ __forceinline__ u64 lanemask_lt() {
  const int lane = threadIdx.x & (WAVE - 1);
  return (lane == 0) ? 0ull : (~0ull >> (WAVE - lane));
}

// Lanes of this wave holding the same `nbits`-bit value `d` (among lanes with `valid`).
template <int NBITS>
__device__ __forceinline__ u64 wave_peers(u32 d, bool valid) {
  u64 m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < NBITS; ++b) {
    const bool bit = (d >> b) & 1u;
    const u64 x = __ballot(bit);
    m &= bit ? x : ~x;
  }
  return m;
}

// Inclusive wave prefix sum (64 lanes).
template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    T y = __shfl_up(v, o, WAVE);
    if (lane >= o) v += y;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
  const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    T y = __shfl_up(v, o, WAVE);
    if (lane >= o) v = v > y ? v : y;
  }
  return v;
}

struct OpSum {
  template <typename T>
  __device__ __forceinline__ static T apply(T a, T b) { return a + b; }
  template <typename T>
  __device__ __forceinline__ static T identity() { return T(0); }
  template <typename T>
  __device__ __forceinline__ static T wave_incl(T v) { return wave_incl_sum(v); }
};

struct OpMax {
  template <typename T>
  __device__ __forceinline__ static T apply(T a, T b) { return a > b ? a : b; }
  template <typename T>
  __device__ __forceinline__ static T identity() { return T(0); }
  template <typename T>
  __device__ __forceinline__ static T wave_incl(T v) { return wave_incl_max(v); }
};

// Block-wide exclusive scan of one value per thread; returns the exclusive prefix,
// writes the block aggregate to *total.  `s` must hold NWAVES+1 entries.
template <typename Op, typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* s, T* total) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x / WAVE;
  T inc = Op::template wave_incl<T>(v);
  if (lane == WAVE - 1) s[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T acc = Op::template identity<T>();
    for (int i = 0; i < NWAVES; ++i) {
      T x = s[i];
      s[i] = acc;
      acc = Op::apply(acc, x);
    }
    s[NWAVES] = acc;
  }
  __syncthreads();
  T wpre = s[w];
  T excl_in_wave = __shfl_up(inc, 1, WAVE);
  if (lane == 0) excl_in_wave = Op::template identity<T>();
  T r = Op::apply(wpre, excl_in_wave);
  *total = s[NWAVES];
  __syncthreads();
  return r;
}

#define SMX_CEIL_DIV(a, b) (((a) + (b)-1) / (b))

// Records the thread-local error message returned by smx_last_error(); returns code.
int smx_set_error(int code, const char* msg);
