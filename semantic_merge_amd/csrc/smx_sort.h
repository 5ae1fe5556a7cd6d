// smx_sort.h — stable LSD radix sort of (u64 key, u32 value) pairs, 8-bit digits.
//
// Used off the fast path: (1) the generic T-order path when a branch log is not
// timestamp-ordered (sort each branch by (ts, oid)), (2) the move-prefix path
// when some moveDecl carries a None newAddress/newFile (group moves by symbol).
// Per pass: per-block digit histogram -> exclusive scan over [digit][block] ->
// stable scatter (wave64 ballot peer ranks, per-wave counts combined in LDS).
#pragma once

#include "smx_scan.h"

#define RADIX_ITEMS 16
#define RADIX_TILE (BLOCK * RADIX_ITEMS)

static __global__ void __launch_bounds__(BLOCK) k_radix_hist(const u64* __restrict__ keys, i64 n, int shift,
                                                      u32* __restrict__ hist, int nblk) {
  __shared__ u32 h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * RADIX_TILE;
#pragma unroll 4
  for (int it = 0; it < RADIX_ITEMS; ++it) {
    const i64 i = base + it * BLOCK + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(i64)threadIdx.x * nblk + blockIdx.x] = h[threadIdx.x];
}

static __global__ void __launch_bounds__(BLOCK) k_radix_scatter(const u64* __restrict__ kin,
                                                         const u32* __restrict__ vin,
                                                         u64* __restrict__ kout,
                                                         u32* __restrict__ vout, i64 n, int shift,
                                                         const u32* __restrict__ offs, int nblk) {
  __shared__ u32 run[256];
  __shared__ u32 wc[NWAVES][256];
  const int t = threadIdx.x;
  const int w = t / WAVE;
  run[t] = offs[(i64)t * nblk + blockIdx.x];
  const i64 base = (i64)blockIdx.x * RADIX_TILE;
  for (int it = 0; it < RADIX_ITEMS; ++it) {
    const i64 i = base + it * BLOCK + t;
    const bool valid = i < n;
    const u64 k = valid ? kin[i] : 0;
    const u32 v = valid ? vin[i] : 0;
    const u32 d = (u32)(k >> shift) & 255u;
#pragma unroll
    for (int q = 0; q < NWAVES; ++q) wc[q][t] = 0;
    __syncthreads();
    const u64 peers = wave_peers<8>(d, valid);
    const u32 rank = __popcll(peers & lanemask_lt());
    if (valid && rank == 0) wc[w][d] = __popcll(peers);
    __syncthreads();
    {
      u32 acc = run[t];
#pragma unroll
      for (int q = 0; q < NWAVES; ++q) {
        const u32 c = wc[q][t];
        wc[q][t] = acc;
        acc += c;
      }
      run[t] = acc;
    }
    __syncthreads();
    if (valid) {
      const u32 pos = wc[w][d] + rank;
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
  }
}

struct RadixTemp {
  u64* k2;
  u32* v2;
  u32* hist;      // 256 * nblk
  u32* partials;  // SCAN_NB
};

static inline size_t radix_temp_bytes(i64 n) {
  const i64 nblk = SMX_CEIL_DIV(n > 0 ? n : 1, (i64)RADIX_TILE);
  return (size_t)n * 12 + (size_t)256 * nblk * 4 + SCAN_NB * 8 + 256;
}

// Sorts (keys, vals) in place by the digits at `shifts` (LSD order: least
// significant first).  Stable.  Counts stay below 2^32 (n < 2^32).
static hipError_t radix_sort_pairs(u64* keys, u32* vals, i64 n, const int* shifts, int nshift,
                                   RadixTemp tmp, hipStream_t st) {
  if (n <= 1 || nshift == 0) return hipSuccess;
  const int nblk = (int)SMX_CEIL_DIV(n, (i64)RADIX_TILE);
  u64* ka = keys;
  u32* va = vals;
  u64* kb = tmp.k2;
  u32* vb = tmp.v2;
  for (int p = 0; p < nshift; ++p) {
    hipLaunchKernelGGL(k_radix_hist, dim3(nblk), dim3(BLOCK), 0, st, ka, n, shifts[p], tmp.hist,
                       nblk);
    hipError_t e = scan_excl<OpSum, u32, u32>(tmp.hist, tmp.hist, (i64)256 * nblk, nullptr,
                                              tmp.partials, (u32*)nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_radix_scatter, dim3(nblk), dim3(BLOCK), 0, st, ka, va, kb, vb, n,
                       shifts[p], tmp.hist, nblk);
    u64* tk = ka; ka = kb; kb = tk;
    u32* tv = va; va = vb; vb = tv;
  }
  if (ka != keys) {
    (void)hipMemcpyAsync(keys, ka, (size_t)n * 8, hipMemcpyDeviceToDevice, st);
    (void)hipMemcpyAsync(vals, va, (size_t)n * 4, hipMemcpyDeviceToDevice, st);
  }
  return hipGetLastError();
}
