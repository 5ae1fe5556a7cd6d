// smx_sort.h — stable LSD radix sort of (u64 key, u32 value) pairs, 8-bit digits.
//
// Used off the fast path: (1) the generic T-order path when a branch log is not
// timestamp-ordered (sort each branch by (ts, oid)), (2) the move-prefix path
// when some moveDecl carries a None newAddress/newFile (group moves by symbol).
// Per pass: per-block digit histogram [block][digit] -> column scan (smx_scan.h) ->
// stable tile-local scatter through LDS, digit runs written contiguously.
#pragma once

#include "smx_scan.h"

#ifndef RADIX_ITEMS
#define RADIX_ITEMS 16
#endif
#ifndef RADIX_HIST_AGG
#define RADIX_HIST_AGG 0
#endif
#define RADIX_TILE (BLOCK * RADIX_ITEMS)   // 4096 pairs per block and pass (16-pair digit runs)
#define RADIX_SEG (RADIX_TILE / NWAVES)     // contiguous elements per wave

// Digit histogram of each block's tile, row-major hist[block][256].
static __global__ void __launch_bounds__(BLOCK) k_radix_hist(const u64* __restrict__ keys, i64 n, int shift,
                                                             u32* __restrict__ hist, int nblk) {
  __shared__ u32 h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * RADIX_TILE;
  u32 d[RADIX_ITEMS];
#pragma unroll
  for (int it = 0; it < RADIX_ITEMS; ++it) {
    const i64 i = base + it * BLOCK + threadIdx.x;
    d[it] = i < n ? (u32)(keys[i] >> shift) & 255u : 256u;
  }
#if RADIX_HIST_AGG
  // one LDS atomic per distinct digit per wave (slow-varying digits, e.g. timestamp
  // bytes, would otherwise serialise on one bin)
  const u64 lt = lanemask_lt();
#pragma unroll
  for (int it = 0; it < RADIX_ITEMS; ++it) {
    const u64 peers = wave_peers<8>(d[it] & 255u, d[it] < 256u);
    if (d[it] < 256u && (peers & lt) == 0) atomicAdd(&h[d[it]], (u32)__popcll(peers));
  }
#else
#pragma unroll
  for (int it = 0; it < RADIX_ITEMS; ++it)
    if (d[it] < 256u) atomicAdd(&h[d[it]], 1u);
#endif
  __syncthreads();
  hist[(i64)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

// Stable scatter of one tile: wave w ranks its contiguous segment of RADIX_SEG
// pairs round by round (ballot peers + a per-wave digit cursor, no block
// barriers), the block combines the per-wave digit counts, stages the tile in LDS
// in digit order, and writes each digit's run contiguously (coalesced) at the
// block's global offset for that digit.
static __global__ void __launch_bounds__(BLOCK) k_radix_scatter(const u64* __restrict__ kin,
                                                                const u32* __restrict__ vin,
                                                                u64* __restrict__ kout,
                                                                u32* __restrict__ vout, i64 n, int shift,
                                                                const u32* __restrict__ offs, int nblk) {
  __shared__ u64 sk[RADIX_TILE];          // 32 KB at 4096 pairs
  __shared__ u32 sv[RADIX_TILE];          // 16 KB
  __shared__ u32 wc[NWAVES][256];         // per-wave digit counts, then offsets
  __shared__ u32 lstart[256];             // local digit starts
  __shared__ u32 gofs[256];               // global start of this block's digit runs
  const int t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  const i64 base = (i64)blockIdx.x * RADIX_TILE;
#pragma unroll
  for (int q = 0; q < NWAVES; ++q) wc[q][t] = 0;
  gofs[t] = offs[(i64)blockIdx.x * 256 + t];
  __syncthreads();
  const u64 lt = lanemask_lt();
  u64 k[RADIX_ITEMS];
  u32 v[RADIX_ITEMS], dr[RADIX_ITEMS];  // digit | rank-in-wave-segment << 8
#pragma unroll
  for (int it = 0; it < RADIX_ITEMS; ++it) {
    const i64 i = base + (i64)w * RADIX_SEG + it * WAVE + lane;
    const bool valid = i < n;
    k[it] = valid ? kin[i] : ~0ull;
    v[it] = valid ? vin[i] : 0u;
  }
#pragma unroll
  for (int it = 0; it < RADIX_ITEMS; ++it) {
    const i64 i = base + (i64)w * RADIX_SEG + it * WAVE + lane;
    const bool valid = i < n;
    const u32 d = (u32)(k[it] >> shift) & 255u;
    const u64 peers = wave_peers<8>(d, valid);
    const u32 before = wc[w][d];  // the wave's cursor for d (wave-private row)
    const u32 r = __popcll(peers & lt);
    dr[it] = d | ((before + r) << 8);
    // the last peer advances the cursor (same wave: visible to the next round)
    if (valid && (peers >> lane) == 1ull) wc[w][d] = before + __popcll(peers);
  }
  __syncthreads();
  {  // per digit: local start + the earlier waves' counts
    u32 tot = 0;
#pragma unroll
    for (int q = 0; q < NWAVES; ++q) tot += wc[q][t];
    lstart[t] = tot;
  }
  __syncthreads();
  if (t < WAVE) {  // exclusive scan of the 256 digit totals (4 per lane)
    u32 x[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = lstart[4 * t + j];
      s += x[j];
    }
    const u32 inc = wave_incl_sum(s);
    u32 run = inc - s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lstart[4 * t + j] = run;
      run += x[j];
    }
  }
  __syncthreads();
  {
    u32 acc = lstart[t];
#pragma unroll
    for (int q = 0; q < NWAVES; ++q) {
      const u32 c = wc[q][t];
      wc[q][t] = acc;
      acc += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < RADIX_ITEMS; ++it) {
    const i64 i = base + (i64)w * RADIX_SEG + it * WAVE + lane;
    if (i < n) {
      const u32 d = dr[it] & 255u, p = wc[w][d] + (dr[it] >> 8);
      sk[p] = k[it];
      sv[p] = v[it];
    }
  }
  __syncthreads();
  const int cnt = (int)(n - base < RADIX_TILE ? n - base : RADIX_TILE);
  for (int p = t; p < cnt; p += BLOCK) {
    const u64 kk = sk[p];
    const u32 d = (u32)(kk >> shift) & 255u;
    const u32 g = gofs[d] + (u32)p - lstart[d];
    kout[g] = kk;
    vout[g] = sv[p];
  }
}

struct RadixTemp {
  u64* k2;
  u32* v2;
  u32* hist;      // radix_hist_bytes(n)
  u32* partials;  // unused (kept for the layout)
};

// hist [nblk][256] + column-scan tile sums + 257 digit starts
static inline size_t radix_hist_bytes(i64 n) {
  const i64 nblk = SMX_CEIL_DIV(n > 0 ? n : 1, (i64)RADIX_TILE);
  return (size_t)256 * nblk * 4 + hscan_tsum_bytes(nblk, 256) + 260 * 4;
}

// Sorts (keys, vals) in place by the digits at `shifts` (LSD order: least
// significant first).  Stable.  Counts stay below 2^32 (n < 2^32).
static hipError_t radix_sort_pairs(u64* keys, u32* vals, i64 n, const int* shifts, int nshift,
                                   RadixTemp tmp, hipStream_t st) {
  if (n <= 1 || nshift == 0) return hipSuccess;
  const int nblk = (int)SMX_CEIL_DIV(n, (i64)RADIX_TILE);
  u32* tsum = tmp.hist + (size_t)256 * nblk;
  u32* dstart = tsum + hscan_tsum_bytes(nblk, 256) / 4;
  u64* ka = keys;
  u32* va = vals;
  u64* kb = tmp.k2;
  u32* vb = tmp.v2;
  for (int p = 0; p < nshift; ++p) {
    hipLaunchKernelGGL(k_radix_hist, dim3(nblk), dim3(BLOCK), 0, st, ka, n, shifts[p], tmp.hist, nblk);
    hscan(tmp.hist, nblk, 256u, tsum, dstart, st);
    hipLaunchKernelGGL(k_radix_scatter, dim3(nblk), dim3(BLOCK), 0, st, ka, va, kb, vb, n, shifts[p], tmp.hist,
                       nblk);
    u64* tk = ka; ka = kb; kb = tk;
    u32* tv = va; va = vb; vb = tv;
  }
  if (ka != keys) {
    (void)hipMemcpyAsync(keys, ka, (size_t)n * 8, hipMemcpyDeviceToDevice, st);
    (void)hipMemcpyAsync(vals, va, (size_t)n * 4, hipMemcpyDeviceToDevice, st);
  }
  return hipGetLastError();
}
