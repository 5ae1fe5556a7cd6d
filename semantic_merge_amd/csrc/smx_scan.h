// smx_scan.h — device-wide exclusive scans (sum / max) with a host- or device-held
// length.  Three launches: per-block reduce, scan of block partials, block scans.
// Each block owns one contiguous chunk; each thread scans 8 consecutive items.
#pragma once

#include "smx_common.h"

#define SCAN_NB 512
#define SCAN_ITEMS 8
#define SCAN_TILE (BLOCK * SCAN_ITEMS)

// n_dev: the length, held on the device, at most n_host (the arrays' capacity)
__device__ __forceinline__ i64 scan_len(const u64* n_dev, i64 n_host) {
  return n_dev ? (i64)min(*n_dev, (u64)n_host) : n_host;
}

template <typename Op, typename TI, typename TO>
__global__ void __launch_bounds__(BLOCK) k_scan_reduce(const TI* __restrict__ in, i64 n_host,
                                                       const u64* n_dev, TO* partials) {
  __shared__ TO s[NWAVES + 1];
  const i64 n = scan_len(n_dev, n_host);
  const i64 chunk = SMX_CEIL_DIV(SMX_CEIL_DIV(n, (i64)SCAN_NB), (i64)SCAN_TILE) * SCAN_TILE;
  const i64 lo = (i64)blockIdx.x * chunk;
  const i64 hi = lo + chunk < n ? lo + chunk : n;
  TO acc = Op::template identity<TO>();
  for (i64 i = lo + threadIdx.x; i < hi; i += BLOCK) acc = Op::apply(acc, (TO)in[i]);
  TO total;
  block_excl_scan<Op, TO>(acc, s, &total);
  if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// Exclusive scan of the SCAN_NB partials in place; optionally stores the grand total.
template <typename Op, typename TO>
__global__ void __launch_bounds__(BLOCK) k_scan_partials(TO* partials, TO* total_out) {
  static_assert(SCAN_NB % BLOCK == 0, "whole partials per thread");
  constexpr int PER = SCAN_NB / BLOCK;
  __shared__ TO s[NWAVES + 1];
  TO v[PER];
  TO acc = Op::template identity<TO>();
#pragma unroll
  for (int j = 0; j < PER; ++j) {  // consecutive partials per thread
    v[j] = partials[threadIdx.x * PER + j];
    acc = Op::apply(acc, v[j]);
  }
  TO total;
  TO run = block_excl_scan<Op, TO>(acc, s, &total);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    partials[threadIdx.x * PER + j] = run;
    run = Op::apply(run, v[j]);
  }
  if (total_out && threadIdx.x == 0) *total_out = total;
}

template <typename Op, typename TI, typename TO>
__global__ void __launch_bounds__(BLOCK) k_scan_down(const TI* __restrict__ in, TO* __restrict__ out,
                                                     i64 n_host, const u64* n_dev,
                                                     const TO* partials) {
  __shared__ TO s[NWAVES + 1];
  const i64 n = scan_len(n_dev, n_host);
  const i64 chunk = SMX_CEIL_DIV(SMX_CEIL_DIV(n, (i64)SCAN_NB), (i64)SCAN_TILE) * SCAN_TILE;
  const i64 lo = (i64)blockIdx.x * chunk;
  const i64 hi = lo + chunk < n ? lo + chunk : n;
  TO carry = partials[blockIdx.x];
  for (i64 t0 = lo; t0 < hi; t0 += SCAN_TILE) {
    const i64 b = t0 + (i64)threadIdx.x * SCAN_ITEMS;
    TO v[SCAN_ITEMS];
    TO acc = Op::template identity<TO>();
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
      v[j] = (b + j < hi) ? (TO)in[b + j] : Op::template identity<TO>();
      acc = Op::apply(acc, v[j]);
    }
    TO total;
    TO pre = block_excl_scan<Op, TO>(acc, s, &total);
    TO run = Op::apply(carry, pre);
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
      if (b + j < hi) out[b + j] = run;
      run = Op::apply(run, v[j]);
    }
    carry = Op::apply(carry, total);
  }
}

// out[i] = op-exclusive-prefix of in[0..i); *total_out (optional) = op over all.
template <typename Op, typename TI, typename TO>
static hipError_t scan_excl(const TI* in, TO* out, i64 n_host, const u64* n_dev, TO* partials,
                            TO* total_out, hipStream_t st) {
  hipLaunchKernelGGL((k_scan_reduce<Op, TI, TO>), dim3(SCAN_NB), dim3(BLOCK), 0, st, in, n_host,
                     n_dev, partials);
  hipLaunchKernelGGL((k_scan_partials<Op, TO>), dim3(1), dim3(BLOCK), 0, st, partials, total_out);
  hipLaunchKernelGGL((k_scan_down<Op, TI, TO>), dim3(SCAN_NB), dim3(BLOCK), 0, st, in, out, n_host,
                     n_dev, partials);
  return hipGetLastError();
}

// Column scan of a row-major [block][bucket] count matrix (written and read
// coalesced by the per-block kernels of the table bucketing and the radix sort):
// each entry becomes the global start of that block's run in that bucket, i.e. an
// exclusive scan in bucket-major order: bstart[bucket] + the counts of the earlier
// blocks in the same bucket.  In tiles of HS_ROWS blocks: tile sums, a per-column
// scan of the tile sums (+ bucket starts, nbk + 1 entries), then the tiles.
#define HS_ROWS 64
#define HS_COLS 256
#define HS_MAXCOLS 1024

static __global__ void __launch_bounds__(HS_COLS) k_hscan_up(const u32* __restrict__ hist, int nblk, u32 nbk,
                                                      u32* __restrict__ tsum) {
  const u32 col = blockIdx.y * HS_COLS + threadIdx.x;
  if (col >= nbk) return;
  const int r0 = blockIdx.x * HS_ROWS, r1 = min(r0 + HS_ROWS, nblk);
  u32 s = 0;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += hist[(u64)r * nbk + col];
  tsum[(u64)blockIdx.x * nbk + col] = s;
}

static __global__ void __launch_bounds__(HS_MAXCOLS) k_hscan_mid(u32* __restrict__ tsum, int ntile, u32 nbk,
                                                        u32* __restrict__ bstart) {
  __shared__ u32 s[HS_MAXCOLS / WAVE + 1];
  const u32 col = threadIdx.x;
  u32 run = 0;
  if (col < nbk) {
#pragma unroll 8
    for (int t = 0; t < ntile; ++t) {
      const u32 v = tsum[(u64)t * nbk + col];
      tsum[(u64)t * nbk + col] = run;
      run += v;
    }
  }
  u32 tot;
  const u32 ex = block_excl_scan<OpSum, u32, HS_MAXCOLS / WAVE>(col < nbk ? run : 0u, s, &tot);
  if (col < nbk) bstart[col] = ex;
  if (col == 0) bstart[nbk] = tot;
}

static __global__ void __launch_bounds__(HS_COLS) k_hscan_down(u32* __restrict__ hist, int nblk, u32 nbk,
                                                        const u32* __restrict__ tsum,
                                                        const u32* __restrict__ bstart) {
  const u32 col = blockIdx.y * HS_COLS + threadIdx.x;
  if (col >= nbk) return;
  const int r0 = blockIdx.x * HS_ROWS, r1 = min(r0 + HS_ROWS, nblk);
  u32 run = bstart[col] + tsum[(u64)blockIdx.x * nbk + col];
  for (int r = r0; r < r1; ++r) {
    const u32 v = hist[(u64)r * nbk + col];
    hist[(u64)r * nbk + col] = run;
    run += v;
  }
}

static inline size_t hscan_tsum_bytes(i64 nrows, i64 ncols) {
  return (size_t)ncols * (SMX_CEIL_DIV(nrows, (i64)HS_ROWS) + 1) * 4;
}

// hist [nrows][ncols] -> bucket-major exclusive offsets in place; bstart[ncols + 1].
static inline void hscan(u32* hist, int nrows, u32 ncols, u32* tsum, u32* bstart, hipStream_t st) {
  const int ntile = (int)SMX_CEIL_DIV((i64)nrows, (i64)HS_ROWS);
  const dim3 g(ntile, (unsigned)SMX_CEIL_DIV((u64)ncols, (u64)HS_COLS));
  hipLaunchKernelGGL(k_hscan_up, g, dim3(HS_COLS), 0, st, hist, nrows, ncols, tsum);
  hipLaunchKernelGGL(k_hscan_mid, dim3(1), dim3(HS_MAXCOLS), 0, st, tsum, ntile, ncols, bstart);
  hipLaunchKernelGGL(k_hscan_down, g, dim3(HS_COLS), 0, st, hist, nrows, ncols, tsum, bstart);
}

