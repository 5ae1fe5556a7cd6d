// smx_tables.h — per-symbol final chain states (compose.py:27-28, 71-82, 99-110).
//
// Every op after the move block sees the symbol's final move state (last
// non-None newAddress / newFile over its moves, in T order) and every
// non-rename sees the last non-skipped rename.  "Last in T order" = max T, so
// each field is a max over packed ((T + 1) << 32 | value).
//
// Scattered 64-bit device atomics run at ~26 G/s on MI355X; instead the
// records are bucketed by symbol range (one counting pass + one scatter pass,
// no global atomics) and each bucket is reduced by one workgroup with LDS
// atomics over a table of at most TB_WIDTH symbols.
#pragma once

#include "smx_scan.h"

#define TB_WIDTH 4096       // symbols per bucket (3 x 32 KB LDS tables)
#define TB_MAXBK 1024       // buckets handled by the bucketed path
#define TB_ITEMS 8
#define TB_TILE (BLOCK * TB_ITEMS)

struct TbArgs {
  const u32* symT;  // moves: T-ordered symbols (T < nMv)
  const i32* mvA;
  const i32* mvF;
  const u32* Msym;  // renames (rename block order)
  const i32* Mstr;
  const u8* skip;
  const ComposeMeta* meta;
  u64 ncap;         // n_a + n_b (bound for device-side counts)
  u32 width;        // symbols per bucket
  u32 nbk;          // buckets
  u32 smax;         // n_sym - 1 (clamp)
  u64 nMv, nR;      // filled on the device by tb_load
};

__device__ __forceinline__ TbArgs tb_load(TbArgs A) {
  const ComposeMeta* m = A.meta;
  const bool fail = m->f_fail | m->bad_sym;
  A.nMv = fail ? 0 : min(m->kcnt[SMX_KIND_MOVE], A.ncap);
  A.nR = fail ? 0 : min(m->kcnt[SMX_KIND_RENAME], A.ncap - A.nMv);
  return A;
}

// record r: r < nMv -> move T = r; else rename m = r - nMv (skipped renames and
// moves with both values None produce no record)
__device__ __forceinline__ bool tb_record(const TbArgs& A, u64 r, u32* sym, i32* v0, i32* v1) {
  if (r < A.nMv) {
    *v0 = A.mvA[r];
    *v1 = A.mvF[r];
    *sym = min(A.symT[r], A.smax);
    return *v0 >= 0 || *v1 >= 0;
  }
  const u64 m = r - A.nMv;
  if (A.skip[m]) return false;
  *sym = min(A.Msym[m], A.smax);
  *v0 = A.Mstr[m];
  *v1 = -1;
  return true;
}

__global__ void __launch_bounds__(BLOCK) k_tb_hist(TbArgs A0, u32* __restrict__ hist, int nblk) {
  const TbArgs A = tb_load(A0);
  __shared__ u32 h[TB_MAXBK];
  for (u32 i = threadIdx.x; i < A.nbk; i += BLOCK) h[i] = 0;
  __syncthreads();
  const u64 nrec = A.nMv + A.nR;
  const u64 base = (u64)blockIdx.x * TB_TILE;
#pragma unroll 4
  for (int it = 0; it < TB_ITEMS; ++it) {
    const u64 r = base + (u64)it * BLOCK + threadIdx.x;
    u32 s;
    i32 a, f;
    if (r < nrec && tb_record(A, r, &s, &a, &f)) atomicAdd(&h[s / A.width], 1u);
  }
  __syncthreads();
  for (u32 i = threadIdx.x; i < A.nbk; i += BLOCK) hist[(u64)i * nblk + blockIdx.x] = h[i];
}

// Scatter into bucket order.  The block's records are first counting-sorted by
// bucket in LDS, then every bucket's run is written contiguously (coalesced),
// instead of one scattered 16-byte store per record.  Order inside a bucket is
// irrelevant (the reduce is a max).
__global__ void __launch_bounds__(BLOCK) k_tb_scatter(TbArgs A0, const u32* __restrict__ offs, int nblk,
                                                      uint4* __restrict__ rec) {
  __shared__ uint4 stage[TB_TILE];      // 64 KB
  __shared__ u32 lstart[TB_MAXBK];      // local bucket starts (then cursors)
  __shared__ u32 gbase[TB_MAXBK];       // global start of this block's run in each bucket
  __shared__ u32 wsum[NWAVES + 1];
  __shared__ u16 sbk[TB_TILE];          // bucket of each staged record
  const TbArgs A = tb_load(A0);
  const u64 nrec = A.nMv + A.nR;
  const u64 base = (u64)blockIdx.x * TB_TILE;
  if (base >= nrec) return;
  const u32 nbk = A.nbk;
  for (u32 i = threadIdx.x; i < nbk; i += BLOCK) {
    lstart[i] = 0;
    gbase[i] = offs[(u64)i * nblk + blockIdx.x];
  }
  __syncthreads();
  // pass 1: local histogram (records kept in registers)
  uint4 q[TB_ITEMS];
  u32 bk[TB_ITEMS];
#pragma unroll
  for (int it = 0; it < TB_ITEMS; ++it) {
    const u64 r = base + (u64)it * BLOCK + threadIdx.x;
    u32 s;
    i32 a, f;
    bk[it] = 0xffffffffu;
    if (r < nrec && tb_record(A, r, &s, &a, &f)) {
      bk[it] = s / A.width;
      q[it] = make_uint4(s, (u32)r, (u32)a, (u32)f);
      atomicAdd(&lstart[bk[it]], 1u);
    }
  }
  __syncthreads();
  // exclusive scan of the local counts (nbk <= TB_MAXBK = 4 per thread)
  {
    u32 v[TB_MAXBK / BLOCK];
    u32 acc = 0;
#pragma unroll
    for (int j = 0; j < TB_MAXBK / BLOCK; ++j) {
      const u32 b = threadIdx.x * (TB_MAXBK / BLOCK) + j;
      v[j] = b < nbk ? lstart[b] : 0u;
      acc += v[j];
    }
    u32 tot;
    u32 run = block_excl_scan<OpSum, u32>(acc, wsum, &tot);
#pragma unroll
    for (int j = 0; j < TB_MAXBK / BLOCK; ++j) {
      const u32 b = threadIdx.x * (TB_MAXBK / BLOCK) + j;
      if (b < nbk) lstart[b] = run;
      run += v[j];
    }
    if (threadIdx.x == 0) wsum[NWAVES] = tot;
  }
  __syncthreads();
  const u32 total = wsum[NWAVES];
  // global position of local slot i of bucket b = gbase[b] + (i - start[b]);
  // precompute gbase[b] - start[b] before the cursors advance
  for (u32 i = threadIdx.x; i < nbk; i += BLOCK) gbase[i] -= lstart[i];
  __syncthreads();
  // pass 2: place records in LDS by bucket
#pragma unroll
  for (int it = 0; it < TB_ITEMS; ++it) {
    if (bk[it] == 0xffffffffu) continue;
    const u32 pos = atomicAdd(&lstart[bk[it]], 1u);
    stage[pos] = q[it];
    sbk[pos] = (u16)bk[it];
  }
  __syncthreads();
  // pass 3: contiguous runs out
  for (u32 i = threadIdx.x; i < total; i += BLOCK) rec[gbase[sbk[i]] + i] = stage[i];
}

#define TBR_NT 1024

// One workgroup per bucket: LDS max-tables, then fin[sym] = (addr, file, ctx, 0).
__global__ void __launch_bounds__(TBR_NT) k_tb_reduce(TbArgs A0, const u32* __restrict__ offs, int nblk,
                                                      const u32* __restrict__ nrec_total,
                                                      const uint4* __restrict__ rec,
                                                      i64 n_sym, int4* __restrict__ fin) {
  const TbArgs A = tb_load(A0);
  __shared__ u64 tA[TB_WIDTH], tF[TB_WIDTH], tC[TB_WIDTH];
  const u32 b = blockIdx.x;
  for (u32 i = threadIdx.x; i < A.width; i += TBR_NT) tA[i] = tF[i] = tC[i] = 0;
  __syncthreads();
  const bool any = A.nMv + A.nR > 0;
  const u32 lo = any ? offs[(u64)b * nblk] : 0u;
  const u32 hi = !any ? 0u : (b + 1 < A.nbk) ? offs[(u64)(b + 1) * nblk] : *nrec_total;
  const u32 s0 = b * A.width;
  for (u32 i = lo + threadIdx.x; i < hi; i += TBR_NT) {
    const uint4 q = rec[i];
    const u32 ls = q.x - s0;
    const u64 key = ((u64)q.y + 1) << 32;
    if ((u64)q.y < A.nMv) {
      if ((i32)q.z >= 0) atomicMax((unsigned long long*)&tA[ls], (unsigned long long)(key | q.z));
      if ((i32)q.w >= 0) atomicMax((unsigned long long*)&tF[ls], (unsigned long long)(key | q.w));
    } else {
      atomicMax((unsigned long long*)&tC[ls], (unsigned long long)(key | q.z));
    }
  }
  __syncthreads();
  for (u32 i = threadIdx.x; i < A.width && (i64)(s0 + i) < n_sym; i += TBR_NT) {
    const u64 a = tA[i], f = tF[i], c = tC[i];
    fin[s0 + i] = make_int4(a ? (i32)(u32)a : -1, f ? (i32)(u32)f : -1, c ? (i32)(u32)c : -1, 0);
  }
}


// Fallback for symbol spaces beyond TB_MAXBK * TB_WIDTH: device-scope atomics.
__global__ void k_tab_atomic(TbArgs A0, u64* __restrict__ tabA, u64* __restrict__ tabF, u64* __restrict__ tabR) {
  const TbArgs A = tb_load(A0);
  const u64 nrec = A.nMv + A.nR;
  for (u64 r = (u64)blockIdx.x * BLOCK + threadIdx.x; r < nrec; r += (u64)gridDim.x * BLOCK) {
    u32 s;
    i32 a, f;
    if (!tb_record(A, r, &s, &a, &f)) continue;
    const u64 key = (r + 1) << 32;
    if (r < A.nMv) {
      if (a >= 0) atomicMax((unsigned long long*)&tabA[s], (unsigned long long)(key | (u32)a));
      if (f >= 0) atomicMax((unsigned long long*)&tabF[s], (unsigned long long)(key | (u32)f));
    } else {
      atomicMax((unsigned long long*)&tabR[s], (unsigned long long)(key | (u32)a));
    }
  }
}

__global__ void k_finalize(const u64* __restrict__ tabA, const u64* __restrict__ tabF,
                           const u64* __restrict__ tabR, i64 n_sym, int4* __restrict__ fin) {
  for (i64 s = (i64)blockIdx.x * BLOCK + threadIdx.x; s < n_sym; s += (i64)gridDim.x * BLOCK) {
    const u64 a = tabA[s], f = tabF[s], r = tabR[s];
    fin[s] = make_int4(a ? (i32)(u32)a : -1, f ? (i32)(u32)f : -1, r ? (i32)(u32)r : -1, 0);
  }
}
