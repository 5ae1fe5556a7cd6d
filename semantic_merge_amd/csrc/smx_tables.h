// smx_tables.h — per-symbol final chain states (compose.py:27-28, 71-82, 99-110).
//
// Every op after the move block sees the symbol's final move state (last
// non-None newAddress / newFile over its moves, in T order) and every
// non-rename sees the last non-skipped rename.  "Last in T order" = max T.
//
// Records: r in [0, nMv) is the move at T = r (msym[r] = symbol | has-address |
// has-file, written by the window kernel), r = nMv + m the rename at M position m
// (tsym[m]; skipped renames, skipbits, carry nothing).  Scattered device atomics
// execute at the memory side; instead the records are bucketed by symbol range
// and each bucket is reduced by one workgroup with 32-bit LDS max over record
// indices; the values are fetched once per symbol at the end (the move's own
// out_addr / out_file, the rename's Rstr).  Bucketing needs no counting pass:
// k_tb_scatter sorts each tile of TB_TILE records by bucket in LDS and writes the
// tile back in place (fully coalesced) with its bucket starts lst[tile][0..nbk];
// k_tb_reduce of bucket b then reads that bucket's run of every tile.  A record
// is 4 bytes, relative to its tile:
//   bits  0..13  index inside the tile          bits 14..25 symbol offset in its bucket
//   bit  26      the move has a newAddress      bit  27     the move has a newFile
// (one bit more for the index, and the fields above it shifted, with 32768-record tiles)
#pragma once

#include "smx_scan.h"

#define TB_WIDTH 4096       // symbols per bucket
#define TB_MAXBK 1024       // buckets handled by the bucketed path
#ifndef TB_NT
#define TB_NT 1024          // scatter workgroup: one 16384-record tile (64 KB LDS)
#endif
#define TB_NW (TB_NT / WAVE)
#ifndef TB_ITEMS
#define TB_ITEMS 16         // 64-record runs per bucket and tile
#endif
#ifndef TB_NBK_TGT
#define TB_NBK_TGT 256      // target bucket count (width = n_sym / this, <= TB_WIDTH)
#endif
#define TB_TILE (TB_NT * TB_ITEMS)
// record bits: the index inside the tile (REC_IB bits), the symbol offset in its bucket
// (12 bits, TB_WIDTH), the two move flags
#define REC_IB (TB_TILE <= (1 << 14) ? 14 : 15)
static_assert(TB_TILE <= (1 << 15), "tile-relative record index is at most 15 bits");
#define REC_IMASK ((1u << REC_IB) - 1u)
#define REC_HAS_A (1u << (REC_IB + 12))
#define REC_HAS_F (1u << (REC_IB + 13))

struct TbArgs {
  const u32* msym;    // moves: T-ordered symbol | has-address << 30 | has-file << 31
  const u32* tsym;    // renames: symbol at M position
  const u64* skipbits;
  const i32* mv_addr;  // the moves' own newAddress / newFile (= out_addr / out_file, T < nMv)
  const i32* mv_file;
  const i32* Rstr;
  const ComposeMeta* meta;
  u64 ncap;         // n_a + n_b (bound for device-side counts)
  u32 width;        // symbols per bucket
  u32 nbk;          // buckets
  u32 smax;         // n_sym - 1 (clamp)
  u32 keep_skip;    // k_tb_scatter keeps every rename (it runs beside the walk; the
                    // skipped renames' records are killed afterwards by k_tb_unskip --
                    // or, when 2, passed over by k_tb_reduce through the skip bits)
  u64 nMv, nR;      // filled on the device by tb_load
};

__device__ __forceinline__ TbArgs tb_load(TbArgs A) {
  const ComposeMeta* m = A.meta;
  const bool fail = m->f_fail | m->bad_sym;
  A.nMv = fail ? 0 : min(m->kcnt[SMX_KIND_MOVE], A.ncap);
  A.nR = fail ? 0 : min(m->kcnt[SMX_KIND_RENAME], A.ncap - A.nMv);
  return A;
}

__device__ __forceinline__ bool tb_skipped(const TbArgs& A, u64 m) {
  return (A.skipbits[m >> 6] >> (m & 63)) & 1ull;
}

// Record r: symbol and flags; false when it carries nothing (skipped rename, move
// with both values None).
__device__ __forceinline__ bool tb_record(const TbArgs& A, u64 r, u32* sym, u32* flags) {
  if (r < A.nMv) {
    const u32 x = A.msym[r];
    *sym = min(x & SYM_MASK, A.smax);
    *flags = (x & MS_HAS_A ? REC_HAS_A : 0u) | (x & MS_HAS_F ? REC_HAS_F : 0u);
    return (x & (MS_HAS_A | MS_HAS_F)) != 0;
  }
  const u64 m = r - A.nMv;
  if (!A.keep_skip && tb_skipped(A, m)) return false;
  *sym = min(A.tsym[m], A.smax);
  *flags = 0;
  return true;
}

// The TB_ITEMS records of a lane (r = base + it * TB_NT + lane), loads issued
// together: a tile is all moves, all renames, or (one tile) mixed.
__device__ __forceinline__ void tb_items(const TbArgs& A, u64 base, u32 (&sym)[TB_ITEMS], u32 (&fl)[TB_ITEMS],
                                         bool (&ok)[TB_ITEMS]) {
  const u64 nrec = A.nMv + A.nR;
  const u64 end = base + (u64)TB_TILE;
  if (end <= A.nMv) {
    u32 x[TB_ITEMS];
#pragma unroll
    for (int it = 0; it < TB_ITEMS; ++it) x[it] = A.msym[base + (u64)it * TB_NT + threadIdx.x];
#pragma unroll
    for (int it = 0; it < TB_ITEMS; ++it) {
      ok[it] = (x[it] & (MS_HAS_A | MS_HAS_F)) != 0;
      fl[it] = (x[it] & MS_HAS_A ? REC_HAS_A : 0u) | (x[it] & MS_HAS_F ? REC_HAS_F : 0u);
      sym[it] = min(x[it] & SYM_MASK, A.smax);
    }
  } else if (base >= A.nMv && end <= nrec) {
    u32 s[TB_ITEMS];
    const u64 m0 = base - A.nMv;
#pragma unroll
    for (int it = 0; it < TB_ITEMS; ++it) s[it] = A.tsym[m0 + (u64)it * TB_NT + threadIdx.x];
#pragma unroll
    for (int it = 0; it < TB_ITEMS; ++it) {
      ok[it] = A.keep_skip || !tb_skipped(A, m0 + (u64)it * TB_NT + threadIdx.x);
      fl[it] = 0;
      sym[it] = min(s[it], A.smax);
    }
  } else {
#pragma unroll
    for (int it = 0; it < TB_ITEMS; ++it) {
      const u64 r = base + (u64)it * TB_NT + threadIdx.x;
      ok[it] = r < nrec && tb_record(A, r, &sym[it], &fl[it]);
    }
  }
}

// Tile-local bucket sort: the tile's records are counting-sorted by bucket in
// LDS and written back to the tile's own range; lst[tile][b] = start of bucket b
// in the tile, lst[tile][nbk] = the tile's record count.  (The value widths of the
// packed final-state table, smx_common.h FinPack, come from the window kernels.)
__global__ void __launch_bounds__(TB_NT) k_tb_scatter(TbArgs A0, u32* __restrict__ lst, u32* __restrict__ rec) {
  __shared__ u32 stage[TB_TILE];        // TB_TILE * 4 bytes
  __shared__ u32 lstart[TB_MAXBK];      // local bucket starts (then cursors)
  __shared__ u32 wsum[TB_NW + 1];
  const TbArgs A = tb_load(A0);
  const u64 nrec = A.nMv + A.nR;
  const u64 base = (u64)blockIdx.x * TB_TILE;
  if (base >= nrec) return;
  const u32 nbk = A.nbk;
  for (u32 i = threadIdx.x; i < nbk; i += TB_NT) lstart[i] = 0;
  __syncthreads();
  u32 q[TB_ITEMS];
  u32 bk[TB_ITEMS];
  {
    u32 s[TB_ITEMS], fl[TB_ITEMS];
    bool ok[TB_ITEMS];
    tb_items(A, base, s, fl, ok);
#pragma unroll
    for (int it = 0; it < TB_ITEMS; ++it) {
      const u32 loc = (u32)(it * TB_NT) + threadIdx.x;
      bk[it] = 0xffffffffu;
      if (ok[it]) {
        const u32 b = s[it] / A.width;
        bk[it] = b;
        q[it] = loc | ((s[it] - b * A.width) << REC_IB) | fl[it];
        atomicAdd(&lstart[b], 1u);
      }
    }
  }
  __syncthreads();
  u32* lt = lst + (u64)blockIdx.x * (nbk + 1);
  {
    u32 v[TB_MAXBK / TB_NT];
    u32 acc = 0;
#pragma unroll
    for (int j = 0; j < TB_MAXBK / TB_NT; ++j) {
      const u32 b = threadIdx.x * (TB_MAXBK / TB_NT) + j;
      v[j] = b < nbk ? lstart[b] : 0u;
      acc += v[j];
    }
    u32 tot;
    u32 run = block_excl_scan<OpSum, u32, TB_NW>(acc, wsum, &tot);
#pragma unroll
    for (int j = 0; j < TB_MAXBK / TB_NT; ++j) {
      const u32 b = threadIdx.x * (TB_MAXBK / TB_NT) + j;
      if (b < nbk) {
        lstart[b] = run;
        lt[b] = run;
      }
      run += v[j];
    }
    if (threadIdx.x == 0) {
      wsum[TB_NW] = tot;
      lt[nbk] = tot;
    }
  }
  __syncthreads();
  const u32 total = wsum[TB_NW];
#pragma unroll
  for (int it = 0; it < TB_ITEMS; ++it) {
    if (bk[it] == 0xffffffffu) continue;
    const u32 pos = atomicAdd(&lstart[bk[it]], 1u);
    stage[pos] = q[it];
  }
  __syncthreads();
  for (u32 i = threadIdx.x; i < total; i += TB_NT) rec[base + i] = stage[i];
}

#define REC_DEAD 0xffffffffu
// After a keep_skip scatter (which ran beside the walk): the record of every rename
// the walk skipped is found in its tile's bucket run (64 records on average) and
// marked dead, so that k_tb_reduce never sees it.  One wave per skip, its lanes
// test 64 records of the run per step.
__global__ void k_tb_unskip(TbArgs A0, const u32* __restrict__ lst, u32* __restrict__ rec,
                            const u32* __restrict__ skiplist) {
  const TbArgs A = tb_load(A0);
  const u64 nskip = min(A.meta->n_skip, A.nR);
  const u32 nb1 = A.nbk + 1;
  const u32 lane = threadIdx.x & (WAVE - 1);
  const u64 nwv = (u64)gridDim.x * (blockDim.x / WAVE);
  for (u64 i = (u64)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE; i < nskip; i += nwv) {
    const u64 m = skiplist[i];
    if (m >= A.nR) continue;
    const u64 r = A.nMv + m;
    const u64 tile = r / TB_TILE;
    const u32 loc = (u32)(r - tile * TB_TILE);
    const u32 sym = min(A.tsym[m], A.smax);
    const u32 b = sym / A.width;
    const u32* lt = lst + tile * nb1;
    const u64 rb = tile * TB_TILE;
    const u32 e = lt[b + 1];
    for (u32 j = lt[b] + lane; j < e; j += WAVE) {
      const u32 q = rec[rb + j];
      if (q != REC_DEAD && (q & REC_IMASK) == loc) rec[rb + j] = REC_DEAD;
    }
  }
}

#define TBR_NT 1024
#ifndef SMX_XCD_TB
#define SMX_XCD_TB 1
#endif
#ifndef TBR_TK
#define TBR_TK 16
#endif
// TBR_TK: tiles per wave step in k_tb_reduce
#ifndef TBR_U
#define TBR_U 2         // records per lane and tile in a k_tb_reduce step (longer runs: the tail loop)
#endif
#ifndef TBR_PREFETCH
#define TBR_PREFETCH 1  // k_tb_reduce loads the next step's run bounds before this step's records are used
#endif

// One workgroup per bucket: LDS max over record indices, then each symbol's
// values are fetched once: fin[sym] = (addr, file, ctx).
// part != nullptr (sharded merge): instead of fin, write this shard's partial
// tables part[3][n_sym] = (tag << 32) | (value + 1), 0 = no record; the MAX
// all-reduce over shards then keeps the last writer (highest shard).  tagbits > 0:
// 32-bit entries tag << (31 - tagbits) | (value + 1) instead (smx_shard.tab32).
struct PartTab {
  void* p;
  u32 tag;
  int tagbits;  // 0: u64 entries
  ComposeMeta* meta;
  __device__ __forceinline__ void put(i64 n_sym, i64 s, int va, int vf, int vc) const {
    if (tagbits == 0) {
      u64* part = (u64*)p;
      const u64 tg = (u64)tag << 32;
      part[s] = va >= 0 ? tg | (u32)(va + 1) : 0ull;
      part[n_sym + s] = vf >= 0 ? tg | (u32)(vf + 1) : 0ull;
      part[2 * n_sym + s] = vc >= 0 ? tg | (u32)(vc + 1) : 0ull;
      return;
    }
    u32* part = (u32*)p;
    const u32 vb = 31u - (u32)tagbits, tg = tag << vb, lim = 1u << vb;
    const u32 a1 = (u32)(va + 1), f1 = (u32)(vf + 1), c1 = (u32)(vc + 1);
    if ((a1 | f1 | c1) >= lim) meta->tab_over = 1;  // the caller redoes the step with u64 entries
    part[s] = va >= 0 ? tg | (a1 & (lim - 1)) : 0u;
    part[n_sym + s] = vf >= 0 ? tg | (f1 & (lim - 1)) : 0u;
    part[2 * n_sym + s] = vc >= 0 ? tg | (c1 & (lim - 1)) : 0u;
  }
};

__global__ void __launch_bounds__(TBR_NT) k_tb_reduce(TbArgs A0, const u32* __restrict__ lst,
                                                      const u32* __restrict__ rec, i64 n_sym,
                                                      int4* __restrict__ fin, PartTab part) {
  const FinPack FP = fin_pack_of(A0.meta->vbits, true);
  __shared__ u32 tA[TB_WIDTH], tF[TB_WIDTH], tC[TB_WIDTH];
  const TbArgs A = tb_load(A0);
  // neighbouring buckets on one XCD: a tile's runs of buckets b and b + 1 share their
  // boundary lines, which are then fetched into one L2 only
  const u32 b = SMX_XCD_TB ? (u32)xcd_item(blockIdx.x, gridDim.x) : blockIdx.x;
  for (u32 i = threadIdx.x; i < A.width; i += TBR_NT) tA[i] = tF[i] = tC[i] = 0;
  __syncthreads();
  auto put = [&](u32 q, u64 rb) {
    const u32 r1 = (u32)(rb + (q & REC_IMASK)) + 1u;
    const u32 ls = (q >> REC_IB) & 0xfffu;
    if ((u64)(r1 - 1) < A.nMv) {
      if (q & REC_HAS_A) atomicMax(&tA[ls], r1);
      if (q & REC_HAS_F) atomicMax(&tF[ls], r1);
    } else if (A.keep_skip != 2u || !tb_skipped(A, (u64)(r1 - 1) - A.nMv)) {
      atomicMax(&tC[ls], r1);
    }
  };
  // bucket b's run in every tile: each wave takes TBR_TK tiles per step, up to
  // 2 * WAVE records of each in flight together, longer runs finish in a tail loop
  const u64 nrec = A.nMv + A.nR;
  const int nt = nrec ? (int)SMX_CEIL_DIV(nrec, (u64)TB_TILE) : 0;
  const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
  const u32 nb1 = A.nbk + 1;
  constexpr int NW = TBR_NT / WAVE;
  // the run bounds of a step's tiles (lanes < TBR_TK), loaded one step ahead so that a
  // step's record loads do not wait for its bounds
  auto bounds = [&](int t0, u32* lo, u32* hi) {
    *lo = *hi = 0;
    if (lane < TBR_TK && t0 + lane < nt) {
      const u32* lt = lst + (u64)(t0 + lane) * nb1;
      *lo = lt[b];
      *hi = lt[b + 1];
    }
  };
  u32 lo_n = 0, hi_n = 0;
  if (TBR_PREFETCH) bounds(wv * TBR_TK, &lo_n, &hi_n);
  for (int t0 = wv * TBR_TK; t0 < nt; t0 += NW * TBR_TK) {
    u32 lo = lo_n, hi = hi_n;
    if (!TBR_PREFETCH) bounds(t0, &lo, &hi);
    u32 q[TBR_TK][TBR_U];
#pragma unroll
    for (int k = 0; k < TBR_TK; ++k) {
      const u32 lk = __builtin_amdgcn_readlane(lo, k), hk = __builtin_amdgcn_readlane(hi, k);
      const u64 rb = (u64)(t0 + k) * TB_TILE;
#pragma unroll
      for (int u = 0; u < TBR_U; ++u) {
        const u32 i = lk + (u32)lane + (u32)(u * WAVE);
        q[k][u] = i < hk ? __builtin_nontemporal_load(&rec[rb + i]) : ~0u;
      }
    }
    if (TBR_PREFETCH) bounds(t0 + NW * TBR_TK, &lo_n, &hi_n);
#pragma unroll
    for (int k = 0; k < TBR_TK; ++k)
#pragma unroll
      for (int u = 0; u < TBR_U; ++u)
        if (q[k][u] != ~0u) put(q[k][u], (u64)(t0 + k) * TB_TILE);
#pragma unroll
    for (int k = 0; k < TBR_TK; ++k) {
      const u32 lk = __builtin_amdgcn_readlane(lo, k), hk = __builtin_amdgcn_readlane(hi, k);
      const u64 rb = (u64)(t0 + k) * TB_TILE;
      for (u32 i = lk + TBR_U * WAVE + (u32)lane; i < hk; i += WAVE) {
        const u32 x = rec[rb + i];
        if (x != REC_DEAD) put(x, rb);
      }
    }
  }
  __syncthreads();
  const u32 s0 = b * A.width;
  for (u32 i = threadIdx.x; i < A.width && (i64)(s0 + i) < n_sym; i += TBR_NT) {
    const u32 a = tA[i], f = tF[i], c = tC[i];
    const int va = a ? A.mv_addr[a - 1] : -1, vf = f ? A.mv_file[f - 1] : -1;
    const int vc = c ? A.Rstr[(u64)(c - 1) - A.nMv] : -1;
    if (part.p) part.put(n_sym, s0 + i, va, vf, vc);
    else fin_put(FP, fin, s0 + i, va, vf, vc);
  }
}

// Fallback for symbol spaces beyond TB_MAXBK * TB_WIDTH: device-scope atomics.
__global__ void k_tab_atomic(TbArgs A0, u32* __restrict__ tabA, u32* __restrict__ tabF, u32* __restrict__ tabR) {
  const TbArgs A = tb_load(A0);
  const u64 nrec = A.nMv + A.nR;
  for (u64 r = (u64)blockIdx.x * BLOCK + threadIdx.x; r < nrec; r += (u64)gridDim.x * BLOCK) {
    u32 s, fl;
    if (!tb_record(A, r, &s, &fl)) continue;
    const u32 r1 = (u32)r + 1u;
    if (r < A.nMv) {
      if (fl & REC_HAS_A) atomicMax(&tabA[s], r1);
      if (fl & REC_HAS_F) atomicMax(&tabF[s], r1);
    } else {
      atomicMax(&tabR[s], r1);
    }
  }
}

__global__ void k_finalize(TbArgs A0, const u32* __restrict__ tabA, const u32* __restrict__ tabF,
                           const u32* __restrict__ tabR, i64 n_sym, int4* __restrict__ fin, PartTab part) {
  const TbArgs A = tb_load(A0);
  for (i64 s = (i64)blockIdx.x * BLOCK + threadIdx.x; s < n_sym; s += (i64)gridDim.x * BLOCK) {
    const u32 a = tabA[s], f = tabF[s], c = tabR[s];
    const int va = a ? A.mv_addr[a - 1] : -1, vf = f ? A.mv_file[f - 1] : -1;
    const int vc = c ? A.Rstr[(u64)(c - 1) - A.nMv] : -1;
    if (part.p) part.put(n_sym, s, va, vf, vc);
    else fin[s] = make_int4(va, vf, vc, 0);
  }
}
