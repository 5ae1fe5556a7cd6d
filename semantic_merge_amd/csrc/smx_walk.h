// smx_walk.h — DivergentRename detection over the rename block (compose.py:60-70, 88-98).
//
// The reference compares the two branch heads at every merge step; a conflict
// consumes both heads.  Restricted to renames (all moves come first in T and no
// other kind can conflict) the loop is a transducer over M = renames in T order
// with state (ahead branch, d): d of the ahead branch's next renames were already
// consumed as "other heads".  From a d = 0 state the walk only depends on the
// natural-head test of each element, so: flag every natural-head conflict,
// replay from each flagged start until d returns to 0 (region end q), and keep
// the starts not covered by an earlier real region (resolved per cluster).
#pragma once

#include "smx_common.h"

// ---------------------------------------------------------------------------
// kernels: DivergentRename walk over the rename block M (T order)

struct WalkArgs {
  const u32* Msym;
  const i32* Mcls;
  const u8* Mside;
  const u32* Mown;
  const u32* RA;
  const u32* RB;
  const ComposeMeta* meta;
  u64 na_cap, nb_cap;   // host sizes: bounds for the device-side counts
  u64 nR, nRA, nRB;     // filled on the device by walk_load
  u64 fail;
};

// Sizes come from the device (no host sync before the walk); a failed
// presorted plan or invalid input turns every walk kernel into a no-op.
__device__ __forceinline__ WalkArgs walk_load(WalkArgs W) {
  const ComposeMeta* m = W.meta;
  W.fail = m->f_fail | m->bad_sym;
  W.nRA = min(m->n_ren_side[0], W.na_cap);
  W.nRB = min(m->n_ren_side[1], W.nb_cap);
  W.nR = W.nRA + W.nRB;
  return W;
}

// Natural-head test: element m against the other branch's head when no skip
// has happened yet (d = 0): that head is R_other[m - own(m)].  Each block owns a
// contiguous range of FLAG_TILE renames and also reports how many it flagged.
#define FLAG_TILE (BLOCK * 8)

__global__ void __launch_bounds__(BLOCK) k_flags(WalkArgs W0, u8* __restrict__ flags, u32* __restrict__ bcnt) {
  const WalkArgs W = walk_load(W0);
  if (W.fail || (u64)blockIdx.x * FLAG_TILE >= W.nR) return;
  __shared__ u32 c;
  if (threadIdx.x == 0) c = 0;
  __syncthreads();
  const u64 base = (u64)blockIdx.x * FLAG_TILE;
  u32 mine = 0;
  for (int it = 0; it < FLAG_TILE / BLOCK; ++it) {
    const u64 m = base + (u64)it * BLOCK + threadIdx.x;
    if (m >= W.nR) break;
    const int s = W.Mside[m];
    const u64 k = m - W.Mown[m];
    const u64 no = s ? W.nRA : W.nRB;
    u8 f = 0;
    if (k < no) {
      const u32 u = (s ? W.RA : W.RB)[k];
      f = (W.Msym[u] == W.Msym[m]) && (W.Mcls[u] != W.Mcls[m]);
    }
    flags[m] = f;
    mine += f;
  }
  if (mine) atomicAdd(&c, mine);
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = c;
}

// Exclusive scan of the per-block flag counts (one block; nb is small) and the
// candidate total into meta->n_cand.
__global__ void __launch_bounds__(BLOCK) k_flag_offsets(WalkArgs W0, u32* __restrict__ bcnt, ComposeMeta* meta) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  const u32 nb = (u32)SMX_CEIL_DIV(W.nR, (u64)FLAG_TILE);
  __shared__ u32 s[NWAVES + 1];
  u32 carry = 0;
  for (u32 r0 = 0; r0 < nb; r0 += BLOCK * 8) {
    const u32 b = r0 + threadIdx.x * 8;
    u32 v[8];
    u32 acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = b + j < nb ? bcnt[b + j] : 0u;
      acc += v[j];
    }
    u32 tot;
    u32 run = carry + block_excl_scan<OpSum, u32>(acc, s, &tot);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (b + j < nb) bcnt[b + j] = run;
      run += v[j];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) meta->n_cand = carry;
}

__global__ void __launch_bounds__(BLOCK) k_compact(WalkArgs W0, const u8* __restrict__ flags,
                                                   const u32* __restrict__ boff, u32* __restrict__ out) {
  const WalkArgs W = walk_load(W0);
  const u64 n = W.nR;
  if (W.fail || (u64)blockIdx.x * FLAG_TILE >= n) return;
  __shared__ u32 wbase[NWAVES + 1];
  const u64 base = (u64)blockIdx.x * FLAG_TILE;
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  u32 run = boff[blockIdx.x];
  for (int it = 0; it < FLAG_TILE / BLOCK; ++it) {
    const u64 m = base + (u64)it * BLOCK + threadIdx.x;
    const bool f = m < n && flags[m];
    const u64 b = __ballot(f);
    if (lane == 0) wbase[w] = __popcll(b);
    __syncthreads();
    u32 before = 0, tot = 0;
    for (int q = 0; q < NWAVES; ++q) {
      before += q < w ? wbase[q] : 0u;
      tot += wbase[q];
    }
    if (f) out[run + before + __popcll(b & lanemask_lt())] = (u32)m;
    run += tot;
    __syncthreads();
  }
}

// Replays the reference loop restricted to renames from a d = 0 candidate start
// p: state (ahead branch, d = how many of its next renames were consumed early).
// Returns the end q (first position after which d is back to 0).
template <bool WRITE>
__device__ u32 replay_region(const WalkArgs& W, u32 p, u32* nconf, const i32* order_ren,
                             i32* pairs, u64 pair_cap, u32 pair_off, u8* skip) {
  int ahead = -1;
  u32 d = 0;
  u32 m = p;
  u32 nc = 0;
  do {
    const int s = W.Mside[m];
    if (d > 0 && s == ahead) {
      --d;  // consumed as the other head of an earlier conflict
    } else {
      const int o = 1 - s;
      const u64 k = (u64)(m - W.Mown[m]) + (o == ahead ? d : 0u);
      const u64 no = s ? W.nRA : W.nRB;
      if (k < no) {
        const u32 u = (s ? W.RA : W.RB)[k];
        if (W.Msym[u] == W.Msym[m] && W.Mcls[u] != W.Mcls[m]) {
          if (WRITE) {
            const u64 slot = (u64)pair_off + nc;
            if (slot < pair_cap) {
              pairs[2 * slot] = order_ren[s ? u : m];
              pairs[2 * slot + 1] = order_ren[s ? m : u];
            }
            skip[m] = 1;
            skip[u] = 1;
          }
          ++nc;
          ++d;
          ahead = o;
        }
      }
    }
    ++m;
  } while (d > 0 && m < W.nR);
  *nconf = nc;
  return m;
}

__global__ void k_replay_q(WalkArgs W0, const u32* __restrict__ cand, const ComposeMeta* meta,
                           u32* __restrict__ q, u32* __restrict__ nconf) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  const u64 nc = meta->n_cand;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    u32 k;
    q[c] = replay_region<false>(W, cand[c], &k, nullptr, nullptr, 0, 0, nullptr);
    nconf[c] = k;
  }
}

// Real region starts: the first candidate of each cluster (no earlier candidate's
// region reaches it) is real; inside a cluster, walk sequentially.
__global__ void k_cluster(const u32* __restrict__ cand, const u32* __restrict__ q,
                          const u32* __restrict__ pm, const u32* __restrict__ nconf,
                          const ComposeMeta* meta, u32* __restrict__ nreal) {
  const u64 nc = meta->n_cand;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    if (pm[c] > cand[c]) continue;  // not a cluster start
    u32 last_q = 0;
    for (u64 j = c; j < nc && (j == c || pm[j] > cand[j]); ++j) {
      if (cand[j] >= last_q) {
        nreal[j] = nconf[j];
        last_q = q[j];
      } else {
        nreal[j] = 0;
      }
    }
  }
}

// Writes the conflict pairs of every real region and its skipped positions:
// a region's skips lie in [p, q) and regions are disjoint and ordered, so
// listing [p, q) in order yields the globally sorted skip list (2 per conflict).
__global__ void k_replay_write(WalkArgs W0, const u32* __restrict__ cand, const u32* __restrict__ nreal,
                               const u32* __restrict__ coff, const ComposeMeta* meta,
                               const i32* __restrict__ order, i32* __restrict__ pairs,
                               u64 pair_cap, u8* __restrict__ skip, u32* __restrict__ skiplist) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  const i32* order_ren = order + meta->base[SMX_KIND_RENAME];
  const u64 nc = meta->n_cand;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    if (nreal[c] == 0) continue;
    u32 k;
    const u32 p = cand[c];
    const u32 q = replay_region<true>(W, p, &k, order_ren, pairs, pair_cap, coff[c], skip);
    u32 o = 2 * coff[c];
    for (u32 m = p; m < q; ++m)
      if (skip[m]) skiplist[o++] = m;
  }
}

