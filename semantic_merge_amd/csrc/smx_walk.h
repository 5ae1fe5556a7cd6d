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
  u64 nR, nRA, nRB;
};

// Natural-head test: element m against the other branch's head when no skip
// has happened yet (d = 0): that head is R_other[m - own(m)].
__global__ void k_flags(WalkArgs W, u8* __restrict__ flags) {
  for (u64 m = (u64)blockIdx.x * BLOCK + threadIdx.x; m < W.nR; m += (u64)gridDim.x * BLOCK) {
    const int s = W.Mside[m];
    const u64 k = m - W.Mown[m];
    const u64 no = s ? W.nRA : W.nRB;
    u8 f = 0;
    if (k < no) {
      const u32 u = (s ? W.RA : W.RB)[k];
      f = (W.Msym[u] == W.Msym[m]) && (W.Mcls[u] != W.Mcls[m]);
    }
    flags[m] = f;
  }
}

__global__ void k_compact(const u8* __restrict__ flags, const u32* __restrict__ pos, u64 n,
                          u32* __restrict__ out) {
  for (u64 m = (u64)blockIdx.x * BLOCK + threadIdx.x; m < n; m += (u64)gridDim.x * BLOCK)
    if (flags[m]) out[pos[m]] = (u32)m;
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

__global__ void k_replay_q(WalkArgs W, const u32* __restrict__ cand, const ComposeMeta* meta,
                           u32* __restrict__ q, u32* __restrict__ nconf) {
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

__global__ void k_replay_write(WalkArgs W, const u32* __restrict__ cand, const u32* __restrict__ nreal,
                               const u32* __restrict__ coff, const ComposeMeta* meta,
                               const i32* __restrict__ order_ren, i32* __restrict__ pairs,
                               u64 pair_cap, u8* __restrict__ skip) {
  const u64 nc = meta->n_cand;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    if (nreal[c] == 0) continue;
    u32 k;
    replay_region<true>(W, cand[c], &k, order_ren, pairs, pair_cap, coff[c], skip);
  }
}

