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
  // Sharded merge (smx_shard_step): the renames of each branch that follow this
  // shard's in the global rename order (halo_n[b] of them; halo_more[b] when the
  // halo is a strict prefix of the rest), and the global source index of local
  // op j: j < na_cap ? src_a + j : src_b + (j - na_cap).  Single merge: no halo,
  // src_a = 0, src_b = na_cap.
  const u32* halo_sym[2];
  const i32* halo_cls[2];
  const i32* halo_src[2];
  u64 halo_n[2];
  int halo_more[2];
  i64 src_a, src_b;
};

__device__ __forceinline__ i32 walk_gsrc(const WalkArgs& W, i32 j) {
  return (u64)j < W.na_cap ? (i32)(W.src_a + j) : (i32)(W.src_b + ((i64)j - (i64)W.na_cap));
}

// The k-th rename (local numbering) of branch o: a local M position, or an entry
// of the halo (the next shard's renames).  ok = false when branch o has no k-th
// rename; a halo too short to tell flags meta->halo_overflow.
struct WalkHead {
  bool ok, local;
  u32 sym;
  i32 cls;
  u32 u;  // local M position, or halo index
};

__device__ __forceinline__ WalkHead walk_head(const WalkArgs& W, int o, u64 k) {
  WalkHead h{false, false, 0u, 0, 0u};
  const u64 no = o ? W.nRB : W.nRA;
  if (k < no) {
    const u32 u = (o ? W.RB : W.RA)[k];
    return WalkHead{true, true, W.Msym[u], W.Mcls[u], u};
  }
  // selects, not W.halo_*[o]: a dynamic index into the argument struct would put
  // it in scratch memory
  const u64 x = k - no;
  const u64 hn = o ? W.halo_n[1] : W.halo_n[0];
  if (x < hn) {
    const u32* hs = o ? W.halo_sym[1] : W.halo_sym[0];
    const i32* hc = o ? W.halo_cls[1] : W.halo_cls[0];
    return WalkHead{true, false, hs[x], hc[x], (u32)x};
  }
  if (o ? W.halo_more[1] : W.halo_more[0]) const_cast<ComposeMeta*>(W.meta)->halo_overflow = 1;
  return h;
}

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

// The block's flagged positions go, in order, to its FLAG_TILE-slot range of
// slots[] (k_compact then moves the few of them to their scanned offsets).
// zskip != null: also clears the skip flags of the block's positions.
__global__ void __launch_bounds__(BLOCK) k_flags(WalkArgs W0, u32* __restrict__ slots, u32* __restrict__ bcnt,
                                                 u8* __restrict__ zskip) {
  const WalkArgs W = walk_load(W0);
  if (W.fail || (u64)blockIdx.x * FLAG_TILE >= W.nR) return;
  constexpr int NI = FLAG_TILE / BLOCK;
  __shared__ u32 wc[NI][NWAVES];
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  const u64 base = (u64)blockIdx.x * FLAG_TILE;
  u64 fb[NI];  // this wave's flag ballots
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const u64 m = base + (u64)it * BLOCK + threadIdx.x;
    bool f = false;
    if (m < W.nR) {
      if (zskip) zskip[m] = 0;
      const int s = W.Mside[m];
      const u64 k = m - W.Mown[m];
      const WalkHead h = walk_head(W, 1 - s, k);
      f = h.ok && h.sym == W.Msym[m] && h.cls != W.Mcls[m];
    }
    fb[it] = __ballot(f);
    if (lane == 0) wc[it][w] = (u32)__popcll(fb[it]);
  }
  __syncthreads();
  u32 before = 0;  // flags of this block before (it, wave w)
  const u64 lt = lanemask_lt();
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    if ((fb[it] >> lane) & 1ull) {
      u32 r = before + (u32)__popcll(fb[it] & lt);
      for (int q = 0; q < w; ++q) r += wc[it][q];
      slots[base + r] = (u32)(base + (u64)it * BLOCK + threadIdx.x);
    }
#pragma unroll
    for (int q = 0; q < NWAVES; ++q) before += wc[it][q];
  }
  if (threadIdx.x == 0) bcnt[blockIdx.x] = before;
}

// Exclusive scan of the per-block flag counts (one block; nb is small) and the
// candidate total into meta->n_cand.
#define FO_NT 1024  // k_flag_offsets: one block, 16 counts per thread and round
__global__ void __launch_bounds__(FO_NT) k_flag_offsets(WalkArgs W0, u32* __restrict__ bcnt, u64* total) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  const u32 nb = (u32)SMX_CEIL_DIV(W.nR, (u64)FLAG_TILE);
  __shared__ u32 s[FO_NT / WAVE + 1];
  u32 carry = 0;
  for (u32 r0 = 0; r0 < nb; r0 += FO_NT * 16) {
    const u32 b = r0 + threadIdx.x * 16;
    u32 v[16];
    u32 acc = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      v[j] = b + j < nb ? bcnt[b + j] : 0u;
      acc += v[j];
    }
    u32 tot;
    u32 run = carry + block_excl_scan<OpSum, u32, FO_NT / WAVE>(acc, s, &tot);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (b + j < nb) bcnt[b + j] = run;
      run += v[j];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

// One wave per k_flags block: its slots[] run -> cand[] at the block's offset
// (boff = exclusive scan of the counts; the total is meta->n_cand).
__global__ void __launch_bounds__(BLOCK) k_compact(WalkArgs W0, const u32* __restrict__ slots,
                                                   const u32* __restrict__ boff, const u64* __restrict__ total,
                                                   u32* __restrict__ out) {
  const WalkArgs W = walk_load(W0);
  const u64 fbk = (u64)blockIdx.x * NWAVES + threadIdx.x / WAVE;
  const u64 nfb = SMX_CEIL_DIV(W.nR, (u64)FLAG_TILE);
  if (W.fail || fbk >= nfb) return;
  const u32 o = boff[fbk];
  const u32 e = fbk + 1 < nfb ? boff[fbk + 1] : (u32)*total;
  for (u32 i = threadIdx.x & (WAVE - 1); o + i < e; i += WAVE) out[o + i] = slots[fbk * FLAG_TILE + i];
}

// Replays the reference loop restricted to renames from position p with state
// (ahead branch, d = how many of its next renames were consumed early); a
// candidate start has d = 0.  Returns the end q (the first position after which
// d is back to 0, or nR if the region is still open at the shard's end; the
// final state is left in *ahead_io / *d_io).  WRITE: conflict pairs (global
// source indices) and skip flags of local positions.
template <bool WRITE>
__device__ u32 replay_region(const WalkArgs& W, u32 p, int* ahead_io, u32* d_io, u32* nconf,
                             const i32* order_ren, i32* pairs, u64 pair_cap, u64 pair_off, u8* skip) {
  int ahead = *ahead_io;
  u32 d = *d_io;
  u32 m = p;
  u32 nc = 0;
  while (m < W.nR) {
    const int s = W.Mside[m];
    if (d > 0 && s == ahead) {
      --d;  // consumed as the other head of an earlier conflict
      if (WRITE) skip[m] = 1;
    } else {
      const int o = 1 - s;
      const u64 k = (u64)(m - W.Mown[m]) + (o == ahead ? d : 0u);
      const WalkHead h = walk_head(W, o, k);
      if (h.ok && h.sym == W.Msym[m] && h.cls != W.Mcls[m]) {
        if (WRITE) {
          const u64 slot = pair_off + nc;
          if (slot < pair_cap) {
            const i32 mu = walk_gsrc(W, order_ren[m]);
            const i32 hu = h.local ? walk_gsrc(W, order_ren[h.u]) : (o ? W.halo_src[1] : W.halo_src[0])[h.u];
            pairs[2 * slot] = s ? hu : mu;
            pairs[2 * slot + 1] = s ? mu : hu;
          }
          skip[m] = 1;
          if (h.local) skip[h.u] = 1;
        }
        ++nc;
        ++d;
        ahead = o;
      }
    }
    ++m;
    if (d == 0) break;
  }
  *ahead_io = ahead;
  *d_io = d;
  *nconf = nc;
  return m;
}

// Incoming open region (sharded merge): the previous shards' walk ended with
// state (ahead, d > 0); continue it from position 0.  Its conflicts come first in
// this shard's list; candidates before its end are covered.
__global__ void k_replay_in(WalkArgs W0, int in_ahead, u32 in_d, ComposeMeta* meta, const i32* __restrict__ order,
                            i32* __restrict__ pairs, u64 pair_cap, u8* __restrict__ skip,
                            u32* __restrict__ skiplist) {
  const WalkArgs W = walk_load(W0);
  if (W.fail || in_d == 0 || threadIdx.x != 0 || blockIdx.x != 0) return;
  const i32* order_ren = order + meta->base[SMX_KIND_RENAME];
  int ahead = in_ahead;
  u32 d = in_d, nc = 0;
  const u32 q = replay_region<true>(W, 0, &ahead, &d, &nc, order_ren, pairs, pair_cap, 0, skip);
  meta->q_in = q;
  meta->nconf_in = nc;
  u32 o = 0;  // its skips head the sorted skip list
  for (u32 m = 0; m < q; ++m)
    if (skip[m]) skiplist[o++] = m;
  meta->nskip_in = o;
  atomicAdd((unsigned long long*)&meta->n_skip, (unsigned long long)o);
  if (d > 0) {  // still open at this shard's end: hand it on
    meta->out_open = 1;
    meta->out_ahead = (u64)ahead;
    meta->out_d = d;
  }
}

__global__ void k_replay_q(WalkArgs W0, const u32* __restrict__ cand, const ComposeMeta* meta,
                           u32* __restrict__ q, u32* __restrict__ nconf) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  const u64 nc = meta->n_cand;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    u32 k, d = 0;
    int ahead = -1;
    q[c] = replay_region<false>(W, cand[c], &ahead, &d, &k, nullptr, nullptr, 0, 0, nullptr);
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
    u32 last_q = (u32)meta->q_in;   // an incoming region (sharded merge) covers [0, q_in)
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

// Writes the conflict pairs, skip flags and skip-list entries of every real
// region.  Regions are disjoint and ordered and a closed region's skips (2 per
// conflict) lie in [p, q), so listing [p, q) in order yields the sorted skip list
// after the incoming region's entries.  The last real region may still be open
// at the shard's end (sharded merge): its heads beyond the end belong to the next
// shard, its state is handed on, and its entries (fewer) end the list.
__global__ void k_replay_write(WalkArgs W0, const u32* __restrict__ cand, const u32* __restrict__ nreal,
                               const u32* __restrict__ coff, ComposeMeta* meta,
                               const i32* __restrict__ order, i32* __restrict__ pairs,
                               u64 pair_cap, u8* __restrict__ skip, u32* __restrict__ skiplist) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  const i32* order_ren = order + meta->base[SMX_KIND_RENAME];
  const u64 nc = meta->n_cand;
  const u64 off0 = meta->nconf_in, soff0 = meta->nskip_in;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    if (nreal[c] == 0) continue;
    u32 k, d = 0;
    int ahead = -1;
    const u32 p = cand[c];
    const u32 q = replay_region<true>(W, p, &ahead, &d, &k, order_ren, pairs, pair_cap, off0 + coff[c], skip);
    if (d > 0) {
      meta->out_open = 1;
      meta->out_ahead = (u64)ahead;
      meta->out_d = d;
    }
    u64 o = soff0 + 2 * (u64)coff[c];
    u32 cnt = 0;
    for (u32 m = p; m < q; ++m)
      if (skip[m]) {
        skiplist[o++] = m;
        ++cnt;
      }
    atomicAdd((unsigned long long*)&meta->n_skip, (unsigned long long)cnt);
  }
}

