// smx_walk.h — DivergentRename detection over the rename block (compose.py:60-70, 88-98).
//
// The reference compares the two branch heads at every merge step; a conflict
// consumes both heads.  Restricted to renames (all moves come first in T and no
// other kind can conflict) the loop is a transducer over M = renames in T order
// with state (ahead branch, d): d of the ahead branch's next renames were already
// consumed as "other heads".  From a d = 0 state the walk only depends on the
// natural-head test of each element (its other-branch head is then that branch's
// next rename), so: flag every natural-head conflict (k_window_* inside a window,
// k_boundary for the renames whose head lies in a later window), replay from each
// flagged start until d returns to 0 (region end q), and keep the starts not
// covered by an earlier real region (resolved per cluster).
//
// M is held as tsrc[m] (local source op: its branch and, through v0, its newName
// equality class) and tsym[m].  A replay keeps one cursor per branch: the first
// not-yet-consumed rename of that branch after the current position, found by a
// forward scan of tsrc (short on real logs; a long gap switches to a rank lookup
// over the per-window rename counts wren, O(log W + window)).
#pragma once

#include "smx_common.h"

#define WALK_SCAN 256         // forward-scan steps before the rank lookup
#define REPLAY_CAP 256        // k_replay_q: steps before a region counts as long
#define CUR_NONE 0xffffffffu  // cursor: no such rename
#define CUR_HALO 0x80000000u  // cursor: halo index (| h); local positions are < 2^31
#define Q_LONG 0xffffffffu    // k_replay_q: region not closed within REPLAY_CAP steps

struct WalkArgs {
  const i32* tsrc;      // M position -> local source op (renames are tsrc[0, nR))
  const u32* tsym;
  const i32* v0;        // field array: local op j at j (A) or j + bgap (B)
  const u32* wren;      // [W][2]: renames, A renames before window w
  const u32* wbnd;      // [W]: boundary start | branch << 31
  const ComposeMeta* meta;
  u64 na_cap, nb_cap;   // host sizes: bounds for the device-side counts
  i64 bgap;
  u64 nR, nRA, nRB, Wn; // filled on the device by walk_load
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
  const i64* halo_dev;  // device-held halo_n / halo_more (smx_shard.halo_dev), or null
  i64 src_a, src_b;
  const i32* src_map;   // sample-sorted shard: global source of local op j, or null
  // k_replay_q's staged outputs (candidates c < stage_cap): a region that closes with at
  // most RS_CONF conflicts leaves its conflict pairs and skip positions at
  // stage[c * RS_W ..], sok[c] = 1, and k_replay_write copies them instead of replaying
  u32* stage;
  u32* sok;
  u64 stage_cap;
};
#ifndef RS_CONF
#define RS_CONF 2                 // conflicts of a staged region (0: no staging)
#endif
#define RS_W (4 * RS_CONF)        // words per candidate: 2 per conflict pair, 2 skips per conflict

__device__ __forceinline__ i32 walk_gsrc(const WalkArgs& W, i32 j) {
  if (W.src_map) return W.src_map[j];
  return (u64)j < W.na_cap ? (i32)(W.src_a + j) : (i32)(W.src_b + ((i64)j - (i64)W.na_cap));
}

// Sizes come from the device (no host sync before the walk); a failed
// presorted plan or invalid input turns every walk kernel into a no-op.
__device__ __forceinline__ WalkArgs walk_load(WalkArgs W) {
  const ComposeMeta* m = W.meta;
  W.fail = m->f_fail | m->bad_sym;
  W.nRA = min(m->n_ren_side[0], W.na_cap);
  W.nRB = min(m->n_ren_side[1], W.nb_cap);
  W.nR = W.nRA + W.nRB;
  W.Wn = m->n_win;
  if (W.halo_dev) {
    for (int b = 0; b < 2; ++b) {
      W.halo_n[b] = W.halo_sym[b] ? (u64)max(W.halo_dev[b], (i64)0) : 0;
      W.halo_more[b] = W.halo_dev[2 + b] != 0;
    }
  }
  return W;
}

__device__ __forceinline__ int walk_side(const WalkArgs& W, u64 m) { return (u64)W.tsrc[m] >= W.na_cap; }
__device__ __forceinline__ i32 walk_cls_of_src(const WalkArgs& W, i32 j) {
  return W.v0[(u64)j < W.na_cap ? (i64)j : (i64)j + W.bgap];
}

// Halo entry h of branch o (or CUR_NONE; a halo too short to tell flags overflow).
// Selects, not W.halo_*[o]: a dynamic index into the argument struct would put it
// in scratch memory.
__device__ __forceinline__ u32 walk_halo(const WalkArgs& W, int o, u64 h) {
  if (h < (o ? W.halo_n[1] : W.halo_n[0])) return CUR_HALO | (u32)h;
  if (o ? W.halo_more[1] : W.halo_more[0]) const_cast<ComposeMeta*>(W.meta)->halo_overflow = 1;
  return CUR_NONE;
}

// Renames of branch o before window w (w <= Wn; window Wn = the end of M).
__device__ __forceinline__ u64 walk_before(const WalkArgs& W, int o, u64 w) {
  if (w >= W.Wn) return o ? W.nRB : W.nRA;
  const u64 a = W.wren[2 * w + 1];
  return o ? (u64)W.wren[2 * w] - a : a;
}

// First rename of branch o at a position >= x, by counts: x's window, o-renames
// before x, then the window holding the next one.
__device__ u32 walk_rank_next(const WalkArgs& W, int o, u64 x) {
  u64 lo = 0, hi = W.Wn;  // largest w with wren[2w] <= x
  while (hi - lo > 1) {
    const u64 mid = (lo + hi) >> 1;
    if (W.wren[2 * mid] <= x) lo = mid;
    else hi = mid;
  }
  u64 c = walk_before(W, o, lo);
  for (u64 m = W.wren[2 * lo]; m < x; ++m) c += walk_side(W, m) == o;
  const u64 no = o ? W.nRB : W.nRA;
  if (c >= no) return walk_halo(W, o, c - no);
  lo = 0, hi = W.Wn;  // largest w with before(w) <= c: the window holding o-rename c
  while (hi - lo > 1) {
    const u64 mid = (lo + hi) >> 1;
    if (walk_before(W, o, mid) <= c) lo = mid;
    else hi = mid;
  }
  u64 k = c - walk_before(W, o, lo);
  for (u64 m = W.wren[2 * lo];; ++m)
    if (walk_side(W, m) == o && k-- == 0) return (u32)m;
}

// First rename of branch o at a local position >= from, else the halo.  WALK_NEXT_VEC
// sources are read per step, all in flight together (the scan usually ends within a
// step: the branches' renames interleave), instead of one dependent load per position.
#ifndef WALK_NEXT_VEC
#define WALK_NEXT_VEC 1  // 8: config 3 walk 0.145 -> 0.163 ms, config 2 0.046 -> 0.052 ms (round 4); off
#endif
__device__ __forceinline__ u32 walk_next(const WalkArgs& W, int o, u64 from) {
  u64 m = from;
  if (WALK_NEXT_VEC > 1) {
    static_assert(WALK_SCAN % (WALK_NEXT_VEC > 1 ? WALK_NEXT_VEC : 1) == 0, "whole steps");
    for (int i = 0; i < WALK_SCAN; i += WALK_NEXT_VEC, m += WALK_NEXT_VEC) {
      i32 js[WALK_NEXT_VEC > 1 ? WALK_NEXT_VEC : 1];
#pragma unroll
      for (int k = 0; k < WALK_NEXT_VEC; ++k) js[k] = m + k < W.nR ? W.tsrc[m + k] : 0;
#pragma unroll
      for (int k = 0; k < WALK_NEXT_VEC; ++k) {
        if (m + k >= W.nR) return walk_halo(W, o, 0);
        if (((u64)js[k] >= W.na_cap) == (o != 0)) return (u32)(m + k);
      }
    }
    return walk_rank_next(W, o, m);
  }
  for (int i = 0; i < WALK_SCAN; ++i, ++m) {
    if (m >= W.nR) return walk_halo(W, o, 0);
    if (walk_side(W, m) == o) return (u32)m;
  }
  return walk_rank_next(W, o, m);
}

// The o-rename after cursor c.
__device__ __forceinline__ u32 walk_adv(const WalkArgs& W, int o, u32 c) {
  if (c == CUR_NONE) return CUR_NONE;
  if (c & CUR_HALO) return walk_halo(W, o, (u64)(c & ~CUR_HALO) + 1);
  return walk_next(W, o, (u64)c + 1);
}

struct WalkHead {
  u32 sym;
  i32 cls;
};
__device__ __forceinline__ WalkHead walk_at(const WalkArgs& W, int o, u32 c) {
  if (c & CUR_HALO) {
    const u32 h = c & ~CUR_HALO;
    return WalkHead{(o ? W.halo_sym[1] : W.halo_sym[0])[h], (o ? W.halo_cls[1] : W.halo_cls[0])[h]};
  }
  return WalkHead{W.tsym[c], walk_cls_of_src(W, W.tsrc[c])};
}
__device__ __forceinline__ i32 walk_src_at(const WalkArgs& W, int o, u32 c) {
  if (c & CUR_HALO) return (o ? W.halo_src[1] : W.halo_src[0])[c & ~CUR_HALO];
  return walk_gsrc(W, W.tsrc[c]);
}

#define CUR_UNSET (CUR_NONE - 1)  // cursor not computed yet

struct ReplayState {
  int ahead;
  u32 d;
  u32 h[2];  // first not-yet-consumed rename of each branch after the position (lazy)
};

__device__ __forceinline__ ReplayState replay_fresh() { return ReplayState{-1, 0u, {CUR_UNSET, CUR_UNSET}}; }

// Replays the reference loop restricted to renames from position p with state st
// (a candidate start has d = 0).  Returns the end q (the first position after which
// d is back to 0, or nR if the region is still open at the shard's end; the final
// state is left in st), or Q_LONG when CAP and the region is longer than
// REPLAY_CAP steps.  WRITE: conflict pairs (global source indices) at pair_off..,
// skipped positions in increasing order at skip_out.., and their skip bits.
// STAGE: the first RS_CONF conflicts' pairs and their skip positions go to stg (no
// other side effects).
template <bool WRITE, bool CAP, bool STAGE = false>
__device__ u32 replay_region(const WalkArgs& W, u32 p, ReplayState& st, u32* nconf, i32* pairs, u64 pair_cap,
                             u64 pair_off, u32* skip_out, u64* skipbits, u32* nskip, u32* stg = nullptr) {
  u32 m = p;
  u32 nc = 0, ns = 0, steps = 0;
  while (m < W.nR) {
    const i32 j = W.tsrc[m];
    const int s = (u64)j >= W.na_cap;
    if (st.d > 0 && s == st.ahead) {
      --st.d;  // consumed as the other head of an earlier conflict
      if (WRITE) {
        skip_out[ns] = m;
        atomicOr((unsigned long long*)&skipbits[m >> 6], 1ull << (m & 63));
      }
      if (STAGE && ns < 2 * RS_CONF) stg[2 * RS_CONF + ns] = m;
      ++ns;
    } else {
      const int o = 1 - s;
      if (st.h[o] == CUR_UNSET) st.h[o] = walk_next(W, o, (u64)m + 1);
      const u32 hc = st.h[o];
      if (hc != CUR_NONE) {
        const WalkHead hd = walk_at(W, o, hc);
        if (hd.sym == W.tsym[m] && hd.cls != walk_cls_of_src(W, j)) {
          if (WRITE) {
            const u64 slot = pair_off + nc;
            if (slot < pair_cap) {
              const i32 mu = walk_gsrc(W, j), hu = walk_src_at(W, o, hc);
              pairs[2 * slot] = s ? hu : mu;
              pairs[2 * slot + 1] = s ? mu : hu;
            }
            skip_out[ns] = m;
            atomicOr((unsigned long long*)&skipbits[m >> 6], 1ull << (m & 63));
          }
          if (STAGE && nc < RS_CONF) {
            const i32 mu = walk_gsrc(W, j), hu = walk_src_at(W, o, hc);
            stg[2 * nc] = (u32)(s ? hu : mu);
            stg[2 * nc + 1] = (u32)(s ? mu : hu);
            stg[2 * RS_CONF + ns] = m;
          }
          ++ns;
          ++nc;
          if (st.ahead != o) {
            st.ahead = o;
            st.d = 0;
          }
          ++st.d;
          st.h[o] = walk_adv(W, o, hc);
        }
      }
      st.h[s] = walk_next(W, s, (u64)m + 1);
    }
    ++m;
    if (st.d == 0) break;
    if (CAP && ++steps >= REPLAY_CAP) return Q_LONG;
  }
  *nconf = nc;
  if (nskip) *nskip = ns;
  return m;
}

// ---------------------------------------------------------------------------
// kernels

// Renames after the other branch's last rename of their window: their natural
// head is that branch's first rename after the window.  Flagged ones follow the
// window's in-window candidates in its slots; wtot[w] = all of the window's
// candidates.  Re-running it (sharded walk rounds) rewrites the same slots.  Block
// 0 also resets the walk's counters in meta.
// (cslot and wtot carry no __restrict__: k_boundary_cc's last block reads what the
// other blocks wrote there)
__device__ __forceinline__ void boundary_body(WalkArgs W0, ComposeMeta* meta, u32* cslot,
                                              const u32* __restrict__ wcand, u32* wtot,
                                              u64* __restrict__ skipbits, u64 nskipw) {
  // the skip bits of the walk (k_replay_in / k_replay_write set them) start cleared:
  // done here rather than by a zero-fill launch of its own
  for (u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x; i < nskipw; i += (u64)gridDim.x * BLOCK) skipbits[i] = 0ull;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    meta->n_cand = 0;
    meta->n_conf = 0;
    meta->n_conf_loc = 0;
    meta->n_skip = 0;
    meta->q_in = 0;
    meta->nconf_in = 0;
    meta->out_open = 0;
    meta->out_ahead = 0;
    meta->out_d = 0;
    meta->halo_overflow = 0;
    meta->nskip_in = 0;
  }
  const WalkArgs W = walk_load(W0);
  for (u64 w = (u64)blockIdx.x * BLOCK + threadIdx.x; w < W.Wn; w += (u64)gridDim.x * BLOCK) {
    if (W.fail) {  // a failed plan: no candidates (the scan below still runs)
      wtot[w] = 0;
      continue;
    }
    const u64 Mb = W.wren[2 * w], Me = w + 1 < W.Wn ? (u64)W.wren[2 * (w + 1)] : W.nR;
    const u32 c0 = wcand[w];
    u32 cnt = 0;
    if (Me > Mb) {
      const u32 wb = W.wbnd[w];
      const int o = 1 - (int)(wb >> 31);
      const u32 hc = walk_next(W, o, Me);
      if (hc != CUR_NONE) {
        const WalkHead hd = walk_at(W, o, hc);
        u32* out = cslot + Mb + c0;
        for (u64 m = Mb + (wb & 0x7fffffffu); m < Me; ++m)
          if (W.tsym[m] == hd.sym && walk_cls_of_src(W, W.tsrc[m]) != hd.cls) out[cnt++] = (u32)m;
      }
    }
    wtot[w] = c0 + cnt;
  }
}
__global__ void __launch_bounds__(BLOCK) k_boundary(WalkArgs W0, ComposeMeta* meta, u32* cslot,
                                                    const u32* __restrict__ wcand, u32* wtot,
                                                    u64* __restrict__ skipbits, u64 nskipw) {
  boundary_body(W0, meta, cslot, wcand, wtot, skipbits, nskipw);
}

// Fused steps of small merges (launch-bound): every block counts itself done and the
// last one runs the next single-block step, after a device-scope fence each side (the
// other blocks' writes are then visible to it); it also resets the counter, which the
// plan's meta zero-fill started at 0.
__device__ __forceinline__ bool walk_last_block(u32* ctr) {
  __shared__ u32 last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(ctr, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!last) return false;
  __threadfence();
  if (threadIdx.x == 0) *ctr = 0u;
  return true;
}

// One thread per window: its candidate slots -> cand[] at the window's offset
// (woff = exclusive scan of wtot; the total is meta->n_cand).
__global__ void __launch_bounds__(BLOCK) k_cand_compact(WalkArgs W0, const u32* __restrict__ cslot,
                                                        const u32* __restrict__ woff, const u64* __restrict__ total,
                                                        u32* __restrict__ out) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  for (u64 w = (u64)blockIdx.x * BLOCK + threadIdx.x; w < W.Wn; w += (u64)gridDim.x * BLOCK) {
    const u32 o = woff[w];
    const u32 e = w + 1 < W.Wn ? woff[w + 1] : (u32)*total;
    const u64 Mb = W.wren[2 * w];
    for (u32 i = 0; o + i < e; ++i) out[o + i] = cslot[Mb + i];
  }
}

// Single-block exclusive scan (sum or max) of n = *n_dev values; *total_lo (low
// word of a zeroed u64) = the total.  For the candidate arrays, which are short on
// real logs (one block, no extra launches); long ones loop.
#define S1_NT 1024
#ifndef WALK_SCAN1_MAXW
#define WALK_SCAN1_MAXW 65536        // window-count scan in one block up to this many windows
#endif
#ifndef WALK_FUSED_MAXN
#define WALK_FUSED_MAXN (1ll << 22)  // k_cluster_fused up to this many ops
#endif
template <typename Op, int NT = S1_NT>
__device__ __forceinline__ void scan1_block(const u32* __restrict__ in, u32* __restrict__ out, u64 n,
                                            u32* total_lo, u32* s) {
  u32 carry = Op::template identity<u32>();
  for (u64 r0 = 0; r0 < n; r0 += NT * 8) {
    const u64 b = r0 + threadIdx.x * 8;
    u32 v[8];
    u32 acc = Op::template identity<u32>();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = b + j < n ? in[b + j] : Op::template identity<u32>();
      acc = Op::apply(acc, v[j]);
    }
    u32 tot;
    u32 run = Op::apply(carry, block_excl_scan<Op, u32, NT / WAVE>(acc, s, &tot));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (b + j < n) out[b + j] = run;
      run = Op::apply(run, v[j]);
    }
    carry = Op::apply(carry, tot);
  }
  if (total_lo && threadIdx.x == 0) *total_lo = carry;
}
template <typename Op>
__global__ void __launch_bounds__(S1_NT) k_scan1(const u32* __restrict__ in, u32* __restrict__ out,
                                                 const u64* n_dev, u64 cap, u32* total_lo) {
  __shared__ u32 s[S1_NT / WAVE + 1];
  scan1_block<Op>(in, out, min(*n_dev, cap), total_lo, s);  // cap: the arrays' capacity
}

// Small merges (launch-bound): the window-count scan and the candidate compaction in one
// block (k_scan1<OpSum> then k_cand_compact), a barrier between them.
#ifndef WALK_CC_FUSED_MAXW
#define WALK_CC_FUSED_MAXW 4096
#endif
template <int NT>
__device__ __forceinline__ void cand_scan_compact_body(const WalkArgs& W, const u32* wtot, u32* woff, u64 cap,
                                                       u32* total_lo, const u32* cslot, u32* out, u32* s) {
  const u64 nw = min(W.Wn, cap);
  scan1_block<OpSum, NT>(wtot, woff, nw, total_lo, s);
  __syncthreads();  // (global writes of this block: visible to it after the barrier)
  if (W.fail) return;
  const u32 total = *total_lo;
  for (u64 w = threadIdx.x; w < nw; w += NT) {
    const u32 o = woff[w];
    const u32 e = w + 1 < nw ? woff[w + 1] : total;
    const u64 Mb = W.wren[2 * w];
    for (u32 i = 0; o + i < e; ++i) out[o + i] = cslot[Mb + i];
  }
}
__global__ void __launch_bounds__(S1_NT) k_cand_scan_compact(WalkArgs W0, const u32* __restrict__ wtot,
                                                             u32* __restrict__ woff, u64 cap, u32* total_lo,
                                                             const u32* __restrict__ cslot, u32* __restrict__ out) {
  __shared__ u32 s[S1_NT / WAVE + 1];
  cand_scan_compact_body<S1_NT>(walk_load(W0), wtot, woff, cap, total_lo, cslot, out, s);
}
// k_boundary, then (its last block) k_cand_scan_compact: one launch
__global__ void __launch_bounds__(BLOCK) k_boundary_cc(WalkArgs W0, ComposeMeta* meta, u32* cslot,
                                                       const u32* __restrict__ wcand, u32* wtot,
                                                       u64* __restrict__ skipbits, u64 nskipw, u32* woff, u64 cap,
                                                       u32* total_lo, u32* cand) {
  boundary_body(W0, meta, cslot, wcand, wtot, skipbits, nskipw);
  if (!walk_last_block(&meta->wk_done[0])) return;
  __shared__ u32 s[NWAVES + 1];
  cand_scan_compact_body<BLOCK>(walk_load(W0), wtot, woff, cap, total_lo, cslot, cand, s);
}

// Incoming open region (sharded merge): the previous shards' walk ended with
// state (ahead, d > 0); continue it from position 0.  Its conflicts come first in
// this shard's list; candidates before its end are covered.
__global__ void k_replay_in(WalkArgs W0, int in_ahead, u32 in_d, const i64* in_dev, ComposeMeta* meta,
                            i32* __restrict__ pairs, u64 pair_cap, u32* __restrict__ skiplist,
                            u64* __restrict__ skipbits) {
  const WalkArgs W = walk_load(W0);
  if (in_dev) {  // device-held incoming state
    in_ahead = (int)in_dev[0];
    in_d = in_dev[1] > 0 ? (u32)in_dev[1] : 0u;
  }
  if (W.fail || in_d == 0 || threadIdx.x != 0 || blockIdx.x != 0) return;
  ReplayState st = replay_fresh();
  st.ahead = in_ahead;
  st.d = in_d;
  // the ahead branch's first in_d renames were consumed before this shard
  u32 c = walk_next(W, in_ahead, 0);
  for (u32 i = 0; i < in_d && c != CUR_NONE; ++i) c = walk_adv(W, in_ahead, c);
  st.h[in_ahead] = c;
  st.h[1 - in_ahead] = walk_next(W, 1 - in_ahead, 0);
  u32 nc = 0, ns = 0;
  const u32 q = replay_region<true, false>(W, 0, st, &nc, pairs, pair_cap, 0, skiplist, skipbits, &ns);
  meta->q_in = q;
  meta->nconf_in = nc;
  meta->nskip_in = ns;
  atomicAdd((unsigned long long*)&meta->n_skip, (unsigned long long)ns);
  if (st.d > 0) {  // still open at this shard's end: hand it on
    meta->out_open = 1;
    meta->out_ahead = (u64)st.ahead;
    meta->out_d = st.d;
  }
}

__device__ __forceinline__ void replay_q_body(WalkArgs W0, const u32* __restrict__ cand, const ComposeMeta* meta,
                                              u32* q, u32* nconf) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  const u64 nc = meta->n_cand;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    u32 k = 0;
    ReplayState st = replay_fresh();
    if (c < W.stage_cap) {
      const u32 qq = replay_region<false, true, true>(W, cand[c], st, &k, nullptr, 0, 0, nullptr, nullptr, nullptr,
                                                      W.stage + c * RS_W);
      q[c] = qq;
      // staged: closed (d back to 0) within the step cap, with few enough conflicts
      W.sok[c] = qq != Q_LONG && st.d == 0 && k <= RS_CONF;
    } else {
      q[c] = replay_region<false, true>(W, cand[c], st, &k, nullptr, 0, 0, nullptr, nullptr, nullptr);
    }
    nconf[c] = k;
  }
}
__global__ void k_replay_q(WalkArgs W0, const u32* __restrict__ cand, const ComposeMeta* meta,
                           u32* __restrict__ q, u32* __restrict__ nconf) {
  replay_q_body(W0, cand, meta, q, nconf);
}

// Real region starts: the first candidate of each cluster (no earlier candidate's
// region reaches it) is real; inside a cluster, walk sequentially.  A long region
// (Q_LONG; it joins every later candidate to its cluster) is replayed in full here,
// once, by the cluster's thread.
__device__ __forceinline__ void cluster_walk(const WalkArgs& W, const u32* __restrict__ cand, u32* __restrict__ q,
                                             const u32* __restrict__ pm, u32* __restrict__ nconf,
                                             const ComposeMeta* meta, u32* __restrict__ nreal, u64 c0, u64 cstep) {
  const u64 nc = meta->n_cand;
  for (u64 c = c0; c < nc; c += cstep) {
    if (pm[c] > cand[c]) continue;  // not a cluster start
    u32 last_q = (u32)meta->q_in;   // an incoming region (sharded merge) covers [0, q_in)
    for (u64 j = c; j < nc && (j == c || pm[j] > cand[j]); ++j) {
      if (cand[j] >= last_q) {
        if (q[j] == Q_LONG) {
          u32 k = 0;
          ReplayState st = replay_fresh();
          q[j] = replay_region<false, false>(W, cand[j], st, &k, nullptr, 0, 0, nullptr, nullptr, nullptr);
          nconf[j] = k;
        }
        nreal[j] = nconf[j];
        last_q = q[j];
      } else {
        nreal[j] = 0;
      }
    }
  }
}
__global__ void k_cluster(WalkArgs W0, const u32* __restrict__ cand, u32* __restrict__ q,
                          const u32* __restrict__ pm, u32* __restrict__ nconf, const ComposeMeta* meta,
                          u32* __restrict__ nreal) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  cluster_walk(W, cand, q, pm, nconf, meta, nreal, (u64)blockIdx.x * blockDim.x + threadIdx.x,
               (u64)gridDim.x * blockDim.x);
}
// Small merges (launch-bound): k_scan1<OpMax> (pm), k_cluster and k_scan1<OpSum> (coff,
// the conflict total) in one block, barriers between the phases.
template <int NT>
__device__ __forceinline__ void cluster_fused_body(WalkArgs W0, const u32* __restrict__ cand, u32* q, u32* pm,
                                                   u32* nconf, const ComposeMeta* meta, u32* nreal, u32* coff,
                                                   u64 cap, u32* total_lo, u32* s) {
  const WalkArgs W = walk_load(W0);
  const u64 nc = min(meta->n_cand, cap);
  scan1_block<OpMax, NT>(q, pm, nc, nullptr, s);
  __syncthreads();  // (global writes of this block: visible to it after the barrier)
  if (!W.fail) cluster_walk(W, cand, q, pm, nconf, meta, nreal, threadIdx.x, NT);
  __syncthreads();
  scan1_block<OpSum, NT>(nreal, coff, W.fail ? 0 : nc, total_lo, s);
}
__global__ void __launch_bounds__(S1_NT) k_cluster_fused(WalkArgs W0, const u32* __restrict__ cand,
                                                         u32* __restrict__ q, u32* __restrict__ pm,
                                                         u32* __restrict__ nconf, const ComposeMeta* meta,
                                                         u32* __restrict__ nreal, u32* __restrict__ coff, u64 cap,
                                                         u32* total_lo) {
  __shared__ u32 s[S1_NT / WAVE + 1];
  cluster_fused_body<S1_NT>(W0, cand, q, pm, nconf, meta, nreal, coff, cap, total_lo, s);
}
// k_replay_q, then (its last block) k_cluster_fused: one launch
__global__ void __launch_bounds__(BLOCK) k_replay_q_cl(WalkArgs W0, const u32* __restrict__ cand, ComposeMeta* meta,
                                                       u32* q, u32* nconf, u32* pm, u32* nreal, u32* coff, u64 cap,
                                                       u32* total_lo) {
  replay_q_body(W0, cand, meta, q, nconf);
  if (!walk_last_block(&meta->wk_done[1])) return;
  __shared__ u32 s[NWAVES + 1];
  cluster_fused_body<BLOCK>(W0, cand, q, pm, nconf, meta, nreal, coff, cap, total_lo, s);
}

// Writes the conflict pairs, skip-list entries and skip bits of every real
// region.  Regions are disjoint and ordered and a closed region's skips (2 per
// conflict) lie in [p, q) in increasing order, so each region writes its entries
// at 2 x (conflicts before it), after the incoming region's.  The last real region
// may still be open at the shard's end (sharded merge): its heads beyond the end
// belong to the next shard, its state is handed on, and its entries (fewer) end
// the list.
__global__ void k_replay_write(WalkArgs W0, const u32* __restrict__ cand, const u32* __restrict__ nreal,
                               const u32* __restrict__ coff, ComposeMeta* meta, i32* __restrict__ pairs,
                               u64 pair_cap, u32* __restrict__ skiplist, u64* __restrict__ skipbits) {
  const WalkArgs W = walk_load(W0);
  if (blockIdx.x == 0 && threadIdx.x == 0) meta->n_conf = meta->nconf_in + meta->n_conf_loc;
  if (W.fail) return;
  const u64 nc = meta->n_cand;
  const u64 off0 = meta->nconf_in, soff0 = meta->nskip_in;
  for (u64 c = (u64)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (u64)gridDim.x * BLOCK) {
    if (nreal[c] == 0) continue;
    if (c < W.stage_cap && W.sok[c]) {  // k_replay_q's staged outputs: copies, no replay
      const u32 k = nreal[c];
      const u32* g = W.stage + c * RS_W;
      const u64 off = off0 + coff[c];
      u32* sk = skiplist + soff0 + 2 * (u64)coff[c];
      for (u32 i = 0; i < k; ++i)
        if (off + i < pair_cap) {
          pairs[2 * (off + i)] = (i32)g[2 * i];
          pairs[2 * (off + i) + 1] = (i32)g[2 * i + 1];
        }
      for (u32 i = 0; i < 2 * k; ++i) {
        const u32 m = g[2 * RS_CONF + i];
        sk[i] = m;
        atomicOr((unsigned long long*)&skipbits[m >> 6], 1ull << (m & 63));
      }
      atomicAdd((unsigned long long*)&meta->n_skip, (unsigned long long)(2 * k));
      continue;
    }
    u32 k = 0, ns = 0;
    ReplayState st = replay_fresh();
    replay_region<true, false>(W, cand[c], st, &k, pairs, pair_cap, off0 + coff[c],
                               skiplist + soff0 + 2 * (u64)coff[c], skipbits, &ns);
    if (st.d > 0) {
      meta->out_open = 1;
      meta->out_ahead = (u64)st.ahead;
      meta->out_d = st.d;
    }
    atomicAdd((unsigned long long*)&meta->n_skip, (unsigned long long)ns);
  }
}

// Sharded merge: the first `cap` renames of each branch in M order (symbol,
// newName class, global source) -- the previous shards' halo.  One block scans M.
#define EX_NT 1024
__global__ void __launch_bounds__(EX_NT) k_halo_export(WalkArgs W0, u32* __restrict__ xsym,
                                                       i32* __restrict__ xcls, i32* __restrict__ xsrc, u64 cap) {
  const WalkArgs W = walk_load(W0);
  if (W.fail) return;
  __shared__ u32 s[EX_NT / WAVE + 1];
  u64 got[2] = {0, 0};
  for (u64 m0 = 0; m0 < W.nR && (got[0] < cap || got[1] < cap); m0 += EX_NT) {
    const u64 m = m0 + threadIdx.x;
    const bool valid = m < W.nR;
    const int b = valid ? walk_side(W, m) : 0;
    u32 tot;
    const u32 rb = block_excl_scan<OpSum, u32, EX_NT / WAVE>(valid && b ? 1u : 0u, s, &tot);
    const u32 nvalid = (u32)min((u64)EX_NT, W.nR - m0);
    const u64 k = b ? got[1] + rb : got[0] + (u64)(threadIdx.x - rb);
    if (valid && k < cap) {
      const i32 j = W.tsrc[m];
      xsym[b * cap + k] = W.tsym[m];
      xcls[b * cap + k] = walk_cls_of_src(W, j);
      xsrc[b * cap + k] = walk_gsrc(W, j);
    }
    got[1] += tot;
    got[0] += nvalid - tot;
  }
}
