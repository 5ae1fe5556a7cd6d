// smx_small.h — a whole merge in one workgroup, for merges of at most SMALL_N ops (the
// CLI's merges: one op log per branch from a single diff, thousands of ops).
//
// The pipeline of the large merges (plan, windows, walk, tables, emit: ~25 launches)
// is latency, not work, at these sizes.  Here one 1024-thread workgroup holds the merge
// in LDS and runs the reference's composition (semmerge/compose.py:11-114) start to end:
//   1. T = the stable order of A||B by (precedence, timestamp, id, side, index)
//      (compose.py:16-21 sorted() per branch + the A-first merge :51-56).  Branch logs
//      whose timestamps do not decrease (lift.ts emits them so) are ordered in merged
//      runs of equal timestamps (a binary search in the other branch places each run;
//      interpolation buckets on the id order it), then split stably by precedence (wave
//      ballots per kind, one scan); logs in any other order, or ids whose top bits
//      cluster, take a bitonic sort of the op indices on the full key;
//   2. the DivergentRename walk (compose.py:60-70, 88-98) over the rename block of T:
//      the reference's two heads, restricted to renames (T is ordered by precedence
//      first, so both heads are renames exactly while both branches are in their rename
//      blocks); a conflict skips both heads and records (A-op, B-op).  Between two
//      conflicts the heads step through the rename block in T order, so one wave tests
//      the next 64 head pairs at once (each lane's pair from a prefix count of A's
//      renames) and jumps to the first conflict: one step per conflict or per 64 renames;
//   3. the chains (compose.py:27-28, 71-82, 99-110): per-symbol last writers in T order
//      in an LDS hash table on the symbol -- the final move address / file and the final
//      non-skipped rename; a move with a None value looks back for its symbol's last
//      non-None one (the inclusive prefix the reference's move_chain holds);
//   4. materialize (compose.py:30-49): each op of T that is not skipped, at T minus the
//      skips before it, with the ids it sees.
// Same outputs, same meta fields as smx_compose's large-merge path.
#pragma once

#include "smx_common.h"

#define SMALL_N 2048  // ops per merge
#define SMALL_NT 1024
#define SMALL_HT 4096  // hash slots (symbols), a power of two >= 2 * SMALL_N
#define SMALL_EMPTY 0xffffffffu
#define SMALL_BKT 32  // largest interpolation bucket ranked by counting (larger: bitonic sort)

#ifdef SMALL_STAMPS  // phase timestamps of the last call (diagnostic builds, tools/small_phases.py)
__device__ u64 g_small_stamp[16];
#define SMALL_STAMP(i) \
  do {                 \
    if (threadIdx.x == 0) g_small_stamp[i] = wall_clock64(); \
  } while (0)
#else
#define SMALL_STAMP(i) \
  do {                 \
  } while (0)
#endif

__global__ void __launch_bounds__(SMALL_NT) k_compose_small(smx_ops ops, smx_compose_out out, ComposeMeta* meta,
                                                                u64* hrec, u64 hseq) {
  constexpr int IT = SMALL_N / SMALL_NT;
  constexpr int NW = SMALL_NT / WAVE;
  // keys of the sort (dead after it: the hash table takes their place)
  __shared__ __attribute__((aligned(16))) u64 keys[3][SMALL_N];
  u64* kts = keys[0];
  u64* khi = keys[1];
  u64* klo = keys[2];
  __shared__ u8 skd[SMALL_N];     // kind by element
  __shared__ u16 ord[SMALL_N];    // T -> element
  __shared__ u16 mrg[SMALL_N];    // ordered logs: (ts, id, index) order -> element
  __shared__ u32 ssym[SMALL_N];   // by element
  __shared__ i32 sv0[SMALL_N], sv1[SMALL_N];
  __shared__ u8 skip[SMALL_N];    // by T: a rename the walk skipped
  __shared__ u16 rat[SMALL_N + 1];  // rename block: A's renames before T (1a, 1b: run ends)
  __shared__ u16 posA[SMALL_N], posB[SMALL_N];  // the i-th rename of a side: its T
  __shared__ u64 sn[SMALL_N];                   // rename block, by T: symbol << 32 | newName
                                                // (1b: bucket counts and fill)
  __shared__ u32 nxtA[SMALL_N + 1], nxtB[SMALL_N + 1];  // next rename of a side at or after T
  __shared__ u32 wcnt[SMX_N_KINDS * NW];          // per (kind, wave): ops, then their start
  __shared__ u32 sscan[NW + 1];
  __shared__ u32 sinfo[8];  // [2] nmv, [3] rend
  u32* hkey = reinterpret_cast<u32*>(keys[0]);              // [SMALL_HT] symbol of the slot
  u16* hw = reinterpret_cast<u16*>(keys[1]);                 // [3][SMALL_HT]: T + 1 of the last
                                                             // addr / file writer and of the
                                                             // last kept rename (0: none)
  static_assert(SMALL_HT * 4 <= SMALL_N * 8 && 3 * SMALL_HT * 2 <= 2 * SMALL_N * 8, "hash table in the keys");
  static_assert(SMX_N_KINDS * NW <= 5 * WAVE, "kind scan: 5 counters per lane");
  static_assert(sizeof(ComposeMeta) % 4 == 0 && sizeof(ComposeMeta) / 4 <= SMALL_NT, "meta zeroed one word per thread");
  const int t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  const i64 na = ops.n_a, nb = ops.n_b;
  const int n = (int)(na + nb);
  if (t < 8) sinfo[t] = 0;
  if (t < (int)(sizeof(ComposeMeta) / 4)) reinterpret_cast<u32*>(meta)[t] = 0u;
  SMALL_STAMP(0);
  // 1. load (B op j is stored at j + b_gap)
  u32 bad = 0;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int e = t + SMALL_NT * i;
    if (e < n) {
      const i64 j = e < na ? (i64)e : (i64)e + ops.b_gap;
      const u32 k = ops.kind[j], s = ops.sym[j];
      bad |= (k >= SMX_N_KINDS) | (s >= (u64)ops.n_sym);
      skd[e] = (u8)(k < SMX_N_KINDS ? k : SMX_N_KINDS - 1);
      kts[e] = ops.ts[j];
      khi[e] = ops.oid_hi[j];
      klo[e] = ops.oid_lo[j];
      ssym[e] = s;
      sv0[e] = ops.v0[j];
      sv1[e] = ops.v1[j];
    }
    skip[e] = 0;
    reinterpret_cast<u32*>(sn)[e] = 0u;  // (1b's bucket counts and fill)
    reinterpret_cast<u32*>(sn)[SMALL_N + e] = 0u;
  }
  if (__syncthreads_or(bad)) {  // invalid input: the call fails (as the large path: counts -1)
    if (t == 0) {
      meta->bad_sym = 1;
      out.counts[0] = -1;
      out.counts[1] = -1;
      if (hrec) *hrec = hseq << 1 | 1u;  // the verdict word (smx_compose's synchronous call)
    }
    return;
  }
  SMALL_STAMP(1);
  auto key_lt = [&](u32 x, u32 y) -> bool {  // (ts, id) of x < that of y
    if (kts[x] != kts[y]) return kts[x] < kts[y];
    if (khi[x] != khi[y]) return khi[x] < khi[y];
    return klo[x] < klo[y];
  };
  // 1a. the runs of equal timestamps of each branch (blocked: thread t holds ops IT t ..):
  //     a run's start from a max-scan of the start flags, its end stored at its start (in
  //     rat, free until step 2).  A decreasing timestamp sends the merge to the bitonic sort.
  bool slow = false;
  u32 rs[IT];
  {
    u32 mx = 0;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = t * IT + i;
      const bool first = e == 0 || e == (int)na;
      rs[i] = e < n && (first || kts[e] != kts[e - 1]) ? (u32)e : 0u;
      slow |= e < n && !first && kts[e] < kts[e - 1];
      mx = rs[i] > mx ? rs[i] : mx;
    }
    u32 tot;
    u32 run = block_excl_scan<OpMax, u32, NW>(mx, sscan, &tot);  // (syncs)
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = t * IT + i;
      run = rs[i] > run ? rs[i] : run;
      rs[i] = run;
      if (e < n && (e + 1 == n || e + 1 == (int)na || kts[e + 1] != kts[e])) rat[run] = (u16)(e + 1);
    }
    slow = __syncthreads_or(slow);
  }
  SMALL_STAMP(2);
  if (!slow) {
    // 1b. each op's merged run: the ops of both branches with its timestamp, which start at
    //     (own ops before its run) + (the other branch's ops with a smaller timestamp, by a
    //     binary search); inside it, interpolation buckets on the top 32 id bits (one op per
    //     bucket on random ids; counts in LDS, one scan), then each op ranks itself on
    //     (id, index) among its bucket's ops.  Ties: A before B = the lower index.
    u32* bcnt = reinterpret_cast<u32*>(sn);  // [SMALL_N] bucket counts, then starts
    u32* bfill = bcnt + SMALL_N;             // [SMALL_N] bucket fill
    u32 bk[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = t * IT + i;
      bk[i] = 0;
      if (e >= n) continue;
      const bool sa = e < (int)na;
      const u64 ts = kts[e];
      int lo = sa ? (int)na : 0, hi = sa ? n : (int)na;  // the other branch: first ts >= ours
      const int base = lo;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (kts[mid] < ts) lo = mid + 1;
        else hi = mid;
      }
      const u32 eq = lo < (sa ? n : (int)na) && kts[lo] == ts ? (u32)rat[lo] - (u32)lo : 0u;
      const u32 s0 = rs[i], len = (u32)rat[s0] - s0 + eq;
      const u32 m0 = (s0 - (sa ? 0u : (u32)na)) + (u32)(lo - base);
      bk[i] = m0 + (u32)(((u64)len * (u32)(khi[e] >> 32)) >> 32);
      atomicAdd(&bcnt[bk[i]], 1u);
    }
    __syncthreads();
    {
      u32 c[IT], a = 0;
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        c[i] = bcnt[t * IT + i];
        a += c[i];
      }
      u32 tot;
      u32 run = block_excl_scan<OpSum, u32, NW>(a, sscan, &tot);  // (syncs)
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        bcnt[t * IT + i] = run;
        run += c[i];
      }
    }
    __syncthreads();
    bool big = false;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = t * IT + i;
      if (e >= n) continue;
      const u32 b = bk[i], b0 = bcnt[b], b1 = b + 1 < (u32)SMALL_N ? bcnt[b + 1] : (u32)n;
      ord[b0 + atomicAdd(&bfill[b], 1u)] = (u16)e;
      big |= b1 - b0 > SMALL_BKT;
    }
    slow = __syncthreads_or(big);
    if (!slow) {
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int e = t * IT + i;
        if (e >= n) continue;
        const u32 b = bk[i], b0 = bcnt[b], b1 = b + 1 < (u32)SMALL_N ? bcnt[b + 1] : (u32)n;
        const u64 h = khi[e], l = klo[e];
        u32 r = 0;
        for (u32 q = b0; q < b1; ++q) {
          const u32 x = ord[q];
          const u64 hx = khi[x], lx = klo[x];
          r += hx < h || (hx == h && (lx < l || (lx == l && x < (u32)e)));
        }
        mrg[b0 + r] = (u16)e;
      }
    }
  }
  if (!slow) {
    __syncthreads();
    // 1d. stable split by kind: the rank inside the wave from one ballot pair per kind,
    //     the wave's start from a scan over (kind, wave)
    u32 k0, k1, r0 = 0, r1 = 0;
    {
      const int m = 2 * t;
      k0 = m < n ? skd[mrg[m]] : 0xffu;
      k1 = m + 1 < n ? skd[mrg[m + 1]] : 0xffu;
      const u64 lt = lanemask_lt();
#pragma unroll 1
      for (u32 k = 0; k < SMX_N_KINDS; ++k) {
        const u64 b0 = __ballot(k0 == k), b1 = __ballot(k1 == k);
        const u32 c = (u32)__popcll(b0 & lt) + (u32)__popcll(b1 & lt);
        if (k0 == k) r0 = c;
        if (k1 == k) r1 = c + (k0 == k);
        if (lane == 0) wcnt[k * NW + w] = (u32)__popcll(b0) + (u32)__popcll(b1);
      }
    }
    __syncthreads();
    if (w == 0) {
      u32 v[5], s = 0;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int x = 5 * lane + q;
        v[q] = x < SMX_N_KINDS * NW ? wcnt[x] : 0u;
        s += v[q];
      }
      u32 run = wave_incl_sum_u32(s) - s;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int x = 5 * lane + q;
        if (x < SMX_N_KINDS * NW) wcnt[x] = run;
        run += v[q];
      }
    }
    __syncthreads();
    if (2 * t < n) ord[wcnt[k0 * NW + w] + r0] = mrg[2 * t];
    if (2 * t + 1 < n) ord[wcnt[k1 * NW + w] + r1] = mrg[2 * t + 1];
  } else {
    // logs in any order: a bitonic sort of the op indices on the full key; elements
    // past n sort last (their slots are never read)
    auto less = [&](u32 x, u32 y) -> bool {  // x before y in T (x != y)
      if ((int)x >= n || (int)y >= n) return (int)y >= n && (int)x < n;
      if (skd[x] != skd[y]) return skd[x] < skd[y];
      if (kts[x] != kts[y]) return kts[x] < kts[y];
      if (khi[x] != khi[y]) return khi[x] < khi[y];
      if (klo[x] != klo[y]) return klo[x] < klo[y];
      return x < y;  // (side, index): A before B, then the branch index
    };
#pragma unroll
    for (int i = 0; i < IT; ++i) ord[t + SMALL_NT * i] = (u16)(t + SMALL_NT * i);
    __syncthreads();
    int P = 1;
    while (P < n) P <<= 1;
    for (int k = 2; k <= P; k <<= 1) {
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          const int a = t + SMALL_NT * i;
          const int b = a ^ jj;
          if (a < P && b > a) {
            const u32 x = ord[a], y = ord[b];
            const bool up = (a & k) == 0;
            if (up ? less(y, x) : less(x, y)) {
              ord[a] = (u16)y;
              ord[b] = (u16)x;
            }
          }
        }
        __syncthreads();
      }
    }
  }
  __syncthreads();
  SMALL_STAMP(3);
#ifdef SMALL_STAMPS
  if (t == 0) g_small_stamp[15] = slow;
#endif
  // the move block [0, nmv), the rename block [nmv, rend): at the kind boundaries
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int T = t * IT + i;
    if (T >= n) continue;
    const u32 k = skd[ord[T]], kn = T + 1 < n ? skd[ord[T + 1]] : 0xffu;
    if (k <= SMX_KIND_MOVE && kn > SMX_KIND_MOVE) sinfo[2] = (u32)T + 1u;
    if (k <= SMX_KIND_RENAME && kn > SMX_KIND_RENAME) sinfo[3] = (u32)T + 1u;
  }
  __syncthreads();
  const int nmv = (int)sinfo[2], rend = (int)sinfo[3];
  SMALL_STAMP(4);
  // 2. the rename lists of the two sides, in T order, and each rename's (symbol, newName)
  u32 isa[IT], acc = 0;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int T = t * IT + i;
    isa[i] = T >= nmv && T < rend && ord[T] < (u32)na;
    acc += isa[i];
  }
  u32 n_ren_a;
  u32 ra = block_excl_scan<OpSum, u32, NW>(acc, sscan, &n_ren_a);  // (syncs)
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int T = t * IT + i;
    if (T >= nmv && T <= rend) rat[T] = (u16)ra;
    if (T >= nmv && T < rend) {
      const u32 e = ord[T];
      sn[T] = (u64)ssym[e] << 32 | (u32)sv0[e];
      if (isa[i]) posA[ra] = (u16)T;
      else posB[T - nmv - (int)ra] = (u16)T;
    }
    ra += isa[i];
  }
  if (t == 0 && rend == n) rat[n] = (u16)n_ren_a;  // (T == n is no thread's)
  __syncthreads();
  // the next rename of each side at or after T: its position << 16 | its index
  const int nA = (int)__builtin_amdgcn_readfirstlane((int)n_ren_a), nB = rend - nmv - nA;
#pragma unroll
  for (int i = 0; i <= IT; ++i) {
    const int T = i < IT ? t * IT + i : n;
    if (T < nmv || T > rend || (i == IT && (t != 0 || rend != n))) continue;
    const int ia = rat[T], ib = T - nmv - ia;
    nxtA[T] = (u32)(ia < nA ? posA[ia] : rend) << 16 | (u32)ia;
    nxtB[T] = (u32)(ib < nB ? posB[ib] : rend) << 16 | (u32)ib;
  }
  __syncthreads();
  SMALL_STAMP(5);
  if (w == 0) {
    // the walk.  The heads (position << 16 | index in the side's list) are wave-uniform.
    // Lane k takes the heads after k steps without a conflict: the leading side's renames
    // before the other head first (its list, read ahead), then every rename of the block
    // in T order (the next renames of both sides at that position).
    u32 hA = (u32)__builtin_amdgcn_readfirstlane((int)nxtA[nmv]);
    u32 hB = (u32)__builtin_amdgcn_readfirstlane((int)nxtB[nmv]);
    u32 nc = 0;
    while ((int)(hA & 0xffffu) < nA && (int)(hB & 0xffffu) < nB) {
      const int pa = (int)(hA >> 16), pb = (int)(hB >> 16);
      const bool ldA = pa < pb;
      const int il = (int)((ldA ? hA : hB) & 0xffffu) + lane;
      const int cl = il < (ldA ? nA : nB) ? (int)(ldA ? posA[il] : posB[il]) : rend;
      const int other = ldA ? pb : pa;
      const int g = (int)__popcll(__ballot(cl < other));
      const int q = other + lane - g;
      const int qc = q < rend ? q : rend;
      const u32 xA2 = nxtA[qc], xB2 = nxtB[qc];
      const u32 xl = (u32)cl << 16 | (u32)il;
      const u32 xA = lane < g ? (ldA ? xl : hA) : xA2;
      const u32 xB = lane < g ? (ldA ? hB : xl) : xB2;
      const int pA = (int)(xA >> 16), pB = (int)(xB >> 16);
      const bool valid = (int)(xA & 0xffffu) < nA && (int)(xB & 0xffffu) < nB;
      const u64 sa = sn[valid ? pA : nmv], sb = sn[valid ? pB : nmv];
      // the heads after a conflict here, and its ops: loaded beside the pair (the compiler
      // would sink them into the conflict branch, one more LDS round trip there)
      u32 nA1 = nxtA[valid ? pA + 1 : rend], nB1 = nxtB[valid ? pB + 1 : rend];
      u32 oA = ord[valid ? pA : 0], oB = ord[valid ? pB : 0];
      asm volatile("" : "+v"(nA1), "+v"(nB1), "+v"(oA), "+v"(oB));
      const bool conf = valid && (sa >> 32) == (sb >> 32) && (u32)sa != (u32)sb;
      // after a conflict here, are both heads past this pair?  Then the walk goes on at
      // the merged state of position max + 1, which a later lane already holds: the wave
      // follows a run of conflicts with scalar steps over the ballots, not one pass each
      const int pmax = pA > pB ? pA : pB;
      const bool jmp = (nA1 >> 16) > (u32)pmax && (nB1 >> 16) > (u32)pmax;
      const u64 cm = __ballot(conf), im = __ballot(!valid), jm = __ballot(jmp);
      const int knl = g + (pmax + 1 - other);  // the lane of position max + 1
      u64 rec = 0;  // the lanes whose pair conflicts on this pass, in walk order
      int k = 0;
      bool done = false;
      while (true) {
        const u64 ge = ~0ull << k;  // (k < WAVE)
        const int jc = (cm & ge) ? __builtin_ctzll(cm & ge) : WAVE;
        const int ji = (im & ge) ? __builtin_ctzll(im & ge) : WAVE;
        if (jc < ji) {
          rec |= 1ull << jc;
          const int kn = __builtin_amdgcn_readlane(knl, jc);
          if (((jm >> jc) & 1) && kn < WAVE) {
            k = kn;
            continue;
          }
          hA = (u32)__builtin_amdgcn_readlane((int)nA1, jc);
          hB = (u32)__builtin_amdgcn_readlane((int)nB1, jc);
        } else if (ji < WAVE) {
          done = true;
        } else {
          hA = (u32)__builtin_amdgcn_readlane((int)xA, WAVE - 1);
          hB = (u32)__builtin_amdgcn_readlane((int)xB, WAVE - 1);
        }
        break;
      }
      if ((rec >> lane) & 1) {  // the pass's conflicts, each by its own lane
        const u32 ci = nc + (u32)__popcll(rec & lanemask_lt());
        if ((i64)ci < out.conflict_cap) {
          out.conflicts[2 * ci] = (i32)oA;
          out.conflicts[2 * ci + 1] = (i32)oB;
        }
        skip[pA] = 1;
        skip[pB] = 1;
      }
      nc += (u32)__popcll(rec);
      if (done) break;
    }
    if (lane == 0) {
      out.counts[0] = (i64)(n - 2 * (int)nc);
      out.counts[1] = (i64)nc;
      meta->n_conf = nc;
      meta->n_skip = 2 * nc;
      if (hrec) *hrec = hseq << 1;  // read after the stream wait: the kernel's end publishes it
    }
    SMALL_STAMP(6);
  }
  // the keys are dead: the hash table takes their LDS
  for (int i = t; i < SMALL_HT; i += SMALL_NT) {
    hkey[i] = SMALL_EMPTY;
    hw[i] = hw[SMALL_HT + i] = hw[2 * SMALL_HT + i] = 0;
  }
  __syncthreads();
  SMALL_STAMP(7);
  // 3. the chains: every op's symbol slot (moves and renames insert, the rest look up)
  auto slot_of = [&](u32 s, bool ins) -> int {
    u32 h = (s * 2654435761u) >> (32 - 12);
    for (int probe = 0; probe < SMALL_HT; ++probe, h = (h + 1) & (SMALL_HT - 1)) {
      const u32 cur = hkey[h];
      if (cur == s) return (int)h;
      if (cur == SMALL_EMPTY) {
        if (!ins) return -1;
        const u32 old = atomicCAS(&hkey[h], SMALL_EMPTY, s);
        if (old == SMALL_EMPTY || old == s) return (int)h;
      }
    }
    return -1;  // (unreachable: at most SMALL_N symbols in SMALL_HT slots)
  };
  int slot_r[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int T = t + SMALL_NT * i;
    slot_r[i] = -1;
    if (T >= rend) continue;
    slot_r[i] = slot_of(ssym[ord[T]], true);
  }
  __syncthreads();
  SMALL_STAMP(8);
  // last writers: T + 1 packed in u16 (T < SMALL_N); an atomic max on a u16 is emulated
  // with a CAS loop on its 32-bit word
  auto max16 = [&](u16* base, int h, u32 v) {
    u32* wd = reinterpret_cast<u32*>(base) + (h >> 1);
    const u32 sh = 16u * (u32)(h & 1);
    u32 old = *wd;
    while (((old >> sh) & 0xffffu) < v) {
      const u32 nw = (old & ~(0xffffu << sh)) | (v << sh);
      const u32 got = atomicCAS(wd, old, nw);
      if (got == old) break;
      old = got;
    }
  };
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int T = t + SMALL_NT * i;
    if (slot_r[i] < 0) continue;
    const u32 e = ord[T];
    if (T < nmv) {
      if (sv0[e] >= 0) max16(hw, slot_r[i], (u32)T + 1u);
      if (sv1[e] >= 0) max16(hw + SMALL_HT, slot_r[i], (u32)T + 1u);
    } else if (!skip[T]) {  // a kept rename (compose.py:71-72)
      max16(hw + 2 * SMALL_HT, slot_r[i], (u32)T + 1u);
    }
  }
  // The moves' inclusive prefixes (compose.py:73-82), only when a move has a None value:
  // one wave walks the move block in T order, 64 moves a step.  A move's last earlier
  // non-None writer of its symbol is the highest earlier lane of the step with its slot
  // and a value (peers ballots), else the slot's running writer; the step's last writer
  // per slot then becomes the running one.  O(moves / 64) steps, whatever the values.
  u16* pwa = posA;  // by T: T' + 1 of the move's prefix addr / file writer (0: none);
  u16* pwf = posB;  // (posA / posB are dead after the walk)
  u16* la = reinterpret_cast<u16*>(sn);  // by slot: the running writers (sn is dead after
  u16* lf = la + SMALL_HT;               // the walk; klo is not: hw's third table lies in it)
  static_assert(2 * SMALL_HT * 2 <= SMALL_N * 8, "running writers in sn");
  bool none_here = false;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int T = t + SMALL_NT * i;
    if (T < nmv) none_here |= (sv0[ord[T]] < 0) | (sv1[ord[T]] < 0);
  }
  const bool any_none = __syncthreads_or(none_here);  // (also orders the last-writer maxes)
  if (any_none) {
    for (int i = t; i < SMALL_HT; i += SMALL_NT) la[i] = lf[i] = 0;
    __syncthreads();
    if (w == 0) {
      const u64 lt = lanemask_lt();
      for (int c0 = 0; c0 < nmv; c0 += WAVE) {
        const int T = c0 + lane;
        const bool v = T < nmv;
        const u32 e = v ? ord[T] : 0u;
        const int h = v ? slot_of(ssym[e], false) : 0;  // (every move inserted its slot)
        const bool ha = v && sv0[e] >= 0, hf = v && sv1[e] >= 0;
        const u64 peers = wave_peers_n((u32)h, v, 12);
        const u64 pa = __ballot(ha) & peers, pf = __ballot(hf) & peers;
        const u32 ra = v ? la[h] : 0u, rf = v ? lf[h] : 0u;  // (read before the step's updates)
        if (v) {
          pwa[T] = (u16)((pa & lt) ? (u32)(c0 + 63 - __clzll(pa & lt)) + 1u : ra);
          pwf[T] = (u16)((pf & lt) ? (u32)(c0 + 63 - __clzll(pf & lt)) + 1u : rf);
        }
        __builtin_amdgcn_wave_barrier();
        if (ha && (pa >> lane) == 1ull) la[h] = (u16)(T + 1);
        if (hf && (pf >> lane) == 1ull) lf[h] = (u16)(T + 1);
        wave_lds_sync();
      }
    }
    __syncthreads();
  }
  // skips before each T (renames only): exclusive scan of the skip flags, IT per thread
  u32 sk[IT];
  acc = 0;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    sk[i] = (t * IT + i) < n ? skip[t * IT + i] : 0u;
    acc += sk[i];
  }
  u32 tot;
  const u32 sbase = block_excl_scan<OpSum, u32, NW>(acc, sscan, &tot);  // (syncs)
  SMALL_STAMP(9);
  // 4. materialize: T -> T - skips before it
  u32 run = sbase;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int T = t * IT + i;
    const u32 before = run;
    run += sk[i];
    if (T >= n || sk[i]) continue;
    const u32 e = ord[T];
    const u32 k = skd[e], s = ssym[e];
    i32 a = SMX_NONE, f = SMX_NONE, c = SMX_NONE;
    if (T < nmv) {
      // the inclusive prefix of the symbol's moves: its own value, else the last earlier
      // non-None one (compose.py:73-82 then 37-41)
      a = sv0[e];
      f = sv1[e];
      if (a < 0 && pwa[T]) a = sv0[ord[pwa[T] - 1]];  // (any_none: a None value was seen)
      if (f < 0 && pwf[T]) f = sv1[ord[pwf[T] - 1]];
    } else {
      const int h = slot_of(s, false);
      if (h >= 0) {
        const u32 wa = hw[h], wf = hw[SMALL_HT + h], wr = hw[2 * SMALL_HT + h];
        if (wa) a = sv0[ord[wa - 1]];
        if (wf) f = sv1[ord[wf - 1]];
        if (k != SMX_KIND_RENAME && wr) c = sv1[ord[wr - 1]];  // renameContext: non-renames only
      }
    }
    const u32 o = (u32)T - before;
    out.order[o] = (i32)e;
    out.addr[o] = a;
    out.file[o] = f;
    out.ctx[o] = c;
  }
#ifdef SMALL_STAMPS
  __syncthreads();
  SMALL_STAMP(10);
#endif
}
