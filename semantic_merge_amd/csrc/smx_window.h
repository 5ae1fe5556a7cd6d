// smx_window.h — per-window T-order construction (the dominant kernel).
//
// T = stable order of A||B by (precedence, timestamp, id, side, index)
// (semmerge/compose.py:16-21 sorted() per branch + the A-first merge of :51-56).
// A window is a pair of contiguous ranges, one per branch, such that every op of
// the window precedes, in (timestamp, id, side, index) order, every op of the
// next window.  Inside one window (all in LDS):
//   1. merge the A part and the B part by timestamp (A first on ties)   -> S
//   2. stable multisplit of S by precedence rank (wave64 ballots)       -> slots
//   3. equal-(rank, timestamp) groups are contiguous slot ranges; order each by
//      (id, side, index) with a counting rank over the group
//   4. T position = base[rank] + (ops of that rank in earlier windows) + local
// The presorted kernel (k_window_f) handles branch logs whose timestamps never
// decrease (lift.ts emits them in order); k_window_g handles branch logs that the
// generic path pre-sorted by (timestamp, id), where step 3 is not needed.
#pragma once

#include "smx_common.h"

#define WIN_CAP 2048               // max ops per window held in LDS
#define WIN_TGT 1792               // default target window size, presorted path (SMX_WIN_TGT)
#define WIN_TGT_MIN 256
#define NCNT (SMX_N_KINDS + 3)     // kinds, renames per branch, moves with a None value
#define CNT_REN_A SMX_N_KINDS
#define CNT_REN_B (SMX_N_KINDS + 1)
#define CNT_NONE_MV (SMX_N_KINDS + 2)
#define KMOVE SMX_KIND_MOVE
#define KREN SMX_KIND_RENAME
#define NCHUNK (WIN_CAP / WAVE)
#define CH 256                     // chunk of the presorted kind histogram
#ifndef SMX_KEY64
#define SMX_KEY64 1                // group-rank keys: 0 = 21-bit id prefix (u32), 1 = 42-bit (u64)
#endif
#ifndef SMX_LATE_PAYLOAD
#define SMX_LATE_PAYLOAD 0         // 1: load sym/v0/v1 after the rank phase
#endif
#if SMX_KEY64
typedef u64 rkey_t;
#define RK_PREFIX_SHIFT 22         // hi >> 22: top 42 bits of oid_hi
#else
typedef u32 rkey_t;
#define RK_PREFIX_SHIFT 43         // top 21 bits of oid_hi
#endif
#define RK_PER16 (16 / (int)sizeof(rkey_t))   // keys per 16-byte LDS read
#ifndef RK_NRD
#define RK_NRD (SMX_KEY64 ? 4 : 2)           // 16-byte reads per rank-loop step
#endif

// Number of keys < kp among the first m (<= RK_PER16) keys of a 16-byte LDS read.
__device__ __forceinline__ int rk_count(const uint4 x, u32 kp, int m) {
  return (m > 0 && x.x < kp) + (m > 1 && x.y < kp) + (m > 2 && x.z < kp) + (m > 3 && x.w < kp);
}
__device__ __forceinline__ int rk_count(const ulonglong2 x, u64 kp, int m) {
  return (m > 0 && x.x < kp) + (m > 1 && x.y < kp);
}
__device__ __forceinline__ int rk_count(const uint4 x, u32 kp) {
  return (x.x < kp) + (x.y < kp) + (x.z < kp) + (x.w < kp);
}
__device__ __forceinline__ int rk_count(const ulonglong2 x, u64 kp) { return (x.x < kp) + (x.y < kp); }
#if SMX_KEY64
typedef ulonglong2 rkey16_t;
#else
typedef uint4 rkey16_t;
#endif

struct WinArgs {
  const u8* kind;
  const u32* sym;
  const i32* v0;
  const i32* v1;
  // branch view: presorted -> keys at op index j; generic -> sorted copies at j
  const u64* kts;
  const u64* khi;
  const u64* klo;
  const u32* perm;  // generic only: op index of sorted position (A at [0,na), B at [na,n))
  i64 na;
  i64 nb;
  i64 bgap;         // B op j is stored at j + bgap of the field arrays (presorted plan)
  i64 W;
  i64 n_sym;
  int ablate;       // diagnostics only (SMX_ABLATE): skip phases, results invalid
  const i64* bnd;
  const u32* woff;  // [NCNT][W] exclusive offsets over windows (generic plan)
  const u32* cpre;  // presorted plan: [2][kinds][CM] chunk prefixes (256-op chunks)
  i64 CM;
  ComposeMeta* meta;
  i32* order;
  u32* symT;
  i32* mvA;
  i32* mvF;
  u32* Msym;
  i32* Mcls;
  i32* Mstr;
  u8* Mside;
  u32* Mown;
  u32* RA;
  u32* RB;
  u64* dbg;         // diagnostics only: phase timestamps (k_window_f<true>)
};

// Writes one op's T-ordered records (registers -> HBM).
__device__ __forceinline__ void win_emit(const WinArgs& P, const u64* base, i64 w, u32 k, u32 x,
                                         u32 kb, u32 src, u32 s, i32 a, i32 f, int side, u32 own) {
  const u64 T = base[k] + P.woff[(i64)k * P.W + w] + (x - kb);
  // Bounds guards: only a failed (and later discarded) presorted plan can trip them.
  if (T >= (u64)(P.na + P.nb) || own >= (u64)(side ? P.nb : P.na)) return;
  P.order[T] = (i32)src;
  P.symT[T] = s;
  if (k == KMOVE) {
    P.mvA[T] = a;
    P.mvF[T] = f;
  } else if (k == KREN) {
    const u64 m = T - base[KREN];
    P.Msym[m] = s;
    P.Mcls[m] = a;
    P.Mstr[m] = f;
    P.Mside[m] = (u8)side;
    P.Mown[m] = own;
    (side ? P.RB : P.RA)[own] = (u32)m;
  }
}

// ---------------------------------------------------------------------------
// presorted windows (timestamps non-decreasing in each branch log)

#define WF_NT 512
#define WF_WAVES (WF_NT / WAVE)
#define WF_ITEMS (WIN_CAP / WF_NT)

// LDS ~34 KB (buffers are reused across phases) so 4 workgroups fit a CU: while
// some workgroups run their LDS phases, others stream their windows from HBM.
// DBG: phase timestamps of every window (diagnostics, tools/window_phases.py):
// lane 0 of wave 0 stores s_memtime after each phase into P.dbg[w * WF_NSTAMP + i].
#define WF_NSTAMP 24
#define WSTAMP(i)                                                                  \
  do {                                                                             \
    if (DBG && t == 0) P.dbg[w * WF_NSTAMP + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

template <bool DBG>
__global__ void __launch_bounds__(WF_NT, 8) k_window_f(WinArgs P) {
  __shared__ __attribute__((aligned(16))) u64 sts[WIN_CAP];  // element space: timestamps; later slot-space rank keys
  __shared__ u16 sord[WIN_CAP];       // S order (merge), later the final order
  __shared__ u16 fin[WIN_CAP];        // slot -> element, later rename ranks
  __shared__ u16 sl[WIN_CAP];         // element -> slot, later rank -> slot
  __shared__ u8 skind[WIN_CAP];
  __shared__ u8 srank[WIN_CAP];
  __shared__ u64 gbits[NCHUNK];       // group-start bits over slots
  __shared__ u16 ccnt[NCHUNK][SMX_N_KINDS];
  __shared__ u16 rc[NCHUNK][2];
  __shared__ u32 kbase[SMX_N_KINDS + 1];
  __shared__ u32 wck[SMX_N_KINDS];
  __shared__ u64 base[SMX_N_KINDS + 1];
  __shared__ u32 woffk[SMX_N_KINDS + 2];  // this window's offsets: kinds, renames of A, of B
  rkey_t* pkey = (rkey_t*)sts;        // slot space: rank keys (after step 4)
  u16* rown = fin;                    // rename rank within its branch (after step 5)

  const int t = threadIdx.x;
  const int lane = t & (WAVE - 1);
  const int wv = t / WAVE;
  const i64 w = blockIdx.x;
  const i64 a0 = P.bnd[2 * w], b0 = P.bnd[2 * w + 1];
  const int na = (int)(P.bnd[2 * w + 2] - a0);
  const int nb = (int)(P.bnd[2 * w + 3] - b0);
  const int sz = na + nb;
  if (na < 0 || nb < 0 || sz > WIN_CAP) {  // the presorted plan does not hold
    // bit 0: branch logs not timestamp-ordered; bit 1: window too large for LDS;
    // bit 2: ... and it holds one timestamp only, so smaller windows cannot help
    if (threadIdx.x == 0) {
      u64 f = 1;
      if (na >= 0 && nb >= 0) {
        const u64* A = P.kts + a0;
        const u64* B = P.kts + P.na + P.bgap + b0;
        const u64 v = na ? A[0] : B[0];
        const bool one = (!na || (A[0] == v && A[na - 1] == v)) && (!nb || (B[0] == v && B[nb - 1] == v));
        f = one ? 6 : 2;
      }
      atomicOr((unsigned long long*)&P.meta->f_fail, (unsigned long long)f);
    }
    return;
  }
  if (sz == 0) return;
  const i64 bpos = P.na + b0 - na;  // op index of B element e is bpos + e
  const i64 bld = bpos + P.bgap;    // ... stored at field index bld + e
  WSTAMP(0);

  // 1. load the sort keys (kind, timestamp, top of the id) to LDS.  The payload
  //    (sym, v0, v1) is loaded after the rank phase, so its HBM latency overlaps
  //    the later LDS phases and it holds no registers across the rank loop.
  u64 hi_r[WF_ITEMS];
  u32 sym_r[WF_ITEMS];
  i32 v0_r[WF_ITEMS], v1_r[WF_ITEMS];
  u32 k_r[WF_ITEMS];
  bool bad = false;
  // all loads are issued unconditionally (clamped to a valid op) so that the
  // loads of a lane are in flight together; the guards apply to the LDS stores only
  u64 ts_r[WF_ITEMS];
  auto op_index = [&](int e) -> i64 {
    const int ec = e < sz ? e : 0;
    return ec < na ? a0 + ec : bld + ec;
  };
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const i64 j = op_index(t + WF_NT * i);
    k_r[i] = P.kind[j];
    ts_r[i] = P.kts[j];
    hi_r[i] = P.khi[j];
#if !SMX_LATE_PAYLOAD
    sym_r[i] = P.sym[j];
    v0_r[i] = P.v0[j];
    v1_r[i] = P.v1[j];
#endif
  }
  auto load_payload = [&]() {
    if (!SMX_LATE_PAYLOAD) return;
#pragma unroll
    for (int i = 0; i < WF_ITEMS; ++i) {
      // opaque element index: the compiler must not keep the key loads' 64-bit
      // addresses alive (in registers or scratch) across the LDS phases
      int e = t + WF_NT * i;
      asm volatile("" : "+v"(e));
      const i64 j = op_index(e);
      sym_r[i] = P.sym[j];
      v0_r[i] = P.v0[j];
      v1_r[i] = P.v1[j];
    }
  };
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e < sz) {
      bad |= k_r[i] >= SMX_N_KINDS;
      k_r[i] = k_r[i] < SMX_N_KINDS ? k_r[i] : SMX_N_KINDS - 1;
      sts[e] = ts_r[i];
      skind[e] = (u8)k_r[i];
    }
  }
  // kinds of the <= 255 ops between each branch's chunk start and the window start
  // (window offsets below); lanes 0..255 branch A, 256..511 branch B
  u32 kpart = 0xffffffffu;
  {
    const int pa = (int)(a0 % CH), pb = (int)(b0 % CH);
    const int side = t >= CH;
    const int q = t - side * CH;
    if (q < (side ? pb : pa)) kpart = P.kind[side ? (P.na + P.bgap + b0 - pb + q) : (a0 - pa + q)];
  }
  // timestamps just before the window on each branch (issued with the loads above)
  u64 prev_a = 0, prev_b = 0;
  if (t == 0 && a0 > 0) prev_a = P.kts[a0 - 1];
  if (t == 0 && b0 > 0) prev_b = P.kts[P.na + P.bgap + b0 - 1];
  if (bad) P.meta->bad_sym = 1;
  for (int i = t; i < NCHUNK * SMX_N_KINDS; i += WF_NT) (&ccnt[0][0])[i] = 0;
  if (t <= SMX_N_KINDS) base[t] = P.meta->base[t];
  if (t < SMX_N_KINDS) wck[t] = 0;
  // window offsets = chunk prefix at the window start + kinds of the <= 255 ops
  // between that chunk start and the window start (per branch)
  if (t < SMX_N_KINDS) {
    woffk[t] = P.cpre[(i64)t * P.CM + a0 / CH] + P.cpre[(i64)(SMX_N_KINDS + t) * P.CM + b0 / CH];
  } else if (t < SMX_N_KINDS + 2) {
    const int sd = t - SMX_N_KINDS;
    woffk[t] = P.cpre[(i64)(sd * SMX_N_KINDS + KREN) * P.CM + (sd ? b0 : a0) / CH];
  }
  __syncthreads();
  WSTAMP(1);
  // window offsets: the partial-chunk kinds; presorted-layout check: every adjacent
  // pair of each branch log is non-decreasing (the pair straddling a window start
  // is checked here too); moves with a None value are counted for the prefix fix-up
  if (kpart != 0xffffffffu) {
    const u32 k = kpart < SMX_N_KINDS ? kpart : SMX_N_KINDS - 1;
    atomicAdd(&woffk[k], 1u);
    if (k == KREN) atomicAdd(&woffk[SMX_N_KINDS + (t >= CH)], 1u);
  }
  if (P.ablate & 8) {  // load + write only
    load_payload();
    __syncthreads();
#pragma unroll
    for (int i = 0; i < WF_ITEMS; ++i) {
      const int e = t + WF_NT * i;
      if (e >= sz) continue;
      const u32 src = (u32)(e < na ? a0 + e : bpos + e);
      win_emit(P, base, w, k_r[i], (u32)e, 0, src, sym_r[i], v0_r[i], v1_r[i], e >= na, 0);
    }
    return;
  }

  // 2. merge A part [0,na) with B part [na,sz) by timestamp, A first on ties:
  //    merge path, WF_ITEMS outputs per lane.  (Per-element rank searches, four
  //    interleaved binary searches per lane, measured 2-3x slower: LDS-bound.)
  //    Shares its barrier with the layout check: a window that fails the check
  //    discards the merge.
  bool dec = false;
  if (t == 0) dec = (a0 > 0 && na > 0 && prev_a > ts_r[0]) || (b0 > 0 && nb > 0 && prev_b > sts[na]);
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e >= sz) continue;
    if (!(P.ablate & 1) && e != 0 && e != na && sts[e - 1] > ts_r[i]) dec = true;
  }
  {
    const int d0 = t * WF_ITEMS < sz ? t * WF_ITEMS : sz;
    const int d1 = d0 + WF_ITEMS < sz ? d0 + WF_ITEMS : sz;
    int lo = d0 - nb > 0 ? d0 - nb : 0, hi = d0 < na ? d0 : na;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sts[mid] <= sts[na + d0 - 1 - mid]) lo = mid + 1;
      else hi = mid;
    }
    int ia = lo, ib = d0 - lo;
    for (int d = d0; d < d1; ++d) {
      const bool take_a = ia < na && (ib >= nb || sts[ia] <= sts[na + ib]);
      sord[d] = (u16)(take_a ? ia++ : na + ib++);
    }
  }
  if (__syncthreads_or(dec)) {
    if (t == 0) atomicOr((unsigned long long*)&P.meta->f_fail, 1ull);
    return;
  }
  WSTAMP(20);
  WSTAMP(3);

  // 3. stable multisplit of S by rank (wave ballots); element, kind and rank stay in
  //    registers for the scatter (m = t + WF_NT * j is chunk wv + WF_WAVES * j)
  const int nch = (sz + WAVE - 1) / WAVE;
  int me[WF_ITEMS];
  u32 mkr[WF_ITEMS];  // kind | rank << 8
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) {
    const int m = t + WF_NT * j;
    me[j] = m < sz ? sord[m] : 0;
  }
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) mkr[j] = t + WF_NT * j < sz ? skind[me[j]] : 0u;
  const u64 ltm = lanemask_lt();
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) {
    const int m = t + WF_NT * j;
    const int c = wv + WF_WAVES * j;
    const bool valid = m < sz;
    const u32 k = mkr[j];
    const u64 peers = wave_peers<5>(k, valid);
    const u32 r = __popcll(peers & ltm);
    mkr[j] = k | (r << 8);
    if (valid && r == 0) {
      ccnt[c][k] = (u16)__popcll(peers);
      atomicAdd(&wck[k], (u32)__popcll(peers));
    }
  }
  __syncthreads();
  WSTAMP(4);
  for (int k = wv; k < SMX_N_KINDS; k += WF_WAVES) {
    const u32 x = lane < nch ? ccnt[lane][k] : 0u;
    const u32 inc = wave_incl_sum(x);
    if (lane < nch) ccnt[lane][k] = (u16)(inc - x);
  }
  if (wv == WF_WAVES - 1) {  // (kinds 7 and 15 only on this wave)
    const u32 x = lane < SMX_N_KINDS ? wck[lane] : 0u;
    const u32 inc = wave_incl_sum(x);
    if (lane < SMX_N_KINDS) kbase[lane] = inc - x;
    if (lane == SMX_N_KINDS - 1) kbase[SMX_N_KINDS] = inc;
  }
  __syncthreads();
  WSTAMP(5);
  WSTAMP(6);
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) {
    const int m = t + WF_NT * j;
    if (m < sz) {
      const u32 k = mkr[j] & 0xffu;
      const int p = kbase[k] + ccnt[wv + WF_WAVES * j][k] + (mkr[j] >> 8);
      fin[p] = (u16)me[j];
      sl[me[j]] = (u16)p;
    }
  }
  __syncthreads();
  WSTAMP(7);

  // 4. group-start bits (a group = equal (rank, timestamp), contiguous in slots),
  //    then the timestamps are dead and their buffer takes the slot-space oid prefix
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) {
    const int p = t + WF_NT * j;
    bool f = false;
    if (p < sz) {
      const int e = fin[p];
      f = (p == (int)kbase[skind[e]]) || (sts[fin[p - 1]] != sts[e]);
    }
    const u64 b = __ballot(f);
    if (lane == 0 && (p >> 6) < NCHUNK) gbits[p >> 6] = b;
  }
  __syncthreads();
  WSTAMP(8);
  // slot-space rank keys: a prefix of oid_hi, then the slot (unique per window)
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e < sz) {
      const int p = sl[e];
      pkey[p] = ((rkey_t)(hi_r[i] >> RK_PREFIX_SHIFT) << 11) | (rkey_t)p;
    }
  }
  __syncthreads();
  WSTAMP(9);

  // 5. order each group by (oid, side, index).  Counting rank on 32-bit keys (21-bit
  //    oid prefix, slot), four per LDS read; slot order is (side, index) order inside
  //    a group.  If two adjacent ranks share the prefix (about 1 window in 100 on
  //    random ids; always for duplicate ids) the window is re-ranked exactly on the
  //    full oid.
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) {
    const int p = t + WF_NT * j;
    if (p >= sz) break;
    int r = p;
    const int bit = p & 63;
    int wi = p >> 6;
    u64 word = gbits[wi] & (bit == 63 ? ~0ull : ((1ull << (bit + 1)) - 1));
    while (word == 0) word = gbits[--wi];
    const int gs = wi * 64 + 63 - __clzll(word);
    wi = p >> 6;
    word = bit == 63 ? 0ull : (gbits[wi] & ~((1ull << (bit + 1)) - 1));
    while (word == 0 && ++wi < nch) word = gbits[wi];
    int ge = word ? wi * 64 + __ffsll((unsigned long long)word) - 1 : sz;
    ge = ge < sz ? ge : sz;
    if (ge - gs > 1 && !(P.ablate & 2)) {
      const rkey_t kp = pkey[p];
      const rkey16_t* pv = reinterpret_cast<const rkey16_t*>(pkey);
      constexpr int K = RK_PER16;
      const int q0 = gs & ~(K - 1);
      int c = 0;
      int q = q0;
      // RK_NRD x 16 bytes of keys per step: independent LDS reads in flight
      constexpr int NR = RK_NRD;
      for (; q + NR * K <= ge; q += NR * K) {
        rkey16_t x[NR];
#pragma unroll
        for (int u = 0; u < NR; ++u) x[u] = pv[q / K + u];
#pragma unroll
        for (int u = 0; u < NR; ++u) c += rk_count(x[u], kp);
      }
#pragma unroll
      for (int u = 0; u < NR; ++u) {  // fewer left: up to NR more reads, masked
        const int qq = q + K * u;
        if (qq < ge) c += rk_count(pv[qq / K], kp, ge - qq);
      }
      if (q0 < gs) c -= rk_count(pv[q0 / K], kp, gs - q0);  // slots before the group
      r = gs + c;
    }
    sord[r] = fin[p];
    sl[r] = (u16)p;  // sl now maps rank -> slot
  }
  load_payload();
  __syncthreads();
  WSTAMP(10);
  // Ranks are exact unless two elements of a group share the key prefix: then
  // they sit at adjacent ranks in slot order.  Such runs (rare on random ids;
  // every duplicate id) are re-sorted on the full oid, stably.
  auto run_next = [&](int r) -> bool {  // rank r + 1 continues r's prefix run
    const int r1 = r + 1;
    if (r1 >= sz || ((gbits[r1 >> 6] >> (r1 & 63)) & 1ull)) return false;  // next group
    return (pkey[sl[r]] >> 11) == (pkey[sl[r1]] >> 11);
  };
  // 6. renames: rank among the window's renames of the same branch (final order).
  //    Computed in the tie-detection phase; redone after a (rare) tie fix.
  const int R0 = kbase[KREN], RN = wck[KREN];
  const int nrc = (RN + WAVE - 1) / WAVE;
  auto rename_ranks = [&]() {
    for (int c = wv; c < nrc; c += WF_WAVES) {
      const int x = c * WAVE + lane;
      const bool valid = x < RN;
      const int e = valid ? sord[R0 + x] : 0;
      const bool sb = valid && e >= na;
      const u64 bm = __ballot(sb), vm = __ballot(valid);
      const u64 lt = lanemask_lt();
      if (valid) rown[x] = (u16)(sb ? __popcll(bm & lt) : __popcll(vm & ~bm & lt));
      if (lane == 0) {
        rc[c][0] = (u16)__popcll(vm & ~bm);
        rc[c][1] = (u16)__popcll(bm);
      }
    }
  };
  bool tie = false;
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) {  // detection: prefixes of adjacent ranks (any group)
    const int r = t + WF_NT * j;
    if (r + 1 < sz) tie |= (pkey[sl[r]] >> 11) == (pkey[sl[r + 1]] >> 11);
  }
  rename_ranks();
  const bool any_tie = __syncthreads_or(tie);
  WSTAMP(21);
  if (any_tie) {
    for (int r0 = t; r0 + 1 < sz; r0 += WF_NT) {
      if (!run_next(r0) || (r0 > 0 && run_next(r0 - 1))) continue;  // not a run start
      int r1 = r0 + 1;
      while (run_next(r1)) ++r1;
      // insertion sort of sord[r0..r1] by (oid_hi, oid_lo); equal ids keep slot order
      for (int x = r0 + 1; x <= r1; ++x) {
        const int ex = sord[x];
        const i64 jx = ex < na ? a0 + ex : bld + ex;
        const u64 hx = P.khi[jx], lx = P.klo[jx];
        int y = x - 1;
        while (y >= r0) {
          const int ey = sord[y];
          const i64 jy = ey < na ? a0 + ey : bld + ey;
          const u64 hy = P.khi[jy], ly = P.klo[jy];
          if (hy < hx || (hy == hx && ly <= lx)) break;
          sord[y + 1] = (u16)ey;
          --y;
        }
        sord[y + 1] = (u16)ex;
      }
    }
    __syncthreads();
    rename_ranks();
    __syncthreads();
  }
  WSTAMP(11);
  if (wv == 0) {
    const u32 x0 = lane < nrc ? rc[lane][0] : 0u;
    const u32 x1 = lane < nrc ? rc[lane][1] : 0u;
    const u32 i0 = wave_incl_sum(x0), i1 = wave_incl_sum(x1);
    if (lane < nrc) {
      rc[lane][0] = (u16)(i0 - x0);
      rc[lane][1] = (u16)(i1 - x1);
    }
  }
  __syncthreads();
  WSTAMP(12);

  // 7. write T-ordered records in final order (consecutive lanes -> consecutive T
  //    inside each kind: coalesced).  The register payload is staged through the
  //    now-free timestamp buffer in two rounds (sym + v0, then v1).
  if (P.ablate & 4) return;
  {
    // payload checks: symbols in range; moves with a None value (prefix fix-up)
    u32 none_mv = 0;
#pragma unroll
    for (int i = 0; i < WF_ITEMS; ++i) {
      if (t + WF_NT * i >= sz) continue;
      bad |= sym_r[i] >= (u64)P.n_sym;
      none_mv += (skind[t + WF_NT * i] == KMOVE && (v0_r[i] < 0 || v1_r[i] < 0));
    }
    if (bad) P.meta->bad_sym = 1;
    if (none_mv) atomicAdd((unsigned long long*)&P.meta->n_move_none, (unsigned long long)none_mv);
  }
  u32* st_a = (u32*)sts;             // [WIN_CAP] sym
  i32* st_b = (i32*)sts + WIN_CAP;   // [WIN_CAP] v0, then v1
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e < sz) {
      st_a[e] = sym_r[i];
      st_b[e] = v0_r[i];
    }
  }
  __syncthreads();
  WSTAMP(13);
  const u64 wofs_ra = woffk[SMX_N_KINDS], wofs_rb = woffk[SMX_N_KINDS + 1];
  const u64 nall = (u64)(P.na + P.nb);
  for (int x = t; x < sz; x += WF_NT) {
    const int e = sord[x];
    const u32 k = skind[e];
    const u64 T = base[k] + woffk[k] + (u32)(x - kbase[k]);
    if (T >= nall) continue;  // only a failed (discarded) presorted plan can trip this
    const u32 s = st_a[e];
    P.order[T] = (i32)(e < na ? a0 + e : bpos + e);
    P.symT[T] = s;
    if (k == KMOVE) {
      P.mvA[T] = st_b[e];
    } else if (k == KREN) {
      const int side = e >= na;
      const int xr = x - R0;
      const u32 own = (u32)((side ? wofs_rb : wofs_ra) + rc[xr / WAVE][side] + rown[xr]);
      const u64 m = T - base[KREN];
      P.Msym[m] = s;
      P.Mcls[m] = st_b[e];
      P.Mside[m] = (u8)side;
      P.Mown[m] = own;
      if (own < (u64)(side ? P.nb : P.na)) (side ? P.RB : P.RA)[own] = (u32)m;
    }
  }
  __syncthreads();
  WSTAMP(14);
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e < sz) st_b[e] = v1_r[i];
  }
  __syncthreads();
  WSTAMP(15);
  for (int x = t; x < sz; x += WF_NT) {
    const int e = sord[x];
    const u32 k = skind[e];
    if (k != KMOVE && k != KREN) continue;
    const u64 T = base[k] + woffk[k] + (u32)(x - kbase[k]);
    if (T >= nall) continue;
    if (k == KMOVE) P.mvF[T] = st_b[e];
    else P.Mstr[T - base[KREN]] = st_b[e];
  }
  if (DBG) {
    __syncthreads();
    WSTAMP(16);
  }
}

// ---------------------------------------------------------------------------
// generic windows: branch logs pre-sorted by (timestamp, oid); fixed diagonals

__device__ __forceinline__ bool key_le(u64 ta, u64 ha, u64 la, u64 tb, u64 hb, u64 lb) {
  if (ta != tb) return ta < tb;
  if (ha != hb) return ha < hb;
  return la <= lb;
}

#ifndef WG_NT
#define WG_NT 1024
#endif
#define WG_ITEMS (WIN_CAP / WG_NT)

__global__ void __launch_bounds__(WG_NT) k_window_g(WinArgs P) {
  __shared__ u64 sts[WIN_CAP];
  __shared__ u64 shi[WIN_CAP];
  __shared__ u64 slo[WIN_CAP];
  __shared__ u32 ssrc[WIN_CAP];
  __shared__ u16 sord[WIN_CAP];
  __shared__ u16 fin[WIN_CAP];
  __shared__ u16 rown[WIN_CAP];
  __shared__ u8 skind[WIN_CAP];
  __shared__ u8 srank[WIN_CAP];
  __shared__ u16 ccnt[NCHUNK][SMX_N_KINDS];
  __shared__ u16 rc[NCHUNK][2];
  __shared__ u32 kbase[SMX_N_KINDS + 1];
  __shared__ u32 wck[SMX_N_KINDS];
  __shared__ u64 base[SMX_N_KINDS + 1];

  const int t = threadIdx.x;
  const int lane = t & (WAVE - 1);
  const int wv = t / WAVE;
  const i64 w = blockIdx.x;
  const i64 a0 = P.bnd[2 * w], b0 = P.bnd[2 * w + 1];
  const int na = (int)(P.bnd[2 * w + 2] - a0);
  const int nb = (int)(P.bnd[2 * w + 3] - b0);
  const int sz = na + nb;
  if (sz == 0) return;

  bool bad = false;
  for (int e = t; e < sz; e += WG_NT) {
    const i64 j = e < na ? a0 + e : P.na + b0 + (e - na);
    const u32 src = P.perm[j];
    sts[e] = P.kts[j];
    shi[e] = P.khi[j];
    slo[e] = P.klo[j];
    ssrc[e] = src;
    const u32 k = P.kind[src];
    bad |= (k >= SMX_N_KINDS) || (P.sym[src] >= (u64)P.n_sym);
    skind[e] = (u8)(k < SMX_N_KINDS ? k : SMX_N_KINDS - 1);
  }
  if (bad) P.meta->bad_sym = 1;
  for (int i = t; i < NCHUNK * SMX_N_KINDS; i += WG_NT) (&ccnt[0][0])[i] = 0;
  if (t <= SMX_N_KINDS) base[t] = P.meta->base[t];
  __syncthreads();

  {
    const int d0 = t * WG_ITEMS < sz ? t * WG_ITEMS : sz;
    const int d1 = d0 + WG_ITEMS < sz ? d0 + WG_ITEMS : sz;
    int lo = d0 - nb > 0 ? d0 - nb : 0, hi = d0 < na ? d0 : na;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const int j = na + d0 - 1 - mid;
      if (key_le(sts[mid], shi[mid], slo[mid], sts[j], shi[j], slo[j])) lo = mid + 1;
      else hi = mid;
    }
    int ia = lo, ib = d0 - lo;
    for (int d = d0; d < d1; ++d) {
      bool take_a;
      if (ia >= na) take_a = false;
      else if (ib >= nb) take_a = true;
      else {
        const int j = na + ib;
        take_a = key_le(sts[ia], shi[ia], slo[ia], sts[j], shi[j], slo[j]);
      }
      sord[d] = (u16)(take_a ? ia++ : na + ib++);
    }
  }
  __syncthreads();

  const int nch = (sz + WAVE - 1) / WAVE;
  for (int c = wv; c < nch; c += WG_NT / WAVE) {
    const int m = c * WAVE + lane;
    const bool valid = m < sz;
    const int e = valid ? sord[m] : 0;
    const u32 k = valid ? skind[e] : 0u;
    const u64 peers = wave_peers<5>(k, valid);
    const u32 r = __popcll(peers & lanemask_lt());
    if (valid) {
      srank[m] = (u8)r;
      if (r == 0) ccnt[c][k] = (u16)__popcll(peers);
    }
  }
  __syncthreads();
  for (int k = wv; k < SMX_N_KINDS; k += WG_NT / WAVE) {
    const u32 x = lane < nch ? ccnt[lane][k] : 0u;
    const u32 inc = wave_incl_sum(x);
    if (lane < nch) ccnt[lane][k] = (u16)(inc - x);
    if (lane == WAVE - 1) wck[k] = inc;
  }
  __syncthreads();
  if (wv == 0) {
    const u32 x = lane < SMX_N_KINDS ? wck[lane] : 0u;
    const u32 inc = wave_incl_sum(x);
    if (lane < SMX_N_KINDS) kbase[lane] = inc - x;
    if (lane == SMX_N_KINDS - 1) kbase[SMX_N_KINDS] = inc;
  }
  __syncthreads();
  for (int m = t; m < sz; m += WG_NT) {
    const int e = sord[m];
    const u32 k = skind[e];
    fin[kbase[k] + ccnt[m / WAVE][k] + srank[m]] = (u16)e;
  }
  __syncthreads();

  const int R0 = kbase[KREN], RN = wck[KREN];
  const int nrc = (RN + WAVE - 1) / WAVE;
  for (int c = wv; c < nrc; c += WG_NT / WAVE) {
    const int x = c * WAVE + lane;
    const bool valid = x < RN;
    const int e = valid ? fin[R0 + x] : 0;
    const bool sb = valid && e >= na;
    const u64 bm = __ballot(sb), vm = __ballot(valid);
    const u64 lt = lanemask_lt();
    if (valid) rown[x] = (u16)(sb ? __popcll(bm & lt) : __popcll(vm & ~bm & lt));
    if (lane == 0) {
      rc[c][0] = (u16)__popcll(vm & ~bm);
      rc[c][1] = (u16)__popcll(bm);
    }
  }
  __syncthreads();
  if (wv == 0) {
    const u32 x0 = lane < nrc ? rc[lane][0] : 0u;
    const u32 x1 = lane < nrc ? rc[lane][1] : 0u;
    const u32 i0 = wave_incl_sum(x0), i1 = wave_incl_sum(x1);
    if (lane < nrc) {
      rc[lane][0] = (u16)(i0 - x0);
      rc[lane][1] = (u16)(i1 - x1);
    }
  }
  __syncthreads();

  for (int x = t; x < sz; x += WG_NT) {
    const int e = fin[x];
    const u32 k = skind[e];
    const u32 src = ssrc[e];
    const int side = e >= na;
    u32 own = 0;
    if (k == KREN) {
      const int xr = x - R0;
      own = P.woff[(i64)(CNT_REN_A + side) * P.W + w] + rc[xr / WAVE][side] + rown[xr];
    }
    win_emit(P, base, w, k, (u32)x, kbase[k], src, P.sym[src], P.v0[src], P.v1[src], side, own);
  }
}
