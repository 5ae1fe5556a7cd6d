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
__global__ void __launch_bounds__(WF_NT, 8) k_window_f(WinArgs P) {
  __shared__ u64 sts[WIN_CAP];        // element space: timestamp keys; later slot-space oid prefix
  __shared__ u16 sord[WIN_CAP];       // S order (merge), later the final order
  __shared__ u16 fin[WIN_CAP];        // slot -> element, later rename ranks
  __shared__ u16 sl[WIN_CAP];         // element -> slot, later element -> final
  __shared__ u8 skind[WIN_CAP];
  __shared__ u8 srank[WIN_CAP];
  __shared__ u64 gbits[NCHUNK];       // group-start bits over slots
  __shared__ u16 ccnt[NCHUNK][SMX_N_KINDS];
  __shared__ u16 rc[NCHUNK][2];
  __shared__ u32 kbase[SMX_N_KINDS + 1];
  __shared__ u32 wck[SMX_N_KINDS];
  __shared__ u64 base[SMX_N_KINDS + 1];
  __shared__ u32 woffk[SMX_N_KINDS + 2];  // this window's offsets: kinds, renames of A, of B
  __shared__ u32 vor[3];              // OR of (value + 1): moves' addr, file; renames' name
  u32* phi = (u32*)sts;               // slot space: top 32 bits of oid_hi (after step 4)
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
    // bit 0: branch logs not timestamp-ordered; bit 1: window too large for LDS
    if (threadIdx.x == 0)
      atomicOr((unsigned long long*)&P.meta->f_fail, (na < 0 || nb < 0) ? 1ull : 2ull);
    return;
  }
  if (sz == 0) return;
  const i64 bpos = P.na + b0 - na;  // op index of B element e is bpos + e

  // 1. load: keys to LDS, payload stays in registers
  u32 hi_r[WF_ITEMS];
  u32 sym_r[WF_ITEMS];
  i32 v0_r[WF_ITEMS], v1_r[WF_ITEMS];
  u32 k_r[WF_ITEMS];
  bool bad = false;
  // all loads are issued unconditionally (clamped to a valid op) so that the
  // WF_ITEMS x 6 loads of a lane are in flight together; the guards apply to the
  // LDS stores only
  u64 ts_r[WF_ITEMS];
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    const int ec = e < sz ? e : 0;
    const i64 j = ec < na ? a0 + ec : bpos + ec;
    k_r[i] = P.kind[j];
    ts_r[i] = P.kts[j];
    hi_r[i] = (u32)(P.khi[j] >> 32);
    sym_r[i] = P.sym[j];
    v0_r[i] = P.v0[j];
    v1_r[i] = P.v1[j];
  }
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e < sz) {
      bad |= (k_r[i] >= SMX_N_KINDS) || (sym_r[i] >= (u64)P.n_sym);
      k_r[i] = k_r[i] < SMX_N_KINDS ? k_r[i] : SMX_N_KINDS - 1;
      sts[e] = ts_r[i];
      skind[e] = (u8)k_r[i];
    }
  }
  // timestamps just before the window on each branch (issued with the loads above)
  u64 prev_a = 0, prev_b = 0;
  if (t == 0 && a0 > 0) prev_a = P.kts[a0 - 1];
  if (t == 0 && b0 > 0) prev_b = P.kts[P.na + b0 - 1];
  if (bad) P.meta->bad_sym = 1;
  for (int i = t; i < NCHUNK * SMX_N_KINDS; i += WF_NT) (&ccnt[0][0])[i] = 0;
  if (t <= SMX_N_KINDS) base[t] = P.meta->base[t];
  if (t < 3) vor[t] = 0;
  // window offsets = chunk prefix at the window start + kinds of the <= 255 ops
  // between that chunk start and the window start (per branch)
  if (t < SMX_N_KINDS) {
    woffk[t] = P.cpre[(i64)t * P.CM + a0 / CH] + P.cpre[(i64)(SMX_N_KINDS + t) * P.CM + b0 / CH];
  } else if (t < SMX_N_KINDS + 2) {
    const int sd = t - SMX_N_KINDS;
    woffk[t] = P.cpre[(i64)(sd * SMX_N_KINDS + KREN) * P.CM + (sd ? b0 : a0) / CH];
  }
  __syncthreads();
  {
    const int pa = (int)(a0 % CH), pb = (int)(b0 % CH);
    // lanes 0..255: branch A partial chunk, lanes 256..511: branch B
    const int side = t >= CH;
    const int q = t - side * CH;
    if (q < (side ? pb : pa)) {
      const i64 j = side ? (P.na + b0 - pb + q) : (a0 - pa + q);
      u32 k = P.kind[j];
      k = k < SMX_N_KINDS ? k : SMX_N_KINDS - 1;
      atomicAdd(&woffk[k], 1u);
      if (k == KREN) atomicAdd(&woffk[SMX_N_KINDS + side], 1u);
    }
  }
  __syncthreads();

  // presorted-layout check: every adjacent pair of each branch log is
  // non-decreasing (the pair straddling a window start is checked here too);
  // moves with a None value are counted for the prefix fix-up
  if (!(P.ablate & 1)) {
    bool dec = false;
    u32 none_mv = 0;
    if (t == 0) dec = (a0 > 0 && na > 0 && prev_a > sts[0]) || (b0 > 0 && nb > 0 && prev_b > sts[na]);
#pragma unroll
    for (int i = 0; i < WF_ITEMS; ++i) {
      const int e = t + WF_NT * i;
      if (e >= sz) continue;
      if (e != 0 && e != na && sts[e - 1] > sts[e]) dec = true;
      none_mv += (k_r[i] == KMOVE && (v0_r[i] < 0 || v1_r[i] < 0));
    }
    if (none_mv) atomicAdd((unsigned long long*)&P.meta->n_move_none, (unsigned long long)none_mv);
    // value bit widths for the packed final-state table (smx_common.h FinPack)
    u32 oa = 0, of = 0, oc = 0;
#pragma unroll
    for (int i = 0; i < WF_ITEMS; ++i) {
      if (t + WF_NT * i >= sz) continue;
      if (k_r[i] == KMOVE) {
        oa |= (u32)(v0_r[i] + 1);
        of |= (u32)(v1_r[i] + 1);
      } else if (k_r[i] == KREN) {
        oc |= (u32)(v1_r[i] + 1);
      }
    }
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) {
      oa |= __shfl_xor(oa, o, WAVE);
      of |= __shfl_xor(of, o, WAVE);
      oc |= __shfl_xor(oc, o, WAVE);
    }
    if (lane == 0) {
      if (oa) atomicOr(&vor[0], oa);
      if (of) atomicOr(&vor[1], of);
      if (oc) atomicOr(&vor[2], oc);
    }
    if (__syncthreads_or(dec)) {
      if (t == 0) atomicOr((unsigned long long*)&P.meta->f_fail, 1ull);
      return;
    }
  }

  if (P.ablate & 8) {  // load + write only
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

  // 2. merge A part [0,na) with B part [na,sz) by timestamp, A first on ties
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
  __syncthreads();

  // 3. stable multisplit of S by rank
  const int nch = (sz + WAVE - 1) / WAVE;
  for (int c = wv; c < nch; c += WF_WAVES) {
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
  for (int k = wv; k < SMX_N_KINDS; k += WF_WAVES) {
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
  for (int m = t; m < sz; m += WF_NT) {
    const int e = sord[m];
    const u32 k = skind[e];
    const int p = kbase[k] + ccnt[m / WAVE][k] + srank[m];
    fin[p] = (u16)e;
    sl[e] = (u16)p;
  }
  __syncthreads();

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
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e < sz) phi[sl[e]] = hi_r[i];
  }
  __syncthreads();

  // 5. order each group by (oid, side, index): counting rank on the top 32 bits of
  //    oid_hi; elements sharing that prefix (rare) are resolved on the full oid and
  //    then on slot order (= side, index order)
#pragma unroll
  for (int j = 0; j < WF_ITEMS; ++j) {
    const int p = t + WF_NT * j;
    if (p >= sz) continue;
    const int e = fin[p];
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
    int r = p;
    if (ge - gs > 1 && !(P.ablate & 2)) {
      const u32 h = phi[p];
      u32 lt = 0, eq = 0;
      for (int q = gs; q < ge; ++q) {
        const u32 hq = phi[q];
        lt += hq < h;
        eq += hq == h;
      }
      r = gs + (int)lt;
      if (eq > 1) {  // shared 32-bit prefix: exact compare on (oid_hi, oid_lo), then slot
        const i64 jp = e < na ? a0 + e : bpos + e;
        const u64 hp = P.khi[jp], lp = P.klo[jp];
        for (int q = gs; q < ge; ++q) {
          if (q == p || phi[q] != h) continue;
          const int eq2 = fin[q];
          const i64 jq = eq2 < na ? a0 + eq2 : bpos + eq2;
          const u64 hq = P.khi[jq], lq = P.klo[jq];
          r += hq < hp || (hq == hp && (lq < lp || (lq == lp && q < p)));
        }
      }
    }
    sord[r] = (u16)e;
    sl[e] = (u16)r;
  }
  __syncthreads();

  // the window's value bits: one device atomic per word, only when it adds bits
  if (t < 3) {
    u32* vb = P.meta->vbits;
    const u32 mine = vor[t];
    const u32 cur = __hip_atomic_load(&vb[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((cur | mine) != cur) atomicOr(&vb[t], mine);
  }

  // 6. renames: rank among the window's renames of the same branch (final order)
  const int R0 = kbase[KREN], RN = wck[KREN];
  const int nrc = (RN + WAVE - 1) / WAVE;
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

  // 7. write T-ordered records in final order (consecutive lanes -> consecutive T
  //    inside each kind: coalesced).  The register payload is staged through the
  //    now-free timestamp buffer in two rounds (sym + v0, then v1).
  if (P.ablate & 4) return;
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
#pragma unroll
  for (int i = 0; i < WF_ITEMS; ++i) {
    const int e = t + WF_NT * i;
    if (e < sz) st_b[e] = v1_r[i];
  }
  __syncthreads();
  for (int x = t; x < sz; x += WF_NT) {
    const int e = sord[x];
    const u32 k = skind[e];
    if (k != KMOVE && k != KREN) continue;
    const u64 T = base[k] + woffk[k] + (u32)(x - kbase[k]);
    if (T >= nall) continue;
    if (k == KMOVE) P.mvF[T] = st_b[e];
    else P.Mstr[T - base[KREN]] = st_b[e];
  }
}

// ---------------------------------------------------------------------------
// generic windows: branch logs pre-sorted by (timestamp, oid); fixed diagonals

__device__ __forceinline__ bool key_le(u64 ta, u64 ha, u64 la, u64 tb, u64 hb, u64 lb) {
  if (ta != tb) return ta < tb;
  if (ha != hb) return ha < hb;
  return la <= lb;
}

#define WG_NT 256
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
  if (w == 0 && t < 3) P.meta->vbits[t] = ~0u;  // generic plan: value widths not tracked -> int4 table
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
