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
//
// What a window writes, T-ordered:
//   moves (T < nMv)     the FINAL composed records: no skip precedes the rename
//                       block, so a move's output index is T, and it carries its own
//                       newAddress / newFile (compose.py:37-43; a None value is
//                       patched later from the symbol's prefix, k_mv_fix); plus
//                       msym[T] = sym | has-address << 30 | has-file << 31 for the
//                       last-writer tables
//   every other op      tsrc / tsym at P = T - nMv (renames first, then the rest):
//                       the source op and the symbol that k_emit needs
//   renames             Rstr[m] (the rename-chain value, compose.py:71-72), m = P
//   DivergentRename     the natural-head test (compose.py:60-70, 88-98 at d = 0) of
//                       each rename against the other branch's next rename inside
//                       the window; flagged positions go to the window's candidate
//                       slots; the renames after the other branch's last rename of
//                       the window are tested by k_boundary (smx_walk.h)
//   per window          wren (renames / A renames before it), wbnd (where its
//                       boundary renames start)
#pragma once

#include "smx_common.h"

#define WIN_CAP 2048               // max ops per window held in LDS
#ifndef SMX_XCD_WIN
#define SMX_XCD_WIN 1              // generic-plan windows dealt to XCDs in consecutive runs
#endif
#ifndef WIN_TGT
#define WIN_TGT 1792               // default target window size, presorted path (SMX_WIN_TGT)
#endif
#define WIN_TGT_MIN 256
#define NCNT (SMX_N_KINDS + 3)     // kinds, renames per branch, moves with a None value
#define CNT_REN_A SMX_N_KINDS
#define CNT_REN_B (SMX_N_KINDS + 1)
#define CNT_NONE_MV (SMX_N_KINDS + 2)
#define KMOVE SMX_KIND_MOVE
#define KREN SMX_KIND_RENAME
#define NCHUNK (WIN_CAP / WAVE)
#define CH 256                     // chunk of the presorted kind histogram
#define SYM_MASK 0x3fffffffu       // msym: symbol bits (n_sym <= 2^30)
#define MS_HAS_A (1u << 30)
#define MS_HAS_F (1u << 31)

// Keys < kp among the four (or the first m) of a 16-byte LDS read.
__device__ __forceinline__ int rk4(const uint4 x, u32 kp) {
  return (x.x < kp) + (x.y < kp) + (x.z < kp) + (x.w < kp);
}
__device__ __forceinline__ int rk4(const uint4 x, u32 kp, int m) {
  return (m > 0 && x.x < kp) + (m > 1 && x.y < kp) + (m > 2 && x.z < kp) + (m > 3 && x.w < kp);
}

// Four consecutive i32 stores as one 16-byte store (4-byte aligned address).
typedef i32 __attribute__((ext_vector_type(4))) win_v4i;
typedef win_v4i __attribute__((aligned(4))) win_v4i_a4;
__device__ __forceinline__ void st4(i32* p, i32 a, i32 b, i32 c, i32 d) {
  *reinterpret_cast<win_v4i_a4*>(p) = win_v4i{a, b, c, d};
}

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
  i64 src_a, src_b; // global source index of local op j (sharded merge; 0 / na otherwise)
  const i32* src_map;  // sample-sorted shard: global source of local op j, or null
  int ablate;       // diagnostic builds only (SMX_ABLATE): skip phases, results invalid
  const i64* bnd;
  const u32* woff;  // [NCNT][W] exclusive offsets over windows (generic plan)
  const u32* cpre;  // presorted plan: [2][kinds][CM] chunk prefixes (256-op chunks)
  i64 CM;
  ComposeMeta* meta;
  // outputs (module comment)
  i32* out_order;
  i32* out_addr;
  i32* out_file;
  i32* out_ctx;
  u32* msym;
  i32* tsrc;
  u32* tsym;
  i32* Rstr;
  u32* wren;        // [W][2]
  u32* wbnd;        // [W]: first boundary rename (window-local) | its branch << 31
  u32* cslot;       // candidate M positions, window w's from M offset wren[2w]
  u32* wcand;       // [W] in-window candidates
  u64* dbg;         // diagnostics only: phase timestamps (k_window_f<true>)
};

// OR of the per-wave value widths into meta->vbits (k_tb_reduce packs the final-state
// table with them); an atomic only when it adds bits.
__device__ __forceinline__ void win_publish_widths(ComposeMeta* meta, const u32* vbw, int nw) {
  for (int q = 0; q < 3; ++q) {
    u32 m = 0;
    for (int w = 0; w < nw; ++w) m |= vbw[w * 3 + q];
    const u32 cur = __hip_atomic_load(&meta->vbits[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((cur | m) != cur) atomicOr(&meta->vbits[q], m);
  }
}
// ... with the published widths read beforehand (cur[3]): no global round trip here
__device__ __forceinline__ void win_publish_widths(ComposeMeta* meta, const u32* vbw, int nw, const u32* cur) {
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    u32 m = 0;
    for (int w = 0; w < nw; ++w) m |= vbw[w * 3 + q];
    if ((cur[q] | m) != cur[q]) atomicOr(&meta->vbits[q], m);
  }
}

__device__ __forceinline__ i32 win_gsrc(const WinArgs& P, i64 j) {
  if (P.src_map) return P.src_map[j];
  return j < P.na ? (i32)(P.src_a + j) : (i32)(P.src_b + (j - P.na));
}

// The window's renames in final order, x = 0 .. RN-1: branch s(x), rank own(x) in
// its branch's renames of the window, posl = the window-local x of each branch's
// renames (A's first, then B's).  Natural head of x: the other branch's next
// rename, the (x - own(x))-th of that branch in the window if there is one.
// Flags -> candidate slots in M order; thread 0 writes where the boundary renames
// (after the other branch's last rename of the window) start.
// SymCls(x) -> (symbol, newName class) of rename x.
template <int NT, int NCHK, typename SideOwn, typename SymCls>
__device__ __forceinline__ void win_rename_flags(const WinArgs& P, i64 w, u64 Mbase, int RN, int cntA,
                                                 int cntB, const u16* posl, u64* cb, SideOwn side_own,
                                                 SymCls sym_cls) {
  constexpr int NW = NT / WAVE;
  const int t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  const int nrc = (RN + WAVE - 1) / WAVE;
  for (int c = wv; c < nrc; c += NW) {
    const int x = c * WAVE + lane;
    bool f = false;
    if (x < RN) {
      int s, own;
      side_own(x, &s, &own);
      const int k = x - own;
      if (k < (s ? cntA : cntB)) {
        const int h = posl[(s ? 0 : cntA) + k];
        const uint2 me = sym_cls(x), hd = sym_cls(h);
        f = me.x == hd.x && me.y != hd.y;
      }
    }
    const u64 b = __ballot(f);
    if (lane == 0) cb[c] = b;
  }
  if (t == 0) {
    // boundary renames: those after the other branch's last rename of the window
    u32 bnd = 0;
    if (RN) {
      int s, own;
      side_own(RN - 1, &s, &own);
      const int cnt_o = s ? cntA : cntB;
      const u32 bx = cnt_o ? (u32)posl[(s ? 0 : cntA) + cnt_o - 1] + 1u : 0u;
      bnd = bx | ((u32)s << 31);
    }
    P.wbnd[w] = bnd;
  }
  __syncthreads();
  const u64 nall = (u64)(P.na + P.nb);
  for (int c = wv; c < nrc; c += NW) {
    const u64 b = cb[c];
    if (!b) continue;
    u32 before = lane < c ? (u32)__popcll(cb[lane]) : 0u;  // chunks before c
    if (NCHK > WAVE) before += WAVE + lane < c ? (u32)__popcll(cb[WAVE + lane]) : 0u;
    before = wave_incl_sum(before);
    before = __builtin_amdgcn_readlane(before, WAVE - 1);
    if ((b >> lane) & 1ull) {
      const u64 slot = Mbase + before + (u32)__popcll(b & lanemask_lt());
      if (slot < nall) P.cslot[slot] = (u32)(Mbase + (u64)(c * WAVE + lane));
    }
  }
  if (t == 0) {
    u32 tot = 0;
    for (int c = 0; c < nrc; ++c) tot += (u32)__popcll(cb[c]);
    P.wcand[w] = tot;
  }
}

// ---------------------------------------------------------------------------
// presorted windows (timestamps non-decreasing in each branch log)

#ifndef WF_NT
#define WF_NT 512
#endif
#ifndef WF_CAP
#define WF_CAP WIN_CAP              // max ops per presorted window
#endif
#ifndef WF_WIDE_CAP
#define WF_WIDE_CAP 8192  // the wide presorted window (run_presorted(wide)): one per CU
#endif
#define WF_WIDE_NT 1024
#ifndef WF_SMALL_CAP
#define WF_SMALL_CAP 512  // small merges' windows (latency-bound: more windows in flight per CU)
#endif
#define WF_SMALL_NT 128
#ifndef WF_SMALL_TGT
#define WF_SMALL_TGT 256
#endif
#ifndef WF_SMALL_MAXN
#define WF_SMALL_MAXN 0  // merges up to this many ops start with the small windows: off, config 2's
                         // window stage 0.048 -> 0.218 ms with them (profiles/r04_h/ab_c2.txt)
#endif
#define WF_NCH (WF_CAP / WAVE)
#define WF_WAVES (WF_NT / WAVE)
#define WF_ITEMS (WF_CAP / WF_NT)
#define WF_KP ((2 * CH + WF_NT - 1) / WF_NT)  // partial-chunk kinds per lane

// LDS ~34 KB (buffers are reused across phases) so 4 workgroups fit a CU: while
// some workgroups run their LDS phases, others stream their windows from HBM.
// DBG: phase timestamps of every window (diagnostics, tools/window_phases.py):
// lane 0 of wave 0 stores s_memtime after each phase into P.dbg[w * WF_NSTAMP + i].
#define WF_NSTAMP 24
// Diagnostic builds: SMX_ABLATE = 100 + N leaves the kernel after phase N (timing of
// the phases by difference, tools/window_ablate.py); results invalid.
#define WF_EXIT(N)                                                         \
  do {                                                                     \
    if (SMX_DIAG && P.ablate == 100 + (N)) {                               \
      if (t == 0 && sord[0] == 0xfffeu && fin[1] == 0xfffeu) P.meta->dup_key = 1; \
      return;                                                              \
    }                                                                      \
  } while (0)
// the run-grouped order's phase exits (diagnostic builds: SMX_ABLATE = 0x10000 + N, a value
// clear of the bit-tested ablations 1, 2, 4 (N <= 3 only) and 16)
#define RX_EXIT(N)                                                          \
  do {                                                                      \
    if (SMX_DIAG && P.ablate == 0x10000 + (N)) {                            \
      if (t == 0 && sord[0] == 0xfffeu && fin[1] == 0xfffeu) P.meta->dup_key = 1; \
      return;                                                               \
    }                                                                       \
  } while (0)
#define WSTAMP(i)                                                                  \
  do {                                                                             \
    if (DBG && t == 0) P.dbg[w * WF_NSTAMP + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// MAP: the sample-sorted shard's source map (P.src_map) is read; a separate instance so
// that the plain path's store loop has no load whose wait would also drain its stores
#ifndef WF_MINB
#define WF_MINB 8
#endif
#ifndef WF_DENSE_KINDS
#define WF_DENSE_KINDS 1  // step 3's ballots over the dense index of the present kinds
#endif
#ifndef WF_BUCKET
#define WF_BUCKET 1  // step 5 by interpolation buckets (0: counting rank over each group)
#endif
#ifndef WF_BF
#define WF_BF 1      // branch-free per-item code in the load and merge phases
#endif
#ifndef WF_ONEATOM
#define WF_ONEATOM 1 // step 5 places each slot at start + arrival rank (one LDS atomic per element, not two)
#endif
#ifndef WF_TIEFIX
#define WF_TIEFIX 1  // wide windows: equal 32-bit keys in a bucket ranked on the full ids right there (no window re-rank)
#endif
#ifndef WF_LATEARGS
#define WF_LATEARGS 0  // step 9 re-reads its kernel arguments: 63 -> 17 SGPR spills, but 28 B/lane of VGPR scratch spills (off)
#endif
#ifndef WF_RUNMERGE
#define WF_RUNMERGE 0  // step 2 by timestamp-run heads (a search per run, not a merge path per thread):
                       // config 3 window 1.225 -> 1.230 ms, config 5 wide 0.907 -> 0.960 ms; off (profiles/r04_e, r04_f)
#endif
#ifndef WF_KPBAL
#define WF_KPBAL 0   // partial-chunk kinds counted by peers ballots (one LDS atomic per (wave, kind)): 1.225 -> 1.235 ms,
                     // and 1.395 ms together with WF_RUNMERGE (+21% VALU in that build); off (profiles/r04_f)
#endif
#ifndef WF_RANK8
#define WF_RANK8 0   // step 5's bucket rank by 8 predicated compares (the loop only for larger buckets): window 1.223 -> 1.260 ms, off (profiles/r04_d)
#endif
#ifndef WF_BK16
#define WF_BK16 1    // bucket-ordered 16-bit key prefixes for the rank loop (window 1.329 -> 1.286 ms, profiles/r03_e/ab.txt)
#endif
#ifndef WF_FUSEFIN
#define WF_FUSEFIN 1  // step 5's final order written by the rank loop itself: window 1.248 -> 1.227 ms (profiles/r03_q)
#endif
#ifndef WF_BZ4
#define WF_BZ4 1     // step 5's bucket counters zeroed in step 4's last phase (one barrier fewer)
#endif
#ifndef WF_OUT2
#define WF_OUT2 1    // steps 7-9 staged by final slot (inv), four slots per thread, 16-byte stores: window 1.271 -> 1.233 ms (profiles/r03_m/ab.txt)
#endif
#ifndef WF_RUNS
#define WF_RUNS 1    // the normal presorted windows order by runs and (kind, run) groups (no merge / multisplit)
#endif
#ifndef WF_HBATCH
#define WF_HBATCH 0  // run-grouped step h, 1: the ITEMS buckets' ends and first members read together:
                     // window 1.181 -> 1.439 ms on config 3 (more live registers), off
#endif
#ifndef WF_LOREG
#define WF_LOREG 1  // run-grouped step h: a bucket's start from the op's slot and arrival rank (no LDS read)
#endif
#ifndef WF_HEADLIST
#define WF_HEADLIST 0  // run-grouped step a, 1: every head binary-searches a list of the other part's
                       // heads at once (three more barriers): window 1.196 -> 1.241 ms on config 3,
                       // wide 0.409 -> 0.416 on config 5 (profiles/r05_x), off; 0: one head at a time
                       // with the whole wave, a 64-way search of the other part's timestamps
#endif
#ifndef WF_GAGG
#define WF_GAGG 1  // step c's group counts aggregated per wave: 1 the wide windows, 2 every window
#endif
#ifndef WF_RUNS_WIDE
#define WF_RUNS_WIDE 1  // ... and the wide ones (config 5: one run per window)
#endif
#ifndef WF_STB_KIND
#define WF_STB_KIND 1  // v0 / v1 staged for moves and renames only (the other kinds output neither)
#endif
#ifdef WF_WPE
#define WF_BOUNDS __launch_bounds__(WF_NT) __attribute__((amdgpu_waves_per_eu(WF_WPE, WF_WPE)))
#else
#define WF_BOUNDS __launch_bounds__(WF_NT, WF_MINB)
#endif
template <int CAP, int NT, bool DBG, bool MAP, bool RUNS = false>
__global__ void __launch_bounds__(NT, CAP > WF_CAP ? 4 : WF_MINB) k_window_f(WinArgs P) {
  // CAP ops per window on NT threads: (2048, 512) four windows per CU; (8192, 1024) one
  // window per CU for logs whose equal-timestamp groups need it (config 5)
  constexpr int ITEMS = CAP / NT, NCH = CAP / WAVE, WAVES = NT / WAVE, KP = (2 * CH + NT - 1) / NT;
  // equal 32-bit rank keys resolved in the rank loop itself (the wide window, whose
  // 8192-op groups see ~1 such pair in 128 and whose exact re-rank would be quadratic);
  // the small windows flag them for the window re-rank (fewer registers in the loop)
  constexpr bool TIEFIX = WF_TIEFIX && CAP > WF_CAP;
  static_assert(CAP % NT == 0 && NCH <= 2 * WAVE && CAP <= 65536, "window geometry");
  __shared__ __attribute__((aligned(16))) u64 sts[CAP];  // element space: timestamps; later slot-space rank keys
  __shared__ __attribute__((aligned(16))) u16 sord[CAP];  // S order (merge), later the final order
  __shared__ u16 fin[CAP];        // slot -> element, later rename ranks
  __shared__ u16 sl[CAP];         // element -> slot, later rank -> slot, later posl
  __shared__ u8 skind[CAP];
  __shared__ __attribute__((aligned(16))) u8 skS[CAP];  // kinds in S order, later by slot (WF_OUT2)
#if WF_OUT2
  __shared__ u16 inv[CAP];        // element -> final slot
  __shared__ u64 tbase[SMX_N_KINDS]; // T of a kind's slot x = tbase[kind] + x
#endif
  __shared__ u64 gbits[NCH];       // group-start bits over slots, later candidate ballots
  __shared__ u16 ccnt[NCH][SMX_N_KINDS];
  __shared__ u16 rc[NCH][2];
  __shared__ u32 kbase[SMX_N_KINDS + 1];
  __shared__ u32 wck[SMX_N_KINDS];
  __shared__ u64 base[SMX_N_KINDS + 1];
  __shared__ u32 woffk[SMX_N_KINDS + 2];  // this window's offsets: kinds, renames of A, of B
  __shared__ u32 wtot[2];                 // the window's renames of A, of B
  __shared__ u32 vbw[WAVES][3];        // per wave: value widths (addr, file, name)
  u16* rown = fin;                    // rename rank within its branch (after step 5)

  const int t = threadIdx.x;
  const int lane = t & (WAVE - 1);
  const int wv = t / WAVE;
  const i64 w = blockIdx.x;  // (XCD-ordered presorted windows measured slower: 1.241 -> 1.269 ms, profiles/r03_p)
  // the plan already failed (k_khist saw a timestamp group no window holds, or an
  // earlier window overflowed): leave before any load; a scalar read, in flight with
  // the window bounds' (a stale 0 only defers the exit to the check after the loads)
  if (P.meta->f_fail) return;
  const i64 a0 = P.bnd[2 * w], b0 = P.bnd[2 * w + 1];
  const int na = (int)(P.bnd[2 * w + 2] - a0);
  const int nb = (int)(P.bnd[2 * w + 3] - b0);
  const int sz = na + nb;
  if (na < 0 || nb < 0 || sz > CAP) {  // the presorted plan does not hold
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
  const i64 bpos = P.na + b0 - na;  // op index of B element e is bpos + e
  const i64 bld = bpos + P.bgap;    // ... stored at field index bld + e
  WSTAMP(0);

  // 1. load the sort keys (kind, timestamp, top of the id) and the payload
  u32 hi_r[ITEMS];  // the top 32 bits of oid_hi: the rank key (only they are loaded)
  u32 sym_r[ITEMS];
  i32 v0_r[ITEMS], v1_r[ITEMS];
  u32 k_r[ITEMS];
  bool bad = false;
  // every global read of the window is issued here, before any loaded value is used:
  // the load phase is one round trip to memory, and the later phases find their
  // operands in registers (no dependent global reads between barriers).  The few side
  // reads go first, so that their address arithmetic never waits on the bulk loads.
  // kinds of the <= 255 ops between each branch's chunk start and the window start
  // (window offsets below); entries 0..255 branch A, 256..511 branch B
  u32 kpart[KP];
#pragma unroll
  for (int u = 0; u < KP; ++u) {
    const int x = t + NT * u;
    const int pa = (int)(a0 % CH), pb = (int)(b0 % CH);
    const int side = x >= CH;
    const int q = x - side * CH;
    kpart[u] = 0xffffffffu;
    if (x < 2 * CH && q < (side ? pb : pa)) kpart[u] = P.kind[side ? (P.na + P.bgap + b0 - pb + q) : (a0 - pa + q)];
  }
  // timestamps just before the window on each branch
  u64 prev_a = 0, prev_b = 0;
  if (t == 0 && a0 > 0) prev_a = P.kts[a0 - 1];
  if (t == 0 && b0 > 0) prev_b = P.kts[P.na + P.bgap + b0 - 1];
  // T-order segment starts; window offsets = chunk prefix at the window start + kinds
  // of the <= 255 ops between that chunk start and the window start (per branch)
  const u64 base_v = t <= SMX_N_KINDS ? P.meta->base[t] : 0ull;
#if WF_DENSE_KINDS
  const u32 kmask_r = P.meta->kmask[0] | P.meta->kmask[1];
#endif
  // a window that already failed the plan (dense groups: every window does) makes the
  // rest of the launch pointless: checked after the load phase, no extra round trip
  const u64 failed = t == 0 ? P.meta->f_fail : 0ull;
  u32 woff_x = 0, woff_y = 0;  // (added where stored: an add here would wait for every load)
  // (32-bit chunk indices: 2 * kinds * CM < 2^32 for any n < 2^31, the i32 output limit)
  if (t < SMX_N_KINDS) {
    woff_x = P.cpre[(u32)t * (u32)P.CM + (u32)(a0 / CH)];
    woff_y = P.cpre[(u32)(SMX_N_KINDS + t) * (u32)P.CM + (u32)(b0 / CH)];
  } else if (t < SMX_N_KINDS + 2) {
    const int sd = t - SMX_N_KINDS;
    woff_x = P.cpre[(u32)(sd * SMX_N_KINDS + KREN) * (u32)P.CM + (u32)((sd ? b0 : a0) / CH)];
  }
  // value widths published so far (a stale read only costs a redundant atomicOr)
  u32 vcur[3] = {0u, 0u, 0u};
  if (t == 0) {
#pragma unroll
    for (int q = 0; q < 3; ++q) vcur[q] = __hip_atomic_load(&P.meta->vbits[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // all loads are issued unconditionally (clamped to a valid op) so that the
  // loads of a lane are in flight together; the guards apply to the LDS stores only
  u64 ts_r[ITEMS];
  auto op_index = [&](int e) -> i64 {  // (an empty window still writes its exports)
    const int ec = e < sz ? e : 0;
    return sz == 0 ? 0 : (ec < na ? a0 + ec : bld + ec);
  };
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const i64 j = op_index(t + NT * i);
    k_r[i] = P.kind[j];
    ts_r[i] = P.kts[j];
    hi_r[i] = reinterpret_cast<const u32*>(P.khi)[2 * j + 1];
    sym_r[i] = P.sym[j];
    v0_r[i] = P.v0[j];
    v1_r[i] = P.v1[j];
  }
  u32 none_mv = 0;  // moves with a None value (prefix fix-up)
  u32 vb_a = 0, vb_f = 0, vb_c = 0;  // OR of (value + 1): widths of the packed final-state table
#if WF_BF
  // branch-free: the LDS slots past sz take harmless values (every later phase reads
  // slots < sz only), the rest is selects -- no exec-mask bookkeeping per item
  static_assert(NT * ITEMS <= CAP, "item slots inside the LDS arrays");
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    const bool ok = e < sz;
    const u32 kr = k_r[i];
    bad |= ok & ((kr >= SMX_N_KINDS) | (sym_r[i] >= (u64)P.n_sym));
    const u32 k = kr < SMX_N_KINDS ? kr : SMX_N_KINDS - 1;
    sts[e] = ts_r[i];
    if constexpr (!RUNS) skind[e] = (u8)k;  // (the run-grouped order keeps the kinds in registers)
    const bool mv = ok & (k == KMOVE), rn = ok & (k == KREN);
    const bool ha = v0_r[i] >= 0, hf = v1_r[i] >= 0;
    sym_r[i] = (sym_r[i] & SYM_MASK) | ((mv & ha) ? MS_HAS_A : 0u) | ((mv & hf) ? MS_HAS_F : 0u);
    none_mv += (mv & !(ha & hf)) ? 1u : 0u;
    vb_a |= mv ? (u32)(v0_r[i] + 1) : 0u;
    vb_f |= mv ? (u32)(v1_r[i] + 1) : 0u;
    vb_c |= rn ? (u32)(v1_r[i] + 1) : 0u;
  }
#else
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    if (e < sz) {
      bad |= k_r[i] >= SMX_N_KINDS || sym_r[i] >= (u64)P.n_sym;
      const u32 k = k_r[i] < SMX_N_KINDS ? k_r[i] : SMX_N_KINDS - 1;
      sts[e] = ts_r[i];
      skind[e] = (u8)k;
      // the payload's first word: sym | the move's has-value bits (msym)
      if (k == KMOVE) {
        sym_r[i] = (sym_r[i] & SYM_MASK) | (v0_r[i] >= 0 ? MS_HAS_A : 0u) | (v1_r[i] >= 0 ? MS_HAS_F : 0u);
        none_mv += v0_r[i] < 0 || v1_r[i] < 0;
        vb_a |= (u32)(v0_r[i] + 1);
        vb_f |= (u32)(v1_r[i] + 1);
      } else {
        sym_r[i] &= SYM_MASK;
        if (k == KREN) vb_c |= (u32)(v1_r[i] + 1);
      }
    }
  }
#endif
  vb_a = wave_or_to_last(vb_a);
  vb_f = wave_or_to_last(vb_f);
  vb_c = wave_or_to_last(vb_c);
  if (lane == WAVE - 1) {
    vbw[wv][0] = vb_a;
    vbw[wv][1] = vb_f;
    vbw[wv][2] = vb_c;
  }
  if (bad) P.meta->bad_sym = 1;
  for (int i = t; i < NCH * SMX_N_KINDS; i += NT) (&ccnt[0][0])[i] = 0;
  if constexpr (RUNS)  // the run-grouped order's bucket counters (fin is next written by step 6)
    for (int i = t; i < CAP / 2; i += NT) reinterpret_cast<u32*>(fin)[i] = 0u;
  if (t <= SMX_N_KINDS) base[t] = base_v;
  if (t < SMX_N_KINDS) wck[t] = 0;
  if (t < SMX_N_KINDS + 2) woffk[t] = woff_x + woff_y;
  if (t == 0) wtot[0] = failed != 0;
  __syncthreads();
  if (wtot[0]) return;  // (wtot is written again in step 6)
  WSTAMP(1);
  if (SMX_DIAG && (P.ablate & 16)) {  // diagnostics: load only (keeps every load live)
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) x += sym_r[i] + (u32)v0_r[i] + (u32)v1_r[i] + (u32)hi_r[i];
    if (x == 0x9e3779b9u) P.meta->dup_key = 1;
    return;
  }
  // window offsets: the partial-chunk kinds
#if WF_KPBAL && WF_DENSE_KINDS
  {
    // one LDS atomic per (wave, kind) from the peers ballots over the dense index of the
    // present kinds (per-lane atomics on a few hot counters serialise in the LDS);
    // a wave's slots x = t + NT * u lie on one side of CH (WAVE divides CH)
    static_assert(CH % WAVE == 0, "one side per wave");
    const u32 kp0 = __builtin_amdgcn_readfirstlane(kmask_r);
    const int kb0 = 32 - __clz((int)(max(__popc(kp0), 1u) - 1u));
#pragma unroll
    for (int u = 0; u < KP; ++u) {
      const bool v = kpart[u] != 0xffffffffu;
      const u32 k = v ? (kpart[u] < SMX_N_KINDS ? kpart[u] : SMX_N_KINDS - 1) : 0u;
      const u64 peers = wave_peers_n((u32)__popc(kp0 & ((1u << k) - 1u)), v, kb0);
      if (v && (peers & lanemask_lt()) == 0) atomicAdd(&woffk[k], (u32)__popcll(peers));
      const u64 rb = __ballot(v && k == KREN);
      if (lane == 0 && rb) atomicAdd(&woffk[SMX_N_KINDS + (t + NT * u >= CH)], (u32)__popcll(rb));
    }
  }
#else
#pragma unroll
  for (int u = 0; u < KP; ++u) {
    if (kpart[u] != 0xffffffffu) {
      const u32 k = kpart[u] < SMX_N_KINDS ? kpart[u] : SMX_N_KINDS - 1;
      atomicAdd(&woffk[k], 1u);
      if (k == KREN) atomicAdd(&woffk[SMX_N_KINDS + (t + NT * u >= CH)], 1u);
    }
  }
#endif

  const int nch = (sz + WAVE - 1) / WAVE;
  auto group_of = [&](int p, int* gs_o, int* ge_o) {
    const int bit = p & 63;
    int wi = p >> 6;
    u64 word = gbits[wi] & (bit == 63 ? ~0ull : ((1ull << (bit + 1)) - 1));
    while (word == 0) word = gbits[--wi];
    *gs_o = wi * 64 + 63 - __clzll(word);
    wi = p >> 6;
    word = bit == 63 ? 0ull : (gbits[wi] & ~((1ull << (bit + 1)) - 1));
    while (word == 0 && ++wi < nch) word = gbits[wi];
    const int ge = word ? wi * 64 + __ffsll((unsigned long long)word) - 1 : sz;
    *ge_o = ge < sz ? ge : sz;
  };
  bool btie = false;  // two equal 32-bit keys in one group (steps 2-5: the exact re-rank below)
  // ---- Run-grouped order (RUNS): no merge, no multisplit.  Inside a branch part the
  // timestamps never decrease, so the equal-timestamp ops of both parts form one run of
  // the merged order S, which starts at S position spos(v) = #{A ops < v} + #{B ops < v}
  // (A first on ties, compose.py:54).  Each run's heads (the first op of its value in a
  // part) find spos by a 64-way search of the other part; the runs' dense index r comes
  // from an occupancy mask over S positions.  An op's group is (kind, r) and the
  // groups laid out kind-major ARE the window's T order of groups (T is ordered by kind,
  // then timestamp): one histogram + scan of KD * R counters gives every group's start,
  // then each group is ordered by (id, side, index) with interpolation buckets (one op
  // per bucket on random ids) and a rank inside the bucket, equal 32-bit keys on the
  // full ids.  A window with more than GMAX groups (very many distinct timestamps) fails
  // the plan as a window too large (f_fail 2): the host retries with smaller windows.
  constexpr bool runs_ok = RUNS;
  if constexpr (RUNS) {
    constexpr int OW = CAP / 32;     // occupancy words over S positions
    constexpr int GMAX = 4 * CAP;    // group counters (u16, in sts once the timestamps are dead)
    u32* occ = reinterpret_cast<u32*>(&ccnt[0][0]);  // (zeroed with ccnt before the load barrier)
    static_assert(sizeof(ccnt) >= OW * sizeof(u32), "occupancy words inside ccnt");
    __shared__ u16 occpre[OW];
    __shared__ u16 lasth[NCH];       // last head at or before the end of each 64-op chunk
    __shared__ u32 rinfo[2];         // groups fit, R
#if WF_HEADLIST
    __shared__ u16 hpre[NCH + 1];    // heads before each chunk (and in all)
    __shared__ u32 hna;              // the A part's heads (index of B's first head)
#endif
    u16* sp = sl;                    // S position of each head's run (element space)
    u32* gcnt = reinterpret_cast<u32*>(sts);             // group counters, two u16 per word
    static_assert(GMAX / 2 * sizeof(u32) <= sizeof(sts), "group counters inside sts");
    u32* bcnt = reinterpret_cast<u32*>(fin);             // bucket counters, two u16 per word (zeroed before the load barrier)
    u32* mkey = reinterpret_cast<u32*>(sts);             // bucket order: 32-bit keys (after the group starts are dead)
    u16* mel = reinterpret_cast<u16*>(reinterpret_cast<u32*>(sts) + CAP);  // ... and elements
    // a. run heads, the order check, each head's run position
    bool dec = false;
    if (t == 0) {
      dec = (a0 > 0 && na > 0 && prev_a > sts[0]) || (b0 > 0 && nb > 0 && prev_b > sts[na]);
      win_publish_widths(P.meta, &vbw[0][0], WAVES, vcur);
    }
    u64 hbr[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int e = t + NT * i;
      const bool valid = e < sz;
      const bool first = e == 0 || e == na;
      const u64 pv = sts[valid && !first ? e - 1 : 0];
      const bool head = valid && (first || pv != ts_r[i]);
      dec |= valid && !first && pv > ts_r[i];
      hbr[i] = __ballot(head);
      // this item's 64-op chunk: wave-uniform, and said so (t / WAVE is a lane value to the
      // compiler, which would then run the head searches below as lane-divergent loops)
      const int c = __builtin_amdgcn_readfirstlane((NT * i) / WAVE + wv);
      if (lane == 0 && c < NCH) gbits[c] = hbr[i];
#if !WF_HEADLIST
      // the heads of this chunk, one at a time with the whole wave: a 64-way search of
      // the other part for #{ops < v} (two or three rounds of one LDS read per lane)
      u64 hb = hbr[i];
      while (hb) {
        const int hl = __ffsll((unsigned long long)hb) - 1;
        hb &= hb - 1;
        const int eh = c * WAVE + hl;
        const u64 v = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(ts_r[i] >> 32), hl) << 32) |
                      (u64)(u32)__builtin_amdgcn_readlane((int)(u32)ts_r[i], hl);
        const bool sa = eh < na;
        const int o0 = sa ? na : 0, no = sa ? nb : na;
        int lo = 0, len = no;  // answer in [lo, lo + len]; everything before lo is < v
        while (len > 0) {
          const int S = (len + WAVE - 1) / WAVE;
          const int q = lane * S;
          const bool pr = q < len && sts[o0 + lo + (q < len ? q : 0)] < v;
          const int cnt = __popcll(__ballot(pr));
          if (cnt == 0) break;
          const int qp = lo + (cnt - 1) * S;  // the last sample below v
          const int hi = min(qp + S, lo + len);
          lo = qp + 1;
          len = hi - lo;
        }
        const int spos = (sa ? eh : eh - na) + lo;
        if (lane == 0) {
          sp[eh] = (u16)spos;
          atomicOr(&occ[spos >> 5], 1u << (spos & 31));
        }
      }
#endif
    }
#if WF_HEADLIST
    if (t == 0) hna = 0xffffu;  // (no B part: every head is A's)
#endif
    if (__syncthreads_or(dec)) {
      if (t == 0) atomicOr((unsigned long long*)&P.meta->f_fail, 1ull);
      return;
    }
#if WF_HEADLIST
    // the heads of both parts in one list, element order (A's first): hel[j], with the
    // heads before each chunk from one wave's scan of the chunk ballots
    u16* hel = sord;  // (free until step h)
    if (wv == 0) {
      const u32 h0 = lane < NCH ? (u32)__popcll(gbits[lane]) : 0u;
      const u32 h1 = lane + WAVE < NCH ? (u32)__popcll(gbits[lane + WAVE]) : 0u;
      const u32 i0 = wave_incl_sum_u32(h0), i1 = wave_incl_sum_u32(h1);
      const u32 t0 = (u32)__builtin_amdgcn_readlane((int)i0, WAVE - 1);
      if (lane < NCH) hpre[lane] = (u16)(i0 - h0);
      if (lane + WAVE < NCH) hpre[lane + WAVE] = (u16)(t0 + i1 - h1);
      if (lane == WAVE - 1) hpre[NCH] = (u16)(t0 + i1);
    }
    __syncthreads();
    {
      const u64 lt = lanemask_lt();
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int e = t + NT * i;
        const int c = __builtin_amdgcn_readfirstlane((NT * i) / WAVE + wv);
        if ((hbr[i] >> lane) & 1ull) {
          const u32 j = (u32)hpre[c] + (u32)__popcll(hbr[i] & lt);
          hel[j] = (u16)e;
          if (e == na) hna = j;
        }
      }
    }
    __syncthreads();
    {
      // each head: #{other part's ops < v} = the index of the other part's first head
      // whose timestamp is >= v (that op starts a run), by a binary search of the head list
      const u32 nH = hpre[NCH], nHA = hna == 0xffffu ? nH : hna;
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int e = t + NT * i;
        if (!((hbr[i] >> lane) & 1ull)) continue;
        const u64 v = ts_r[i];
        const bool sa = e < na;
        const u32 end = sa ? nH : nHA;
        u32 lo = sa ? nHA : 0u, hi = end;
        while (lo < hi) {
          const u32 mid = (lo + hi) >> 1;
          if (sts[hel[mid]] < v) lo = mid + 1;
          else hi = mid;
        }
        const int o0 = sa ? na : 0, no = sa ? nb : na;
        const int cnt = lo < end ? (int)hel[lo] - o0 : no;
        const int spos = (sa ? e : e - na) + cnt;
        sp[e] = (u16)spos;
        atomicOr(&occ[spos >> 5], 1u << (spos & 31));
      }
    }
    __syncthreads();
#endif
    RX_EXIT(1);
    // b. (wave 0) the last head of each chunk, the runs' dense index, the group count
    const u32 kpres = __builtin_amdgcn_readfirstlane(kmask_r);
    const int KD = __popc(kpres);
    const int kbits_r = 32 - __clz((int)(max(KD, 1) - 1));  // bits of a dense kind
    if (wv == 0) {
      static_assert(NCH <= 2 * WAVE && OW <= 4 * WAVE, "one wave covers the chunks and occupancy words");
      u32 carry = 0;  // (last head + 1; 0 = none yet)
#pragma unroll
      for (int c0 = 0; c0 < NCH; c0 += WAVE) {
        const int c = c0 + lane;
        const u64 hw = c < nch ? gbits[c] : 0ull;
        u32 lh = hw ? (u32)(c * WAVE + 63 - __clzll(hw)) + 1u : 0u;
        lh = max(wave_incl_max_u32(lh), carry);
        if (c < NCH) lasth[c] = (u16)(lh ? lh - 1u : 0u);
        carry = (u32)__builtin_amdgcn_readlane((int)lh, WAVE - 1);
      }
      u32 rsum = 0;
#pragma unroll
      for (int w0 = 0; w0 < OW; w0 += WAVE) {
        const int x = w0 + lane;
        const u32 o = x < OW ? occ[x] : 0u;
        const u32 pc = (u32)__popc(o), inc = wave_incl_sum_u32(pc);
        if (x < OW) occpre[x] = (u16)(rsum + inc - pc);
        rsum += (u32)__builtin_amdgcn_readlane((int)inc, WAVE - 1);
      }
      if (lane == 0) {
        rinfo[0] = (u32)KD * rsum <= (u32)GMAX && !(SMX_DIAG && P.ablate == 200);
        rinfo[1] = rsum;
      }
    }
    {  // the group counters (the timestamps are dead: every head has searched)
      typedef u32 __attribute__((ext_vector_type(4))) z4;
      for (int i = t; i < GMAX / 8; i += NT) reinterpret_cast<z4*>(gcnt)[i] = z4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    if (!rinfo[0]) {  // more (kind, run) groups than counters: smaller windows (f_fail 2)
      if (t == 0) atomicOr((unsigned long long*)&P.meta->f_fail, 2ull);
      return;
    }
    RX_EXIT(2);
    {
      const u32 R = rinfo[1];
      // c. each op's run (its head: in its chunk, else the last head of the earlier
      //    chunks), group g = dense kind * R + run, counted
      const u64 lem = lanemask_lt() | (1ull << lane);
      u32 g_r[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const int e = t + NT * i;
        const int c = __builtin_amdgcn_readfirstlane((NT * i) / WAVE + wv);
        const u64 m = hbr[i] & lem;
        const int h = m ? c * WAVE + 63 - __clzll(m) : (int)lasth[c > 0 ? c - 1 : 0];
        const u32 k = k_r[i] < SMX_N_KINDS ? k_r[i] : SMX_N_KINDS - 1;
        g_r[i] = 0xffffffffu;
        u32 r = 0, dk = 0;
        if (e < sz) {
          const u32 s = sp[h];
          r = occpre[s >> 5] + (u32)__popc(occ[s >> 5] & ((1u << (s & 31)) - 1u));
          dk = (u32)__popc(kpres & ((1u << k) - 1u));
          g_r[i] = dk * R + r;
        }
        // the wide windows: a wave inside one run (config 5: one run per window) has at
        // most KD distinct groups, counted per group by its lowest lane (a per-lane LDS
        // atomic on a handful of words serialises: wide window 0.422 -> 0.406 ms on config 5);
        // otherwise, and in the normal windows (many runs, where the test costs more than it
        // saves), one atomic per op
        bool agg = false;
        u32 r0 = 0;
        if constexpr (WF_GAGG >= 2 || (WF_GAGG == 1 && CAP > WF_CAP)) {
          const u64 vm = __ballot(e < sz);
          r0 = (u32)__builtin_amdgcn_readfirstlane((int)r);
          // (WF_GAGG 2: also a wave over two runs, one more ballot)
          agg = vm && __ballot(e < sz && r - r0 > (WF_GAGG >= 2 ? 1u : 0u)) == 0;
        }
        if (agg) {
          const u64 peers = WF_GAGG >= 2 ? wave_peers_n(dk << 1 | (r - r0), e < sz, kbits_r + 1)
                                         : wave_peers_n(dk, e < sz, kbits_r);
          if (e < sz && (peers & lanemask_lt()) == 0)
            atomicAdd(&gcnt[g_r[i] >> 1], (u32)__popcll(peers) << (16 * (g_r[i] & 1)));
        } else if (e < sz) {
          atomicAdd(&gcnt[g_r[i] >> 1], 1u << (16 * (g_r[i] & 1)));
        }
      }
      __syncthreads();
      RX_EXIT(3);
      // d. group starts: exclusive scan of the KD * R counters (kind-major = T order), in
      //    passes of 4 * NT counters (one pass on config 3's windows: 6 kinds x 14 runs)
      const int GS = KD * (int)R;
      {
        u32 carry = 0;
        for (int g0 = 0; g0 < GS; g0 += 4 * NT) {  // (block-uniform)
          const int x = g0 / 2 + 2 * t;  // words x, x + 1: counters 2x .. 2x + 3
          const u32 w0 = 2 * x < GS ? gcnt[x] : 0u, w1 = 2 * x + 2 < GS ? gcnt[x + 1] : 0u;
          const u32 c0 = w0 & 0xffffu, c1 = w0 >> 16, c2 = w1 & 0xffffu, c3 = w1 >> 16;
          u32 tot;
          const u32 run = carry + block_excl_scan<OpSum, u32, WAVES>(c0 + c1 + c2 + c3, &vbw[0][0], &tot);
          if (2 * x < GS) gcnt[x] = run | ((run + c0) << 16);
          if (2 * x + 2 < GS) gcnt[x + 1] = (run + c0 + c1) | ((run + c0 + c1 + c2) << 16);
          carry += tot;
        }
      }
      __syncthreads();
      auto gstart = [&](int g) -> u32 {
        return g < GS ? (gcnt[g >> 1] >> (16 * (g & 1))) & 0xffffu : (u32)sz;
      };
      // kinds: window-local start and count (kind k's groups are d(k) * R .. + R)
      if (t <= SMX_N_KINDS) {
        u32 s = (u32)sz, e = (u32)sz;
        if (t < SMX_N_KINDS) {
          const int d = __popc(kpres & ((1u << t) - 1u));
          s = R ? gstart(d * (int)R) : 0u;
          e = ((kpres >> t) & 1u) && R ? gstart((d + 1) * (int)R) : s;
          wck[t] = e - s;
        }
        kbase[t] = s;
      }
      RX_EXIT(4);
      // e. interpolation bucket inside the group: b = gs + (ge - gs) * key / 2^32
      u32 b_r[ITEMS], ar_r[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        b_r[i] = 0xffffffffu;
        ar_r[i] = 0u;
        if (g_r[i] == 0xffffffffu) continue;
        const u32 gs = gstart((int)g_r[i]), ge = gstart((int)g_r[i] + 1);
        const u32 b = gs + (u32)(((u64)(ge - gs) * hi_r[i]) >> 32);
        b_r[i] = b;
        ar_r[i] = (atomicAdd(&bcnt[b >> 1], 1u << (16 * (b & 1))) >> (16 * (b & 1))) & 0xffffu;
      }
      __syncthreads();
      RX_EXIT(5);
      // f. bucket starts
      {
        constexpr int WPT = CAP / (2 * NT);
        u32 cw[WPT], sum = 0;
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
          cw[i] = bcnt[WPT * t + i];
          sum += (cw[i] & 0xffffu) + (cw[i] >> 16);
        }
        u32 tot;
        u32 run = block_excl_scan<OpSum, u32, WAVES>(sum, &vbw[0][0], &tot);
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
          const u32 c0 = cw[i] & 0xffffu, c1 = cw[i] >> 16;
          bcnt[WPT * t + i] = run | ((run + c0) << 16);
          run += c0 + c1;
        }
      }
      __syncthreads();
      auto bstart = [&](u32 b) -> u32 {
        return b < (u32)CAP ? (bcnt[b >> 1] >> (16 * (b & 1))) & 0xffffu : (u32)sz;
      };
      RX_EXIT(6);
      // g. members in bucket order: key and element
      u32 slot_r[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        slot_r[i] = 0u;
        if (b_r[i] == 0xffffffffu) continue;
        const u32 s = bstart(b_r[i]) + ar_r[i];
        slot_r[i] = s;
        mkey[s] = hi_r[i];
        mel[s] = (u16)(t + NT * i);
      }
      __syncthreads();
      RX_EXIT(7);
      // h. rank inside the bucket on (key, full id, side, index); the final order
      //    (per-lane loops: one op per bucket on average; a wave-uniform loop over the
      //    ITEMS buckets together spilled registers)
#if WF_HBATCH
      // every item's bucket end and first member read together (independent LDS reads:
      // one round trip for the ITEMS buckets; a bucket holds one op on average), the
      // rest of a bucket by the loop below
      u32 hw_r[ITEMS], x0_r[ITEMS];
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 b = b_r[i] == 0xffffffffu ? 0u : b_r[i];
        const u32 b1 = b + 1 < (u32)CAP ? b + 1 : (u32)CAP - 1;
        hw_r[i] = bcnt[b1 >> 1];
        x0_r[i] = mkey[slot_r[i] - ar_r[i]];
      }
#endif
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const u32 b = b_r[i];
        if (b == 0xffffffffu) continue;
        const int e = t + NT * i;
        const u32 b1 = b + 1 < (u32)CAP ? b + 1 : (u32)CAP - 1;  // (branch-free bucket bounds)
#if WF_LOREG
        const u32 lo = slot_r[i] - ar_r[i];  // (the bucket's start: this op's slot less its arrival rank)
#else
        const u32 lo = (bcnt[b >> 1] >> (16 * (b & 1))) & 0xffffu;
#endif
#if WF_HBATCH
        const u32 hw = (hw_r[i] >> (16 * (b1 & 1))) & 0xffffu;
#else
        const u32 hw = (bcnt[b1 >> 1] >> (16 * (b1 & 1))) & 0xffffu;
#endif
        const u32 hi = b + 1 < (u32)CAP ? hw : (u32)sz, kp = hi_r[i];
        u32 c = 0;
        bool tie = false;
#if WF_HBATCH
        {  // the first member (lo < hi: this op is in the bucket)
          const u32 x = x0_r[i];
          c += x < kp;
          tie |= (x == kp) & (lo != slot_r[i]);
        }
#pragma unroll 1
        for (u32 q = lo + 1; q < hi; ++q) {
#else
#pragma unroll 1
        for (u32 q = lo; q < hi; ++q) {  // (own slot: x == kp, not a tie)
#endif
          const u32 x = mkey[q];
          c += x < kp;
          tie |= (x == kp) & (q != slot_r[i]);
        }
        if (tie) {  // equal top 32 bits (rare): the full ids, then element order = (side, index)
          c = 0;
          const i64 jm = e < na ? a0 + e : bld + e;
          const u64 hm = P.khi[jm], lm = P.klo[jm];
#pragma unroll 1
          for (u32 q = lo; q < hi; ++q) {
            const u32 x = mkey[q];
            if (x != kp || q == slot_r[i]) {
              c += x < kp;
              continue;
            }
            const int eo = mel[q];
            const i64 jo = eo < na ? a0 + eo : bld + eo;
            const u64 ho = P.khi[jo], lo2 = P.klo[jo];
            c += ho < hm || (ho == hm && (lo2 < lm || (lo2 == lm && eo < e)));
          }
        }
        const u32 f = lo + c;
        sord[f] = (u16)e;
        inv[e] = (u16)f;
        skS[f] = (u8)(k_r[i] < SMX_N_KINDS ? k_r[i] : SMX_N_KINDS - 1);
      }
      __syncthreads();
      RX_EXIT(8);
    }
  }
  if constexpr (!RUNS) {  // steps 2-5: merge, multisplit, group order
  // 2. merge A part [0,na) with B part [na,sz) by timestamp, A first on ties
  //    (compose.py:54): merge path, ITEMS outputs per lane, with the kinds
  //    copied into S order.  Presorted-layout check: every adjacent pair of each
  //    branch log is non-decreasing (the pair straddling a window start is checked
  //    here too); it shares the merge's barrier and a window that fails it discards
  //    the merge.
  bool dec = false;
  if (t == 0) {
    dec = (a0 > 0 && na > 0 && prev_a > sts[0]) || (b0 > 0 && nb > 0 && prev_b > sts[na]);
    win_publish_widths(P.meta, &vbw[0][0], WAVES, vcur);
  }
#if WF_RUNMERGE
  // Run-head merge.  Inside a branch the timestamps never decrease, so an op's merged
  // position is its branch index plus the other branch's ops before its timestamp run
  // (A first on ties: for an A op the B ops with a smaller timestamp, for a B op the A
  // ops with a smaller or equal one).  Only the first op of each run (a head) searches
  // the other branch; the rest read their head's count.  (Config 2 / 3 windows hold ~14
  // runs per branch, config 5's wide windows one: a few searches instead of a merge-path
  // search and a merge step chain per thread.)
  u64* rbits = gbits;  // [NCH] head bits over elements (gbits is next written in step 4)
  u16* hl = fin;       // per wave: its heads' elements (fin is next written in step 3)
  u16* roff = sl;      // per head element: the other branch's ops before its run (sl: step 3)
  u64 hb[ITEMS];
  int nh = 0;  // this wave's heads (wave-uniform)
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    const bool valid = e < sz;
    const u64 pv = sts[valid && e > 0 ? e - 1 : 0];
    const bool head = valid && (e == 0 || e == na || pv != ts_r[i]);
    if (!(SMX_DIAG && (P.ablate & 1))) dec |= valid && e != 0 && e != na && pv > ts_r[i];
    hb[i] = __ballot(head);
    if (lane == 0) rbits[(NT * i) / WAVE + wv] = hb[i];
    if (head) hl[wv * (ITEMS * WAVE) + nh + (int)__popcll(hb[i] & lanemask_lt())] = (u16)e;
    nh += (int)__popcll(hb[i]);
  }
  wave_lds_sync();  // this wave's head list, for its own lanes
  for (int r = 0; r < nh; r += WAVE) {
    if (r + lane < nh) {
      const int e = hl[wv * (ITEMS * WAVE) + r + lane];
      const u64 x = sts[e];
      int lo = 0, hi = e < na ? nb : na;
      if (e < na) {  // B ops with a smaller timestamp
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (sts[na + mid] < x) lo = mid + 1;
          else hi = mid;
        }
      } else {  // A ops with a smaller or equal timestamp
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (sts[mid] <= x) lo = mid + 1;
          else hi = mid;
        }
      }
      roff[e] = (u16)lo;
    }
  }
#else
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    if (e >= sz) continue;
    if (!(SMX_DIAG && (P.ablate & 1)) && e != 0 && e != na && sts[e - 1] > ts_r[i]) dec = true;
  }
  {
    const int d0 = t * ITEMS < sz ? t * ITEMS : sz;
    const int d1 = d0 + ITEMS < sz ? d0 + ITEMS : sz;
    int lo = d0 - nb > 0 ? d0 - nb : 0, hi = d0 < na ? d0 : na;
    // (a fixed count of predicated halving steps measured slower: window 1.225 -> 1.270 ms,
    //  profiles/r03_x/ab_merge_search_fixed_steps.txt)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sts[mid] <= sts[na + d0 - 1 - mid]) lo = mid + 1;
      else hi = mid;
    }
    int ia = lo, ib = d0 - lo;
#if WF_BF
    // ITEMS outputs, predicated (a thread past sz stores nothing)
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
      const int d = d0 + u;
      const u64 ta = sts[ia < na ? ia : 0], tb = sts[na + (ib < nb ? ib : 0)];
      const bool take_a = ia < na && (ib >= nb || ta <= tb);
      const int e = take_a ? ia : na + ib;
      ia += take_a ? 1 : 0;
      ib += take_a ? 0 : 1;
      if (d < d1) {
        sord[d] = (u16)e;
        skS[d] = skind[e];
      }
    }
#else
    for (int d = d0; d < d1; ++d) {
      const bool take_a = ia < na && (ib >= nb || sts[ia] <= sts[na + ib]);
      const int e = take_a ? ia++ : na + ib++;
      sord[d] = (u16)e;
      skS[d] = skind[e];
    }
#endif
  }
#endif
  if (__syncthreads_or(dec)) {
    if (t == 0) atomicOr((unsigned long long*)&P.meta->f_fail, 1ull);
    return;
  }
#if WF_RUNMERGE
  {
    // each op's head: the last head at or before it -- in its own 64-op chunk (the
    // ballot), else the last head of the nearest earlier chunk that has one (every
    // chunk's head word read once per wave; lane broadcasts with the whole wave active)
    const int nchw = (sz + WAVE - 1) / WAVE;
    const u64 rw0 = lane < nchw ? rbits[lane] : 0ull;
    const u64 rnz0 = __ballot(rw0 != 0);
    const u64 rw1 = NCH > WAVE && WAVE + lane < nchw ? rbits[(WAVE + lane) % NCH] : 0ull;
    const u64 rnz1 = NCH > WAVE ? __ballot(rw1 != 0) : 0ull;
    auto bc64 = [](u64 v, int l) -> u64 {
      return (u64)(u32)__builtin_amdgcn_readlane((int)(u32)v, l) |
             ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), l) << 32);
    };
    const u64 lem = lanemask_lt() | (1ull << lane);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int c = (NT * i) / WAVE + wv;  // this wave's chunk (uniform)
      if (c * WAVE >= sz) break;          // (uniform)
      // the last non-empty chunk before c (chunk 0 starts with a head, so c > 0 has one)
      const int cl = c & (WAVE - 1);
      const u64 b0 = c < WAVE ? rnz0 & ((1ull << cl) - 1) : rnz0;
      const u64 b1 = c < WAVE ? 0ull : rnz1 & ((1ull << cl) - 1);
      const int wp = b1 ? WAVE + 63 - __clzll(b1) : (b0 ? 63 - __clzll(b0) : 0);
      const u64 wpw = wp < WAVE ? bc64(rw0, wp & (WAVE - 1)) : bc64(rw1, wp & (WAVE - 1));
      const int hprev = wp * WAVE + 63 - __clzll(wpw | 1ull);
      const u64 below = hb[i] & lem;
      const int e = t + NT * i;
      if (e < sz) {
        const int h = below ? c * WAVE + 63 - __clzll(below) : hprev;
        const int pos = (e < na ? e : e - na) + (int)roff[h];
        const u32 kr = k_r[i] < SMX_N_KINDS ? k_r[i] : SMX_N_KINDS - 1;
        sord[pos] = (u16)e;
        skS[pos] = (u8)kr;
      }
    }
  }
  __syncthreads();
#endif
  WSTAMP(3);
  WF_EXIT(2);

  // 3. stable multisplit of S by rank (wave ballots); element, kind and rank stay in
  //    registers for the scatter (m = t + NT * j is chunk wv + WAVES * j)
  int me[ITEMS];
  u32 mkr[ITEMS];  // kind | rank << 8
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int m = t + NT * j;
    me[j] = m < sz ? sord[m] : 0;
    mkr[j] = m < sz ? skS[m] : 0u;
  }
  const u64 ltm = lanemask_lt();
#if WF_DENSE_KINDS
  // the ballots run over the dense index of the kinds present in the merge (k_khist's
  // kind masks): 6 kinds take 3 ballots instead of 5
  const u32 kpres = __builtin_amdgcn_readfirstlane(kmask_r);
  const int kbits = 32 - __clz((int)(max(__popc(kpres), 1u) - 1u));
#endif
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int m = t + NT * j;
    const int c = wv + WAVES * j;
    const bool valid = m < sz;
    const u32 k = mkr[j];
#if WF_DENSE_KINDS
    const u64 peers = wave_peers_n((u32)__popc(kpres & ((1u << k) - 1u)), valid, kbits);
#else
    const u64 peers = wave_peers<5>(k, valid);
#endif
    const u32 r = __popcll(peers & ltm);
    mkr[j] = k | (r << 8);
    if (valid && r == 0) {
      ccnt[c][k] = (u16)__popcll(peers);
      atomicAdd(&wck[k], (u32)__popcll(peers));
    }
  }
  __syncthreads();
  WSTAMP(4);
  WF_EXIT(3);
  for (int k = wv; k < SMX_N_KINDS; k += WAVES) {
    u32 carry = 0;
#pragma unroll
    for (int c0 = 0; c0 < NCH; c0 += WAVE) {  // (one pass when NCH <= 64)
      const int c = c0 + lane;
      const u32 x = c < nch ? ccnt[c][k] : 0u;
      const u32 inc = wave_incl_sum(x);
      if (c < nch) ccnt[c][k] = (u16)(carry + inc - x);
      if (NCH > WAVE) carry += (u32)__builtin_amdgcn_readlane((int)inc, WAVE - 1);
    }
  }
  if (wv == WAVES - 1) {  // (kinds 7 and 15 only on this wave)
    const u32 x = lane < SMX_N_KINDS ? wck[lane] : 0u;
    const u32 inc = wave_incl_sum(x);
    if (lane < SMX_N_KINDS) kbase[lane] = inc - x;
    if (lane == SMX_N_KINDS - 1) kbase[SMX_N_KINDS] = inc;
  }
  __syncthreads();
  WSTAMP(6);
  WF_EXIT(4);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int m = t + NT * j;
    if (m < sz) {
      const u32 k = mkr[j] & 0xffu;
      const int p = kbase[k] + ccnt[wv + WAVES * j][k] + (mkr[j] >> 8);
      fin[p] = (u16)me[j];
      sl[me[j]] = (u16)p;
      if (WF_OUT2) skS[p] = (u8)k;  // (skS was read in the prologue, before two barriers)
    }
  }
  __syncthreads();
  WSTAMP(7);
  WF_EXIT(5);

  // 4. group-start bits (a group = equal (rank, timestamp), contiguous in slots),
  //    then the timestamps are dead and their buffer takes the slot-space oid prefix
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int p = t + NT * j;
    bool f = false;
    if (p < sz) {
      const int e = fin[p];
#if WF_OUT2
      f = (p == (int)kbase[skS[p]]) || (sts[fin[p - 1]] != sts[e]);  // (skS: kinds by slot)
#else
      f = (p == (int)kbase[skind[e]]) || (sts[fin[p - 1]] != sts[e]);
#endif
    }
    const u64 b = __ballot(f);
    if (lane == 0 && (p >> 6) < NCH) gbits[p >> 6] = b;
  }
  __syncthreads();
  WSTAMP(8);
  WF_EXIT(6);
  // slot-space rank keys: the top 32 bits of oid_hi; sl is reset to "no slot" for
  // the rank phase's collision check
  u32* pkey = (u32*)sts;
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    if (e < sz) {
      const int p = sl[e];
      pkey[p] = hi_r[i];
      sl[e] = 0xffffu;
    }
  }
#if WF_BUCKET && WF_BZ4
  // step 5's bucket counters (the upper half of sts: the timestamps are dead)
  for (int i = t; i < CAP / 2; i += NT) reinterpret_cast<u32*>(sts)[CAP + i] = 0u;
#endif
  __syncthreads();
  WSTAMP(9);
  WF_EXIT(7);

  // 5. order each group by (oid, side, index): counting rank over the group on the
  //    32-bit keys, four per LDS read.  Two keys of a group that are equal (about one
  //    window in 10^4 on random ids; every duplicate id) get the same rank and leave
  //    a rank without a slot: such a window is re-ranked exactly on (oid_hi, oid_lo,
  //    slot) -- slot order is (side, index) order inside a group.
  // the group bounds of a wave's 64 consecutive slots from one read of every
  // group-start word (nch <= 32) and lane broadcasts: no dependent LDS chain
  // (NCH > 64: a second word per lane, gw1 / gnz1 for chunks 64..127)
  const u64 gw = lane < nch ? gbits[lane] : 0ull;
  const u64 gnz = __ballot(gw != 0);
  const u64 gw1 = NCH > WAVE && WAVE + lane < nch ? gbits[(WAVE + lane) % NCH] : 0ull;
  const u64 gnz1 = NCH > WAVE ? __ballot(gw1 != 0) : 0ull;
  auto bcast64 = [](u64 v, int l) -> u64 {
    return (u64)(u32)__builtin_amdgcn_readlane((int)(u32)v, l) |
           ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), l) << 32);
  };
  // group-start word i (wave-uniform i < NCH), with the whole wave active
  auto gword = [&](int i) -> u64 {
    if (NCH <= WAVE) return bcast64(gw, i);
    const u64 a = bcast64(gw, i & (WAVE - 1)), b = bcast64(gw1, i & (WAVE - 1));
    return i < WAVE ? a : b;
  };
  const u64 le_mask = lanemask_lt() | (1ull << lane);
#if WF_BUCKET
#endif
#if WF_BUCKET
  // interpolation buckets over slot space: slot p of group [gs, ge) goes to bucket
  // gs + (ge - gs) * key / 2^32 (one op per bucket on random ids); 16-bit counters,
  // two per word, in the upper half of sts (free until step 7)
  u32* bcnt = reinterpret_cast<u32*>(sts) + CAP;
#if WF_BK16
  // the top 16 bits of each key in bucket order (the last quarter of sts): the rank
  // loop compares them without the slot -> key chain, the full key only on a tie
  u16* bk16 = reinterpret_cast<u16*>(reinterpret_cast<u32*>(sts) + CAP + CAP / 2);
  u32 own_r[ITEMS];
#endif
#if !WF_BZ4
  for (int i = t; i < CAP / 2; i += NT) bcnt[i] = 0u;
  __syncthreads();
#endif
  u32 bk_r[ITEMS];
  u32 kp_r[ITEMS];
#if WF_ONEATOM
  u32 ar_r[ITEMS];  // arrival rank inside the bucket (the count atomic's return value)
#endif
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) bk_r[j] = 0xffffffffu, kp_r[j] = 0u;
#endif
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int wi = __builtin_amdgcn_readfirstlane((NT * j) / WAVE + wv);  // this wave's slot chunk
    if (wi >= nch) break;  // wave-uniform
    const int p = wi * WAVE + lane;
    // Group bounds, branch-free: every lane broadcast (v_readlane) runs with the whole
    // wave active.  (Lane reads inside the lanes' divergent branches mis-ordered groups
    // in some builds: a register's value in lanes outside the branch is not defined.)
    // The last group start before the chunk and the first one after it are scalar.
    const u64 W = gword(wi);
    int wp, wn;
    bool has_next;
    if (NCH <= WAVE) {
      const u64 prevm = gnz & ((1ull << wi) - 1);  // (slot 0 always starts a group)
      wp = prevm ? 63 - __clzll(prevm) : 0;
      const u64 nxtm = wi + 1 < WAVE ? gnz & ~((2ull << wi) - 1) : 0ull;
      has_next = nxtm != 0;
      wn = nxtm ? __ffsll((unsigned long long)nxtm) - 1 : 0;
    } else {
      // the last non-empty word before wi and the first after it, over 128 words
      const int wl = wi & (WAVE - 1);
      const u64 below0 = wi < WAVE ? gnz & ((1ull << wl) - 1) : gnz;
      const u64 below1 = wi < WAVE ? 0ull : gnz1 & ((1ull << wl) - 1);
      wp = below1 ? WAVE + 63 - __clzll(below1) : (below0 ? 63 - __clzll(below0) : 0);
      const u64 above0 = wi < WAVE ? (wl + 1 < WAVE ? gnz & ~((2ull << wl) - 1) : 0ull) : 0ull;
      const u64 above1 = wi < WAVE ? gnz1 : (wl + 1 < WAVE ? gnz1 & ~((2ull << wl) - 1) : 0ull);
      has_next = (above0 | above1) != 0;
      wn = above0 ? __ffsll((unsigned long long)above0) - 1
                  : (above1 ? WAVE + __ffsll((unsigned long long)above1) - 1 : 0);
    }
    const int prevS = wp * WAVE + 63 - __clzll(gword(wp) | 1ull);
    const u64 Wn = gword(wn);
    const int nextS = has_next ? wn * WAVE + __ffsll((unsigned long long)(Wn | (1ull << 63))) - 1 : sz;
    const u64 below = W & le_mask, above = W & ~le_mask;
    const int gs = below ? wi * WAVE + 63 - __clzll(below | 1ull) : prevS;
    int ge = above ? wi * WAVE + __ffsll((unsigned long long)(above | (1ull << 63))) - 1 : nextS;
    ge = ge < sz ? ge : sz;
    if (p >= sz) continue;
#if WF_BUCKET
    {
      const u32 kp = pkey[p];
      const u32 b = (u32)gs + (u32)(((u64)(u32)(ge - gs) * kp) >> 32);
      kp_r[j] = kp;
      bk_r[j] = b;
#if WF_ONEATOM
      ar_r[j] = (atomicAdd(&bcnt[b >> 1], 1u << (16 * (b & 1))) >> (16 * (b & 1))) & 0xffffu;
#else
      atomicAdd(&bcnt[b >> 1], 1u << (16 * (b & 1)));
#endif
      continue;
    }
#endif
    int r = p;
    if (ge - gs > 1 && !(SMX_DIAG && (P.ablate & 2))) {
      const u32 kp = pkey[p];
      const uint4* pv = reinterpret_cast<const uint4*>(pkey);
      const int q0 = gs & ~3;
      int c = 0;
      int q = q0;
      for (; q + 8 <= ge; q += 8) {  // 2 x 16 bytes of keys per step in flight
        const uint4 x0 = pv[q / 4], x1 = pv[q / 4 + 1];
        c += rk4(x0, kp) + rk4(x1, kp);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // fewer left: up to 2 more reads, masked
        const int qq = q + 4 * u;
        if (qq < ge) c += rk4(pv[qq / 4], kp, ge - qq);
      }
      if (q0 < gs) c -= rk4(pv[q0 / 4], kp, gs - q0);  // slots before the group
      r = gs + c;
    }
    sord[r] = fin[p];
    sl[r] = (u16)p;  // sl now maps rank -> slot
#if WF_OUT2
    inv[fin[p]] = (u16)r;
#endif
  }
#if WF_BUCKET
  {
    __syncthreads();
    // exclusive scan of the CAP counters: CAP / NT per thread (two 16-bit ones per word)
    constexpr int WPT = CAP / (2 * NT);
    u32 cw[WPT], sum = 0;
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      cw[i] = bcnt[WPT * t + i];
      sum += (cw[i] & 0xffffu) + (cw[i] >> 16);
    }
    u32 tot;
    u32 run = block_excl_scan<OpSum, u32, WAVES>(sum, &vbw[0][0], &tot);  // (vbw is dead after step 2)
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const u32 c0 = cw[i] & 0xffffu, c1 = cw[i] >> 16;
      bcnt[WPT * t + i] = run | ((run + c0) << 16);
      run += c0 + c1;
    }
    __syncthreads();
    // scatter the slots into their buckets (sl: bucket position -> slot); the counters
    // become the bucket ends (WF_ONEATOM: they stay the starts; position = start +
    // arrival rank, no second atomic)
    u32 lo_r[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const u32 b = bk_r[j];
      lo_r[j] = 0;
      if (b == 0xffffffffu) continue;
      const u32 sh = 16 * (b & 1);
#if WF_ONEATOM
      lo_r[j] = (bcnt[b >> 1] >> sh) & 0xffffu;
      const u32 pos = lo_r[j] + ar_r[j];
#else
      const u32 old = atomicAdd(&bcnt[b >> 1], 1u << sh);
      const u32 pos = (old >> sh) & 0xffffu;
#endif
      sl[pos] = (u16)((NT * j) / WAVE * WAVE + wv * WAVE + lane);
#if WF_BK16
      own_r[j] = pos;
      bk16[pos] = (u16)(kp_r[j] >> 16);
#endif
    }
    __syncthreads();
    // rank inside the bucket on the 32-bit key
    int rr[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const u32 b = bk_r[j];
      rr[j] = -1;
      if (b == 0xffffffffu) continue;
#if WF_ONEATOM
      // bucket [start(b), start(b + 1)); the starts are an exclusive scan over every
      // bucket of the window (buckets past the last slot start at the total)
      const u32 lo = lo_r[j];
      const u32 e = b + 1 < (u32)CAP ? (bcnt[(b + 1) >> 1] >> (16 * ((b + 1) & 1))) & 0xffffu : (u32)sz;
#else
      const u32 e = (bcnt[b >> 1] >> (16 * (b & 1))) & 0xffffu;
      const u32 lo = b ? (bcnt[(b - 1) >> 1] >> (16 * ((b - 1) & 1))) & 0xffffu : 0u;
#endif
      const u32 kp = kp_r[j];
      u32 c = 0, eq = 0;
#if WF_BK16
      const u32 k16 = kp >> 16, own = own_r[j];
      eq = 1;
#if WF_RANK8
      // buckets of at most 8 (all but ~1e-5 of the elements on random ids): eight
      // predicated compares, no lane-divergent loop (whose exec-mask bookkeeping is
      // scalar work, the window's scarcest issue slot); larger buckets and equal top
      // halves take the general loop below
      {
        const u32 nb = e - lo;
        bool gen = nb > 8;
#pragma unroll
        for (u32 i = 0; i < 8; ++i) {
          const u32 q = lo + i;
          const u32 x = bk16[q];  // (past the bucket: masked; LDS reads never fault)
          const bool in = i < nb && q != own;
          c += (in && x < k16) ? 1u : 0u;
          gen |= in && x == k16;
        }
        if (gen) c = 0;
        for (u32 q = gen ? lo : e; q < e; ++q) {
#else
      {
      for (u32 q = lo; q < e; ++q) {
#endif
        const u32 x = bk16[q];
        if (q == own) continue;
        if (x != k16) {
          c += x < k16;
        } else {  // equal top halves: the full keys (rare)
          const u32 k = pkey[sl[q]];
          if (!TIEFIX || k != kp) {
            c += k < kp;
            eq += k == kp;
          } else {
            // equal 32-bit keys (duplicate ids; ~1 pair in 2^33 per group on random
            // ids): the full ids, then slot order -- (side, index) order in a group
            const int pm = (NT * j) / WAVE * WAVE + wv * WAVE + lane, po = sl[q];
            const int em = fin[pm], eo = fin[po];
            const i64 jm = em < na ? a0 + em : bld + em, jo = eo < na ? a0 + eo : bld + eo;
            const u64 hm = P.khi[jm], ho = P.khi[jo], lm = P.klo[jm], lo2 = P.klo[jo];
            c += ho < hm || (ho == hm && (lo2 < lm || (lo2 == lm && po < pm)));
          }
        }
      }
      }
#else
      for (u32 q = lo; q < e; ++q) {
        const u32 k = pkey[sl[q]];
        c += k < kp;
        eq += k == kp;
      }
#endif
      btie |= eq > 1;
      rr[j] = (int)(lo + c);
      if (WF_FUSEFIN && !DBG) {
        // the final order at once: nothing in this loop reads sord or inv, and the
        // rank -> slot map is not needed after step 5 (the exact re-rank rebuilds it)
        const int e = fin[(NT * j) / WAVE * WAVE + wv * WAVE + lane];
        sord[rr[j]] = (u16)e;
#if WF_OUT2
        inv[e] = (u16)rr[j];
#endif
      }
    }
    if (!(WF_FUSEFIN && !DBG)) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        if (rr[j] < 0) continue;
        const int p = (NT * j) / WAVE * WAVE + wv * WAVE + lane;
        const int e = fin[p];
        sord[rr[j]] = (u16)e;
        sl[rr[j]] = (u16)p;  // sl maps rank -> slot (the diagnostic order check)
#if WF_OUT2
        inv[e] = (u16)rr[j];
#endif
      }
    }
  }
#endif
  __syncthreads();
  if (DBG) {  // diagnostics: the group order against the slot-space keys (dbg words 5, 17, 18)
    for (int r = t + 1; r < sz; r += NT) {
      const bool start = (gbits[r >> 6] >> (r & 63)) & 1ull;
      if (!start && pkey[sl[r - 1]] > pkey[sl[r]]) atomicAdd((unsigned long long*)&P.dbg[w * WF_NSTAMP + 5], 1ull);
      if (!start && sts[0] == 0x12345ull) P.meta->dup_key = 3;  // (keeps sts live)
    }
    for (int r = t; r < sz; r += NT) {
      const int p0 = sl[r];
      if (p0 >= sz) atomicAdd((unsigned long long*)&P.dbg[w * WF_NSTAMP + 17], 1ull);
      else if (fin[p0] != sord[r]) atomicAdd((unsigned long long*)&P.dbg[w * WF_NSTAMP + 18], 1ull);
    }
  }
  WSTAMP(10);
  WF_EXIT(8);
  }  // (!RUNS)
  // 6. renames: rank among the window's renames of the same branch (final order).
  //    Computed in the collision-check phase into registers (rown aliases fin, which
  //    the exact re-rank still reads) and stored once no tie is known; redone after a
  //    (rare) exact re-rank.
  const int R0 = kbase[KREN], RN = wck[KREN];
  const int nrc = (RN + WAVE - 1) / WAVE;
  constexpr int RQ = (NCH + WAVES - 1) / WAVES;  // rename chunks per wave
  u32 rown_r[RQ];
  auto rename_ranks = [&](bool store) {
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int c = wv + q * WAVES;
      rown_r[q] = 0;
      if (c >= nrc) continue;  // wave-uniform
      const int x = c * WAVE + lane;
      const bool valid = x < RN;
      const int e = valid ? sord[R0 + x] : 0;
      const bool sb = valid && e >= na;
      const u64 bm = __ballot(sb), vm = __ballot(valid);
      const u64 lt = lanemask_lt();
      rown_r[q] = (u32)(sb ? __popcll(bm & lt) : __popcll(vm & ~bm & lt));
      if (store && valid) rown[x] = (u16)rown_r[q];
      if (lane == 0) {
        rc[c][0] = (u16)__popcll(vm & ~bm);
        rc[c][1] = (u16)__popcll(bm);
      }
    }
  };
  bool tie = false;
#if WF_BUCKET
  tie = btie;
#else
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const int r = t + NT * j;
    if (r < sz) tie |= sl[r] == 0xffffu;
  }
#endif
  rename_ranks(false);
  const bool any_tie = __syncthreads_or(tie);
  WSTAMP(21);
  if (any_tie) {
    // exact ranks from the full ids (global memory; rare)
    for (int p = t; p < sz; p += NT) {
      int gs, ge;
      group_of(p, &gs, &ge);
      const int ex = fin[p];
      const i64 jx = ex < na ? a0 + ex : bld + ex;
      const u64 hx = P.khi[jx], lx = P.klo[jx];
      int c = 0;
      for (int q = gs; q < ge; ++q) {
        if (q == p) continue;
        const int ey = fin[q];
        const i64 jy = ey < na ? a0 + ey : bld + ey;
        const u64 hy = P.khi[jy], ly = P.klo[jy];
        c += hy < hx || (hy == hx && (ly < lx || (ly == lx && q < p)));
      }
      sl[gs + c] = (u16)p;
    }
    __syncthreads();
    for (int r = t; r < sz; r += NT) {
      const int e = fin[sl[r]];
      sord[r] = (u16)e;
#if WF_OUT2
      inv[e] = (u16)r;
#endif
    }
    __syncthreads();
    rename_ranks(true);
    __syncthreads();
  } else {
#pragma unroll
    for (int q = 0; q < RQ; ++q) {  // fin is dead now: the ranks go to rown
      const int x = (wv + q * WAVES) * WAVE + lane;
      if (wv + q * WAVES < nrc && x < RN) rown[x] = (u16)rown_r[q];
    }
  }
  WSTAMP(11);
  if (wv == 0) {
    u32 c0s = 0, c1s = 0;  // carries over 64-chunk passes
#pragma unroll
    for (int cb0 = 0; cb0 < NCH; cb0 += WAVE) {
      const int c = cb0 + lane;
      const u32 x0 = c < nrc ? rc[c][0] : 0u;
      const u32 x1 = c < nrc ? rc[c][1] : 0u;
      const u32 i0 = wave_incl_sum(x0), i1 = wave_incl_sum(x1);
      if (c < nrc) {
        rc[c][0] = (u16)(c0s + i0 - x0);
        rc[c][1] = (u16)(c1s + i1 - x1);
      }
      c0s += (u32)__builtin_amdgcn_readlane((int)i0, WAVE - 1);
      c1s += (u32)__builtin_amdgcn_readlane((int)i1, WAVE - 1);
    }
    if (lane == WAVE - 1) {
      wtot[0] = c0s;
      wtot[1] = c1s;
    }
  }
  if (none_mv) atomicAdd((unsigned long long*)&P.meta->n_move_none, (unsigned long long)none_mv);
  __syncthreads();
  WSTAMP(12);
  WF_EXIT(9);

  // 7. payload by element, round 1: sym (| the move's has-value bits) and v0; the
  //    position of each rename in its branch's list (posl)
  if (SMX_DIAG && (P.ablate & 4)) return;
  u32* st_a = (u32*)sts;             // [CAP] sym | flags
  i32* st_b = (i32*)sts + CAP;   // [CAP] v0, then v1
  u16* posl = sl;
#if WF_OUT2
  // by final slot: each element's owner stores its payload at inv[element]
  int xi[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    xi[i] = e < sz ? inv[e] : CAP;
    if (e < sz) {
      st_a[xi[i]] = sym_r[i];
      if (!WF_STB_KIND || k_r[i] <= KREN) st_b[xi[i]] = v0_r[i];
    }
  }
  if (t < SMX_N_KINDS) tbase[t] = base[t] + woffk[t] - kbase[t];
#else
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    if (e < sz) {
      st_a[e] = sym_r[i];
      st_b[e] = v0_r[i];
    }
  }
#endif
  const int cntA = wtot[0], cntB = wtot[1];
  for (int x = t; x < RN; x += NT) {
    const int e = sord[R0 + x];
    const int s = e >= na;
    posl[(s ? cntA : 0) + rc[x >> 6][s] + rown[x]] = (u16)x;
  }
  if (t == 0) {
    P.wren[2 * w] = woffk[KREN];
    P.wren[2 * w + 1] = woffk[CNT_REN_A];
  }
  __syncthreads();
  WSTAMP(13);
  WF_EXIT(10);
  RX_EXIT(9);
  // 8. natural-head DivergentRename flags -> candidate slots; window exports
  win_rename_flags<NT, NCH>(
      P, w, woffk[KREN], RN, cntA, cntB, posl, gbits,
      [&](int x, int* s, int* own) {
        const int e = sord[R0 + x];
        *s = e >= na;
        *own = rc[x >> 6][*s] + rown[x];
      },
      [&](int x) -> uint2 {
#if WF_OUT2
        return make_uint2(st_a[R0 + x] & SYM_MASK, (u32)st_b[R0 + x]);
#else
        const int e = sord[R0 + x];
        return make_uint2(st_a[e] & SYM_MASK, (u32)st_b[e]);
#endif
      });
  WSTAMP(14);
  WF_EXIT(11);
  RX_EXIT(10);

  // The output phases' kernel arguments are read again here from the kernarg segment
  // (scalar loads through an opaque pointer): held from the kernel's start they were
  // spilled to VGPR lanes and reloaded one v_readlane each in these phases.
#if WF_LATEARGS == 2
  // only the eight output pointers re-read here (the rest of the arguments as loaded)
  WinArgs Q = P;
  {
    const WinArgs* K = kernarg_late<WinArgs>();
    Q.out_order = K->out_order;
    Q.out_addr = K->out_addr;
    Q.out_file = K->out_file;
    Q.out_ctx = K->out_ctx;
    Q.msym = K->msym;
    Q.tsrc = K->tsrc;
    Q.tsym = K->tsym;
    Q.Rstr = K->Rstr;
  }
#else
  const WinArgs& Q = WF_LATEARGS ? *kernarg_late<WinArgs>() : P;
#endif
  // 9. T-ordered records in final order (consecutive lanes -> consecutive T inside
  //    each kind: coalesced)
  const u64 nall = (u64)(Q.na + Q.nb);
  const u64 nmv = base[KREN];
#if WF_OUT2
  // four consecutive slots per thread (CAP = 4 * NT): one LDS read of each array,
  // and when the four share a kind (kinds are contiguous slot ranges) one 16-byte
  // store per output array
  // (CAP = 4 * NT * OP: OP passes of four slots per thread)
  constexpr int OP = CAP / (4 * NT);
  static_assert(CAP == 4 * NT * OP, "four slots per thread and pass");
  auto gsrc = [&](i32 j) -> i32 {
    return MAP ? Q.src_map[j] : (j < Q.na ? (i32)(Q.src_a + j) : (i32)(Q.src_b + (j - Q.na)));
  };
  u32 k4[OP][4];
  u64 T4[OP][4];
  bool uni[OP];
#pragma unroll
  for (int ps = 0; ps < OP; ++ps) {
    const int x0 = 4 * (t + NT * ps);
    const int m4 = sz - x0 < 4 ? sz - x0 : 4;
    uni[ps] = false;
    if (m4 <= 0) continue;
    const uint2 ew = *reinterpret_cast<const uint2*>(&sord[x0]);
    const u32 kw = *reinterpret_cast<const u32*>(&skS[x0]);
    const uint4 av = *reinterpret_cast<const uint4*>(&st_a[x0]);
    const uint4 bv = *reinterpret_cast<const uint4*>(&st_b[x0]);
    const u32 ee[4] = {ew.x & 0xffffu, ew.x >> 16, ew.y & 0xffffu, ew.y >> 16};
    const u32 aa[4] = {av.x, av.y, av.z, av.w};
    const i32 bb[4] = {(i32)bv.x, (i32)bv.y, (i32)bv.z, (i32)bv.w};
    i32 j4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      u32 k = (kw >> (8 * u)) & 0xffu;
      k = k < SMX_N_KINDS ? k : 0u;  // (slots past sz)
      k4[ps][u] = k;
      T4[ps][u] = tbase[k] + (u64)(x0 + u);
      j4[u] = (i32)(ee[u] < (u32)na ? a0 + ee[u] : bpos + ee[u]);
    }
    uni[ps] = m4 == 4 && k4[ps][3] == k4[ps][0] && T4[ps][0] + 3 < nall;
    if (uni[ps]) {
      const u64 T = T4[ps][0];
      if (k4[ps][0] == KMOVE) {
        st4(Q.out_order + T, gsrc(j4[0]), gsrc(j4[1]), gsrc(j4[2]), gsrc(j4[3]));
        st4(Q.out_addr + T, bb[0], bb[1], bb[2], bb[3]);
        st4(Q.out_ctx + T, -1, -1, -1, -1);
        st4((i32*)Q.msym + T, (i32)aa[0], (i32)aa[1], (i32)aa[2], (i32)aa[3]);
      } else {
        st4(Q.tsrc + (T - nmv), j4[0], j4[1], j4[2], j4[3]);
        st4((i32*)Q.tsym + (T - nmv), (i32)(aa[0] & SYM_MASK), (i32)(aa[1] & SYM_MASK), (i32)(aa[2] & SYM_MASK),
            (i32)(aa[3] & SYM_MASK));
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const u64 T = T4[ps][u];
        if (u >= m4 || T >= nall) continue;  // (T >= nall: only a failed, discarded plan)
        if (k4[ps][u] == KMOVE) {
          Q.out_order[T] = gsrc(j4[u]);
          Q.out_addr[T] = bb[u];
          Q.out_ctx[T] = -1;
          Q.msym[T] = aa[u];
        } else {
          Q.tsrc[T - nmv] = j4[u];
          Q.tsym[T - nmv] = aa[u] & SYM_MASK;
        }
      }
    }
  }
  __syncthreads();
  WSTAMP(15);
  WF_EXIT(12);
  // round 2: v1 -> the move's newFile, the rename's chain value
#pragma unroll
  for (int i = 0; i < ITEMS; ++i)
    if (xi[i] < CAP && (!WF_STB_KIND || k_r[i] <= KREN)) st_b[xi[i]] = v1_r[i];
  __syncthreads();
#pragma unroll
  for (int ps = 0; ps < OP; ++ps) {
    const int x0 = 4 * (t + NT * ps);
    const int m4 = sz - x0 < 4 ? sz - x0 : 4;
    if (m4 <= 0 || (k4[ps][0] > KREN && k4[ps][m4 - 1] > KREN)) continue;
    const uint4 bv = *reinterpret_cast<const uint4*>(&st_b[x0]);
    const i32 bb[4] = {(i32)bv.x, (i32)bv.y, (i32)bv.z, (i32)bv.w};
    if (uni[ps]) {
      const u64 T = T4[ps][0];
      st4(k4[ps][0] == KMOVE ? Q.out_file + T : Q.Rstr + (T - nmv), bb[0], bb[1], bb[2], bb[3]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const u64 T = T4[ps][u];
        if (u >= m4 || T >= nall || k4[ps][u] > KREN) continue;
        if (k4[ps][u] == KMOVE) Q.out_file[T] = bb[u];
        else Q.Rstr[T - nmv] = bb[u];
      }
    }
  }
#else
  // 9. T-ordered records in final order (consecutive lanes -> consecutive T inside
  //    each kind: coalesced)
  for (int x = t; x < sz; x += NT) {
    const int e = sord[x];
    const u32 k = skind[e];
    const u64 T = base[k] + woffk[k] + (u32)(x - kbase[k]);
    if (T >= nall) continue;  // only a failed (discarded) presorted plan can trip this
    const i64 j = e < na ? a0 + e : bpos + e;
    const u32 sa = st_a[e];
    if (k == KMOVE) {
      Q.out_order[T] = MAP ? Q.src_map[j] : (j < Q.na ? (i32)(Q.src_a + j) : (i32)(Q.src_b + (j - Q.na)));
      Q.out_addr[T] = st_b[e];
      Q.out_ctx[T] = -1;
      Q.msym[T] = sa;
    } else {
      Q.tsrc[T - nmv] = (i32)j;
      Q.tsym[T - nmv] = sa & SYM_MASK;
    }
  }
  __syncthreads();
  WSTAMP(15);
  WF_EXIT(12);
  // round 2: v1 -> the move's newFile, the rename's chain value
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const int e = t + NT * i;
    if (e < sz) st_b[e] = v1_r[i];
  }
  __syncthreads();
  for (int x = t; x < sz; x += NT) {
    const int e = sord[x];
    const u32 k = skind[e];
    if (k != KMOVE && k != KREN) continue;
    const u64 T = base[k] + woffk[k] + (u32)(x - kbase[k]);
    if (T >= nall) continue;
    if (k == KMOVE) Q.out_file[T] = st_b[e];
    else Q.Rstr[T - nmv] = st_b[e];
  }
#endif
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

// 1024-op windows on 512 threads: 38 KB of LDS, four windows per CU (2048-op windows
// took 75 KB, two per CU; config 5 window stage 0.80 -> 0.61 ms, profiles/r02_i)
#ifndef WG_CAP
#define WG_CAP 1024                 // ops per generic window (fixed diagonals, k_gpart)
#endif
#ifndef WG_NT
#define WG_NT 512
#endif
#define WG_ITEMS (WG_CAP / WG_NT)
#define WG_NCH (WG_CAP / WAVE)

__global__ void __launch_bounds__(WG_NT) k_window_g(WinArgs P) {
  __shared__ u64 sts[WG_CAP];
  __shared__ u64 shi[WG_CAP];
  __shared__ u64 slo[WG_CAP];
  __shared__ u32 ssrc[WG_CAP];
  __shared__ u16 sord[WG_CAP];       // merge order, later posl
  __shared__ u16 fin[WG_CAP];
  __shared__ u16 rown[WG_CAP];
  __shared__ u8 skind[WG_CAP];
  __shared__ u8 srank[WG_CAP];
  __shared__ u16 ccnt[WG_NCH][SMX_N_KINDS];
  __shared__ u16 rc[WG_NCH][2];
  __shared__ u32 kbase[SMX_N_KINDS + 1];
  __shared__ u32 wck[SMX_N_KINDS];
  __shared__ u64 base[SMX_N_KINDS + 1];
  __shared__ u64 cb[WG_NCH];
  __shared__ u32 wtot[2];
  __shared__ u32 vbw[WG_NT / WAVE][3];
  __shared__ u32 woffk[NCNT];
  // after the merge the id words are dead: the payload by element takes their place
  u32* st_sym = reinterpret_cast<u32*>(shi);
  i32* st_v0 = reinterpret_cast<i32*>(shi) + WG_CAP;
  i32* st_v1 = reinterpret_cast<i32*>(slo);

  const int t = threadIdx.x;
  const int lane = t & (WAVE - 1);
  const int wv = t / WAVE;
  // consecutive windows on one XCD: a timestamp group spans several windows, whose
  // gathers through the permutation then hit the same L2
  const i64 w = SMX_XCD_WIN ? xcd_item(blockIdx.x, P.W) : (i64)blockIdx.x;
  if (P.meta->f_fail) return;  // the segmented sort failed: no permutation to gather through
  const i64 a0 = P.bnd[2 * w], b0 = P.bnd[2 * w + 1];
  const int na = (int)(P.bnd[2 * w + 2] - a0);
  const int nb = (int)(P.bnd[2 * w + 3] - b0);
  const int sz = na + nb;

  // loads: the sorted keys and the permutation, then the op fields through it (two
  // round trips, every item's loads in flight together; the payload stays in registers
  // until the merge is done)
  bool bad = false;
  u32 vb_a = 0, vb_f = 0, vb_c = 0;
  u32 src_r[WG_ITEMS], k_r[WG_ITEMS], sym_r[WG_ITEMS];
  i32 v0_r[WG_ITEMS], v1_r[WG_ITEMS];
  u64 kt_r[WG_ITEMS], kh_r[WG_ITEMS], kl_r[WG_ITEMS];
#pragma unroll
  for (int i = 0; i < WG_ITEMS; ++i) {
    const int e = t + WG_NT * i;
    const int ec = e < sz ? e : 0;
    const i64 j = sz == 0 ? 0 : (ec < na ? a0 + ec : P.na + b0 + (ec - na));
    src_r[i] = P.perm[j];
    kt_r[i] = P.kts[j];
    kh_r[i] = P.khi[j];
    kl_r[i] = P.klo[j];
  }
  if (t < NCNT) woffk[t] = P.woff[(i64)t * P.W + w];
#pragma unroll
  for (int i = 0; i < WG_ITEMS; ++i) {
    const u32 src = src_r[i];
    k_r[i] = P.kind[src];
    sym_r[i] = P.sym[src];
    v0_r[i] = P.v0[src];
    v1_r[i] = P.v1[src];
  }
#pragma unroll
  for (int i = 0; i < WG_ITEMS; ++i) {
    const int e = t + WG_NT * i;
    if (e >= sz) continue;
    sts[e] = kt_r[i];
    shi[e] = kh_r[i];
    slo[e] = kl_r[i];
    ssrc[e] = src_r[i];
    const u32 k = k_r[i];
    bad |= (k >= SMX_N_KINDS) || (sym_r[i] >= (u64)P.n_sym);
    skind[e] = (u8)(k < SMX_N_KINDS ? k : SMX_N_KINDS - 1);
    if (k == KMOVE) {
      vb_a |= (u32)(v0_r[i] + 1);
      vb_f |= (u32)(v1_r[i] + 1);
    } else if (k == KREN) {
      vb_c |= (u32)(v1_r[i] + 1);
    }
  }
  vb_a = wave_or_to_last(vb_a);
  vb_f = wave_or_to_last(vb_f);
  vb_c = wave_or_to_last(vb_c);
  if (lane == WAVE - 1) {
    vbw[wv][0] = vb_a;
    vbw[wv][1] = vb_f;
    vbw[wv][2] = vb_c;
  }
  if (bad) P.meta->bad_sym = 1;
  for (int i = t; i < WG_NCH * SMX_N_KINDS; i += WG_NT) (&ccnt[0][0])[i] = 0;
  if (t <= SMX_N_KINDS) base[t] = P.meta->base[t];
  __syncthreads();

  if (t == 0) win_publish_widths(P.meta, &vbw[0][0], WG_NT / WAVE);
  if (sz > 0) {
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
#pragma unroll
  for (int i = 0; i < WG_ITEMS; ++i) {  // (visible after the multisplit's barriers)
    const int e = t + WG_NT * i;
    if (e < sz) {
      st_sym[e] = sym_r[i];
      st_v0[e] = v0_r[i];
      st_v1[e] = v1_r[i];
    }
  }

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
    if (lane == WAVE - 1) {
      wtot[0] = i0;
      wtot[1] = i1;
    }
  }
  __syncthreads();
  const int cntA = wtot[0], cntB = wtot[1];
  u16* posl = sord;
  for (int x = t; x < RN; x += WG_NT) {
    const int e = fin[R0 + x];
    const int s = e >= na;
    posl[(s ? cntA : 0) + rc[x >> 6][s] + rown[x]] = (u16)x;
  }
  if (t == 0) {
    P.wren[2 * w] = woffk[KREN];
    P.wren[2 * w + 1] = woffk[CNT_REN_A];
  }
  __syncthreads();
  win_rename_flags<WG_NT, WG_NCH>(
      P, w, woffk[KREN], RN, cntA, cntB, posl, cb,
      [&](int x, int* s, int* own) {
        const int e = fin[R0 + x];
        *s = e >= na;
        *own = rc[x >> 6][*s] + rown[x];
      },
      [&](int x) -> uint2 {
        const int e = fin[R0 + x];
        return make_uint2(st_sym[e], (u32)st_v0[e]);
      });

  const u64 nall = (u64)(P.na + P.nb);
  const u64 nmv = base[KREN];
  for (int x = t; x < sz; x += WG_NT) {
    const int e = fin[x];
    const u32 k = skind[e];
    const u32 src = ssrc[e];
    const u64 T = base[k] + woffk[k] + (u32)(x - kbase[k]);
    if (T >= nall) continue;
    const u32 s = st_sym[e];
    if (k == KMOVE) {
      const i32 a = st_v0[e], f = st_v1[e];
      P.out_order[T] = win_gsrc(P, src);
      P.out_addr[T] = a;
      P.out_file[T] = f;
      P.out_ctx[T] = -1;
      P.msym[T] = (s & SYM_MASK) | (a >= 0 ? MS_HAS_A : 0u) | (f >= 0 ? MS_HAS_F : 0u);
    } else {
      P.tsrc[T - nmv] = (i32)src;
      P.tsym[T - nmv] = s;
      if (k == KREN) P.Rstr[T - nmv] = st_v1[e];
    }
  }
}
