// smx_compose.hip — MI355X (gfx950) implementation of semmerge's compose_oplogs
// (semmerge/compose.py:11-114) behind the C ABI of include/smx.h.
//
// Exact data-parallel restatement of the reference's sequential loop:
//   T      = stable order of A||B by (precedence, timestamp, id, side, index)
//            (per-branch sorted() + merge with A on ties, compose.py:16-21,51-56)
//   moves  precede renames precede everything else in T, so
//            moveDecl k sees the inclusive per-symbol prefix of last non-None
//            newAddress/newFile; every later op sees the final move state;
//            non-renames see the final non-skipped rename (compose.py:27-49,71-82)
//   DivergentRename skips (compose.py:60-70,88-98) are found by replaying a
//            two-state transducer (ahead side, depth d) over the rename block
//            from every "natural-head" candidate, and resolving overlapping
//            regions cluster by cluster.
//
// Pipeline (one merge):
//   k_stats     kind histogram, per-branch timestamp monotonicity, key masks
//   k_fpart     presorted windows: merge-path on timestamps, cut at ts boundaries
//   k_wcount    per-window kind counts          k_wscan   window offsets, T bases
//   [generic]   radix-sort each branch by (ts, oid) and cut fixed windows
//   k_window    per window, in LDS: merge A/B parts, multisplit by kind, sort
//               equal-timestamp groups by id, write T-ordered arrays
//   walk        k_flags -> compact -> k_replay_q -> max-scan -> k_cluster ->
//               scan -> k_replay_write (conflict pairs, skip flags)
//   tables      per-symbol last writers (packed (T+1)<<32|value atomicMax)
//   k_emit      compacted output: order, addr, file, ctx
#include <mutex>
#include <string>
#include <vector>

#include "smx_sort.h"

#define WIN_CAP 2048               // max ops per window held in LDS
#define WIN_TGT 1024               // target window size, presorted path
#define WIN_ITEMS (WIN_CAP / BLOCK)
#define NCNT (SMX_N_KINDS + 2)     // kinds + renames per side
#define KMOVE SMX_KIND_MOVE
#define KREN SMX_KIND_RENAME

// ---------------------------------------------------------------------------
// error / profiling state
static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIP_TRY(x)                                                                 \
  do {                                                                             \
    hipError_t _e = (x);                                                           \
    if (_e != hipSuccess)                                                          \
      return set_err(SMX_E_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

enum Stage { ST_PLAN, ST_GSORT, ST_WINDOW, ST_WALK, ST_TABLES, ST_MVPREFIX, ST_EMIT, ST_N };
static const char* kStageNames[ST_N] = {"plan",   "gsort",     "window", "walk",
                                        "tables", "mvprefix", "emit"};
static std::mutex g_prof_mu;
static int g_prof = 0;
static double g_stage_ms[ST_N];
static int64_t g_stage_calls[ST_N];

struct StageTimer {
  hipStream_t st;
  bool on;
  hipEvent_t ev[ST_N][2];
  bool used[ST_N];
  StageTimer(hipStream_t s, bool enabled) : st(s), on(enabled) {
    for (int i = 0; i < ST_N; ++i) used[i] = false;
    if (!on) return;
    for (int i = 0; i < ST_N; ++i) {
      (void)hipEventCreate(&ev[i][0]);
      (void)hipEventCreate(&ev[i][1]);
    }
  }
  void begin(int i) {
    if (on) (void)hipEventRecord(ev[i][0], st);
  }
  void end(int i) {
    if (on) {
      (void)hipEventRecord(ev[i][1], st);
      used[i] = true;
    }
  }
  void flush() {
    if (!on) return;
    (void)hipStreamSynchronize(st);
    std::lock_guard<std::mutex> g(g_prof_mu);
    for (int i = 0; i < ST_N; ++i) {
      if (used[i]) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ev[i][0], ev[i][1]);
        g_stage_ms[i] += ms;
        g_stage_calls[i] += 1;
      }
    }
  }
  ~StageTimer() {
    if (!on) return;
    for (int i = 0; i < ST_N; ++i) {
      (void)hipEventDestroy(ev[i][0]);
      (void)hipEventDestroy(ev[i][1]);
    }
  }
};

// ---------------------------------------------------------------------------
// kernels: planning

__global__ void __launch_bounds__(BLOCK) k_stats(const u8* __restrict__ kind, const u64* __restrict__ ts,
                                                 const u64* __restrict__ hi, const u64* __restrict__ lo,
                                                 const u32* __restrict__ sym, const i32* __restrict__ v0,
                                                 const i32* __restrict__ v1, i64 na, i64 n, i64 n_sym,
                                                 ComposeMeta* meta) {
  __shared__ u32 cnt[SMX_N_KINDS + 4];
  __shared__ u64 kor[2][3], kand[2][3];
  const int t = threadIdx.x;
  if (t < SMX_N_KINDS + 4) cnt[t] = 0;
  if (t < 6) {
    kor[t / 3][t % 3] = 0;
    kand[t / 3][t % 3] = ~0ull;
  }
  __syncthreads();
  u64 ro[2][3] = {{0, 0, 0}, {0, 0, 0}};
  u64 ra[2][3] = {{~0ull, ~0ull, ~0ull}, {~0ull, ~0ull, ~0ull}};
  bool nonmono0 = false, nonmono1 = false, badsym = false;
  u32 none_moves = 0;
  for (i64 i = (i64)blockIdx.x * BLOCK + t; i < n; i += (i64)gridDim.x * BLOCK) {
    const u32 k = kind[i];
    const int side = i >= na;
    atomicAdd(&cnt[k < SMX_N_KINDS ? k : SMX_N_KINDS - 1], 1u);
    const u64 tv = ts[i], hv = hi[i], lv = lo[i];
    if (side) {
      ro[1][0] |= tv; ro[1][1] |= hv; ro[1][2] |= lv;
      ra[1][0] &= tv; ra[1][1] &= hv; ra[1][2] &= lv;
    } else {
      ro[0][0] |= tv; ro[0][1] |= hv; ro[0][2] |= lv;
      ra[0][0] &= tv; ra[0][1] &= hv; ra[0][2] &= lv;
    }
    if (i != 0 && i != na && ts[i - 1] > tv) {
      if (side) nonmono1 = true; else nonmono0 = true;
    }
    if (sym[i] >= (u64)n_sym || k >= SMX_N_KINDS) badsym = true;
    if (k == KMOVE && (v0[i] < 0 || v1[i] < 0)) ++none_moves;
    if (k == KREN) atomicAdd(&cnt[SMX_N_KINDS + side], 1u);
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      atomicOr((unsigned long long*)&kor[s][q], (unsigned long long)ro[s][q]);
      atomicAnd((unsigned long long*)&kand[s][q], (unsigned long long)ra[s][q]);
    }
  if (none_moves) atomicAdd(&cnt[SMX_N_KINDS + 2], none_moves);
  if (nonmono0) meta->nonmono[0] = 1;
  if (nonmono1) meta->nonmono[1] = 1;
  if (badsym) meta->bad_sym = 1;
  __syncthreads();
  if (t < SMX_N_KINDS && cnt[t]) atomicAdd((unsigned long long*)&meta->kcnt[t], (unsigned long long)cnt[t]);
  if (t < 2 && cnt[SMX_N_KINDS + t])
    atomicAdd((unsigned long long*)&meta->n_ren_side[t], (unsigned long long)cnt[SMX_N_KINDS + t]);
  if (t == 2 && cnt[SMX_N_KINDS + 2])
    atomicAdd((unsigned long long*)&meta->n_move_none, (unsigned long long)cnt[SMX_N_KINDS + 2]);
  if (t < 6) {
    atomicOr((unsigned long long*)&meta->key_or[t / 3][t % 3], (unsigned long long)kor[t / 3][t % 3]);
    atomicAnd((unsigned long long*)&meta->key_and[t / 3][t % 3], (unsigned long long)kand[t / 3][t % 3]);
  }
}

__global__ void k_meta_init(ComposeMeta* meta) {
  for (int s = 0; s < 2; ++s)
    for (int q = 0; q < 3; ++q) meta->key_and[s][q] = ~0ull;
}

// Presorted windows: boundary k sits at the merge-path split of diagonal k*WIN_TGT
// (timestamps, A first on ties), snapped down to the first op of that timestamp on
// both branches, so every (timestamp) group lands whole in one window.
__global__ void k_fpart(const u64* __restrict__ ts, i64 na, i64 nb, i64 W, i64* __restrict__ bnd) {
  const i64 k = (i64)blockIdx.x * BLOCK + threadIdx.x;
  if (k > W) return;
  const i64 n = na + nb;
  const u64* A = ts;
  const u64* B = ts + na;
  const i64 d = k * WIN_TGT;
  if (k == 0) {
    bnd[0] = 0;
    bnd[1] = 0;
    return;
  }
  if (d >= n || k == W) {
    bnd[2 * k] = na;
    bnd[2 * k + 1] = nb;
    return;
  }
  i64 lo = d - nb > 0 ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    i64 mid = (lo + hi) >> 1;
    if (A[mid] <= B[d - 1 - mid]) lo = mid + 1;
    else hi = mid;
  }
  const i64 a = lo, b = d - lo;
  const u64 tau = (a < na && (b >= nb || A[a] <= B[b])) ? A[a] : B[b];
  lo = 0; hi = na;
  while (lo < hi) {
    i64 mid = (lo + hi) >> 1;
    if (A[mid] < tau) lo = mid + 1; else hi = mid;
  }
  bnd[2 * k] = lo;
  lo = 0; hi = nb;
  while (lo < hi) {
    i64 mid = (lo + hi) >> 1;
    if (B[mid] < tau) lo = mid + 1; else hi = mid;
  }
  bnd[2 * k + 1] = lo;
}

__device__ __forceinline__ bool key_le(u64 ta, u64 ha, u64 la, u64 tb, u64 hb, u64 lb) {
  if (ta != tb) return ta < tb;
  if (ha != hb) return ha < hb;
  return la <= lb;
}

// Generic windows over branch logs sorted by (ts, oid): fixed diagonals of WIN_CAP.
__global__ void k_gpart(const u64* __restrict__ sts, const u64* __restrict__ shi,
                        const u64* __restrict__ slo, i64 na, i64 nb, i64 W, i64* __restrict__ bnd) {
  const i64 k = (i64)blockIdx.x * BLOCK + threadIdx.x;
  if (k > W) return;
  const i64 n = na + nb;
  const i64 d = k * WIN_CAP;
  if (k == 0) { bnd[0] = 0; bnd[1] = 0; return; }
  if (d >= n || k == W) { bnd[2 * k] = na; bnd[2 * k + 1] = nb; return; }
  i64 lo = d - nb > 0 ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    i64 mid = (lo + hi) >> 1;
    const i64 j = na + d - 1 - mid;
    if (key_le(sts[mid], shi[mid], slo[mid], sts[j], shi[j], slo[j])) lo = mid + 1;
    else hi = mid;
  }
  bnd[2 * k] = lo;
  bnd[2 * k + 1] = d - lo;
}

// Per-window counts of each kind, plus renames per branch.  perm == nullptr: the
// presorted layout (branch position j is op base+j).  Column-major [c][W].
__global__ void __launch_bounds__(BLOCK) k_wcount(const u8* __restrict__ kind, const u32* __restrict__ perm,
                                                  const i64* __restrict__ bnd, i64 na, i64 W,
                                                  u32* __restrict__ wcnt, ComposeMeta* meta, int check_cap) {
  __shared__ u32 c[NCNT];
  const i64 w = blockIdx.x;
  if (threadIdx.x < NCNT) c[threadIdx.x] = 0;
  __syncthreads();
  const i64 a0 = bnd[2 * w], b0 = bnd[2 * w + 1], a1 = bnd[2 * w + 2], b1 = bnd[2 * w + 3];
  if (check_cap && threadIdx.x == 0 && (a1 - a0) + (b1 - b0) > WIN_CAP) meta->f_fail = 1;
  for (i64 j = a0 + threadIdx.x; j < a1; j += BLOCK) {
    const u32 src = perm ? perm[j] : (u32)j;
    const u32 k = min((u32)kind[src], (u32)SMX_N_KINDS - 1);  // validated in k_stats
    atomicAdd(&c[k], 1u);
    if (k == KREN) atomicAdd(&c[SMX_N_KINDS], 1u);
  }
  for (i64 j = b0 + threadIdx.x; j < b1; j += BLOCK) {
    const u32 src = perm ? perm[na + j] : (u32)(na + j);
    const u32 k = min((u32)kind[src], (u32)SMX_N_KINDS - 1);
    atomicAdd(&c[k], 1u);
    if (k == KREN) atomicAdd(&c[SMX_N_KINDS + 1], 1u);
  }
  __syncthreads();
  if (threadIdx.x < NCNT) wcnt[(i64)threadIdx.x * W + w] = c[threadIdx.x];
}

// Exclusive scan of each count column over windows; block 0 also sets the T bases.
__global__ void __launch_bounds__(BLOCK) k_wscan(const u32* __restrict__ wcnt, u32* __restrict__ woff,
                                                 i64 W, ComposeMeta* meta) {
  __shared__ u32 s[NWAVES + 1];
  const int c = blockIdx.x;
  const u32* in = wcnt + (i64)c * W;
  u32* out = woff + (i64)c * W;
  u32 carry = 0;
  for (i64 r0 = 0; r0 < W; r0 += BLOCK * 8) {
    const i64 b = r0 + (i64)threadIdx.x * 8;
    u32 v[8];
    u32 acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = b + j < W ? in[b + j] : 0u;
      acc += v[j];
    }
    u32 tot;
    u32 run = carry + block_excl_scan<OpSum, u32>(acc, s, &tot);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (b + j < W) out[b + j] = run;
      run += v[j];
    }
    carry += tot;
  }
  if (c == 0 && threadIdx.x == 0) {
    u64 acc = 0;
    for (int k = 0; k < SMX_N_KINDS; ++k) {
      meta->base[k] = acc;
      acc += meta->kcnt[k];
    }
    meta->base[SMX_N_KINDS] = acc;
  }
}

// ---------------------------------------------------------------------------
// kernel: one window -> T-ordered arrays

struct WinArgs {
  const u8* kind;
  const u32* sym;
  const i32* v0;
  const i32* v1;
  // branch views: presorted -> keys at op index base+j; generic -> sorted copies at j
  const u64* kts;
  const u64* khi;
  const u64* klo;
  const u32* perm;  // generic only: op index of sorted position (A at [0,na), B at [na,n))
  i64 na;
  i64 W;
  const i64* bnd;
  const u32* woff;  // [NCNT][W]
  const ComposeMeta* meta;
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

template <bool PRESORTED>
__global__ void __launch_bounds__(BLOCK) k_window(WinArgs P) {
  __shared__ u64 sts[WIN_CAP];
  __shared__ u64 shi[WIN_CAP];
  __shared__ u64 slo[WIN_CAP];
  __shared__ u32 ssrc[WIN_CAP];
  __shared__ u16 sord[WIN_CAP];
  __shared__ u16 fin[WIN_CAP];
  __shared__ u16 rown[WIN_CAP];
  __shared__ u8 skind[WIN_CAP];
  __shared__ u8 srank[WIN_CAP];
  __shared__ u16 ccnt[WIN_CAP / WAVE][SMX_N_KINDS];
  __shared__ u16 rc[WIN_CAP / WAVE][2];
  __shared__ u32 kbase[SMX_N_KINDS + 1];
  __shared__ u32 wck[SMX_N_KINDS];

  const int t = threadIdx.x;
  const int lane = t & (WAVE - 1);
  const int wv = t / WAVE;
  const i64 w = blockIdx.x;
  const i64 a0 = P.bnd[2 * w], b0 = P.bnd[2 * w + 1];
  const int na = (int)(P.bnd[2 * w + 2] - a0);
  const int nb = (int)(P.bnd[2 * w + 3] - b0);
  const int sz = na + nb;
  if (sz == 0) return;

  // 1. stage keys, kinds and op indices of both branch parts
  for (int e = t; e < sz; e += BLOCK) {
    const i64 j = e < na ? a0 + e : P.na + b0 + (e - na);  // position in the branch layout
    u32 src;
    u64 tv, hv, lv;
    if (PRESORTED) {
      src = (u32)j;
      tv = P.kts[j]; hv = P.khi[j]; lv = P.klo[j];
    } else {
      src = P.perm[j];
      tv = P.kts[j]; hv = P.khi[j]; lv = P.klo[j];
    }
    sts[e] = tv; shi[e] = hv; slo[e] = lv;
    ssrc[e] = src;
    skind[e] = P.kind[src];
  }
  for (int i = t; i < (WIN_CAP / WAVE) * SMX_N_KINDS; i += BLOCK) (&ccnt[0][0])[i] = 0;
  __syncthreads();

  // 2. merge the A part [0,na) and B part [na,sz) -> S order (A first on ties)
  {
    const int d0 = t * WIN_ITEMS < sz ? t * WIN_ITEMS : sz;
    const int d1 = d0 + WIN_ITEMS < sz ? d0 + WIN_ITEMS : sz;
    int lo = d0 - nb > 0 ? d0 - nb : 0, hi = d0 < na ? d0 : na;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const int j = na + d0 - 1 - mid;
      const bool af = PRESORTED ? (sts[mid] <= sts[j])
                                : key_le(sts[mid], shi[mid], slo[mid], sts[j], shi[j], slo[j]);
      if (af) lo = mid + 1; else hi = mid;
    }
    int ia = lo, ib = d0 - lo;
    for (int d = d0; d < d1; ++d) {
      bool take_a;
      if (ia >= na) take_a = false;
      else if (ib >= nb) take_a = true;
      else {
        const int j = na + ib;
        take_a = PRESORTED ? (sts[ia] <= sts[j])
                           : key_le(sts[ia], shi[ia], slo[ia], sts[j], shi[j], slo[j]);
      }
      sord[d] = (u16)(take_a ? ia++ : na + ib++);
    }
  }
  __syncthreads();

  // 3. stable multisplit of S by kind (wave ballots), window-local slots
  const int nch = (sz + WAVE - 1) / WAVE;
  for (int c = wv; c < nch; c += NWAVES) {
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
  if (t < SMX_N_KINDS) {
    u32 acc = 0;
    for (int c = 0; c < nch; ++c) {
      const u32 x = ccnt[c][t];
      ccnt[c][t] = (u16)acc;
      acc += x;
    }
    wck[t] = acc;
  }
  __syncthreads();
  if (t == 0) {
    u32 acc = 0;
    for (int k = 0; k < SMX_N_KINDS; ++k) {
      kbase[k] = acc;
      acc += wck[k];
    }
    kbase[SMX_N_KINDS] = acc;
  }
  __syncthreads();
  for (int m = t; m < sz; m += BLOCK) {
    const int e = sord[m];
    const u32 k = skind[e];
    fin[kbase[k] + ccnt[m / WAVE][k] + srank[m]] = (u16)e;
  }
  __syncthreads();

  // 4. presorted path: equal-(kind, ts) groups are contiguous; order them by
  //    (oid, side, index) = (oid, slot) with a counting rank
  const u16* fo = fin;
  if (PRESORTED) {
    for (int p = t; p < sz; p += BLOCK) {
      const int e = fin[p];
      const u32 k = skind[e];
      const int kb = kbase[k], ke = kb + wck[k];
      const u64 t0 = sts[e];
      int gs = p;
      while (gs > kb && sts[fin[gs - 1]] == t0) --gs;
      int ge = p + 1;
      while (ge < ke && sts[fin[ge]] == t0) ++ge;
      int r = p;
      if (ge - gs > 1) {
        const u64 h = shi[e], l = slo[e];
        r = gs;
        for (int q = gs; q < ge; ++q) {
          const int f = fin[q];
          const u64 hq = shi[f], lq = slo[f];
          r += (hq < h) || (hq == h && (lq < l || (lq == l && q < p)));
        }
      }
      sord[r] = (u16)e;
    }
    __syncthreads();
    fo = sord;
  }

  // 5. renames: rank among same-branch renames of this window (final order)
  const int R0 = kbase[KREN], RN = wck[KREN];
  const int nrc = (RN + WAVE - 1) / WAVE;
  for (int c = wv; c < nrc; c += NWAVES) {
    const int x = c * WAVE + lane;
    const bool valid = x < RN;
    const int e = valid ? fo[R0 + x] : 0;
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
  if (t < 2) {
    u32 acc = 0;
    for (int c = 0; c < nrc; ++c) {
      const u32 x = rc[c][t];
      rc[c][t] = (u16)acc;
      acc += x;
    }
  }
  __syncthreads();

  // 6. write T-ordered outputs (coalesced along the final order)
  const u64* base = P.meta->base;
  for (int x = t; x < sz; x += BLOCK) {
    const int e = fo[x];
    const u32 k = skind[e];
    const u64 T = base[k] + P.woff[(i64)k * P.W + w] + (u32)(x - kbase[k]);
    const u32 src = ssrc[e];
    P.order[T] = (i32)src;
    const u32 s = P.sym[src];
    P.symT[T] = s;
    if (k == KMOVE) {
      P.mvA[T] = P.v0[src];
      P.mvF[T] = P.v1[src];
    } else if (k == KREN) {
      const u64 m = T - base[KREN];
      const int side = e >= na;
      const int xr = x - R0;
      const u32 own = P.woff[(i64)(SMX_N_KINDS + side) * P.W + w] + rc[xr / WAVE][side] + rown[xr];
      P.Msym[m] = s;
      P.Mcls[m] = P.v0[src];
      P.Mstr[m] = P.v1[src];
      P.Mside[m] = (u8)side;
      P.Mown[m] = own;
      (side ? P.RB : P.RA)[own] = (u32)m;
    }
  }
}

// ---------------------------------------------------------------------------
// kernels: generic path helpers

__global__ void k_gather_init(const u64* __restrict__ key, u64* __restrict__ kout, u32* __restrict__ vout,
                              i64 n) {
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (i64)gridDim.x * BLOCK) {
    kout[i] = key[i];
    vout[i] = (u32)i;
  }
}

__global__ void k_gather(const u64* __restrict__ key, const u32* __restrict__ idx, u64* __restrict__ kout,
                         i64 n) {
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (i64)gridDim.x * BLOCK)
    kout[i] = key[idx[i]];
}

__global__ void k_offset(u32* __restrict__ v, i64 n, u32 off) {
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (i64)gridDim.x * BLOCK) v[i] += off;
}

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

// ---------------------------------------------------------------------------
// kernels: per-symbol last writers and output

__global__ void k_tab_move(const u32* __restrict__ symT, const i32* __restrict__ mvA,
                           const i32* __restrict__ mvF, u64 nMv, u64* __restrict__ tabA,
                           u64* __restrict__ tabF) {
  for (u64 T = (u64)blockIdx.x * BLOCK + threadIdx.x; T < nMv; T += (u64)gridDim.x * BLOCK) {
    const u32 s = symT[T];
    const i32 a = mvA[T], f = mvF[T];
    if (a >= 0) atomicMax((unsigned long long*)&tabA[s], (unsigned long long)(((T + 1) << 32) | (u32)a));
    if (f >= 0) atomicMax((unsigned long long*)&tabF[s], (unsigned long long)(((T + 1) << 32) | (u32)f));
  }
}

__global__ void k_tab_ren(const u32* __restrict__ Msym, const i32* __restrict__ Mstr,
                          const u8* __restrict__ skip, u64 nR, u64* __restrict__ tabR) {
  for (u64 m = (u64)blockIdx.x * BLOCK + threadIdx.x; m < nR; m += (u64)gridDim.x * BLOCK) {
    if (skip[m]) continue;
    atomicMax((unsigned long long*)&tabR[Msym[m]], (unsigned long long)(((m + 1) << 32) | (u32)Mstr[m]));
  }
}

__global__ void k_finalize(const u64* __restrict__ tabA, const u64* __restrict__ tabF,
                           const u64* __restrict__ tabR, i64 n_sym, int4* __restrict__ fin) {
  for (i64 s = (i64)blockIdx.x * BLOCK + threadIdx.x; s < n_sym; s += (i64)gridDim.x * BLOCK) {
    const u64 a = tabA[s], f = tabF[s], r = tabR[s];
    fin[s] = make_int4(a ? (i32)(u32)a : -1, f ? (i32)(u32)f : -1, r ? (i32)(u32)r : -1, 0);
  }
}

__global__ void k_mv_init(const u32* __restrict__ symT, u64 nMv, u64* __restrict__ keys,
                          u32* __restrict__ vals) {
  for (u64 j = (u64)blockIdx.x * BLOCK + threadIdx.x; j < nMv; j += (u64)gridDim.x * BLOCK) {
    keys[j] = symT[j];
    vals[j] = (u32)j;
  }
}

// Moves grouped by symbol (T order inside a group): inclusive last-non-None scan.
__global__ void k_mv_seg(const u64* __restrict__ keys, const u32* __restrict__ vals, u64 nMv,
                         const i32* __restrict__ mvA, const i32* __restrict__ mvF,
                         i32* __restrict__ prefA, i32* __restrict__ prefF) {
  for (u64 j = (u64)blockIdx.x * BLOCK + threadIdx.x; j < nMv; j += (u64)gridDim.x * BLOCK) {
    if (j != 0 && keys[j - 1] == keys[j]) continue;
    i32 ra = -1, rf = -1;
    for (u64 i = j; i < nMv && keys[i] == keys[j]; ++i) {
      const u32 T = vals[i];
      if (mvA[T] >= 0) ra = mvA[T];
      if (mvF[T] >= 0) rf = mvF[T];
      prefA[T] = ra;
      prefF[T] = rf;
    }
  }
}

struct EmitArgs {
  const i32* order;
  const u32* symT;
  const i32* prefA;
  const i32* prefF;
  const u8* skip;
  const u32* skipex;
  const int4* fin;
  const ComposeMeta* meta;
  u64 n, nMv, nR;
  i32* out_order;
  i32* out_addr;
  i32* out_file;
  i32* out_ctx;
};

__global__ void __launch_bounds__(BLOCK) k_emit(EmitArgs E) {
  const u64 nskip = 2 * E.meta->n_conf;
  for (u64 T = (u64)blockIdx.x * BLOCK + threadIdx.x; T < E.n; T += (u64)gridDim.x * BLOCK) {
    const i32 src = E.order[T];
    i32 a, f, c;
    u64 o;
    if (T < E.nMv) {
      o = T;
      a = E.prefA[T];
      f = E.prefF[T];
      c = -1;
    } else if (T < E.nMv + E.nR) {
      const u64 m = T - E.nMv;
      if (E.skip[m]) continue;
      o = T - E.skipex[m];
      const int4 F = E.fin[E.symT[T]];
      a = F.x;
      f = F.y;
      c = -1;
    } else {
      o = T - nskip;
      const int4 F = E.fin[E.symT[T]];
      a = F.x;
      f = F.y;
      c = F.z;
    }
    E.out_order[o] = src;
    E.out_addr[o] = a;
    E.out_file[o] = f;
    E.out_ctx[o] = c;
  }
}

__global__ void k_counts(const ComposeMeta* meta, u64 n, i64* counts) {
  counts[0] = (i64)(n - 2 * meta->n_conf);
  counts[1] = (i64)meta->n_conf;
}

// ---------------------------------------------------------------------------
// workspace layout

struct Layout {
  size_t off[64];
  size_t total;
};

enum Buf {
  B_META, B_BND, B_WCNT, B_WOFF, B_STS, B_SHI, B_SLO, B_PERM, B_RKEY, B_RVAL, B_RK2, B_RV2,
  B_RHIST, B_PART, B_ORDER, B_SYMT, B_MVA, B_MVF, B_MSYM, B_MCLS, B_MSTR, B_MSIDE, B_MOWN,
  B_RAB, B_FLAGS, B_FPOS, B_CAND, B_Q, B_PM, B_NCONF, B_NREAL, B_COFF, B_SKIP, B_SKIPEX,
  B_TABA, B_TABF, B_TABR, B_FIN, B_PREFA, B_PREFF, B_N
};

static Layout layout(i64 na, i64 nb, i64 n_sym) {
  const i64 n = na + nb;
  const i64 nn = n > 0 ? n : 1;
  const i64 W = SMX_CEIL_DIV(nn, (i64)WIN_TGT) + 2;
  const i64 nblk = SMX_CEIL_DIV(nn, (i64)RADIX_TILE);
  size_t sz[B_N];
  sz[B_META] = sizeof(ComposeMeta);
  sz[B_BND] = (size_t)(W + 1) * 2 * 8;
  sz[B_WCNT] = (size_t)NCNT * W * 4;
  sz[B_WOFF] = (size_t)NCNT * W * 4;
  sz[B_STS] = sz[B_SHI] = sz[B_SLO] = (size_t)nn * 8;
  sz[B_PERM] = (size_t)nn * 4;
  sz[B_RKEY] = (size_t)nn * 8;
  sz[B_RVAL] = (size_t)nn * 4;
  sz[B_RK2] = (size_t)nn * 8;
  sz[B_RV2] = (size_t)nn * 4;
  sz[B_RHIST] = (size_t)256 * nblk * 4;
  sz[B_PART] = (size_t)SCAN_NB * 8;
  sz[B_ORDER] = sz[B_SYMT] = sz[B_MVA] = sz[B_MVF] = (size_t)nn * 4;
  sz[B_MSYM] = sz[B_MCLS] = sz[B_MSTR] = sz[B_MOWN] = sz[B_RAB] = (size_t)nn * 4;
  sz[B_MSIDE] = (size_t)nn;
  sz[B_FLAGS] = (size_t)nn;
  sz[B_FPOS] = sz[B_CAND] = sz[B_Q] = sz[B_PM] = sz[B_NCONF] = sz[B_NREAL] = sz[B_COFF] = (size_t)nn * 4;
  sz[B_SKIP] = (size_t)nn;
  sz[B_SKIPEX] = (size_t)nn * 4;
  const i64 ns = n_sym > 0 ? n_sym : 1;
  sz[B_TABA] = sz[B_TABF] = sz[B_TABR] = (size_t)ns * 8;
  sz[B_FIN] = (size_t)ns * 16;
  sz[B_PREFA] = sz[B_PREFF] = (size_t)nn * 4;
  Layout L;
  size_t acc = 0;
  for (int i = 0; i < B_N; ++i) {
    L.off[i] = acc;
    acc += (sz[i] + 255) & ~(size_t)255;
  }
  L.total = acc;
  return L;
}

// ---------------------------------------------------------------------------
// C ABI

static int grid_for(i64 n, int per_block_items = BLOCK) {
  i64 g = SMX_CEIL_DIV(n > 0 ? n : 1, (i64)per_block_items);
  if (g > 4096) g = 4096;
  return (int)g;
}

extern "C" int smx_compose_workspace_bytes(int64_t n_a, int64_t n_b, int64_t n_sym, size_t* bytes) {
  if (!bytes || n_a < 0 || n_b < 0 || n_sym < 0) return set_err(SMX_E_ARG, "bad argument");
  *bytes = layout(n_a, n_b, n_sym).total;
  return SMX_OK;
}

static int compose_impl(const smx_ops* ops, const smx_compose_out* out, void* ws, size_t ws_bytes,
                        hipStream_t st) {
  const i64 na = ops->n_a, nb = ops->n_b, n = na + nb, n_sym = ops->n_sym;
  if (na < 0 || nb < 0 || n_sym < 0) return set_err(SMX_E_ARG, "negative size");
  if (n >= (i64)0x7fffffff) return set_err(SMX_E_ARG, "n_a + n_b must be < 2^31");
  if (!out || !out->counts) return set_err(SMX_E_ARG, "null output");
  if (n == 0) {
    HIP_TRY(hipMemsetAsync(out->counts, 0, 2 * sizeof(int64_t), st));
    return SMX_OK;
  }
  if (!ops->kind || !ops->ts || !ops->oid_hi || !ops->oid_lo || !ops->sym || !ops->v0 || !ops->v1 ||
      !out->order || !out->addr || !out->file || !out->ctx || (!out->conflicts && out->conflict_cap > 0))
    return set_err(SMX_E_ARG, "null input/output pointer");
  if (n_sym < 1) return set_err(SMX_E_ARG, "n_sym must be >= 1");
  const Layout L = layout(na, nb, n_sym);
  if (!ws || ws_bytes < L.total)
    return set_err(SMX_E_WORKSPACE, "workspace too small: need " + std::to_string(L.total));
  char* base = (char*)ws;
#define WS(T, b) ((T*)(base + L.off[b]))
  ComposeMeta* meta = WS(ComposeMeta, B_META);
  i64* bnd = WS(i64, B_BND);
  u32* wcnt = WS(u32, B_WCNT);
  u32* woff = WS(u32, B_WOFF);

  int prof;
  {
    std::lock_guard<std::mutex> g(g_prof_mu);
    prof = g_prof;
  }
  StageTimer tm(st, prof != 0);

  // ---- plan: stats + presorted partition + counts (one host sync) ----
  tm.begin(ST_PLAN);
  HIP_TRY(hipMemsetAsync(meta, 0, sizeof(ComposeMeta), st));
  hipLaunchKernelGGL(k_meta_init, dim3(1), dim3(1), 0, st, meta);
  hipLaunchKernelGGL(k_stats, dim3(grid_for(n, BLOCK * 16)), dim3(BLOCK), 0, st, ops->kind, ops->ts,
                     ops->oid_hi, ops->oid_lo, ops->sym, ops->v0, ops->v1, na, n, n_sym, meta);
  const i64 Wf = SMX_CEIL_DIV(n, (i64)WIN_TGT);
  hipLaunchKernelGGL(k_fpart, dim3(SMX_CEIL_DIV(Wf + 1, (i64)BLOCK)), dim3(BLOCK), 0, st, ops->ts, na, nb,
                     Wf, bnd);
  hipLaunchKernelGGL(k_wcount, dim3(Wf), dim3(BLOCK), 0, st, ops->kind, (const u32*)nullptr, bnd, na, Wf,
                     wcnt, meta, 1);
  hipLaunchKernelGGL(k_wscan, dim3(NCNT), dim3(BLOCK), 0, st, wcnt, woff, Wf, meta);
  HIP_TRY(hipGetLastError());
  ComposeMeta hm;
  HIP_TRY(hipMemcpyAsync(&hm, meta, sizeof(ComposeMeta), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  tm.end(ST_PLAN);
  if (hm.bad_sym) return set_err(SMX_E_ARG, "invalid input: sym[i] >= n_sym or kind[i] >= 18");
  const bool presorted = !hm.nonmono[0] && !hm.nonmono[1] && !hm.f_fail;
  const u64 nMv = hm.kcnt[KMOVE], nR = hm.kcnt[KREN];
  const u64 nRA = hm.n_ren_side[0], nRB = hm.n_ren_side[1];

  WinArgs P;
  P.kind = ops->kind;
  P.sym = ops->sym;
  P.v0 = ops->v0;
  P.v1 = ops->v1;
  P.na = na;
  P.bnd = bnd;
  P.woff = woff;
  P.meta = meta;
  P.order = WS(i32, B_ORDER);
  P.symT = WS(u32, B_SYMT);
  P.mvA = WS(i32, B_MVA);
  P.mvF = WS(i32, B_MVF);
  P.Msym = WS(u32, B_MSYM);
  P.Mcls = WS(i32, B_MCLS);
  P.Mstr = WS(i32, B_MSTR);
  P.Mside = WS(u8, B_MSIDE);
  P.Mown = WS(u32, B_MOWN);
  P.RA = WS(u32, B_RAB);
  P.RB = WS(u32, B_RAB) + nRA;
  i64 W;
  if (presorted) {
    W = Wf;
    P.kts = ops->ts;
    P.khi = ops->oid_hi;
    P.klo = ops->oid_lo;
    P.perm = nullptr;
  } else {
    // ---- generic: stable radix sort of each branch by (ts, oid_hi, oid_lo) ----
    tm.begin(ST_GSORT);
    u64* sts = WS(u64, B_STS);
    u64* shi = WS(u64, B_SHI);
    u64* slo = WS(u64, B_SLO);
    u32* perm = WS(u32, B_PERM);
    RadixTemp rt{WS(u64, B_RK2), WS(u32, B_RV2), WS(u32, B_RHIST), WS(u32, B_PART)};
    const u64* words[3] = {ops->oid_lo, ops->oid_hi, ops->ts};
    for (int side = 0; side < 2; ++side) {
      const i64 off = side ? na : 0, cnt = side ? nb : na;
      if (cnt == 0) continue;
      u64* key = WS(u64, B_RKEY) + off;
      u32* val = perm + off;
      for (int wi = 0; wi < 3; ++wi) {
        const int q = 2 - wi;  // meta order: 0 = ts, 1 = hi, 2 = lo
        const u64 varying = hm.key_or[side][q] ^ hm.key_and[side][q];
        int shifts[8], ns = 0;
        for (int dgt = 0; dgt < 8; ++dgt)
          if ((varying >> (8 * dgt)) & 0xffull) shifts[ns++] = 8 * dgt;
        if (wi == 0)
          hipLaunchKernelGGL(k_gather_init, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, words[wi] + off, key,
                             val, cnt);
        else
          hipLaunchKernelGGL(k_gather, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, words[wi], val, key, cnt);
        if (wi == 0 && off) {
          // values are op indices of A||B
          hipLaunchKernelGGL(k_offset, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, val, cnt, (u32)off);
        }
        if (ns) HIP_TRY(radix_sort_pairs(key, val, cnt, shifts, ns, rt, st));
      }
      hipLaunchKernelGGL(k_gather, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, ops->ts, val, sts + off, cnt);
      hipLaunchKernelGGL(k_gather, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, ops->oid_hi, val, shi + off, cnt);
      hipLaunchKernelGGL(k_gather, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, ops->oid_lo, val, slo + off, cnt);
    }
    W = SMX_CEIL_DIV(n, (i64)WIN_CAP);
    hipLaunchKernelGGL(k_gpart, dim3(SMX_CEIL_DIV(W + 1, (i64)BLOCK)), dim3(BLOCK), 0, st, sts, shi, slo, na,
                       nb, W, bnd);
    hipLaunchKernelGGL(k_wcount, dim3(W), dim3(BLOCK), 0, st, ops->kind, perm, bnd, na, W, wcnt, meta, 0);
    hipLaunchKernelGGL(k_wscan, dim3(NCNT), dim3(BLOCK), 0, st, wcnt, woff, W, meta);
    HIP_TRY(hipGetLastError());
    P.kts = sts;
    P.khi = shi;
    P.klo = slo;
    P.perm = perm;
    tm.end(ST_GSORT);
  }
  P.W = W;

  // ---- windows -> T-ordered arrays ----
  tm.begin(ST_WINDOW);
  if (presorted)
    hipLaunchKernelGGL(k_window<true>, dim3(W), dim3(BLOCK), 0, st, P);
  else
    hipLaunchKernelGGL(k_window<false>, dim3(W), dim3(BLOCK), 0, st, P);
  HIP_TRY(hipGetLastError());
  tm.end(ST_WINDOW);

  // ---- DivergentRename walk over the rename block ----
  tm.begin(ST_WALK);
  u8* skip = WS(u8, B_SKIP);
  u32* skipex = WS(u32, B_SKIPEX);
  u32* part = WS(u32, B_PART);
  const i32* order_ren = P.order + hm.base[KREN];
  if (nR > 0) {
    HIP_TRY(hipMemsetAsync(skip, 0, nR, st));
    WalkArgs Wk{P.Msym, P.Mcls, P.Mside, P.Mown, P.RA, P.RB, nR, nRA, nRB};
    u8* flags = WS(u8, B_FLAGS);
    u32* fpos = WS(u32, B_FPOS);
    u32* cand = WS(u32, B_CAND);
    u32* q = WS(u32, B_Q);
    u32* pm = WS(u32, B_PM);
    u32* nconf = WS(u32, B_NCONF);
    u32* nreal = WS(u32, B_NREAL);
    u32* coff = WS(u32, B_COFF);
    // n_cand / n_conf are u64 in meta; the scans produce u32 totals into the low word
    // (little endian) of the zeroed u64 fields.
    u32* ncand32 = (u32*)&meta->n_cand;
    u32* nconf32 = (u32*)&meta->n_conf;
    const u64* ncand_dev = &meta->n_cand;
    hipLaunchKernelGGL(k_flags, dim3(grid_for(nR)), dim3(BLOCK), 0, st, Wk, flags);
    HIP_TRY((scan_excl<OpSum, u8, u32>(flags, fpos, (i64)nR, nullptr, part, ncand32, st)));
    hipLaunchKernelGGL(k_compact, dim3(grid_for(nR)), dim3(BLOCK), 0, st, flags, fpos, nR, cand);
    hipLaunchKernelGGL(k_replay_q, dim3(grid_for(nR)), dim3(BLOCK), 0, st, Wk, cand, meta, q, nconf);
    HIP_TRY((scan_excl<OpMax, u32, u32>(q, pm, 0, ncand_dev, part, (u32*)nullptr, st)));
    hipLaunchKernelGGL(k_cluster, dim3(grid_for(nR)), dim3(BLOCK), 0, st, cand, q, pm, nconf, meta, nreal);
    HIP_TRY((scan_excl<OpSum, u32, u32>(nreal, coff, 0, ncand_dev, part, nconf32, st)));
    hipLaunchKernelGGL(k_replay_write, dim3(grid_for(nR)), dim3(BLOCK), 0, st, Wk, cand, nreal, coff, meta,
                       order_ren, out->conflicts, (u64)out->conflict_cap, skip);
    HIP_TRY((scan_excl<OpSum, u8, u32>(skip, skipex, (i64)nR, nullptr, part, (u32*)nullptr, st)));
    HIP_TRY(hipGetLastError());
  }
  tm.end(ST_WALK);

  // ---- per-symbol final states ----
  tm.begin(ST_TABLES);
  u64* tabA = WS(u64, B_TABA);
  u64* tabF = WS(u64, B_TABF);
  u64* tabR = WS(u64, B_TABR);
  int4* fin = WS(int4, B_FIN);
  HIP_TRY(hipMemsetAsync(tabA, 0, (size_t)n_sym * 8, st));
  HIP_TRY(hipMemsetAsync(tabF, 0, (size_t)n_sym * 8, st));
  HIP_TRY(hipMemsetAsync(tabR, 0, (size_t)n_sym * 8, st));
  if (nMv > 0)
    hipLaunchKernelGGL(k_tab_move, dim3(grid_for(nMv)), dim3(BLOCK), 0, st, P.symT, P.mvA, P.mvF, nMv, tabA,
                       tabF);
  if (nR > 0)
    hipLaunchKernelGGL(k_tab_ren, dim3(grid_for(nR)), dim3(BLOCK), 0, st, P.Msym, P.Mstr, skip, nR, tabR);
  hipLaunchKernelGGL(k_finalize, dim3(grid_for(n_sym)), dim3(BLOCK), 0, st, tabA, tabF, tabR, n_sym, fin);
  HIP_TRY(hipGetLastError());
  tm.end(ST_TABLES);

  // ---- moves with a None value need the per-symbol prefix (rare) ----
  const i32* prefA = P.mvA;
  const i32* prefF = P.mvF;
  if (hm.n_move_none > 0 && nMv > 0) {
    tm.begin(ST_MVPREFIX);
    u64* keys = WS(u64, B_RKEY);
    u32* vals = WS(u32, B_RVAL);
    RadixTemp rt{WS(u64, B_RK2), WS(u32, B_RV2), WS(u32, B_RHIST), WS(u32, B_PART)};
    int shifts[4], ns = 0;
    for (int dgt = 0; dgt < 4; ++dgt)
      if (((u64)(n_sym - 1) >> (8 * dgt)) != 0) shifts[ns++] = 8 * dgt;
    hipLaunchKernelGGL(k_mv_init, dim3(grid_for(nMv)), dim3(BLOCK), 0, st, P.symT, nMv, keys, vals);
    if (ns) HIP_TRY(radix_sort_pairs(keys, vals, (i64)nMv, shifts, ns, rt, st));
    i32* pA = WS(i32, B_PREFA);
    i32* pF = WS(i32, B_PREFF);
    hipLaunchKernelGGL(k_mv_seg, dim3(grid_for(nMv)), dim3(BLOCK), 0, st, keys, vals, nMv, P.mvA, P.mvF, pA,
                       pF);
    HIP_TRY(hipGetLastError());
    prefA = pA;
    prefF = pF;
    tm.end(ST_MVPREFIX);
  }

  // ---- compacted output ----
  tm.begin(ST_EMIT);
  EmitArgs E{P.order, P.symT, prefA, prefF, skip, skipex, fin, meta, (u64)n, nMv, nR,
             out->order, out->addr, out->file, out->ctx};
  hipLaunchKernelGGL(k_emit, dim3(grid_for(n, BLOCK * 4)), dim3(BLOCK), 0, st, E);
  hipLaunchKernelGGL(k_counts, dim3(1), dim3(1), 0, st, meta, (u64)n, out->counts);
  HIP_TRY(hipGetLastError());
  tm.end(ST_EMIT);
  tm.flush();
#undef WS
  return SMX_OK;
}

extern "C" int smx_compose(const smx_ops* ops, const smx_compose_out* out, void* workspace,
                           size_t workspace_bytes, void* stream) {
  if (!ops) return set_err(SMX_E_ARG, "null ops");
  try {
    return compose_impl(ops, out, workspace, workspace_bytes, (hipStream_t)stream);
  } catch (const std::exception& e) {
    return set_err(SMX_E_HIP, e.what());
  }
}

extern "C" int smx_set_profiling(int enabled) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  g_prof = enabled;
  return SMX_OK;
}

extern "C" int smx_reset_stage_times(void) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  for (int i = 0; i < ST_N; ++i) {
    g_stage_ms[i] = 0;
    g_stage_calls[i] = 0;
  }
  return SMX_OK;
}

extern "C" int smx_stage_times(double* ms, int64_t* calls, int cap) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  for (int i = 0; i < ST_N && i < cap; ++i) {
    if (ms) ms[i] = g_stage_ms[i];
    if (calls) calls[i] = g_stage_calls[i];
  }
  return ST_N;
}

extern "C" const char* smx_stage_name(int i) { return (i >= 0 && i < ST_N) ? kStageNames[i] : ""; }

extern "C" const char* smx_last_error(void) { return g_err.c_str(); }

extern "C" const char* smx_version(void) { return "smx 0.1 gfx950"; }
