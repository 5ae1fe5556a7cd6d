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
//   k_fpart     presorted windows: merge-path on timestamps, cut at ts boundaries
//   k_wcount    per-window kind counts + presorted-layout checks
//   k_wscan     window offsets and kind totals  k_bases   T segment starts
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
#include "smx_window.h"


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

// Stage events are recorded on the call's stream and only resolved when the
// caller asks for the times (smx_stage_times), so profiling adds no host sync.
struct PendingEv {
  int stage;
  hipEvent_t a, b;
};
static std::vector<PendingEv> g_pending;

struct StageTimer {
  hipStream_t st;
  bool on;
  hipEvent_t open[ST_N];
  std::vector<PendingEv> done;
  StageTimer(hipStream_t s, bool enabled) : st(s), on(enabled) {}
  void begin(int i) {
    if (!on) return;
    (void)hipEventCreate(&open[i]);
    (void)hipEventRecord(open[i], st);
  }
  void end(int i) {
    if (!on) return;
    hipEvent_t b;
    (void)hipEventCreate(&b);
    (void)hipEventRecord(b, st);
    done.push_back({i, open[i], b});
  }
  void flush() {
    if (!on) return;
    std::lock_guard<std::mutex> g(g_prof_mu);
    for (auto& p : done) g_pending.push_back(p);
    done.clear();
  }
  ~StageTimer() {
    for (auto& p : done) {  // an error path left events unpublished
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
  }
};

static void resolve_pending_locked() {
  for (auto& p : g_pending) {
    (void)hipEventSynchronize(p.b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    g_stage_ms[p.stage] += ms;
    g_stage_calls[p.stage] += 1;
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  g_pending.clear();
}

// ---------------------------------------------------------------------------
// kernels: planning

// Per-branch OR / AND of the key words (generic path: skip constant radix digits).
__global__ void __launch_bounds__(BLOCK) k_keymask(const u64* __restrict__ ts, const u64* __restrict__ hi,
                                                   const u64* __restrict__ lo, i64 na, i64 n,
                                                   ComposeMeta* meta) {
  u64 ro[2][3] = {{0, 0, 0}, {0, 0, 0}};
  u64 ra[2][3] = {{~0ull, ~0ull, ~0ull}, {~0ull, ~0ull, ~0ull}};
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (i64)gridDim.x * BLOCK) {
    const u64 v[3] = {ts[i], hi[i], lo[i]};
    const int s = i >= na;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      ro[s][q] |= v[q];
      ra[s][q] &= v[q];
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      atomicOr((unsigned long long*)&meta->key_or[s][q], (unsigned long long)ro[s][q]);
      atomicAnd((unsigned long long*)&meta->key_and[s][q], (unsigned long long)ra[s][q]);
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

// Per-window counts: each kind, renames per branch, moves with a None value.
// perm == nullptr: presorted layout (branch position j is op j); then the kernel
// also checks what the presorted windows rely on: boundaries non-decreasing,
// window size <= WIN_CAP, timestamps non-decreasing inside each branch (every
// adjacent pair is checked by exactly one window).  Column-major [c][W].
__global__ void __launch_bounds__(BLOCK) k_wcount(const u8* __restrict__ kind, const u64* __restrict__ ts,
                                                  const i32* __restrict__ v0, const i32* __restrict__ v1,
                                                  const u32* __restrict__ perm, const i64* __restrict__ bnd,
                                                  i64 na, i64 W, u32* __restrict__ wcnt, ComposeMeta* meta) {
  __shared__ u32 c[NCNT];
  __shared__ u32 fail;
  const i64 w = blockIdx.x;
  if (threadIdx.x < NCNT) c[threadIdx.x] = 0;
  if (threadIdx.x == 0) fail = 0;
  __syncthreads();
  const i64 a0 = bnd[2 * w], b0 = bnd[2 * w + 1], a1 = bnd[2 * w + 2], b1 = bnd[2 * w + 3];
  const bool presorted = perm == nullptr;
  if (presorted && threadIdx.x == 0 && (a1 < a0 || b1 < b0 || (a1 - a0) + (b1 - b0) > WIN_CAP)) fail = 1;
  bool bad = false, mono_fail = false;
  for (int side = 0; side < 2; ++side) {
    const i64 lo = side ? b0 : a0, hi = side ? b1 : a1, off = side ? na : 0;
    for (i64 j = lo + threadIdx.x; j < hi; j += BLOCK) {
      const u32 src = presorted ? (u32)(off + j) : perm[off + j];
      const u32 k0 = kind[src];
      bad |= k0 >= SMX_N_KINDS;
      const u32 k = k0 < SMX_N_KINDS ? k0 : SMX_N_KINDS - 1;
      atomicAdd(&c[k], 1u);
      if (k == KREN) atomicAdd(&c[CNT_REN_A + side], 1u);
      if (k == KMOVE && (v0[src] < 0 || v1[src] < 0)) atomicAdd(&c[CNT_NONE_MV], 1u);
      if (presorted && j > 0 && ts[src - 1] > ts[src]) mono_fail = true;
    }
  }
  if (mono_fail) fail = 1;
  if (bad) meta->bad_sym = 1;
  __syncthreads();
  if (threadIdx.x == 0 && fail) meta->f_fail = 1;
  if (threadIdx.x < NCNT) wcnt[(i64)threadIdx.x * W + w] = c[threadIdx.x];
}

// Exclusive scan of each count column over windows; column totals into meta.
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
  if (threadIdx.x == 0) {
    if (c < SMX_N_KINDS) meta->kcnt[c] = carry;
    else if (c == CNT_REN_A) meta->n_ren_side[0] = carry;
    else if (c == CNT_REN_B) meta->n_ren_side[1] = carry;
    else meta->n_move_none = carry;
  }
}

// T bases: exclusive prefix of the kind totals.
__global__ void k_bases(ComposeMeta* meta) {
  u64 acc = 0;
  for (int k = 0; k < SMX_N_KINDS; ++k) {
    meta->base[k] = acc;
    acc += meta->kcnt[k];
  }
  meta->base[SMX_N_KINDS] = acc;
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

#include "smx_walk.h"

// ---------------------------------------------------------------------------
// kernels: per-symbol last writers and output

// Invalid syms (flagged by the window kernel, reported through counts) are
// clamped so that every access stays in bounds.
__global__ void k_tab_move(const u32* __restrict__ symT, const i32* __restrict__ mvA,
                           const i32* __restrict__ mvF, u64 nMv, u64* __restrict__ tabA,
                           u64* __restrict__ tabF, u32 smax) {
  for (u64 T = (u64)blockIdx.x * BLOCK + threadIdx.x; T < nMv; T += (u64)gridDim.x * BLOCK) {
    const u32 s = min(symT[T], smax);
    const i32 a = mvA[T], f = mvF[T];
    if (a >= 0) atomicMax((unsigned long long*)&tabA[s], (unsigned long long)(((T + 1) << 32) | (u32)a));
    if (f >= 0) atomicMax((unsigned long long*)&tabF[s], (unsigned long long)(((T + 1) << 32) | (u32)f));
  }
}

__global__ void k_tab_ren(const u32* __restrict__ Msym, const i32* __restrict__ Mstr,
                          const u8* __restrict__ skip, u64 nR, u64* __restrict__ tabR, u32 smax) {
  for (u64 m = (u64)blockIdx.x * BLOCK + threadIdx.x; m < nR; m += (u64)gridDim.x * BLOCK) {
    if (skip[m]) continue;
    atomicMax((unsigned long long*)&tabR[min(Msym[m], smax)], (unsigned long long)(((m + 1) << 32) | (u32)Mstr[m]));
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
  u32 smax;
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
      const int4 F = E.fin[min(E.symT[T], E.smax)];
      a = F.x;
      f = F.y;
      c = -1;
    } else {
      o = T - nskip;
      const int4 F = E.fin[min(E.symT[T], E.smax)];
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
  if (meta->bad_sym) {  // invalid input (sym >= n_sym or kind >= 18)
    counts[0] = -1;
    counts[1] = -1;
    return;
  }
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

  // ---- plan: presorted windows + per-window counts/checks (one host sync) ----
  tm.begin(ST_PLAN);
  HIP_TRY(hipMemsetAsync(meta, 0, sizeof(ComposeMeta), st));
  const i64 Wf = SMX_CEIL_DIV(n, (i64)WIN_TGT);
  hipLaunchKernelGGL(k_fpart, dim3(SMX_CEIL_DIV(Wf + 1, (i64)BLOCK)), dim3(BLOCK), 0, st, ops->ts, na, nb,
                     Wf, bnd);
  hipLaunchKernelGGL(k_wcount, dim3(Wf), dim3(BLOCK), 0, st, ops->kind, ops->ts, ops->v0, ops->v1,
                     (const u32*)nullptr, bnd, na, Wf, wcnt, meta);
  hipLaunchKernelGGL(k_wscan, dim3(NCNT), dim3(BLOCK), 0, st, wcnt, woff, Wf, meta);
  hipLaunchKernelGGL(k_bases, dim3(1), dim3(1), 0, st, meta);
  HIP_TRY(hipGetLastError());
  ComposeMeta hm;
  HIP_TRY(hipMemcpyAsync(&hm, meta, sizeof(ComposeMeta), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  tm.end(ST_PLAN);
  if (hm.bad_sym) return set_err(SMX_E_ARG, "invalid input: kind[i] >= 18");
  const bool presorted = !hm.f_fail;

  WinArgs P;
  P.kind = ops->kind;
  P.sym = ops->sym;
  P.v0 = ops->v0;
  P.v1 = ops->v1;
  P.na = na;
  P.n_sym = n_sym;
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
    HIP_TRY(hipMemsetAsync(meta, 0, sizeof(ComposeMeta), st));
    hipLaunchKernelGGL(k_meta_init, dim3(1), dim3(1), 0, st, meta);
    hipLaunchKernelGGL(k_keymask, dim3(grid_for(n, BLOCK * 8)), dim3(BLOCK), 0, st, ops->ts, ops->oid_hi,
                       ops->oid_lo, na, n, meta);
    HIP_TRY(hipMemcpyAsync(&hm, meta, sizeof(ComposeMeta), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
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
        if (wi == 0) {
          hipLaunchKernelGGL(k_gather_init, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, words[wi] + off, key,
                             val, cnt);
          if (off)  // values are op indices of A||B
            hipLaunchKernelGGL(k_offset, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, val, cnt, (u32)off);
        } else {
          hipLaunchKernelGGL(k_gather, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, words[wi], val, key, cnt);
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
    hipLaunchKernelGGL(k_wcount, dim3(W), dim3(BLOCK), 0, st, ops->kind, ops->ts, ops->v0, ops->v1, perm, bnd,
                       na, W, wcnt, meta);
    hipLaunchKernelGGL(k_wscan, dim3(NCNT), dim3(BLOCK), 0, st, wcnt, woff, W, meta);
    hipLaunchKernelGGL(k_bases, dim3(1), dim3(1), 0, st, meta);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&hm, meta, sizeof(ComposeMeta), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    P.kts = sts;
    P.khi = shi;
    P.klo = slo;
    P.perm = perm;
    tm.end(ST_GSORT);
  }
  P.W = W;
  const u64 nMv = hm.kcnt[KMOVE], nR = hm.kcnt[KREN];
  const u64 nRA = hm.n_ren_side[0], nRB = hm.n_ren_side[1];
  P.RA = WS(u32, B_RAB);
  P.RB = WS(u32, B_RAB) + nRA;

  // ---- windows -> T-ordered arrays ----
  tm.begin(ST_WINDOW);
  if (presorted)
    hipLaunchKernelGGL(k_window_f, dim3(W), dim3(WF_NT), 0, st, P);
  else
    hipLaunchKernelGGL(k_window_g, dim3(W), dim3(WG_NT), 0, st, P);
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
                       tabF, (u32)(n_sym - 1));
  if (nR > 0)
    hipLaunchKernelGGL(k_tab_ren, dim3(grid_for(nR)), dim3(BLOCK), 0, st, P.Msym, P.Mstr, skip, nR, tabR, (u32)(n_sym - 1));
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
  EmitArgs E{P.order, P.symT, prefA, prefF, skip, skipex, fin, meta, (u64)n, nMv, nR, (u32)(n_sym - 1),
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
  resolve_pending_locked();
  for (int i = 0; i < ST_N; ++i) {
    g_stage_ms[i] = 0;
    g_stage_calls[i] = 0;
  }
  return SMX_OK;
}

extern "C" int smx_stage_times(double* ms, int64_t* calls, int cap) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  resolve_pending_locked();
  for (int i = 0; i < ST_N && i < cap; ++i) {
    if (ms) ms[i] = g_stage_ms[i];
    if (calls) calls[i] = g_stage_calls[i];
  }
  return ST_N;
}

extern "C" const char* smx_stage_name(int i) { return (i >= 0 && i < ST_N) ? kStageNames[i] : ""; }

extern "C" const char* smx_last_error(void) { return g_err.c_str(); }

extern "C" const char* smx_version(void) { return "smx 0.1 gfx950"; }
