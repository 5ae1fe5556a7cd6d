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
//               equal-timestamp groups by id; the moves' final records, the other
//               ops' (source, symbol) in T order, natural-head DivergentRename flags
//   walk        k_boundary -> candidate scan/compact -> k_replay_q -> max-scan ->
//               k_cluster -> scan -> k_replay_write (conflict pairs, skip bits,
//               sorted skip list)
//   tables      per-symbol last writers: bucket by symbol range, LDS max-reduce
//   k_emit      compacted output of every op after the move block: order, addr,
//               file, ctx
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "smx_sort.h"
#include "smx_window.h"
#include "smx_small.h"
#include "smx_tables.h"


// ---------------------------------------------------------------------------
// error / profiling state
static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int smx_set_error(int code, const char* msg) { return set_err(code, msg ? msg : ""); }
#define HIP_TRY(x)                                                                 \
  do {                                                                             \
    hipError_t _e = (x);                                                           \
    if (_e != hipSuccess)                                                          \
      return set_err(SMX_E_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

// gsort: the generic plan's sort and window planning; segsort: its segmented sort's
// kernels alone (inside gsort); window_g: the generic window kernel; window: the
// presorted one at the normal or small capacity, including attempts that fail;
// window_wide: its wide (8192-op) instance, a stage of its own so that a merge's
// failed normal attempt is never averaged into the wide launch's time
enum Stage { ST_PLAN, ST_GSORT, ST_WINDOW, ST_WALK, ST_TABLES, ST_MVPREFIX, ST_EMIT, ST_SEGSORT, ST_WINDOW_G,
             ST_WINDOW_WIDE, ST_SMALL, ST_N };
static const char* kStageNames[ST_N] = {"plan",   "gsort",    "window", "walk",    "tables",
                                        "mvprefix", "emit", "segsort", "window_g", "window_wide", "small"};
static std::mutex g_prof_mu;
static int g_prof = 0;
static u32 g_prof_mask = ~0u;  // the stages timed while profiling is on (smx_set_profiling_stages)
static double g_stage_ms[ST_N];
static int64_t g_stage_calls[ST_N];

// Stage events are recorded on the call's stream and only resolved when the
// caller asks for the times (smx_stage_times), so profiling adds no host sync.
struct PendingEv {
  int stage;
  hipEvent_t a, b;
};
static std::vector<PendingEv> g_pending;

// Timing events are reused: creating and destroying a dozen per merge sat on the host
// path between one merge's sync and the next merge's first launch.  (g_prof_mu guards
// the pool.)
static std::vector<hipEvent_t> g_ev_pool;
static hipEvent_t ev_acquire() {
  {
    std::lock_guard<std::mutex> g(g_prof_mu);
    if (!g_ev_pool.empty()) {
      hipEvent_t e = g_ev_pool.back();
      g_ev_pool.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  // timing only (read after the caller's sync): no system-scope fence, whose cache
  // write-back and invalidate at every record cost the timed merges ~40 us on config 3
  // (2.380 ms with the stage timers on against 2.342 ms off, measured in round 5)
  (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return e;
}
static void ev_release_locked(hipEvent_t e) {  // (caller holds g_prof_mu)
  if (e) g_ev_pool.push_back(e);
}

struct StageTimer {
  hipStream_t st;
  bool on;
  u32 mask = ~0u;
  hipEvent_t open[ST_N];
  std::vector<PendingEv> done;
  bool is_open[ST_N] = {};
  StageTimer(hipStream_t s, bool enabled) : st(s), on(enabled) {
    if (on) {
      std::lock_guard<std::mutex> g(g_prof_mu);
      mask = g_prof_mask;
    }
  }
  void begin(int i) {
    if (!on || !((mask >> i) & 1u)) return;
    if (!is_open[i]) open[i] = ev_acquire();  // (a restarted stage re-records its open event)
    (void)hipEventRecord(open[i], st);
    is_open[i] = true;
  }
  void end(int i) {
    if (!on || !is_open[i]) return;
    hipEvent_t b = ev_acquire();
    (void)hipEventRecord(b, st);
    done.push_back({i, open[i], b});
    is_open[i] = false;
  }
  void flush() {
    if (!on) return;
    std::lock_guard<std::mutex> g(g_prof_mu);
    for (auto& p : done) g_pending.push_back(p);
    done.clear();
  }
  ~StageTimer() {  // an error path left events unpublished: back to the pool
    if (done.empty() && !std::any_of(is_open, is_open + ST_N, [](bool b) { return b; })) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
      (void)hipGetLastError();
      return;  // a capturing stream must not be synchronized: these events are left to leak
    }
    (void)hipStreamSynchronize(st);  // (recorded events may still be pending)
    std::lock_guard<std::mutex> g(g_prof_mu);
    for (auto& p : done) {
      ev_release_locked(p.a);
      ev_release_locked(p.b);
    }
    for (int i = 0; i < ST_N; ++i)
      if (is_open[i]) ev_release_locked(open[i]);
  }
};

static void resolve_pending_locked() {
  for (auto& p : g_pending) {
    (void)hipEventSynchronize(p.b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    g_stage_ms[p.stage] += ms;
    g_stage_calls[p.stage] += 1;
    ev_release_locked(p.a);
    ev_release_locked(p.b);
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
  // wave OR of the 12 words (AND = NOT OR NOT) on DPP, then LDS, then one device
  // atomic per word and block (a device atomic per thread serialised on 12 words)
  __shared__ u32 sm[24];
  if (threadIdx.x < 24) sm[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const u64 w[2] = {ro[s][q], ~ra[s][q]};
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const u32 lo32 = wave_or_to_last((u32)w[x]), hi32 = wave_or_to_last((u32)(w[x] >> 32));
        if ((threadIdx.x & (WAVE - 1)) == WAVE - 1) {
          atomicOr(&sm[(s * 3 + q) * 4 + 2 * x], lo32);
          atomicOr(&sm[(s * 3 + q) * 4 + 2 * x + 1], hi32);
        }
      }
    }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int s = threadIdx.x / 3, q = threadIdx.x % 3;
    const u32* v = &sm[threadIdx.x * 4];
    atomicOr((unsigned long long*)&meta->key_or[s][q], ((unsigned long long)v[1] << 32) | v[0]);
    atomicAnd((unsigned long long*)&meta->key_and[s][q], ~(((unsigned long long)v[3] << 32) | v[2]));
  }
}

// Zero fill as a kernel: the asynchronous part of a merge, which is captured into a
// HIP graph, holds kernel nodes only.
__global__ void k_zero(u32* __restrict__ p, u64 nw) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (u64)gridDim.x * blockDim.x) p[i] = 0u;
}
static int zero_async(void* p, size_t bytes, hipStream_t st) {
  if (bytes % 4) return set_err(SMX_E_ARG, "zero_async: size not a multiple of 4");
  const u64 nw = bytes / 4;
  if (nw == 0) return SMX_OK;
  u64 g = SMX_CEIL_DIV(nw, (u64)BLOCK * 4);
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_zero, dim3((u32)g), dim3(BLOCK), 0, st, (u32*)p, nw);
  HIP_TRY(hipGetLastError());
  return SMX_OK;
}

__global__ void k_meta_init(ComposeMeta* meta) {
  for (int s = 0; s < 2; ++s)
    for (int q = 0; q < 3; ++q) meta->key_and[s][q] = ~0ull;
}

#ifndef SMX_KHIST_LONG
#define SMX_KHIST_LONG 1     // k_fpart flags timestamp groups longer than a window (from k_khist's samples)
#endif
#ifndef SMX_FPART_FAILCHK
#define SMX_FPART_FAILCHK 0  // k_fpart skips its snap and writes on a failed plan (off: plan 0.135 -> 0.14 ms on config 3, profiles/r03_x/ab_plan_checks.txt)
#endif
#ifndef SMX_CSCAN_FAILCHK
#define SMX_CSCAN_FAILCHK 0  // the chunk scans leave on a failed plan (off, as k_fpart)
#endif

// Presorted windows: boundary k sits at the merge-path split of diagonal k*tgt
// (timestamps, A first on ties), snapped down to the first op of that timestamp on
// both branches, so every (timestamp) group lands whole in one window.
// tgt is a multiple of CH, so at split candidates m = CH*i the merge-path test
// A[m] <= B[d-1-m] reads only chunk samples (sA[i] = A[CH*i], sB[j] =
// B[CH*j + CH-1]; 1/256 of the keys, cache-resident): the first level of the
// search runs on them, the second inside one chunk.  The snap gallops back over
// the (short) run of equal timestamps.
// LongW (the synchronous merge's early verdict): k_khist made the long-group test; on its
// F_LONG these are the wide plan's boundaries (tgt_w, W_w windows of D_w chunks, its own
// long test flagging F_WLONG) and k_cscan_mid then clears F_LONG, so no normal window, no
// re-arm and no second k_fpart run (config 5's doomed attempt).
struct LongW {
  i64 tgt_w = 0, W_w = 0, D_w = 0;  // tgt_w 0: off
};
__device__ __forceinline__ void fpart_body(const u64* __restrict__ ts, const u64* __restrict__ tsB,
                                           const u64* __restrict__ sA, const u64* __restrict__ sB, i64 na, i64 nb,
                                           i64 W, i64 tgt, i64 D, i64* __restrict__ bnd, ComposeMeta* meta,
                                           u32* long_host, i64 blk, i64 nblk, LongW lw = LongW{}) {
  const i64 k = blk * BLOCK + threadIdx.x;
  bool chk = SMX_KHIST_LONG;
  u64 fl = F_LONG;
  if (lw.tgt_w) {
    if ((__hip_atomic_load(&meta->f_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & F_LONG) == F_LONG) {
      W = lw.W_w, tgt = lw.tgt_w, D = lw.D_w;  // the wide plan, tested at its own capacity
      fl = F_WLONG;
      long_host = nullptr;
    } else {
      chk = false;  // (k_khist tested the normal capacity)
    }
  }
  if (chk) {
    // A chunk sample equal to the sample D chunks (one window capacity) later (A: first
    // ops of chunks c and c + D; B: last ops of full chunks): that timestamp group alone
    // overflows a window, so the presorted plan cannot hold.  Flagged before the windows
    // run: k_window_f then leaves before its loads (6: a window too large, and smaller
    // windows cannot help).  Grid-stride over the samples, off the search's path.
    const i64 nt = nblk * BLOCK, ca = SMX_CEIL_DIV(na, (i64)CH), cb = nb / CH;
    bool lg = false;
    for (i64 c = k; c + D < ca; c += nt) lg |= sA[c] == sA[c + D];
    for (i64 c = k; c + D < cb; c += nt) lg |= sB[c] == sB[c + D];
    const u64 lgw = __ballot(lg);
    if (lgw && (threadIdx.x & (WAVE - 1)) == 0 &&
        (__hip_atomic_load(&meta->f_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & fl) != fl) {
      atomicOr((unsigned long long*)&meta->f_fail, fl);
      // ... and, on the synchronous path, to the host (pinned, coherent), which then
      // launches no tail behind this failed plan
      if (long_host) __hip_atomic_store(long_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // a wave that saw the plan fail leaves its boundaries unsearched, as 0 (k_window_f
    // leaves before its loads on F_LONG, and a zero boundary only ever gives an empty or
    // an oversized window; the wide plan redoes them) -- on config 5 the snap's gallops
    // over 4096-op timestamp runs were most of this kernel
    if (lgw) {
      if (k <= W) bnd[2 * k] = bnd[2 * k + 1] = 0;
      return;
    }
  }
  if (k > W) return;
  const u64 failed = SMX_FPART_FAILCHK ? meta->f_fail : 0ull;  // (k_khist saw a group no window holds; used after the search)
  const i64 n = na + nb;
  const u64* A = ts;
  const u64* B = tsB;
  const i64 d = k * tgt;
  if (k == 0 || d >= n || k == W) {
    bnd[2 * k] = k == 0 ? 0 : na;
    bnd[2 * k + 1] = k == 0 ? 0 : nb;
    return;
  }
  const i64 lo0 = d - nb > 0 ? d - nb : 0, hi0 = d < na ? d : na;
  i64 lo = lo0, hi = hi0;
  if (lo < hi) {
    const i64 ilo = SMX_CEIL_DIV(lo, (i64)CH), ihi = (hi - 1) / CH;  // samples inside [lo, hi)
    if (ilo <= ihi) {
      const i64 dj = d / CH - 1;
      i64 l = ilo, h = ihi + 1;
      while (l < h) {
        const i64 mid = (l + h) >> 1;
        if (sA[mid] <= sB[dj - mid]) l = mid + 1;
        else h = mid;
      }
      // test true at CH*(l-1) (if l > ilo), false at CH*l (if l <= ihi)
      if (l > ilo) lo = CH * (l - 1) + 1;
      if (l <= ihi) hi = CH * l;
    }
    while (lo < hi) {
      const i64 mid = (lo + hi) >> 1;
      if (A[mid] <= B[d - 1 - mid]) lo = mid + 1;
      else hi = mid;
    }
  }
  if (failed) return;
  const i64 a = lo, b = d - lo;
  const u64 tau = (a < na && (b >= nb || A[a] <= B[b])) ? A[a] : B[b];
  // first index of each branch with ts >= tau: at or before the split
  i64 r[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const u64* X = s ? B : A;
    i64 h = s ? b : a;  // X[h] >= tau, or h == branch length
    i64 step = 1, l = 0;
    while (h > 0) {
      const i64 cand = h - step > 0 ? h - step : 0;
      if (X[cand] < tau) {
        l = cand + 1;
        break;
      }
      h = cand;
      step *= 2;
    }
    while (l < h) {
      const i64 mid = (l + h) >> 1;
      if (X[mid] < tau) l = mid + 1;
      else h = mid;
    }
    r[s] = l;
  }
  bnd[2 * k] = r[0];
  bnd[2 * k + 1] = r[1];
}
__global__ void k_fpart(const u64* __restrict__ ts, const u64* __restrict__ tsB, const u64* __restrict__ sA,
                        const u64* __restrict__ sB, i64 na, i64 nb, i64 W, i64 tgt, i64 D, i64* __restrict__ bnd,
                        ComposeMeta* meta, u32* long_host, LongW lw) {
  fpart_body(ts, tsB, sA, sB, na, nb, W, tgt, D, bnd, meta, long_host, blockIdx.x, gridDim.x, lw);
}

// Generic windows over branch logs sorted by (ts, oid): fixed diagonals of WIN_CAP.
__global__ void k_gpart(const u64* __restrict__ sts, const u64* __restrict__ shi,
                        const u64* __restrict__ slo, i64 na, i64 nb, i64 W, i64* __restrict__ bnd,
                        const ComposeMeta* meta) {
  const i64 k = (i64)blockIdx.x * BLOCK + threadIdx.x;
  if (k > W || meta->f_fail) return;  // (the segmented sort failed: nothing to cut)
  const i64 n = na + nb;
  const i64 d = k * WG_CAP;
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

// Presorted plan, counting: kind histogram of fixed 256-op chunks of each branch
// (cnt[side][kind][chunk]), then an exclusive scan over chunks per (side, kind).
// A window derives its T offsets from the chunk prefixes at its start plus the
// kinds of at most 255 ops before it.  Coalesced: iteration j of a block reads
// chunk j, lane t its byte t.
#ifndef KH_NT
#define KH_NT 512                  // 32 chunks per block: a column's counts fill a 128-byte line
#endif
#define CH_PER_BLOCK (KH_NT / 16)   // 16 lanes x 16 kind bytes per 256-op chunk
#ifndef KH_BF
#define KH_BF 0                    // branch-free byte counting: plan 0.134 -> 0.137 ms (round 4); off
#endif
#ifndef KH_R
#define KH_R 1                     // chunk rounds per block (4 measured slower: profiles/r02_k/khist_rounds_ab.txt)
#endif

// Block b counts global chunks [b*CH_PER_BLOCK, ...) (A chunks, then B chunks):
// lane t reads bytes [16*(t%16), +16) of chunk t/16 (one 16-byte load when
// aligned), so a chunk is one 16-lane DPP row.  No atomics: each lane counts its 16
// kinds in packed 5-bit fields (6 kinds per word), widens them to 10-bit fields and
// the row adds them up with DPP shifts; the row's last lane holds the chunk's counts.
// Dl > 0 (the synchronous merge's early verdict): k_fpart's long-group test is made here,
// on the input itself (the timestamp Dl chunks later, one more load per chunk), so that
// the host learns it right behind this kernel and launches the windows that hold the
// groups (smx_compose.hip enqueue_async); f_fail = F_LONG and long_host[0] = 1.
__global__ void __launch_bounds__(KH_NT) k_khist(const u8* __restrict__ kind, const u64* __restrict__ ts,
                                                 i64 na, i64 nb, i64 bgap, i64 CM, u32* __restrict__ cnt,
                                                 u64* __restrict__ sA, u64* __restrict__ sB, ComposeMeta* meta,
                                                 u32* long_host, i64 Dl) {
  __shared__ u32 c[CH_PER_BLOCK * KH_R][SMX_N_KINDS];
  __shared__ u32 km[2];
  __shared__ u32 lgb;  // the block saw a group longer than a window (Dl)
  const i64 CA = SMX_CEIL_DIV(na, (i64)CH), CB = SMX_CEIL_DIV(nb, (i64)CH);
  const int j = threadIdx.x / 16, q = threadIdx.x % 16;
  if (threadIdx.x < 2) km[threadIdx.x] = 0;
  if (threadIdx.x == 0) lgb = 0;
  // KH_R rounds of CH_PER_BLOCK chunks per block; every round's loads are issued first
  u32 w[KH_R][4];
  int nvr[KH_R];
  // timestamp samples for k_fpart: first op of each A chunk, last op of each full B chunk
  // (stored after the counting: their loads then wait beside the kind bytes', not ahead of
  // them; separate registers for A and B, or the second load waits on the first)
  u64 smpA[KH_R], smpB[KH_R], farA[KH_R], farB[KH_R];  // (far: the sample Dl chunks later)
  u64* atA[KH_R];
  u64* atB[KH_R];
  bool chkA[KH_R], chkB[KH_R];
#pragma unroll
  for (int rd = 0; rd < KH_R; ++rd) {
    const i64 g = ((i64)blockIdx.x * KH_R + rd) * CH_PER_BLOCK + j;
    const int side = g >= CA;
    const i64 cc = side ? g - CA : g;
    const i64 len = side ? nb : na;
    const i64 r0 = cc * CH + q * 16;  // branch position of this lane's first byte
    const int nv = g < CA + CB ? (int)(len - r0 < 0 ? 0 : (len - r0 < 16 ? len - r0 : 16)) : 0;
    nvr[rd] = nv;
    const u8* src = kind + (side ? na + bgap : 0) + r0;
    w[rd][0] = w[rd][1] = w[rd][2] = w[rd][3] = 0u;
    if (nv == 16 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
      const uint4 v = *reinterpret_cast<const uint4*>(src);
      w[rd][0] = v.x; w[rd][1] = v.y; w[rd][2] = v.z; w[rd][3] = v.w;
    } else {
#pragma unroll
      for (int y = 0; y < 16; ++y)
        if (y < nv) w[rd][y >> 2] |= (u32)src[y] << (8 * (y & 3));
    }
    atA[rd] = atB[rd] = nullptr;
    smpA[rd] = smpB[rd] = farA[rd] = farB[rd] = 0;
    chkA[rd] = chkB[rd] = false;
    if (g < CA + CB) {
      if (!side && q == 0) {
        atA[rd] = sA + cc;
        smpA[rd] = ts[cc * CH];
        if (Dl > 0 && cc + Dl < CA) {
          chkA[rd] = true;
          farA[rd] = ts[(cc + Dl) * CH];
        }
      }
      if (side && q == 15 && nv == 16) {
        atB[rd] = sB + cc;
        smpB[rd] = ts[na + bgap + cc * CH + CH - 1];
        if (Dl > 0 && cc + Dl < nb / CH) {  // (B samples: last ops of full chunks)
          chkB[rd] = true;
          farB[rd] = ts[na + bgap + (cc + Dl) * CH + CH - 1];
        }
      }
    }
  }
  bool bad = false;
#pragma unroll
  for (int rd = 0; rd < KH_R; ++rd) {
    const int nv = nvr[rd];
    u32 pk[3] = {0u, 0u, 0u};  // kind k: bits 5 * (k % 6) of word k / 6
#pragma unroll
    for (int y = 0; y < 16; ++y) {
      if (!KH_BF && y >= nv) break;
      const bool ok = !KH_BF || y < nv;  // (branch-free: a lane past its chunk's end adds 0)
      u32 k = (w[rd][y >> 2] >> (8 * (y & 3))) & 0xffu;
      bad |= ok & (k >= SMX_N_KINDS);
      k = k < SMX_N_KINDS ? k : SMX_N_KINDS - 1;
      const u32 wd = (k * 43u) >> 8;  // k / 6 for k < 18
      const u32 inc = ok ? 1u << (5u * (k - 6u * wd)) : 0u;
      pk[0] += wd == 0 ? inc : 0u;
      pk[1] += wd == 1 ? inc : 0u;
      pk[2] += wd == 2 ? inc : 0u;
    }
    // 10-bit fields (a chunk count is at most 256), three kinds per word; row sums
    u32 f[6];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      f[2 * i] = (pk[i] & 31u) | ((pk[i] >> 5) & 31u) << 10 | ((pk[i] >> 10) & 31u) << 20;
      f[2 * i + 1] = ((pk[i] >> 15) & 31u) | ((pk[i] >> 20) & 31u) << 10 | ((pk[i] >> 25) & 31u) << 20;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      u32 v = f[i];
      v += dpp_u32<0x111, 0xf>(v);  // row_shr:1
      v += dpp_u32<0x112, 0xf>(v);  // row_shr:2
      v += dpp_u32<0x114, 0xf>(v);  // row_shr:4
      v += dpp_u32<0x118, 0xf>(v);  // row_shr:8
      f[i] = v;
    }
    if (q == 15) {
#pragma unroll
      for (int k = 0; k < SMX_N_KINDS; ++k) c[rd * CH_PER_BLOCK + j][k] = (f[k / 3] >> (10 * (k % 3))) & 1023u;
    }
  }
  bool lg = false;
#pragma unroll
  for (int rd = 0; rd < KH_R; ++rd) {
    if (atA[rd]) *atA[rd] = smpA[rd];
    if (atB[rd]) *atB[rd] = smpB[rd];
    lg |= (chkA[rd] && farA[rd] == smpA[rd]) || (chkB[rd] && farB[rd] == smpB[rd]);
  }
  // a sample equal to the one Dl chunks (one window capacity) later: that timestamp group
  // alone overflows a window (k_fpart's test, SMX_KHIST_LONG); published below, once per
  // block, and to the host by the one block whose atomic set it (thousands of waves
  // storing to the pinned flag over the bus slowed this kernel and its completion)
  if (__ballot(lg) && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(&lgb, 1u);
  if (__ballot(bad) && (threadIdx.x & (WAVE - 1)) == 0) {
    meta->bad_sym = 1;
    if (long_host) __hip_atomic_store(long_host + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (threadIdx.x == 0 && lgb &&
      (__hip_atomic_load(&meta->f_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & F_LONG) != F_LONG) {
    const u64 was = atomicOr((unsigned long long*)&meta->f_fail, F_LONG);
    if ((was & F_LONG) != F_LONG && long_host)
      __hip_atomic_store(long_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // column-major output: consecutive threads write consecutive chunks of one column;
  // the kinds present per branch (the scans skip the all-zero columns)
  u32 m0 = 0, m1 = 0;
  for (int i = threadIdx.x; i < CH_PER_BLOCK * KH_R * SMX_N_KINDS; i += KH_NT) {
    const int jj = i % (CH_PER_BLOCK * KH_R), k = i / (CH_PER_BLOCK * KH_R);
    const i64 gg = (i64)blockIdx.x * CH_PER_BLOCK * KH_R + jj;
    if (gg >= CA + CB) continue;
    const int sd = gg >= CA;
    const u32 v = c[jj][k];
    cnt[((i64)sd * SMX_N_KINDS + k) * CM + (sd ? gg - CA : gg)] = v;
    if (v) (sd ? m1 : m0) |= 1u << k;
  }
  m0 = wave_or_to_last(m0);
  m1 = wave_or_to_last(m1);
  if ((threadIdx.x & (WAVE - 1)) == WAVE - 1) {
    if (m0) atomicOr(&km[0], m0);
    if (m1) atomicOr(&km[1], m1);
  }
  __syncthreads();
  // published only when it adds bits (a stale read costs a redundant atomic): the
  // blocks would otherwise serialise on two words
  if (threadIdx.x < 2 && km[threadIdx.x]) {
    const u32 cur = __hip_atomic_load(&meta->kmask[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((cur | km[threadIdx.x]) != cur) atomicOr(&meta->kmask[threadIdx.x], km[threadIdx.x]);
  }
}

// k_khist as a persistent grid (KH_PERSIST): each block walks groups of CH_PER_BLOCK
// chunks with the next group's kind bytes loaded before the current group is counted,
// counts branch-free, and publishes the kinds present once at its end.
#ifndef KH_PERSIST
#define KH_PERSIST 0  // off: config 3 plan 0.134 -> 0.151 ms with it (profiles/r04_h/ab_c3.txt)
#endif
#define KH_BLOCKS_PER_CU 4
__device__ __forceinline__ void kh_load(const u8* __restrict__ kind, const u64* __restrict__ ts, i64 na, i64 nb,
                                        i64 bgap, i64 CA, i64 CB, i64 g, int q, u64* __restrict__ sA,
                                        u64* __restrict__ sB, uint4* w, int* nv_o) {
  const int side = g >= CA;
  const i64 cc = side ? g - CA : g;
  const i64 len = side ? nb : na;
  const i64 r0 = cc * CH + q * 16;
  const int nv = g < CA + CB ? (int)(len - r0 < 0 ? 0 : (len - r0 < 16 ? len - r0 : 16)) : 0;
  *nv_o = nv;
  const u8* src = kind + (side ? na + bgap : 0) + r0;
  if (g < CA + CB) {
    if (!side && q == 0) sA[cc] = ts[cc * CH];
    if (side && q == 15 && nv == 16) sB[cc] = ts[na + bgap + cc * CH + CH - 1];
  }
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (nv == 16 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    v = *reinterpret_cast<const uint4*>(src);
  } else {
    u32 x[4] = {0u, 0u, 0u, 0u};
    for (int y = 0; y < nv; ++y) x[y >> 2] |= (u32)src[y] << (8 * (y & 3));
    v = make_uint4(x[0], x[1], x[2], x[3]);
  }
  *w = v;
}
__global__ void __launch_bounds__(KH_NT) k_khist2(const u8* __restrict__ kind, const u64* __restrict__ ts,
                                                  i64 na, i64 nb, i64 bgap, i64 CM, u32* __restrict__ cnt,
                                                  u64* __restrict__ sA, u64* __restrict__ sB, ComposeMeta* meta,
                                                  u32* long_host) {
  __shared__ u32 c[CH_PER_BLOCK][SMX_N_KINDS];
  __shared__ u32 km[2];
  const i64 CA = SMX_CEIL_DIV(na, (i64)CH), CB = SMX_CEIL_DIV(nb, (i64)CH);
  const i64 ngrp = SMX_CEIL_DIV(CA + CB, (i64)CH_PER_BLOCK);
  const int j = threadIdx.x / 16, q = threadIdx.x % 16;
  if (threadIdx.x < 2) km[threadIdx.x] = 0;
  u32 m0 = 0, m1 = 0;
  bool bad = false;
  i64 blk = blockIdx.x;
  uint4 w;
  int nv = 0;
  if (blk < ngrp) kh_load(kind, ts, na, nb, bgap, CA, CB, blk * CH_PER_BLOCK + j, q, sA, sB, &w, &nv);
  for (; blk < ngrp; blk += gridDim.x) {
    const uint4 cw = w;
    const int cnv = nv;
    if (blk + gridDim.x < ngrp)  // the next group's bytes, in flight while this one is counted
      kh_load(kind, ts, na, nb, bgap, CA, CB, (blk + gridDim.x) * CH_PER_BLOCK + j, q, sA, sB, &w, &nv);
    const u32 ww[4] = {cw.x, cw.y, cw.z, cw.w};
    u32 pk[3] = {0u, 0u, 0u};  // kind k: bits 5 * (k % 6) of word k / 6
#pragma unroll
    for (int y = 0; y < 16; ++y) {
      const bool ok = y < cnv;
      u32 k = (ww[y >> 2] >> (8 * (y & 3))) & 0xffu;
      bad |= ok & (k >= SMX_N_KINDS);
      k = k < SMX_N_KINDS ? k : SMX_N_KINDS - 1;
      const u32 wd = (k * 43u) >> 8;  // k / 6 for k < 18
      const u32 inc = ok ? 1u << (5u * (k - 6u * wd)) : 0u;
      pk[0] += wd == 0 ? inc : 0u;
      pk[1] += wd == 1 ? inc : 0u;
      pk[2] += wd == 2 ? inc : 0u;
    }
    u32 f[6];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      f[2 * i] = (pk[i] & 31u) | ((pk[i] >> 5) & 31u) << 10 | ((pk[i] >> 10) & 31u) << 20;
      f[2 * i + 1] = ((pk[i] >> 15) & 31u) | ((pk[i] >> 20) & 31u) << 10 | ((pk[i] >> 25) & 31u) << 20;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      u32 v = f[i];
      v += dpp_u32<0x111, 0xf>(v);  // row_shr:1
      v += dpp_u32<0x112, 0xf>(v);  // row_shr:2
      v += dpp_u32<0x114, 0xf>(v);  // row_shr:4
      v += dpp_u32<0x118, 0xf>(v);  // row_shr:8
      f[i] = v;
    }
    if (q == 15) {
#pragma unroll
      for (int k = 0; k < SMX_N_KINDS; ++k) c[j][k] = (f[k / 3] >> (10 * (k % 3))) & 1023u;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < CH_PER_BLOCK * SMX_N_KINDS; i += KH_NT) {
      const int jj = i % CH_PER_BLOCK, k = i / CH_PER_BLOCK;
      const i64 gg = blk * CH_PER_BLOCK + jj;
      if (gg >= CA + CB) continue;
      const int sd = gg >= CA;
      const u32 v = c[jj][k];
      cnt[((i64)sd * SMX_N_KINDS + k) * CM + (sd ? gg - CA : gg)] = v;
      if (v) (sd ? m1 : m0) |= 1u << k;
    }
    __syncthreads();  // (c is rewritten by the next group)
  }
  if (__ballot(bad) && (threadIdx.x & (WAVE - 1)) == 0) {
    meta->bad_sym = 1;
    if (long_host) __hip_atomic_store(long_host + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  m0 = wave_or_to_last(m0);
  m1 = wave_or_to_last(m1);
  if ((threadIdx.x & (WAVE - 1)) == WAVE - 1) {
    if (m0) atomicOr(&km[0], m0);
    if (m1) atomicOr(&km[1], m1);
  }
  __syncthreads();
  if (threadIdx.x < 2 && km[threadIdx.x]) {
    const u32 cur = __hip_atomic_load(&meta->kmask[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((cur | km[threadIdx.x]) != cur) atomicOr(&meta->kmask[threadIdx.x], km[threadIdx.x]);
  }
}

__device__ __forceinline__ bool cs_present(const ComposeMeta* meta, int col) {
  return (meta->kmask[col >= SMX_N_KINDS] >> (col % SMX_N_KINDS)) & 1u;
}

// Exclusive scan of each (side, kind) column of chunk counts in three fully
// parallel phases over tiles of CS_TILE chunks: tile sums; scan of the tile sums
// (+ column totals into meta); tile scans.
#define CS_TILE (BLOCK * 8)

__global__ void __launch_bounds__(BLOCK) k_cscan_up(const u32* __restrict__ cnt, i64 na, i64 nb, i64 CM,
                                                    i64 NT, u32* __restrict__ tsum, const ComposeMeta* meta) {
  __shared__ u32 s[NWAVES + 1];
  const int col = blockIdx.y;
  if (!cs_present(meta, col) || (SMX_CSCAN_FAILCHK && meta->f_fail)) return;  // all-zero column: its prefixes are its counts
  const i64 C = SMX_CEIL_DIV(col >= SMX_N_KINDS ? nb : na, (i64)CH);
  const i64 t0 = (i64)blockIdx.x * CS_TILE;
  if (t0 >= C) return;
  const u32* colp = cnt + (i64)col * CM;
  const i64 b = t0 + (i64)threadIdx.x * 8;
  u32 acc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc += b + j < C ? colp[b + j] : 0u;
  u32 tot;
  block_excl_scan<OpSum, u32>(acc, s, &tot);
  if (threadIdx.x == 0) tsum[(i64)col * NT + blockIdx.x] = tot;
}

// The window count the plan's windows read (meta->n_win): nwin, or after an early
// F_LONG (k_khist) with the wide boundaries in place (nwin_long > 0, k_fpart's LongW) the
// wide plan's -- and F_LONG is cleared so the wide windows and the tail run.
__device__ __forceinline__ void set_n_win(ComposeMeta* meta, u64 nwin, u64 nwin_long) {
  if (nwin_long && meta->f_fail == F_LONG) {
    meta->f_fail = 0;
    nwin = nwin_long;
  }
  meta->n_win = nwin;
}

__global__ void __launch_bounds__(BLOCK) k_cscan_mid(u32* __restrict__ tsum, i64 na, i64 nb, i64 CM, i64 NT,
                                                     u32* __restrict__ cnt, ComposeMeta* meta, u64 nwin,
                                                     u64 nwin_long) {
  __shared__ u32 s[NWAVES + 1];
  const int col = blockIdx.x;
  if (SMX_CSCAN_FAILCHK && meta->f_fail) return;  // (k_khist saw a group no window holds)
  const int side = col / SMX_N_KINDS, k = col % SMX_N_KINDS;
  const i64 C = SMX_CEIL_DIV(side ? nb : na, (i64)CH);
  const i64 nt = cs_present(meta, col) ? SMX_CEIL_DIV(C, (i64)CS_TILE) : 0;  // (absent: total 0)
  u32 carry = 0;
  for (i64 r0 = 0; r0 < nt; r0 += BLOCK) {
    const i64 r = r0 + threadIdx.x;
    const u32 v = r < nt ? tsum[(i64)col * NT + r] : 0u;
    u32 tot;
    const u32 ex = block_excl_scan<OpSum, u32>(v, s, &tot);
    if (r < nt) tsum[(i64)col * NT + r] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    cnt[(i64)col * CM + C] = carry;  // prefix at the end of the branch (a window may start there)
    atomicAdd((unsigned long long*)&meta->kcnt[k], (unsigned long long)carry);
    if (k == KREN) meta->n_ren_side[side] = carry;
    // the last column's block: the T-order segment starts (k_bases), from every total
    __threadfence();
    if (atomicAdd((unsigned long long*)&meta->cs_done, 1ull) == (unsigned long long)gridDim.x - 1) {
      __threadfence();
      set_n_win(meta, nwin, nwin_long);
      u64 acc = 0;
      for (int kk = 0; kk < SMX_N_KINDS; ++kk) {
        meta->base[kk] = acc;
        acc += __hip_atomic_load(&meta->kcnt[kk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      meta->base[SMX_N_KINDS] = acc;
    }
  }
}

__global__ void __launch_bounds__(BLOCK) k_cscan_down(u32* __restrict__ cnt, i64 na, i64 nb, i64 CM, i64 NT,
                                                      const u32* __restrict__ tsum, const ComposeMeta* meta) {
  __shared__ u32 s[NWAVES + 1];
  const int col = blockIdx.y;
  if (!cs_present(meta, col) || (SMX_CSCAN_FAILCHK && meta->f_fail)) return;
  const i64 C = SMX_CEIL_DIV(col >= SMX_N_KINDS ? nb : na, (i64)CH);
  const i64 t0 = (i64)blockIdx.x * CS_TILE;
  if (t0 >= C) return;
  u32* colp = cnt + (i64)col * CM;
  const i64 b = t0 + (i64)threadIdx.x * 8;
  u32 v[8];
  u32 acc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = b + j < C ? colp[b + j] : 0u;
    acc += v[j];
  }
  u32 tot;
  u32 run = tsum[(i64)col * NT + blockIdx.x] + block_excl_scan<OpSum, u32>(acc, s, &tot);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (b + j < C) colp[b + j] = run;
    run += v[j];
  }
}

// Small merges (CM <= CS_SMALL_CM chunks per branch): each (side, kind) column scanned by
// one block in one launch (k_cscan_up / mid / down are three launch latencies); the
// totals and, in the last column's block, the T-order segment starts as in k_cscan_mid.
#ifndef CS_SMALL_CM
#define CS_SMALL_CM 16384
#endif
__device__ __forceinline__ void cscan_small_body(u32* __restrict__ cnt, i64 na, i64 nb, i64 CM, ComposeMeta* meta,
                                                 u64 nwin, int col, u32* s, u64 nwin_long = 0) {
  const int side = col / SMX_N_KINDS, k = col % SMX_N_KINDS;
  const i64 C = SMX_CEIL_DIV(side ? nb : na, (i64)CH);
  u32* colp = cnt + (i64)col * CM;
  u32 carry = 0;
  if (cs_present(meta, col)) {  // (an absent column's prefixes are its zero counts)
    for (i64 t0 = 0; t0 < C; t0 += CS_TILE) {
      const i64 b = t0 + (i64)threadIdx.x * 8;
      u32 v[8];
      u32 acc = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = b + j < C ? colp[b + j] : 0u;
        acc += v[j];
      }
      u32 tot;
      u32 run = carry + block_excl_scan<OpSum, u32>(acc, s, &tot);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (b + j < C) colp[b + j] = run;
        run += v[j];
      }
      carry += tot;
    }
  }
  if (threadIdx.x == 0) {
    colp[C] = carry;  // prefix at the end of the branch (a window may start there)
    atomicAdd((unsigned long long*)&meta->kcnt[k], (unsigned long long)carry);
    if (k == KREN) meta->n_ren_side[side] = carry;
    __threadfence();
    if (atomicAdd((unsigned long long*)&meta->cs_done, 1ull) == (unsigned long long)(2 * SMX_N_KINDS - 1)) {
      __threadfence();
      set_n_win(meta, nwin, nwin_long);
      u64 acc = 0;
      for (int kk = 0; kk < SMX_N_KINDS; ++kk) {
        meta->base[kk] = acc;
        acc += __hip_atomic_load(&meta->kcnt[kk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      meta->base[SMX_N_KINDS] = acc;
    }
  }
}
#ifndef SMX_FPART_CS
#define SMX_FPART_CS 1  // small merges: k_fpart and k_cscan_small in one launch
#endif
__global__ void __launch_bounds__(BLOCK) k_cscan_small(u32* __restrict__ cnt, i64 na, i64 nb, i64 CM,
                                                       ComposeMeta* meta, u64 nwin, u64 nwin_long) {
  __shared__ u32 s[NWAVES + 1];
  cscan_small_body(cnt, na, nb, CM, meta, nwin, blockIdx.x, s, nwin_long);
}
// Small merges (launch-bound): k_fpart and k_cscan_small are independent (both read
// only k_khist's outputs), so one launch runs both: the first nfp blocks are k_fpart's,
// the last 2 * SMX_N_KINDS k_cscan_small's columns.
__global__ void __launch_bounds__(BLOCK) k_fpart_cscan(const u64* __restrict__ ts, const u64* __restrict__ tsB,
                                                       const u64* __restrict__ sA, const u64* __restrict__ sB, i64 na,
                                                       i64 nb, i64 W, i64 tgt, i64 D, i64* __restrict__ bnd,
                                                       ComposeMeta* meta, u32* long_host, u32* __restrict__ cnt,
                                                       i64 CM, i64 nfp) {
  __shared__ u32 s[NWAVES + 1];
  if ((i64)blockIdx.x < nfp) fpart_body(ts, tsB, sA, sB, na, nb, W, tgt, D, bnd, meta, long_host, blockIdx.x, nfp);
  else cscan_small_body(cnt, na, nb, CM, meta, (u64)W, (int)(blockIdx.x - nfp), s);
}

// Per-window counts: each kind and renames per branch (+ moves with a None value
// in the generic layout).  Column-major [c][W].
//  * presorted layout (perm == nullptr): branch position j is op j; only the kind
//    bytes are read, 16 per lane (the layout itself is verified by k_window_f);
//  * generic layout: through the sort permutation, one op per lane.
__device__ __forceinline__ void wc_add_one(u32 k, u32 (&c)[SMX_N_KINDS], bool& bad) {
  bad |= k >= SMX_N_KINDS;
#pragma unroll
  for (int kk = 0; kk < SMX_N_KINDS; ++kk) c[kk] += (k == (u32)kk);
}

__device__ __forceinline__ void wc_add_bytes(u32 x, u32 (&c)[SMX_N_KINDS], bool& bad) {
#pragma unroll
  for (int q = 0; q < 4; ++q) wc_add_one((x >> (8 * q)) & 0xffu, c, bad);
}

#ifndef WC_NT
#define WC_NT BLOCK  // threads per generic window in k_wcount
#endif
__global__ void __launch_bounds__(WC_NT) k_wcount(const u8* __restrict__ kind, const i32* __restrict__ v0,
                                                  const i32* __restrict__ v1, const u32* __restrict__ perm,
                                                  const i64* __restrict__ bnd, i64 na, i64 W,
                                                  u32* __restrict__ wcnt, ComposeMeta* meta) {
  __shared__ u32 c[NCNT];
  if (perm != nullptr && meta->f_fail) return;  // the segmented sort failed: perm is not written
  const i64 w = SMX_XCD_WIN ? xcd_item(blockIdx.x, W) : (i64)blockIdx.x;  // (the window's gathers stay in one L2)
  if (threadIdx.x < NCNT) c[threadIdx.x] = 0;
  __syncthreads();
  const i64 a0 = bnd[2 * w], b0 = bnd[2 * w + 1], a1 = bnd[2 * w + 2], b1 = bnd[2 * w + 3];
  bool bad = false;
  if (perm == nullptr) {
    for (int side = 0; side < 2; ++side) {
      const i64 off = side ? na : 0;
      const i64 lo = off + (side ? b0 : a0), hi = off + (side ? b1 : a1);
      if (hi <= lo) continue;
      u32 cnt[SMX_N_KINDS];
#pragma unroll
      for (int kk = 0; kk < SMX_N_KINDS; ++kk) cnt[kk] = 0;
      const i64 alo = (lo + 15) & ~(i64)15, ahi = hi & ~(i64)15;
      if (alo >= ahi) {  // short range: bytes
        for (i64 j = lo + threadIdx.x; j < hi; j += WC_NT) wc_add_one(kind[j], cnt, bad);
      } else {
        for (i64 j = lo + threadIdx.x; j < alo; j += WC_NT) wc_add_one(kind[j], cnt, bad);
        for (i64 j = ahi + threadIdx.x; j < hi; j += WC_NT) wc_add_one(kind[j], cnt, bad);
        const uint4* v = (const uint4*)(kind + alo);
        for (i64 q = threadIdx.x; q < (ahi - alo) / 16; q += WC_NT) {
          const uint4 x = v[q];
          wc_add_bytes(x.x, cnt, bad);
          wc_add_bytes(x.y, cnt, bad);
          wc_add_bytes(x.z, cnt, bad);
          wc_add_bytes(x.w, cnt, bad);
        }
      }
#pragma unroll
      for (int kk = 0; kk < SMX_N_KINDS; ++kk) {
        const u32 tot = wave_incl_sum(cnt[kk]);
        if ((threadIdx.x & (WAVE - 1)) == WAVE - 1 && tot) {
          atomicAdd(&c[kk], tot);
          if (kk == KREN) atomicAdd(&c[CNT_REN_A + side], tot);
        }
      }
    }
  } else {
    // a window holds at most WG_CAP ops: WC_ITEMS per thread, every load issued before
    // any is used (the perm -> kind -> value chain is one round trip per level, not one
    // per item); the item count is fixed, so the ballots stay wave-uniform
    constexpr int WC_ITEMS = (WG_CAP + WC_NT - 1) / WC_NT;
    const u64 lt = lanemask_lt();
    const i64 nA = a1 - a0, nW = nA + (b1 - b0);
    u32 src[WC_ITEMS], kv[WC_ITEMS];
    i32 x0[WC_ITEMS], x1[WC_ITEMS];
    bool val[WC_ITEMS], sd[WC_ITEMS];
#pragma unroll
    for (int i = 0; i < WC_ITEMS; ++i) {
      const i64 e = (i64)i * WC_NT + threadIdx.x;
      val[i] = e < nW && e < WG_CAP;
      sd[i] = e >= nA;
      src[i] = val[i] ? perm[sd[i] ? na + b0 + (e - nA) : a0 + e] : 0u;
    }
#pragma unroll
    for (int i = 0; i < WC_ITEMS; ++i) kv[i] = kind[src[i]];
#pragma unroll
    for (int i = 0; i < WC_ITEMS; ++i) {  // the values of the moves only
      const bool mv = val[i] && kv[i] == KMOVE;
      x0[i] = mv ? v0[src[i]] : 0;
      x1[i] = mv ? v1[src[i]] : 0;
    }
#pragma unroll
    for (int i = 0; i < WC_ITEMS; ++i) {
      u32 k = 0;
      bool none_mv = false;
      if (val[i]) {
        bad |= kv[i] >= SMX_N_KINDS;
        k = kv[i] < SMX_N_KINDS ? kv[i] : SMX_N_KINDS - 1;
        none_mv = k == KMOVE && (x0[i] < 0 || x1[i] < 0);
      }
      const u64 peers = wave_peers<5>(k, val[i]);
      if (val[i] && (peers & lt) == 0) atomicAdd(&c[k], (u32)__popcll(peers));
      const u64 nm = __ballot(none_mv);
      if (nm && (threadIdx.x & (WAVE - 1)) == 0) atomicAdd(&c[CNT_NONE_MV], (u32)__popcll(nm));
      // renames per branch (a wave may straddle the A/B boundary: split the peers)
      if (val[i] && k == KREN) {
        const u64 sb = __ballot(sd[i]);
        const u64 mine = peers & (sd[i] ? sb : ~sb);
        if ((mine & lt) == 0) atomicAdd(&c[CNT_REN_A + (sd[i] ? 1 : 0)], (u32)__popcll(mine));
      }
    }
    if (nW > WG_CAP) bad = true;  // cannot happen: k_gpart cuts windows of at most WG_CAP ops
  }
  if (bad) meta->bad_sym = 1;
  __syncthreads();
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

// T bases: exclusive prefix of the kind totals; the plan's window count.
__global__ void k_bases(ComposeMeta* meta, u64 nwin) {
  meta->n_win = nwin;
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

// Two columns gathered through one read of the permutation.
__global__ void k_gather2(const u64* __restrict__ a, const u64* __restrict__ b, const u32* __restrict__ idx,
                          u64* __restrict__ aout, u64* __restrict__ bout, i64 n) {
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (i64)gridDim.x * BLOCK) {
    const u32 j = idx[i];
    aout[i] = a[j];
    bout[i] = b[j];
  }
}

__global__ void k_offset(u32* __restrict__ v, i64 n, u32 off) {
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (i64)gridDim.x * BLOCK) v[i] += off;
}

#include "smx_walk.h"

// ---------------------------------------------------------------------------
// kernels: output of the renames and the other kinds; None-value moves

struct EmitArgs {
  const i32* tsrc;     // P = T - nMv: local source op (renames first, then the rest)
  const u32* tsym;
  const u64* skipbits; // renames skipped by the walk
  const u32* skiplist; // ... as a sorted list
  const int4* fin;
  const ComposeMeta* meta;
  u64 n;
  u32 smax;
  int allow_pack;  // the final-state table came from k_tb_reduce (packs when widths fit)
  u64 na_loc;      // local op j -> global j < na_loc ? src_a + j : src_b + j - na_loc
  i64 src_a, src_b;
  const i32* src_map;  // or, for a sample-sorted shard, src_map[j]
  i32* out_order;
  i32* out_addr;
  i32* out_file;
  i32* out_ctx;
  i64* counts;
  int status_none;  // report pending None-value moves (single merge) in counts[0]
  u64* hrec;        // or null: the synchronous call's verdict word (EarlyVerdict)
  u64 hseq;
};

#ifndef SMX_EMIT_NT
#define SMX_EMIT_NT 1
#endif
#ifndef SMX_EMIT_NTST
#define SMX_EMIT_NTST 1
#endif
// Streams read once and outputs written once: non-temporal, so that they do not evict
// the gathered final-state table from L2 (k_emit4's aligned 16-byte stores; plain ones
// measured emit 0.753 -> 0.821 ms on config 3, profiles/r06/ab_c3_emit_stores.txt).  A
// wave's outputs are an aligned range, so no line is shared between waves; the partial
// stores at the range's ends are plain (round 2 measured non-temporal partial-line
// stores 1.4-1.8x slower than plain ones, when ranges were not aligned).
#if SMX_EMIT_NT
#define NTLD(p) __builtin_nontemporal_load(p)
#else
#define NTLD(p) (*(p))
#endif
#if SMX_EMIT_NTST
#define NTST(v, p) __builtin_nontemporal_store((v), (p))
#else
#define NTST(v, p) (*(p) = (v))
#endif
#ifndef SMX_EMIT_NOGATHER
#define SMX_EMIT_NOGATHER 0
#endif
#ifndef EMIT_WT
#define EMIT_WT 1024  // positions per wave (2048: emit 0.753 -> 0.749 ms, within noise, profiles/r06/ab_c3_emit_stores.txt)
#endif
#ifndef EMIT_B
#define EMIT_B 8      // wave steps whose loads are issued together
#endif
static_assert(EMIT_WT % (WAVE * EMIT_B) == 0, "a wave's output range is whole batches of steps");

// Every op after the move block (the moves' records came from the window
// kernel).  Each wave owns EMIT_WT consecutive OUTPUT indices (aligned: no output
// line is shared between waves); output o holds the op at position
//   renames  P = o' + #{skips j : S[j] - j <= o'}   (o' = o - nMv, S = sorted skip list)
//   others   P = o' + nskip                          (every skip is a rename)
// found by one binary search per wave and a scalar walk over the (few) skips of
// each 64-output step.  Renames see their symbol's final move state, the rest
// also its last rename (compose.py:30-49).  Block 0 writes the call's counts.
#ifdef EMIT_WPE
#define EMIT_BOUNDS __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(EMIT_WPE, EMIT_WPE)))
#else
#define EMIT_BOUNDS __launch_bounds__(BLOCK)
#endif
__global__ void EMIT_BOUNDS k_emit(EmitArgs E) {
  const ComposeMeta* M = E.meta;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // -1 invalid input (sym >= n_sym or kind >= 18); -2 the plan failed, -3 moves
    // with a None value still need their prefix fix-up (smx_compose_finish)
    const bool bad = M->bad_sym != 0;
    E.counts[0] = bad ? -1 : M->f_fail ? -2 : (M->n_move_none && E.status_none) ? -3 : (i64)(E.n - M->n_skip);
    E.counts[1] = bad ? -1 : (i64)M->n_conf;
    // seq << 1 | 1: smx_compose_finish has work left (or an error) and reads the meta
    if (E.hrec) *E.hrec = E.hseq << 1 | ((bad || M->f_fail || (M->n_move_none && M->kcnt[KMOVE])) ? 1u : 0u);
  }
  if (M->f_fail | M->bad_sym) return;
  const u64 nskip = M->n_skip;
  const u64 nmv = min(M->kcnt[KMOVE], E.n);
  const u64 nP = E.n - nmv;
  const u64 nR = min(M->kcnt[KREN], nP);
  const u64 nout = E.n - nskip, nRk = nR - nskip;
  auto gsrc = [&](i32 j) -> i32 {
    if (E.src_map) return E.src_map[j];
    return (u64)j < E.na_loc ? (i32)(E.src_a + j) : (i32)(E.src_b + ((i64)j - (i64)E.na_loc));
  };
  const FinPack FP = fin_pack_of(M->vbits, E.allow_pack != 0);
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 w0 = (((u64)blockIdx.x * BLOCK + threadIdx.x) / WAVE) * EMIT_WT;  // output index
  if (w0 + EMIT_WT <= nmv || w0 >= nout || nP == 0) return;
  u64 kk = 0;  // skips with S[j] - j below the next step's first rename output
  {
    const u64 o0 = w0 > nmv ? w0 - nmv : 0;
    if (o0 < nRk) {
      u64 lo = 0, hi = nskip;
      while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if ((u64)E.skiplist[mid] - mid < o0) lo = mid + 1;
        else hi = mid;
      }
      kk = lo;
    }
  }
  for (int bt = 0; bt < EMIT_WT / (WAVE * EMIT_B); ++bt) {
    const u64 ob = w0 + (u64)bt * WAVE * EMIT_B;
    if (ob >= nout) break;
    u64 pp[EMIT_B];
#pragma unroll
    for (int j = 0; j < EMIT_B; ++j) {
      const u64 b = ob + (u64)j * WAVE;  // the step's first output (wave-uniform)
      const u64 o = b + lane;
      const u64 op = o >= nmv ? o - nmv : 0;
      const u64 k0 = kk;
      u64 add = 0;
      if (b + WAVE > nmv && (b > nmv ? b - nmv : 0) < nRk) {
        // rename outputs in this step (o' up to b + 63 - nMv): the skips at or below o'
        const u64 ohi = b + WAVE - 1 - nmv;
        while (kk < nskip) {
          const u64 sj = (u64)(u32)__builtin_amdgcn_readfirstlane((int)E.skiplist[kk]) - kk;
          if (sj > ohi) break;
          add += op >= sj;
          ++kk;
        }
      }
      const bool ok = o >= nmv && o < nout;
      pp[j] = !ok ? 0 : (op < nRk ? op + k0 + add : op + nskip);
    }
    i32 src[EMIT_B];
    u32 sy[EMIT_B];
#pragma unroll
    for (int j = 0; j < EMIT_B; ++j) {
      src[j] = NTLD(&E.tsrc[pp[j]]);
      sy[j] = min(NTLD(&E.tsym[pp[j]]), E.smax);
    }
    int4 F[EMIT_B];
    if (SMX_EMIT_NOGATHER) {  // diagnostics only: the stream without the table lookups
#pragma unroll
      for (int j = 0; j < EMIT_B; ++j) F[j] = make_int4((int)sy[j], 0, 0, 0);
    } else if (FP.packed) {
      u64 x[EMIT_B];
#pragma unroll
      for (int j = 0; j < EMIT_B; ++j) x[j] = fin_word(FP, E.fin, sy[j]);
#pragma unroll
      for (int j = 0; j < EMIT_B; ++j) F[j] = fin_decode(FP, x[j]);
    } else {
#pragma unroll
      for (int j = 0; j < EMIT_B; ++j) F[j] = E.fin[sy[j]];
    }
#pragma unroll
    for (int j = 0; j < EMIT_B; ++j) {
      const u64 o = ob + (u64)j * WAVE + lane;
      if (o >= nmv && o < nout) {
        const bool ren = o - nmv < nRk;
        NTST(gsrc(src[j]), &E.out_order[o]);
        NTST(F[j].x, &E.out_addr[o]);
        NTST(F[j].y, &E.out_file[o]);
        NTST(ren ? -1 : F[j].z, &E.out_ctx[o]);
      }
    }
  }
}

// k_emit with four consecutive outputs per lane: the streams move 16 bytes per lane
// and instruction (the per-lane address work of the texture path is what bounds this
// kernel: a fully divergent 64-lane table gather costs the CU ~150 cycles, a coalesced
// 4-byte stream instruction about as many per byte as a 16-byte one per four).  Each
// wave owns EMIT_WT consecutive output indices; a step is 256 outputs.  Four outputs
// of a lane read four consecutive positions P unless a skipped rename falls between
// them (rare): then each is read on its own.
#ifndef EMIT_VEC
#define EMIT_VEC 1
#endif
#define EMIT4_STEPS (EMIT_WT / (4 * WAVE))
typedef u32 ev4u __attribute__((ext_vector_type(4)));
typedef i32 ev4i __attribute__((ext_vector_type(4)));
typedef ev4u __attribute__((aligned(4))) ev4u_a4;
__global__ void EMIT_BOUNDS k_emit4(EmitArgs E) {
  const ComposeMeta* M = E.meta;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const bool bad = M->bad_sym != 0;
    E.counts[0] = bad ? -1 : M->f_fail ? -2 : (M->n_move_none && E.status_none) ? -3 : (i64)(E.n - M->n_skip);
    E.counts[1] = bad ? -1 : (i64)M->n_conf;
    // seq << 1 | 1: smx_compose_finish has work left (or an error) and reads the meta
    if (E.hrec) *E.hrec = E.hseq << 1 | ((bad || M->f_fail || (M->n_move_none && M->kcnt[KMOVE])) ? 1u : 0u);
  }
  if (M->f_fail | M->bad_sym) return;
  const u64 nskip = M->n_skip;
  const u64 nmv = min(M->kcnt[KMOVE], E.n);
  const u64 nP = E.n - nmv;
  const u64 nR = min(M->kcnt[KREN], nP);
  const u64 nout = E.n - nskip, nRk = nR - nskip;
  auto gsrc = [&](i32 j) -> i32 {
    if (E.src_map) return E.src_map[j];
    return (u64)j < E.na_loc ? (i32)(E.src_a + j) : (i32)(E.src_b + ((i64)j - (i64)E.na_loc));
  };
  const FinPack FP = fin_pack_of(M->vbits, E.allow_pack != 0);
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 w0 = (((u64)blockIdx.x * BLOCK + threadIdx.x) / WAVE) * EMIT_WT;  // output index
  if (w0 + EMIT_WT <= nmv || w0 >= nout || nP == 0) return;
  u64 kk = 0;  // skips with S[j] - j below the next step's first rename output
  {
    const u64 o0 = w0 > nmv ? w0 - nmv : 0;
    if (o0 < nRk) {
      u64 lo = 0, hi = nskip;
      while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if ((u64)E.skiplist[mid] - mid < o0) lo = mid + 1;
        else hi = mid;
      }
      kk = lo;
    }
  }
  u64 pp[EMIT4_STEPS][4];
  bool vec[EMIT4_STEPS];
#pragma unroll
  for (int j = 0; j < EMIT4_STEPS; ++j) {
    const u64 b = w0 + (u64)j * 4 * WAVE;  // the step's first output (wave-uniform)
    const u64 o = b + 4 * (u64)lane;
    u64 add[4] = {0, 0, 0, 0};
    const u64 k0 = kk;
    if (b + 4 * WAVE > nmv && (b > nmv ? b - nmv : 0) < nRk) {
      const u64 ohi = b + 4 * WAVE - 1 - nmv;
      while (kk < nskip) {
        const u64 sj = (u64)(u32)__builtin_amdgcn_readfirstlane((int)E.skiplist[kk]) - kk;
        if (sj > ohi) break;
#pragma unroll
        for (int u = 0; u < 4; ++u) add[u] += (o + u >= nmv ? o + u - nmv : 0) >= sj;
        ++kk;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const u64 ou = o + u;
      const u64 op = ou >= nmv ? ou - nmv : 0;
      const bool ok = ou >= nmv && ou < nout;
      pp[j][u] = !ok ? 0 : (op < nRk ? op + k0 + add[u] : op + nskip);
    }
    vec[j] = o >= nmv && o + 3 < nout && pp[j][3] == pp[j][0] + 3;
  }
  i32 src[EMIT4_STEPS][4];
  u32 sy[EMIT4_STEPS][4];
#pragma unroll
  for (int j = 0; j < EMIT4_STEPS; ++j) {
    if (vec[j]) {
      const ev4u s4 = __builtin_nontemporal_load(reinterpret_cast<const ev4u_a4*>(&E.tsrc[pp[j][0]]));
      const ev4u y4 = __builtin_nontemporal_load(reinterpret_cast<const ev4u_a4*>(&E.tsym[pp[j][0]]));
      src[j][0] = (i32)s4.x, src[j][1] = (i32)s4.y, src[j][2] = (i32)s4.z, src[j][3] = (i32)s4.w;
      sy[j][0] = y4.x, sy[j][1] = y4.y, sy[j][2] = y4.z, sy[j][3] = y4.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        src[j][u] = NTLD(&E.tsrc[pp[j][u]]);
        sy[j][u] = NTLD(&E.tsym[pp[j][u]]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) sy[j][u] = min(sy[j][u], E.smax);
  }
#pragma unroll
  for (int j = 0; j < EMIT4_STEPS; ++j) {
    int4 F[4];
    if (FP.packed) {
      u64 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = fin_word(FP, E.fin, sy[j][u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) F[u] = fin_decode(FP, x[u]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) F[u] = E.fin[sy[j][u]];
    }
    const u64 o = w0 + (u64)j * 4 * WAVE + 4 * (u64)lane;
    i32 vo[4], va[4], vf[4], vc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ren = o + u >= nmv && o + u - nmv < nRk;
      vo[u] = gsrc(src[j][u]);
      va[u] = F[u].x;
      vf[u] = F[u].y;
      vc[u] = ren ? -1 : F[u].z;
    }
    if (o >= nmv && o + 3 < nout) {  // o is a multiple of 4: 16-byte aligned stores
      NTST((ev4i{vo[0], vo[1], vo[2], vo[3]}), reinterpret_cast<ev4i*>(&E.out_order[o]));
      NTST((ev4i{va[0], va[1], va[2], va[3]}), reinterpret_cast<ev4i*>(&E.out_addr[o]));
      NTST((ev4i{vf[0], vf[1], vf[2], vf[3]}), reinterpret_cast<ev4i*>(&E.out_file[o]));
      NTST((ev4i{vc[0], vc[1], vc[2], vc[3]}), reinterpret_cast<ev4i*>(&E.out_ctx[o]));
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (o + u >= nmv && o + u < nout) {
          E.out_order[o + u] = vo[u];
          E.out_addr[o + u] = va[u];
          E.out_file[o + u] = vf[u];
          E.out_ctx[o + u] = vc[u];
        }
      }
    }
  }
}

// Moves whose newAddress or newFile is None see the symbol's inclusive prefix
// (compose.py:73-82 + 37-41): moves grouped by symbol in T order, last-non-None
// scan over the moves' own values (out_addr / out_file with msym's has-value bits);
// the composed output index of move T is T.
// Sharded merge: mvpre[2][n_sym] = the symbol's last non-None (addr, file) on the
// lower shards, as (shard + 1) << 32 | (value + 1), 0 = none.
__global__ void k_mv_init(const u32* __restrict__ msym, u64 nMv, u64* __restrict__ keys, u32* __restrict__ vals) {
  for (u64 j = (u64)blockIdx.x * BLOCK + threadIdx.x; j < nMv; j += (u64)gridDim.x * BLOCK) {
    keys[j] = msym[j] & SYM_MASK;
    vals[j] = (u32)j;
  }
}

__global__ void k_mv_fix(const u64* __restrict__ keys, const u32* __restrict__ vals, u64 nMv,
                         const u32* __restrict__ msym, const u64* __restrict__ mvpre, u64 n_sym,
                         i32* __restrict__ out_addr, i32* __restrict__ out_file) {
  for (u64 j = (u64)blockIdx.x * BLOCK + threadIdx.x; j < nMv; j += (u64)gridDim.x * BLOCK) {
    if (j != 0 && keys[j - 1] == keys[j]) continue;
    i32 ra = -1, rf = -1;
    if (mvpre && keys[j] < n_sym) {
      const u64 pa = mvpre[keys[j]], pf = mvpre[n_sym + keys[j]];
      if (pa) ra = (i32)(u32)pa - 1;
      if (pf) rf = (i32)(u32)pf - 1;
    }
    for (u64 i = j; i < nMv && keys[i] == keys[j]; ++i) {
      const u32 T = vals[i];
      const u32 f = msym[T];
      if (f & MS_HAS_A) ra = out_addr[T];
      else out_addr[T] = ra;
      if (f & MS_HAS_F) rf = out_file[T];
      else out_file[T] = rf;
    }
  }
}

// ---------------------------------------------------------------------------
// workspace layout

struct Layout {
  size_t off[64];
  size_t total;
};

enum Buf {
  B_META, B_BND, B_WCNT, B_WOFF, B_STS, B_SHI, B_SLO, B_PERM, B_RKEY, B_RVAL, B_RK2, B_RV2,
  B_RHIST, B_PART, B_MSYM, B_TSRC, B_TSYM, B_RSTR, B_WREN, B_WBND, B_CSLOT, B_WCAND, B_WCANDB,
  B_WCOFF, B_CAND, B_Q, B_PM, B_NCONF, B_NREAL, B_COFF, B_SKIPBITS, B_SKIPLIST,
  B_TABA, B_TABF, B_TABR, B_FIN, B_REC, B_TBHIST, B_CCNT, B_TSUM, B_SMP, B_N
};

static i64 max_windows(i64 nn) { return SMX_CEIL_DIV(nn, (i64)WIN_TGT_MIN) + 2; }

static Layout layout(i64 na, i64 nb, i64 n_sym) {
  const i64 n = na + nb;
  const i64 nn = n > 0 ? n : 1;
  const i64 W = max_windows(nn);
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
  sz[B_RHIST] = radix_hist_bytes(nn);
  sz[B_PART] = (size_t)SCAN_NB * 8;
  sz[B_MSYM] = sz[B_TSRC] = sz[B_TSYM] = sz[B_RSTR] = (size_t)nn * 4;
  sz[B_WREN] = (size_t)W * 2 * 4;
  sz[B_WBND] = sz[B_WCAND] = sz[B_WCANDB] = sz[B_WCOFF] = (size_t)W * 4;
  sz[B_CSLOT] = sz[B_CAND] = sz[B_Q] = sz[B_PM] = sz[B_NCONF] = sz[B_NREAL] = sz[B_COFF] = (size_t)nn * 4;
  sz[B_SKIPBITS] = (size_t)(SMX_CEIL_DIV(nn, (i64)64) + 1) * 8;
  sz[B_SKIPLIST] = (size_t)nn * 4;
  const i64 ns = n_sym > 0 ? n_sym : 1;
  sz[B_TABA] = sz[B_TABF] = sz[B_TABR] = (size_t)ns * 4;
  sz[B_FIN] = (size_t)ns * 16;
  sz[B_REC] = (size_t)nn * 4;
  sz[B_TBHIST] = (size_t)(TB_MAXBK + 1) * SMX_CEIL_DIV(nn, (i64)TB_TILE) * 4;  // k_tb_scatter's lst
  sz[B_CCNT] = (size_t)2 * SMX_N_KINDS * (SMX_CEIL_DIV(nn, (i64)256) + 2) * 4;
  sz[B_SMP] = (size_t)(SMX_CEIL_DIV(nn, (i64)CH) + 4) * 8;
  sz[B_TSUM] = (size_t)2 * SMX_N_KINDS * (SMX_CEIL_DIV(nn, (i64)CH * CS_TILE) + 2) * 4;
  Layout L{};
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

struct Ctx {
  const smx_ops* ops;
  const smx_compose_out* out;
  hipStream_t st;
  Layout L{};
  char* base;
  i64 na, nb, n, n_sym;
  i64 src_a, src_b;  // global source index of local op j (see WinArgs)
  StageTimer* tm;
  const i32* src_map = nullptr;
  u64* hrec = nullptr;  // the synchronous call's verdict word (k_emit stores it), or null
  u64 hseq = 0;
  template <typename T>
  T* ws(int b) const { return (T*)(base + L.off[b]); }
};

// Diagnostic builds only (tools/window_phases.py): a device buffer for k_window_f
// phase stamps.
#if SMX_DIAG
static void* g_phase_dbg = nullptr;
static size_t g_phase_dbg_bytes = 0;
extern "C" int smx_debug_phase_buffer(void* p, size_t bytes) {
  g_phase_dbg = p;
  g_phase_dbg_bytes = bytes;
  return SMX_OK;
}
#else
static constexpr void* g_phase_dbg = nullptr;
static constexpr size_t g_phase_dbg_bytes = 0;
#endif

static WinArgs win_args(const Ctx& C) {
  WinArgs P{};
  P.kind = C.ops->kind;
  P.sym = C.ops->sym;
  P.v0 = C.ops->v0;
  P.v1 = C.ops->v1;
  P.na = C.na;
  P.nb = C.nb;
  P.bgap = C.ops->b_gap;
  P.n_sym = C.n_sym;
  P.src_a = C.src_a;
  P.src_b = C.src_b;
  P.src_map = C.src_map;
  P.bnd = C.ws<i64>(B_BND);
  P.woff = C.ws<u32>(B_WOFF);
  P.meta = C.ws<ComposeMeta>(B_META);
  P.out_order = C.out->order;
  P.out_addr = C.out->addr;
  P.out_file = C.out->file;
  P.out_ctx = C.out->ctx;
  P.msym = C.ws<u32>(B_MSYM);
  P.tsrc = C.ws<i32>(B_TSRC);
  P.tsym = C.ws<u32>(B_TSYM);
  P.Rstr = C.ws<i32>(B_RSTR);
  P.wren = C.ws<u32>(B_WREN);
  P.wbnd = C.ws<u32>(B_WBND);
  P.cslot = C.ws<u32>(B_CSLOT);
  P.wcand = C.ws<u32>(B_WCAND);
  return P;
}

static WalkArgs walk_args(const Ctx& C, const smx_shard* sh) {
  WalkArgs Wk{};
  Wk.tsrc = C.ws<i32>(B_TSRC);
  Wk.tsym = C.ws<u32>(B_TSYM);
  Wk.v0 = C.ops->v0;
  Wk.wren = C.ws<u32>(B_WREN);
  Wk.wbnd = C.ws<u32>(B_WBND);
  Wk.meta = C.ws<ComposeMeta>(B_META);
  Wk.na_cap = (u64)C.na;
  Wk.nb_cap = (u64)C.nb;
  Wk.bgap = C.ops->b_gap;
  Wk.src_a = C.src_a;
  Wk.src_b = C.src_b;
  Wk.src_map = C.src_map;
  Wk.halo_dev = sh ? sh->halo_dev : nullptr;
  for (int b = 0; b < 2; ++b) {
    Wk.halo_sym[b] = sh ? sh->halo_sym[b] : nullptr;
    Wk.halo_cls[b] = sh ? sh->halo_cls[b] : nullptr;
    Wk.halo_src[b] = sh ? sh->halo_src[b] : nullptr;
    Wk.halo_n[b] = sh && sh->halo_sym[b] ? (u64)sh->halo_n[b] : 0;
    Wk.halo_more[b] = sh ? sh->halo_more[b] : 0;
  }
  // staging for k_replay_q's short regions: buffers of the sorting plans and of the
  // None-value move prefix, free while the walk runs
  Wk.stage = C.ws<u32>(B_RK2);
  Wk.sok = C.ws<u32>(B_RV2);
  Wk.stage_cap = RS_CONF ? (u64)(C.n > 0 ? C.n : 1) * 2 / (RS_CONF ? RS_W : 1) : 0;  // B_RK2: 8 bytes per op
  return Wk;
}

// DivergentRename walk (smx_walk.h): conflicts, skip bits, sorted skip list.
// Every size is read on the device from meta: no host sync.
#ifndef SMX_WALK_LB
#define SMX_WALK_LB 0  // 1: the one-block walk steps run in the last block of the grid before
                       // them; slower: config 2 walk 0.040 -> 0.056 ms (profiles/r05_wlb/ab_c2.txt),
                       // the device-scope fences of every block cost more than the launches
#endif
static int launch_walk(const Ctx& C, const smx_shard* sh) {
  hipStream_t st = C.st;
  ComposeMeta* meta = C.ws<ComposeMeta>(B_META);
  const i64 n = C.n;
  u64* skipbits = C.ws<u64>(B_SKIPBITS);
  u32* skiplist = C.ws<u32>(B_SKIPLIST);
  u32* part = C.ws<u32>(B_PART);
  const u64 nskipw = (u64)SMX_CEIL_DIV(n, (i64)64) + 1;  // (cleared by k_boundary)
  const WalkArgs Wk = walk_args(C, sh);
  u32* cslot = C.ws<u32>(B_CSLOT);
  u32* wcand = C.ws<u32>(B_WCAND);
  u32* wtot = C.ws<u32>(B_WCANDB);
  u32* wcoff = C.ws<u32>(B_WCOFF);
  u32* cand = C.ws<u32>(B_CAND);
  u32* q = C.ws<u32>(B_Q);
  u32* pm = C.ws<u32>(B_PM);
  u32* nconf = C.ws<u32>(B_NCONF);
  u32* nreal = C.ws<u32>(B_NREAL);
  u32* coff = C.ws<u32>(B_COFF);
  // u64 counters of meta: the scans write their u32 totals into the low word
  // (little endian) of the zeroed fields
  u32* nconf32 = (u32*)&meta->n_conf_loc;
  u32* ncand32 = (u32*)&meta->n_cand;
  const u64* ncand_dev = &meta->n_cand;
  const i64 Wmax = max_windows(n);
#ifndef WALK_GSMALL
#define WALK_GSMALL 256  // (64 and 1024 measured the same on configs 2 and 3: profiles/r06/ab_c3_walk_grid.txt)
#endif
  const int gsmall = WALK_GSMALL;  // grid for loops over the (few) candidates
  // small single merges: the one-block steps run in the last block of the grid before
  // them (k_boundary_cc, k_replay_q_cl), two launches fewer
  const bool lb_cc = SMX_WALK_LB && !sh && Wmax <= WALK_CC_FUSED_MAXW;
  const bool lb_cl = SMX_WALK_LB && !sh && n <= WALK_FUSED_MAXN;
  if (lb_cc)
    hipLaunchKernelGGL(k_boundary_cc, dim3(grid_for(Wmax)), dim3(BLOCK), 0, st, Wk, meta, cslot, wcand, wtot,
                       skipbits, nskipw, wcoff, (u64)Wmax, ncand32, cand);
  else
    hipLaunchKernelGGL(k_boundary, dim3(grid_for(Wmax)), dim3(BLOCK), 0, st, Wk, meta, cslot, wcand, wtot, skipbits,
                       nskipw);
  if (sh && (sh->in_d > 0 || sh->in_state_dev))
    hipLaunchKernelGGL(k_replay_in, dim3(1), dim3(1), 0, st, Wk, (int)sh->in_ahead, (u32)sh->in_d,
                       (const i64*)sh->in_state_dev, meta, C.out->conflicts, (u64)C.out->conflict_cap, skiplist,
                       skipbits);
  // (one k_scan1 block over the window counts measured slower on config 3: walk 0.165 ->
  // 0.185 ms, round 3; small merges are launch-bound: one block)
  if (lb_cc) {
    // (k_boundary_cc's last block did the scan and the compaction)
  } else if (Wmax <= WALK_CC_FUSED_MAXW) {
    hipLaunchKernelGGL(k_cand_scan_compact, dim3(1), dim3(S1_NT), 0, st, Wk, wtot, wcoff, (u64)Wmax, ncand32, cslot,
                       cand);
  } else {
    if (Wmax <= WALK_SCAN1_MAXW)
      hipLaunchKernelGGL(k_scan1<OpSum>, dim3(1), dim3(S1_NT), 0, st, wtot, wcoff, (const u64*)&meta->n_win,
                         (u64)Wmax, ncand32);
    else
      HIP_TRY((scan_excl<OpSum, u32, u32>(wtot, wcoff, Wmax, &meta->n_win, part, ncand32, st)));
    hipLaunchKernelGGL(k_cand_compact, dim3(grid_for(Wmax)), dim3(BLOCK), 0, st, Wk, cslot, wcoff, ncand_dev, cand);
  }
  if (lb_cl) {
    hipLaunchKernelGGL(k_replay_q_cl, dim3(gsmall), dim3(BLOCK), 0, st, Wk, cand, meta, q, nconf, pm, nreal, coff,
                       (u64)n, nconf32);
  } else if (n <= WALK_FUSED_MAXN) {  // small merges: max scan, clusters and sum scan in one block
    hipLaunchKernelGGL(k_replay_q, dim3(gsmall), dim3(BLOCK), 0, st, Wk, cand, meta, q, nconf);
    hipLaunchKernelGGL(k_cluster_fused, dim3(1), dim3(S1_NT), 0, st, Wk, cand, q, pm, nconf, meta, nreal, coff,
                       (u64)n, nconf32);
  } else {
    hipLaunchKernelGGL(k_replay_q, dim3(gsmall), dim3(BLOCK), 0, st, Wk, cand, meta, q, nconf);
    hipLaunchKernelGGL(k_scan1<OpMax>, dim3(1), dim3(S1_NT), 0, st, q, pm, ncand_dev, (u64)n, (u32*)nullptr);
    hipLaunchKernelGGL(k_cluster, dim3(gsmall), dim3(BLOCK), 0, st, Wk, cand, q, pm, nconf, meta, nreal);
    hipLaunchKernelGGL(k_scan1<OpSum>, dim3(1), dim3(S1_NT), 0, st, nreal, coff, ncand_dev, (u64)n, nconf32);
  }
  hipLaunchKernelGGL(k_replay_write, dim3(gsmall), dim3(BLOCK), 0, st, Wk, cand, nreal, coff, meta,
                     C.out->conflicts, (u64)C.out->conflict_cap, skiplist, skipbits);
  HIP_TRY(hipGetLastError());
  return SMX_OK;
}

static TbArgs tb_args(const Ctx& C) {
  TbArgs A{};
  A.msym = C.ws<u32>(B_MSYM);
  A.tsym = C.ws<u32>(B_TSYM);
  A.skipbits = C.ws<u64>(B_SKIPBITS);
  A.mv_addr = C.out->addr;
  A.mv_file = C.out->file;
  A.Rstr = C.ws<i32>(B_RSTR);
  A.meta = C.ws<ComposeMeta>(B_META);
  A.ncap = (u64)C.n;
  A.width = 1u;
  A.nbk = 1u;
  A.smax = (u32)(C.n_sym - 1);
  return A;
}

// Bucket geometry of the per-symbol tables: the bucketed path when it returns true.
static bool tb_geometry(const Ctx& C, u64* width_o, u64* nbk_o) {
  u64 width = SMX_CEIL_DIV((u64)C.n_sym, (u64)TB_NBK_TGT);
  if (width < 1) width = 1;
  if (width > TB_WIDTH) width = TB_WIDTH;
  *width_o = width;
  *nbk_o = SMX_CEIL_DIV((u64)C.n_sym, width);
  return *nbk_o <= TB_MAXBK;
}

// The table records bucketed with every rename kept (k_tb_scatter keep_skip): it needs
// only the window outputs, so it can run before or beside the walk; k_tb_unskip then
// applies the walk's skips.  No-op off the bucketed path.
static int launch_tb_prescatter(const Ctx& C) {
  u64 width, nbk;
  if (!tb_geometry(C, &width, &nbk)) return SMX_OK;
  TbArgs A = tb_args(C);
  A.width = (u32)width;
  A.nbk = (u32)nbk;
  A.keep_skip = 1u;
  hipLaunchKernelGGL(k_tb_scatter, dim3((int)SMX_CEIL_DIV((u64)C.n, (u64)TB_TILE)), dim3(TB_NT), 0, C.st, A,
                     C.ws<u32>(B_TBHIST), C.ws<u32>(B_REC));
  HIP_TRY(hipGetLastError());
  return SMX_OK;
}

// Per-symbol last writers.  part == nullptr: the final-state table fin (packed
// when the value widths allow); otherwise this shard's partial tables.  prescattered:
// launch_tb_prescatter already bucketed the records (then only the skips and the
// reduce run here).
static int launch_tables(const Ctx& C, void* part_tab, u32 tag, int tagbits, bool* bucketed,
                         bool prescattered = false) {
  hipStream_t st = C.st;
  const i64 n = C.n;
  int4* fin = C.ws<int4>(B_FIN);
  *bucketed = false;
  const i64 n_sym = C.n_sym;
  TbArgs A = tb_args(C);
  u64 width, nbk;
  if (tb_geometry(C, &width, &nbk)) {
    *bucketed = true;
    A.width = (u32)width;
    A.nbk = (u32)nbk;
    const int nblk = (int)SMX_CEIL_DIV((u64)n, (u64)TB_TILE);
    u32* lst = C.ws<u32>(B_TBHIST);
    u32* rec = C.ws<u32>(B_REC);
    if (prescattered) {
      A.keep_skip = 1u;
      hipLaunchKernelGGL(k_tb_unskip, dim3(1024), dim3(BLOCK), 0, st, A, lst, rec, C.ws<u32>(B_SKIPLIST));
    } else {
      hipLaunchKernelGGL(k_tb_scatter, dim3(nblk), dim3(TB_NT), 0, st, A, lst, rec);
    }
    hipLaunchKernelGGL(k_tb_reduce, dim3(nbk), dim3(TBR_NT), 0, st, A, lst, rec, n_sym, fin,
                       PartTab{part_tab, tag, tagbits, C.ws<ComposeMeta>(B_META)});
  } else {
    // very large symbol spaces: device-scope atomics on the packed keys
    u32* tabA = C.ws<u32>(B_TABA);
    u32* tabF = C.ws<u32>(B_TABF);
    u32* tabR = C.ws<u32>(B_TABR);
    int rc;
    if ((rc = zero_async(tabA, (size_t)n_sym * 4, st)) || (rc = zero_async(tabF, (size_t)n_sym * 4, st)) ||
        (rc = zero_async(tabR, (size_t)n_sym * 4, st)))
      return rc;
    hipLaunchKernelGGL(k_tab_atomic, dim3(grid_for(n)), dim3(BLOCK), 0, st, A, tabA, tabF, tabR);
    hipLaunchKernelGGL(k_finalize, dim3(grid_for(n_sym)), dim3(BLOCK), 0, st, A, tabA, tabF, tabR, n_sym, fin,
                       PartTab{part_tab, tag, tagbits, C.ws<ComposeMeta>(B_META)});
  }
  HIP_TRY(hipGetLastError());
  return SMX_OK;
}

static int launch_emit(const Ctx& C, bool packable, const smx_shard* sh) {
  hipStream_t st = C.st;
  ComposeMeta* meta = C.ws<ComposeMeta>(B_META);
  const i64 n = C.n;
  EmitArgs E{C.ws<i32>(B_TSRC), C.ws<u32>(B_TSYM), C.ws<u64>(B_SKIPBITS), C.ws<u32>(B_SKIPLIST),
             C.ws<int4>(B_FIN), meta, (u64)n, (u32)(C.n_sym - 1), packable ? 1 : 0, (u64)C.na, C.src_a,
             C.src_b, C.src_map, C.out->order, C.out->addr, C.out->file, C.out->ctx, C.out->counts, sh ? 0 : 1,
             sh ? nullptr : C.hrec, C.hseq};
  const i64 ewaves = SMX_CEIL_DIV(n, (i64)EMIT_WT);
  const bool al16 = ((uintptr_t)C.out->order | (uintptr_t)C.out->addr | (uintptr_t)C.out->file |
                     (uintptr_t)C.out->ctx) % 16 == 0;
  if (EMIT_VEC && al16)
    hipLaunchKernelGGL(k_emit4, dim3(SMX_CEIL_DIV(ewaves, (i64)NWAVES)), dim3(BLOCK), 0, st, E);
  else
    hipLaunchKernelGGL(k_emit, dim3(SMX_CEIL_DIV(ewaves, (i64)NWAVES)), dim3(BLOCK), 0, st, E);
  HIP_TRY(hipGetLastError());
  return SMX_OK;
}

// Diagnostic knobs (SMX_ABLATE, SMX_WIN_TGT, SMX_TB_SERIAL, SMX_SIDE_CUS) are read
// from the environment only in a diagnostic build (-DSMX_DIAG=1, tools/build_variants.sh);
// the release library always takes the compiled defaults, so no environment variable
// can change what smx_compose computes.
#if SMX_DIAG
static int knob(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
#else
static constexpr int knob(const char*, int dflt) { return dflt; }
#endif

// A second stream (and its fork/join events) for the table scatter, which runs beside
// the walk: the walk is a chain of small, latency-bound launches that leaves most of
// the chip idle.  One per (device, caller stream), created on first use, so that calls
// on distinct streams never share one (and a graph capture of one caller's stream
// pulls in only that caller's side stream).  `mu` is held from the fork record to the
// join wait: two threads that share a caller stream cannot interleave their records.
// The fork/join is by events, so it also works inside a HIP graph capture.
struct SideStream {
  std::mutex mu;
  int dev = -1;
  hipStream_t caller = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
#define SIDE_MAX 256  // distinct caller streams with a side stream; beyond: no overlap
static std::mutex g_side_mu;
static SideStream* g_side[SIDE_MAX];
static int g_nside = 0;

// *out = the side stream of (current device, caller), or nullptr when the table is
// full (the caller then runs the tables on its own stream).
static int side_stream(hipStream_t caller, SideStream** out) {
  *out = nullptr;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(g_side_mu);
  for (int i = 0; i < g_nside; ++i)
    if (g_side[i]->dev == dev && g_side[i]->caller == caller) {
      *out = g_side[i];
      return SMX_OK;
    }
  if (g_nside == SIDE_MAX) return SMX_OK;
  SideStream* S = new SideStream;
  S->dev = dev;
  S->caller = caller;
  // (the lowest stream priority for it measured the same, profiles/r02_k/side_prio_ab.txt)
  // SMX_SIDE_CUS = k > 0 (diagnostic builds): the side stream runs on the first k CUs
  // only (measured slower, profiles/r02_k/side_cumask_ab.txt)
  int ncu = 0;
  HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int k = knob("SMX_SIDE_CUS", 0);
  if (k > 0 && k < ncu) {
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    for (int i = 0; i < k; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    HIP_TRY(hipExtStreamCreateWithCUMask(&S->s, (uint32_t)mask.size(), mask.data()));
  } else {
    HIP_TRY(hipStreamCreateWithFlags(&S->s, hipStreamNonBlocking));
  }
  // (device-scope events: both streams are on this device.  A default event's record
  // also fences at system scope -- an L2 write-back the next kernel on the recording
  // stream waits behind: ~11 us before k_boundary and ~6 us before the reduce on config 3,
  // profiles/r06/c3_timeline_start.txt)
#ifndef SMX_SIDE_SYSFENCE
#define SMX_SIDE_SYSFENCE 0
#endif
  const unsigned evf = hipEventDisableTiming | (SMX_SIDE_SYSFENCE ? 0u : hipEventDisableSystemFence);
  HIP_TRY(hipEventCreateWithFlags(&S->fork, evf));
  HIP_TRY(hipEventCreateWithFlags(&S->join, evf));
  g_side[g_nside++] = S;
  *out = S;
  return SMX_OK;
}

#ifndef SMX_TB_OVERLAP
#define SMX_TB_OVERLAP 1
#endif
#ifndef SMX_TB_UNSKIP_MAXN
#define SMX_TB_UNSKIP_MAXN (1 << 22)  // up to: k_tb_reduce reads the skip bits; above: k_tb_unskip
#endif
#ifndef SMX_TB_OVERLAP_MIN
#define SMX_TB_OVERLAP_MIN (1 << 18)  // ops (config 2: 0.1746 -> 0.1724 ms with the overlap, profiles/r05_x/c2_overlap_ab.txt; graph replay makes the fork/join cheap)
#endif
// launch_tail forks the table scatter onto the side stream for this merge
static bool n_side_needed(const smx_ops* ops) {
  u64 width = SMX_CEIL_DIV((u64)ops->n_sym, (u64)TB_NBK_TGT);
  if (width < 1) width = 1;
  if (width > TB_WIDTH) width = TB_WIDTH;
  return SMX_TB_OVERLAP && SMX_CEIL_DIV((u64)ops->n_sym, width) <= TB_MAXBK &&
         ops->n_a + ops->n_b >= SMX_TB_OVERLAP_MIN;
}

// Walk, tables, emit of a single merge.  The bucketed tables' scatter keeps every
// rename and runs on the side stream while the walk runs; k_tb_unskip then kills
// the records of the renames the walk skipped (compose.py:60-70: a skipped rename
// never enters rename_chain) before the reduce.
static int launch_tail(const Ctx& C) {
  const i64 n_sym = C.n_sym;
  u64 width = SMX_CEIL_DIV((u64)n_sym, (u64)TB_NBK_TGT);
  if (width < 1) width = 1;
  if (width > TB_WIDTH) width = TB_WIDTH;
  const u64 nbk = SMX_CEIL_DIV((u64)n_sym, width);
  // the smallest merges are launch-bound: below SMX_TB_OVERLAP_MIN the fork/join costs more than the overlap saves
  SideStream* S = nullptr;
  if (SMX_TB_OVERLAP && nbk <= TB_MAXBK && C.n >= SMX_TB_OVERLAP_MIN && !knob("SMX_TB_SERIAL", 0)) {
    int rc = side_stream(C.st, &S);
    if (rc) return rc;
  }
  if (!S) {
    C.tm->begin(ST_WALK);
    int rc = launch_walk(C, nullptr);
    if (rc) return rc;
    C.tm->end(ST_WALK);
    C.tm->begin(ST_TABLES);
    bool bucketed = false;
    if ((rc = launch_tables(C, nullptr, 0, 0, &bucketed))) return rc;
    C.tm->end(ST_TABLES);
    C.tm->begin(ST_EMIT);
    if ((rc = launch_emit(C, bucketed, nullptr))) return rc;
    C.tm->end(ST_EMIT);
    return SMX_OK;
  }
  std::lock_guard<std::mutex> own(S->mu);  // fork record .. join wait
  int rc;
  hipStream_t st = C.st;
  TbArgs A = tb_args(C);
  A.width = (u32)width;
  A.nbk = (u32)nbk;
  // small merges: no k_tb_unskip launch, k_tb_reduce tests the skip bits of the renames
  A.keep_skip = C.n <= SMX_TB_UNSKIP_MAXN ? 2u : 1u;
  u32* lst = C.ws<u32>(B_TBHIST);
  u32* rec = C.ws<u32>(B_REC);
  const int nblk = (int)SMX_CEIL_DIV((u64)C.n, (u64)TB_TILE);
  HIP_TRY(hipEventRecord(S->fork, st));
  HIP_TRY(hipStreamWaitEvent(S->s, S->fork, 0));
  hipLaunchKernelGGL(k_tb_scatter, dim3(nblk), dim3(TB_NT), 0, S->s, A, lst, rec);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(S->join, S->s));
  C.tm->begin(ST_WALK);
  if ((rc = launch_walk(C, nullptr))) {
    (void)hipStreamWaitEvent(st, S->join, 0);  // never leave the side stream unjoined
    return rc;
  }
  C.tm->end(ST_WALK);
  HIP_TRY(hipStreamWaitEvent(st, S->join, 0));
  C.tm->begin(ST_TABLES);
  if (A.keep_skip == 1u)
    hipLaunchKernelGGL(k_tb_unskip, dim3(1024), dim3(BLOCK), 0, st, A, lst, rec, C.ws<u32>(B_SKIPLIST));
  hipLaunchKernelGGL(k_tb_reduce, dim3(nbk), dim3(TBR_NT), 0, st, A, lst, rec, n_sym, C.ws<int4>(B_FIN),
                     PartTab{nullptr, 0u, 0, nullptr});
  HIP_TRY(hipGetLastError());
  C.tm->end(ST_TABLES);
  C.tm->begin(ST_EMIT);
  if ((rc = launch_emit(C, true, nullptr))) return rc;
  C.tm->end(ST_EMIT);
  return SMX_OK;
}

// Presorted plan: branch logs with non-decreasing timestamps (what lift.ts
// emits).  Speculative: k_window_f verifies the layout and flags f_fail.

// early (optional, not inside a graph capture): k_khist raises early->flag[0] when a
// timestamp group is longer than a window (the normal windows cannot hold the log) and
// flag[1] on an invalid kind; early->ev is recorded right behind k_khist, so the host
// knows while k_fpart and the column scans run, and launches the windows that hold the
// groups (run_presorted's Deferred).  (Off the normal level, k_fpart raises flag[0] and
// the event follows it.)
struct EarlyFail {
  u32* flag_host = nullptr;
  u32* flag_dev = nullptr;
  hipEvent_t ev = nullptr;
};
// Presorted window sizes: small (merges up to WF_SMALL_MAXN ops, latency-bound: more,
// shorter windows per CU), normal, wide (timestamp groups no normal window holds).
enum WinLevel { WL_SMALL, WL_NORMAL, WL_WIDE };
static i64 level_cap(int lv) { return lv == WL_SMALL ? WF_SMALL_CAP : lv == WL_WIDE ? WF_WIDE_CAP : WF_CAP; }
// (SMX_FIRST_WIDE, diagnostic builds: start at the wide windows, so that SMX_ABLATE's
// phase exits reach the wide instance)
static int first_level(const Ctx& C) {
  if (knob("SMX_FIRST_WIDE", 0)) return WL_WIDE;
  return C.n <= WF_SMALL_MAXN ? WL_SMALL : WL_NORMAL;
}
static i64 first_tgt(const Ctx& C) {
  if (first_level(C) == WL_WIDE) return knob("SMX_WIN_TGT", WF_WIDE_CAP);
  return first_level(C) == WL_SMALL ? knob("SMX_WIN_TGT", WF_SMALL_TGT) : knob("SMX_WIN_TGT", WIN_TGT);
}

// The presorted windows over the boundaries k_fpart left (W windows).
static int launch_presorted_windows(const Ctx& C, i64 W, i64 CM, int level) {
  const bool wide = level == WL_WIDE;
  hipStream_t st = C.st;
  WinArgs P = win_args(C);
  P.cpre = C.ws<u32>(B_CCNT);
  P.CM = CM;
  P.kts = C.ops->ts;
  P.khi = C.ops->oid_hi;
  P.klo = C.ops->oid_lo;
  P.perm = nullptr;
  P.W = W;
  P.ablate = knob("SMX_ABLATE", 0);
  const int stage = wide ? ST_WINDOW_WIDE : ST_WINDOW;
  C.tm->begin(stage);
#if SMX_DIAG
  if (g_phase_dbg && !P.src_map && (size_t)W * WF_NSTAMP * 8 <= g_phase_dbg_bytes) {
    P.dbg = (u64*)g_phase_dbg;
    if (wide)
      hipLaunchKernelGGL((k_window_f<WF_WIDE_CAP, WF_WIDE_NT, true, false>), dim3(W), dim3(WF_WIDE_NT), 0, st, P);
    else
      hipLaunchKernelGGL((k_window_f<WF_CAP, WF_NT, true, false>), dim3(W), dim3(WF_NT), 0, st, P);
  } else
#endif
  if (wide) {
    if (P.src_map) hipLaunchKernelGGL((k_window_f<WF_WIDE_CAP, WF_WIDE_NT, false, true, WF_RUNS_WIDE>), dim3(W), dim3(WF_WIDE_NT), 0, st, P);
    else hipLaunchKernelGGL((k_window_f<WF_WIDE_CAP, WF_WIDE_NT, false, false, WF_RUNS_WIDE>), dim3(W), dim3(WF_WIDE_NT), 0, st, P);
  } else if (level == WL_SMALL) {
    if (P.src_map) hipLaunchKernelGGL((k_window_f<WF_SMALL_CAP, WF_SMALL_NT, false, true>), dim3(W), dim3(WF_SMALL_NT), 0, st, P);
    else hipLaunchKernelGGL((k_window_f<WF_SMALL_CAP, WF_SMALL_NT, false, false>), dim3(W), dim3(WF_SMALL_NT), 0, st, P);
  } else if (P.src_map) {
    hipLaunchKernelGGL((k_window_f<WF_CAP, WF_NT, false, true, WF_RUNS>), dim3(W), dim3(WF_NT), 0, st, P);
  } else {
    hipLaunchKernelGGL((k_window_f<WF_CAP, WF_NT, false, false, WF_RUNS>), dim3(W), dim3(WF_NT), 0, st, P);
  }
  HIP_TRY(hipGetLastError());
  C.tm->end(stage);
  return SMX_OK;
}



// wide: WF_WIDE_CAP-op windows on WF_WIDE_NT threads (one per CU) for logs whose
// equal-timestamp groups no WF_CAP window holds (config 5: 8192-op groups).
// With `early` at the normal level (the synchronous merge): k_khist makes the long-group
// test and early->ev is recorded behind it; k_fpart and the column scans are enqueued
// for either outcome (normal boundaries, or the wide plan's after F_LONG: LongW), and the
// windows are left to the caller (*defer), which launches the normal or the wide ones
// once the host has read the verdict.
struct Deferred {
  bool on = false;
  i64 W = 0, W_w = 0, CM = 0;
};
static int run_presorted(const Ctx& C, i64 tgt, const EarlyFail* early = nullptr, int level = WL_NORMAL,
                         Deferred* defer = nullptr) {
  hipStream_t st = C.st;
  ComposeMeta* meta = C.ws<ComposeMeta>(B_META);
  i64* bnd = C.ws<i64>(B_BND);
  C.tm->begin(ST_PLAN);
  static_assert(sizeof(ComposeMeta) % 4 == 0, "meta is zeroed by words");
  if (tgt < WIN_TGT_MIN) tgt = WIN_TGT_MIN;
  const i64 cap = level_cap(level);
  if (tgt > cap) tgt = cap;
  tgt -= tgt % CH;  // chunk-aligned diagonals (k_fpart's sampled first level)
  const i64 W = SMX_CEIL_DIV(C.n, tgt);
  const i64 CM = SMX_CEIL_DIV(C.na > C.nb ? C.na : C.nb, (i64)CH) + 1;
  // (a single-pass look-back column scan fused with k_fpart measured slower on config 3:
  // plan 0.133 -> 0.157 ms -- the blocks' tickets and status round trips, profiles/r06)
  const bool cs_small = CM <= CS_SMALL_CM;
  {
    const int rc = zero_async(meta, sizeof(ComposeMeta), st);
    if (rc) return rc;
  }
  const i64 nchunk = SMX_CEIL_DIV(C.na, (i64)CH) + SMX_CEIL_DIV(C.nb, (i64)CH);
  u32* ccnt = C.ws<u32>(B_CCNT);
  u64* sA = C.ws<u64>(B_SMP);
  u64* sB = sA + SMX_CEIL_DIV(C.na, (i64)CH) + 1;
  const bool lmode = early && defer && level == WL_NORMAL && !KH_PERSIST;
  LongW lw{};
  if (lmode) {
    lw.tgt_w = level_cap(WL_WIDE) - level_cap(WL_WIDE) % CH;  // (the first wide attempt of order_fallbacks)
    lw.W_w = SMX_CEIL_DIV(C.n, lw.tgt_w);
    lw.D_w = level_cap(WL_WIDE) / CH;
  }
  if (KH_PERSIST) {
    static int ncu_of[64] = {};  // CUs per device (a benign race: every writer stores the same)
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    int ncu = dev < 64 ? ncu_of[dev] : 0;
    if (ncu == 0) {
      HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      if (dev < 64) ncu_of[dev] = ncu;
    }
    const i64 ngrp = SMX_CEIL_DIV(nchunk, (i64)CH_PER_BLOCK);
    const i64 grid = ngrp < (i64)ncu * KH_BLOCKS_PER_CU ? ngrp : (i64)ncu * KH_BLOCKS_PER_CU;
    hipLaunchKernelGGL(k_khist2, dim3(grid > 0 ? grid : 1), dim3(KH_NT), 0, st, C.ops->kind, C.ops->ts, C.na, C.nb,
                       C.ops->b_gap, CM, ccnt, sA, sB, meta, early ? early->flag_dev : nullptr);
  } else {
    hipLaunchKernelGGL(k_khist, dim3(SMX_CEIL_DIV(nchunk, (i64)CH_PER_BLOCK * KH_R)), dim3(KH_NT), 0, st,
                       C.ops->kind, C.ops->ts, C.na, C.nb, C.ops->b_gap, CM, ccnt, sA, sB, meta,
                       early ? early->flag_dev : nullptr, lmode ? cap / CH : (i64)0);
  }
  if (lmode) HIP_TRY(hipEventRecord(early->ev, st));  // (k_khist's verdict)
  const i64 nfp = SMX_CEIL_DIV(W + 1, (i64)BLOCK);   // (>= the wide plan's W_w + 1 boundaries)
  const bool fused = SMX_FPART_CS && cs_small && !early;
  if (fused)
    hipLaunchKernelGGL(k_fpart_cscan, dim3(nfp + 2 * SMX_N_KINDS), dim3(BLOCK), 0, st, C.ops->ts,
                       C.ops->ts + C.na + C.ops->b_gap, sA, sB, C.na, C.nb, W, tgt, cap / CH, bnd, meta,
                       (u32*)nullptr, ccnt, CM, nfp);
  else
    hipLaunchKernelGGL(k_fpart, dim3(nfp), dim3(BLOCK), 0, st, C.ops->ts, C.ops->ts + C.na + C.ops->b_gap, sA, sB,
                       C.na, C.nb, W, tgt, cap / CH, bnd, meta, (early && !lmode) ? early->flag_dev : nullptr, lw);
  if (early && !lmode) HIP_TRY(hipEventRecord(early->ev, st));
  const u64 nwin_long = lmode ? (u64)lw.W_w : 0ull;
  if (fused) {
    // (k_fpart_cscan scanned the columns)
  } else if (cs_small) {
    hipLaunchKernelGGL(k_cscan_small, dim3(2 * SMX_N_KINDS), dim3(BLOCK), 0, st, ccnt, C.na, C.nb, CM, meta, (u64)W,
                       nwin_long);
  } else {
    const i64 NT = SMX_CEIL_DIV(CM, (i64)CS_TILE);
    u32* tsum = C.ws<u32>(B_TSUM);
    hipLaunchKernelGGL(k_cscan_up, dim3(NT, 2 * SMX_N_KINDS), dim3(BLOCK), 0, st, ccnt, C.na, C.nb, CM, NT, tsum,
                       meta);
    hipLaunchKernelGGL(k_cscan_mid, dim3(2 * SMX_N_KINDS), dim3(BLOCK), 0, st, tsum, C.na, C.nb, CM, NT, ccnt,
                       meta, (u64)W, nwin_long);
    hipLaunchKernelGGL(k_cscan_down, dim3(NT, 2 * SMX_N_KINDS), dim3(BLOCK), 0, st, ccnt, C.na, C.nb, CM, NT,
                       tsum, meta);
  }
  HIP_TRY(hipGetLastError());
  C.tm->end(ST_PLAN);
  if (lmode) {
    *defer = Deferred{true, W, lw.W_w, CM};
    return SMX_OK;
  }
  return launch_presorted_windows(C, W, CM, level);
}

// k_fpart's long-group verdict (f_fail == F_LONG) is given before any window runs, so
// the plan's chunk counts, prefixes and bases stand: only the boundaries and the windows
// are redone, at the wide capacity.
__global__ void k_plan_rearm(ComposeMeta* meta, u64 nwin) {
  if (meta->f_fail == F_LONG) meta->f_fail = 0;
  meta->n_win = nwin;
}
// (the chunk scans must write base[] and the prefixes even when k_fpart flagged F_LONG:
// with SMX_CSCAN_FAILCHK they would leave early and the wide windows read stale prefixes)
static_assert(!SMX_CSCAN_FAILCHK, "run_presorted_rewide reuses the failed plan's chunk prefixes and bases");
static int run_presorted_rewide(const Ctx& C, i64 tgt, int level = WL_WIDE) {
  hipStream_t st = C.st;
  ComposeMeta* meta = C.ws<ComposeMeta>(B_META);
  if (tgt < WIN_TGT_MIN) tgt = WIN_TGT_MIN;
  if (tgt > level_cap(level)) tgt = level_cap(level);
  tgt -= tgt % CH;
  const i64 W = SMX_CEIL_DIV(C.n, tgt);
  const i64 CM = SMX_CEIL_DIV(C.na > C.nb ? C.na : C.nb, (i64)CH) + 1;
  u64* sA = C.ws<u64>(B_SMP);
  u64* sB = sA + SMX_CEIL_DIV(C.na, (i64)CH) + 1;
  C.tm->begin(ST_PLAN);
  hipLaunchKernelGGL(k_plan_rearm, dim3(1), dim3(1), 0, st, meta, (u64)W);
  hipLaunchKernelGGL(k_fpart, dim3(SMX_CEIL_DIV(W + 1, (i64)BLOCK)), dim3(BLOCK), 0, st, C.ops->ts,
                     C.ops->ts + C.na + C.ops->b_gap, sA, sB, C.na, C.nb, W, tgt, level_cap(level) / CH,
                     C.ws<i64>(B_BND), meta, (u32*)nullptr, LongW{});
  HIP_TRY(hipGetLastError());
  C.tm->end(ST_PLAN);
  return launch_presorted_windows(C, W, CM, level);
}

// Generic plan: each branch sorted by (ts, oid_hi, oid_lo, index), then fixed windows
// over the sorted logs (k_window_g).  Used when the presorted plan fails.  Two ways to
// sort a branch:
//  * segmented (GEN_SEG): the branch's timestamps never decrease but its equal-timestamp
//    groups are too long for a presorted window (config 5) -- only each group needs
//    sorting, by oid.  Nominal tiles of SEG_H ops snap back to a group start, so each
//    tile holds whole groups (fewer than SEG_H + the longest group ops); a block sorts
//    its tile with a bitonic network on (group, top 38 bits of oid_hi, tile index), and
//    runs of equal (group, hi38) (rare; every duplicate id) are re-sorted exactly on
//    (oid_hi, oid_lo, index).  A group longer than SEG_CAP - SEG_H ops or a timestamp that decreases sets
//    meta->seg_over and the radix sort runs instead.
//  * radix (GEN_RADIX / GEN_RADIX_LO): stable LSD radix sort on (ts, oid_hi), checked
//    afterwards for adjacent (ts, oid_hi) duplicates, which rerun it with oid_lo.
#define SEG_CAP 8192
#define SEG_H 4096
#define SEG_NT 1024
enum { GEN_SEG, GEN_RADIX, GEN_RADIX_LO };

__global__ void k_dupcheck(const u64* __restrict__ sts, const u64* __restrict__ shi, i64 na, i64 n,
                           ComposeMeta* meta) {
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x + 1; i < n; i += (i64)gridDim.x * BLOCK)
    if (i != na && sts[i] == sts[i - 1] && shi[i] == shi[i - 1]) meta->dup_key = 1;
}

// One pass of the bitonic network over 8 keys per thread: the thread holds keys
// base | m << b (m = 0..7) and runs the stages whose partner bit is b + 2, b + 1, b
// (the top `nbits` of them), ascending where bit k of the index is clear.
__device__ __forceinline__ void seg_pass(u64 (&v)[8], u32 base, u32 b, u32 k, int top, int nbits) {
#pragma unroll
  for (int bit = 2; bit >= 0; --bit) {
    if (bit > top || bit <= top - nbits) continue;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if ((m >> bit) & 1) continue;
      const int m2 = m | (1 << bit);
      const bool asc = ((base | ((u32)m << b)) & k) == 0;
      const u64 x = v[m], y = v[m2];
      const bool sw = asc ? y < x : x < y;
      v[m] = sw ? y : x;
      v[m2] = sw ? x : y;
    }
  }
}

#ifndef SEG_BUCKET
#define SEG_BUCKET 1
#endif
#if SEG_BUCKET
// Interpolation buckets (the default): element x of group [gs, ge) goes to bucket
// (gs + (ge - gs) * hi32 / 2^32) / 2, i.e. two elements per bucket on random ids;
// buckets are ordered like (group, hi), a counting sort places them and each element
// ranks itself on the full key inside its bucket.  A bucket above SEG_BKMAX (ids that
// cluster) sends the tile to the bitonic network.  The key array is unpadded so that two
// blocks (64 KB keys + 8 KB of 16-bit bucket counters each) fit a CU.
#define SEGPAD(i) (i)
#define SEG_NBK (SEG_CAP / 2)
#define SEG_BKMAX 32
#else
#define SEGPAD(i) ((i) + ((i) >> 3))  // one pad word per 8 keys: spreads a thread's 8 keys over banks
#endif

// One tile of one branch (ts, hi, lo: the branch's columns; outputs at the branch's
// offset; off: the branch's first op index in A||B).  Sort key, one u64 per element:
// group (13 bits) | top 38 bits of oid_hi | tile index (13 bits) -- unique, so the
// bitonic network needs no payload; equal (group, hi38) pairs (rare on random ids,
// every duplicate id) are re-sorted exactly afterwards.  Each thread holds 8 keys whose
// indices differ in three consecutive bits b .. b+2, so three stages of the network run
// in registers per LDS round trip (33 round trips for 8192 keys instead of 91 stages).
// The segmented sort cannot order this log: seg_over for the host, and f_fail bit 3 so
// that every kernel queued behind the sort (k_gpart, k_wcount, k_window_g, the tail)
// leaves at once -- the host learns it from the merge's one meta read and runs the
// radix plan then (no host round trip between the sort and the windows).
// seg_over bit 0: a timestamp group longer than a tile holds (the branch is ordered: the
// radix plan orders it); bit 1 (SEG_DECREASE): a timestamp decreases (a sharded range
// slice must then fail, not be radix-sorted locally: smx_shard_step ORDER_FIX).
__device__ __forceinline__ void seg_fail(ComposeMeta* meta, bool decrease) {
  atomicOr((unsigned long long*)&meta->seg_over, decrease ? (unsigned long long)SEG_DECREASE : 1ull);
  atomicOr((unsigned long long*)&meta->f_fail, (unsigned long long)SEG_FAIL_BIT);
}

// One launch per branch (both in one grid measured slower: segsort 0.52 -> 0.60 ms on
// config 5, profiles/r03_v).
__global__ void __launch_bounds__(SEG_NT) k_segsort(const u64* __restrict__ ts, const u64* __restrict__ hi,
                                                    const u64* __restrict__ lo, i64 cnt, u32 off,
                                                    u64* __restrict__ sts, u64* __restrict__ shi,
                                                    u64* __restrict__ slo, u32* __restrict__ perm,
                                                    ComposeMeta* meta) {
  constexpr int PER = SEG_CAP / SEG_NT;  // 8 keys per thread
  static_assert(PER == 8, "the register passes assume 8 keys per thread");
  __shared__ u64 key[SEGPAD(SEG_CAP)];
  __shared__ u32 wsum[SEG_NT / WAVE + 1];
  __shared__ i64 se[2];
#if SEG_BUCKET
  __shared__ u32 bcnt[SEG_NBK / 2];  // two 16-bit bucket counters per word
#endif
  const int t = threadIdx.x, lane = t & (WAVE - 1), wv = t / WAVE;
  const i64 p0 = (i64)blockIdx.x * SEG_H;
  // Layout: every adjacent pair of the nominal range (the nominal ranges cover the
  // branch).  Tile bounds: the group of p0 (and of p0 + SEG_H) starts within the
  // SEG_CAP - SEG_H ops before it, where the ops below its timestamp are counted.
  constexpr int W = SEG_CAP - SEG_H;
  const u64 v0 = ts[p0];
  const bool has_end = p0 + SEG_H < cnt;
  const u64 v1 = has_end ? ts[p0 + SEG_H] : 0;
  bool dec = false, bad = false;
  u32 c0 = 0, c1 = 0;
#pragma unroll
  for (int r = 0; r < SEG_H / SEG_NT; ++r) {
    const i64 i = p0 + r * SEG_NT + t;
    if (i + 1 < cnt) dec |= ts[i + 1] < ts[i];
  }
#pragma unroll
  for (int r = 0; r < W / SEG_NT; ++r) {
    const i64 i0 = p0 - W + r * SEG_NT + t, i1 = p0 + SEG_H - W + r * SEG_NT + t;
    if (i0 >= 0) c0 += ts[i0] < v0;
    if (has_end) c1 += ts[i1] < v1;
  }
  if (t < 2) se[t] = 0;
  __syncthreads();
  c0 = wave_incl_sum(c0);
  c1 = wave_incl_sum(c1);
  if (lane == WAVE - 1) {
    atomicAdd((unsigned long long*)&se[0], (unsigned long long)c0);
    atomicAdd((unsigned long long*)&se[1], (unsigned long long)c1);
  }
  const i64 a0 = p0 - W > 0 ? p0 - W : 0, a1 = p0 + SEG_H - W;
  // a group reaching below its window: longer than the tile scheme allows
  if (t == 0 && p0 - W > 0 && ts[p0 - W - 1] == v0) bad = true;
  if (t == 1 && has_end && a1 > 0 && ts[a1 - 1] == v1) bad = true;
  const bool any_dec = __syncthreads_or(dec);
  if (any_dec | __syncthreads_or(bad)) {
    if (t == 0) seg_fail(meta, any_dec);
    return;
  }
  const i64 s = a0 + se[0], size = (has_end ? a1 + se[1] : cnt) - s;
  if (size <= 0) return;
  if (size > SEG_CAP) {
    if (t == 0) seg_fail(meta, false);
    return;
  }
  u32 P = 8, lgP = 3;
  while (P < (u32)size) P <<= 1, ++lgP;
  const bool own = (u32)t * PER < P;  // this thread holds 8 keys of the network
  // group index of each element: inclusive count of group starts after the first
  u32 f[PER], run = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const i64 x = (i64)t * PER + k;
    f[k] = x > 0 && x < size && ts[s + x] != ts[s + x - 1];
    run += f[k];
  }
  const u32 inc = wave_incl_sum(run);
  if (lane == WAVE - 1) wsum[wv] = inc;
  __syncthreads();
  u32 g = inc - run;
  for (int q = 0; q < wv; ++q) g += wsum[q];
  u64 v[PER];
  u32 gk[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u32 x = t * PER + k;
    g += f[k];
    gk[k] = g;
    v[k] = x < (u32)size ? ((u64)g << 51) | ((hi[s + x] >> 26) << 13) | x : ~0ull;  // padding sorts last
  }
#if SEG_BUCKET
  bool bitonic = false;
  {
    u32 ng = 1;  // groups in the tile
    for (int q = 0; q < SEG_NT / WAVE; ++q) ng += wsum[q];
    u16* gst = reinterpret_cast<u16*>(key);  // group starts (the key array is free until the scatter)
    for (int i = t; i < SEG_NBK / 2; i += SEG_NT) bcnt[i] = 0u;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 x = t * PER + k;
      if (x < (u32)size && (x == 0 || f[k])) gst[gk[k]] = (u16)x;
    }
    __syncthreads();
    u32 bk[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 x = t * PER + k;
      bk[k] = 0;
      if (x < (u32)size) {
        const u32 gs = gst[gk[k]], ge = gk[k] + 1 < ng ? (u32)gst[gk[k] + 1] : (u32)size;
        const u32 h32 = (u32)(v[k] >> 19);  // the top 32 of the 38 id bits
        bk[k] = (gs + (u32)(((u64)(ge - gs) * h32) >> 32)) >> 1;
        atomicAdd(&bcnt[bk[k] >> 1], 1u << (16 * (bk[k] & 1)));
      }
    }
    __syncthreads();
    // exclusive scan of the counters (4 per thread), largest bucket -> fallback
    const u32 nbw = ((u32)size + 3) / 4;  // counter words in use: 2 words per thread
    u32 w0 = 2 * t < nbw ? bcnt[2 * t] : 0u, w1 = 2 * t + 1 < nbw ? bcnt[2 * t + 1] : 0u;
    const u32 c0 = w0 & 0xffffu, c1 = w0 >> 16, c2 = w1 & 0xffffu, c3 = w1 >> 16;
    const u32 mx = max(max(c0, c1), max(c2, c3));
    u32 tot;
    const u32 e0 = block_excl_scan<OpSum, u32, SEG_NT / WAVE>(c0 + c1 + c2 + c3, wsum, &tot);
    const u32 e1 = e0 + c0, e2 = e1 + c1, e3 = e2 + c2;
    if (2 * t < nbw) bcnt[2 * t] = e0 | (e1 << 16);
    if (2 * t + 1 < nbw) bcnt[2 * t + 1] = e2 | (e3 << 16);
    bitonic = __syncthreads_or(mx > SEG_BKMAX);
    if (!bitonic) {
      // scatter: the counters become bucket ends
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const u32 x = t * PER + k;
        if (x < (u32)size) {
          const u32 sh = 16 * (bk[k] & 1);
          const u32 old = atomicAdd(&bcnt[bk[k] >> 1], 1u << sh);
          key[(old >> sh) & 0xffffu] = v[k];
        }
      }
      __syncthreads();
      u32 fp[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const u32 x = t * PER + k;
        fp[k] = 0;
        if (x < (u32)size) {
          const u32 b = bk[k];
          const u32 e = (bcnt[b >> 1] >> (16 * (b & 1))) & 0xffffu;
          const u32 lo = b ? (bcnt[(b - 1) >> 1] >> (16 * ((b - 1) & 1))) & 0xffffu : 0u;
          u32 c = 0;
          for (u32 q = lo; q < e; ++q) c += key[q] < v[k];
          fp[k] = lo + c;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < PER; ++k)
        if (t * PER + k < (u32)size) key[fp[k]] = v[k];
      __syncthreads();
    }
  }
  if (bitonic) {
#endif
  // merge levels k = 2, 4, 8: keys 8t .. 8t+7 (b = 0)
  seg_pass(v, (u32)t * 8, 0, 2, 0, 1);
  seg_pass(v, (u32)t * 8, 0, 4, 1, 2);
  seg_pass(v, (u32)t * 8, 0, 8, 2, 3);
  // later levels: a pass per window b of three partner bits; the keys move between
  // layouts through LDS (write in the old layout, read in the new one)
  u32 cur = 0;  // layout of v
  auto base_of = [&](u32 b) { return ((u32)t >> b << (b + 3)) | ((u32)t & ((1u << b) - 1)); };
  for (u32 lk = 4; lk <= lgP; ++lk) {
    const u32 k = 1u << lk;
    for (int jb = (int)lk - 1; jb >= 0;) {
      const u32 b = jb >= 2 ? (u32)jb - 2 : 0u;
      if (b != cur) {
        __syncthreads();  // the previous layout's reads are done
        if (own) {
          const u32 bo = base_of(cur);
#pragma unroll
          for (int m = 0; m < PER; ++m) key[SEGPAD(bo | ((u32)m << cur))] = v[m];
        }
        __syncthreads();
        if (own) {
          const u32 bn = base_of(b);
#pragma unroll
          for (int m = 0; m < PER; ++m) v[m] = key[SEGPAD(bn | ((u32)m << b))];
        }
        cur = b;
      }
      if (own) seg_pass(v, base_of(b), b, k, jb - (int)b, jb - (int)b + 1);
      jb = (int)b - 1;
    }
  }
  __syncthreads();
  if (own) {
    const u32 bo = base_of(cur);
#pragma unroll
    for (int m = 0; m < PER; ++m) key[SEGPAD(bo | ((u32)m << cur))] = v[m];
  }
  __syncthreads();
#if SEG_BUCKET
  }
#endif
  // runs of equal (group, hi38): exact order on (oid_hi, oid_lo, index)
  for (u32 x = t; x + 1 < (u32)size; x += SEG_NT) {
    const u64 kx = key[SEGPAD(x)] >> 13;
    if ((key[SEGPAD(x + 1)] >> 13) != kx || (x > 0 && (key[SEGPAD(x - 1)] >> 13) == kx)) continue;
    u32 e = x + 2;
    while (e < (u32)size && (key[SEGPAD(e)] >> 13) == kx) ++e;
    for (u32 y = x + 1; y < e; ++y) {
      const u64 ky = key[SEGPAD(y)];
      const u32 vi = (u32)ky & 0x1fffu;
      const u64 vh = hi[s + vi], vl = lo[s + vi];
      u32 z = y;
      while (z > x) {
        const u64 kw = key[SEGPAD(z - 1)];
        const u32 wi = (u32)kw & 0x1fffu;
        const u64 wh = hi[s + wi], wl = lo[s + wi];
        if (!(vh < wh || (vh == wh && (vl < wl || (vl == wl && vi < wi))))) break;
        key[SEGPAD(z)] = kw;
        --z;
      }
      key[SEGPAD(z)] = ky;
    }
  }
  __syncthreads();
  for (u32 x = t; x < (u32)size; x += SEG_NT) {
    const i64 src = s + (key[SEGPAD(x)] & 0x1fffu);
    sts[s + x] = ts[src];
    shi[s + x] = hi[src];
    slo[s + x] = lo[src];
    perm[s + x] = off + (u32)src;
  }
}


// Host wait for a stream: with SMX_SPIN_US > 0 a short spin on hipStreamQuery first, then
// the blocking sync.  Off for the merges: spinning measured slower there (config 2
// 0.161 -> 0.166 ms, profiles/r05_x/spin_ab.txt), while the RGA call gains from it
// (smx_rga.hip RGA_SPIN_US).
#ifndef SMX_SPIN_US
#define SMX_SPIN_US 0
#endif
static hipError_t stream_wait(hipStream_t st) {
  if (SMX_SPIN_US > 0) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipStreamQuery(st);
      if (e != hipErrorNotReady) return e;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(SMX_SPIN_US)) break;
    }
  }
  return hipStreamSynchronize(st);
}

static int read_meta(const Ctx& C, ComposeMeta* hm);

// GEN_SEG: when the segmented sort cannot order this log it flags seg_over and f_fail
// bit 3; every kernel after it leaves at once, and the caller reads seg_over from the
// meta after the tail.
static int run_generic(const Ctx& C, int mode) {
  hipStream_t st = C.st;
  ComposeMeta* meta = C.ws<ComposeMeta>(B_META);
  i64* bnd = C.ws<i64>(B_BND);
  u32* wcnt = C.ws<u32>(B_WCNT);
  u32* woff = C.ws<u32>(B_WOFF);
  const i64 na = C.na, nb = C.nb, n = C.n;
  u64* sts = C.ws<u64>(B_STS);
  u64* shi = C.ws<u64>(B_SHI);
  u64* slo = C.ws<u64>(B_SLO);
  u32* perm = C.ws<u32>(B_PERM);
  C.tm->begin(ST_GSORT);
  HIP_TRY(hipMemsetAsync(meta, 0, sizeof(ComposeMeta), st));
  if (mode == GEN_SEG) {
    C.tm->begin(ST_SEGSORT);
    for (int side = 0; side < 2; ++side) {
      const i64 off = side ? na : 0, cnt = side ? nb : na;
      if (cnt == 0) continue;
      hipLaunchKernelGGL(k_segsort, dim3(SMX_CEIL_DIV(cnt, (i64)SEG_H)), dim3(SEG_NT), 0, st, C.ops->ts + off,
                         C.ops->oid_hi + off, C.ops->oid_lo + off, cnt, (u32)off, sts + off, shi + off, slo + off,
                         perm + off, meta);
    }
    C.tm->end(ST_SEGSORT);
  } else {
    const bool with_lo = mode == GEN_RADIX_LO;
    hipLaunchKernelGGL(k_meta_init, dim3(1), dim3(1), 0, st, meta);
    hipLaunchKernelGGL(k_keymask, dim3(grid_for(n, BLOCK * 8)), dim3(BLOCK), 0, st, C.ops->ts, C.ops->oid_hi,
                       C.ops->oid_lo, na, n, meta);
    ComposeMeta hm;
    HIP_TRY(hipMemcpyAsync(&hm, meta, sizeof(ComposeMeta), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    RadixTemp rt{C.ws<u64>(B_RK2), C.ws<u32>(B_RV2), C.ws<u32>(B_RHIST), C.ws<u32>(B_PART)};
    const u64* words[3] = {C.ops->oid_lo, C.ops->oid_hi, C.ops->ts};
    const int w0 = with_lo ? 0 : 1;
    for (int side = 0; side < 2; ++side) {
      const i64 off = side ? na : 0, cnt = side ? nb : na;
      if (cnt == 0) continue;
      u64* key = C.ws<u64>(B_RKEY) + off;
      u32* val = perm + off;
      for (int wi = w0; wi < 3; ++wi) {
        const int q = 2 - wi;  // meta order: 0 = ts, 1 = hi, 2 = lo
        const u64 varying = hm.key_or[side][q] ^ hm.key_and[side][q];
        int shifts[8], ns = 0;
        for (int dgt = 0; dgt < 8; ++dgt)
          if ((varying >> (8 * dgt)) & 0xffull) shifts[ns++] = 8 * dgt;
        if (wi == w0) {
          hipLaunchKernelGGL(k_gather_init, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, words[wi] + off, key, val,
                             cnt);
          if (off)  // values are op indices of A||B
            hipLaunchKernelGGL(k_offset, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, val, cnt, (u32)off);
        } else {
          hipLaunchKernelGGL(k_gather, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, words[wi], val, key, cnt);
        }
        if (ns) HIP_TRY(radix_sort_pairs(key, val, cnt, shifts, ns, rt, st));
      }
      // the last key word is ts, so the sorted keys are ts in sorted order already
      HIP_TRY(hipMemcpyAsync(sts + off, key, (size_t)cnt * 8, hipMemcpyDeviceToDevice, st));
      hipLaunchKernelGGL(k_gather2, dim3(grid_for(cnt)), dim3(BLOCK), 0, st, C.ops->oid_hi, C.ops->oid_lo, val,
                         shi + off, slo + off, cnt);
    }
    if (!with_lo) hipLaunchKernelGGL(k_dupcheck, dim3(grid_for(n)), dim3(BLOCK), 0, st, sts, shi, na, n, meta);
  }
  const i64 W = SMX_CEIL_DIV(n, (i64)WG_CAP);
  hipLaunchKernelGGL(k_gpart, dim3(SMX_CEIL_DIV(W + 1, (i64)BLOCK)), dim3(BLOCK), 0, st, sts, shi, slo, na, nb,
                     W, bnd, meta);
  hipLaunchKernelGGL(k_wcount, dim3(W), dim3(WC_NT), 0, st, C.ops->kind, C.ops->v0, C.ops->v1, perm, bnd, na, W,
                     wcnt, meta);
  hipLaunchKernelGGL(k_wscan, dim3(NCNT), dim3(BLOCK), 0, st, wcnt, woff, W, meta);
  hipLaunchKernelGGL(k_bases, dim3(1), dim3(1), 0, st, meta, (u64)W);
  HIP_TRY(hipGetLastError());
  C.tm->end(ST_GSORT);
  WinArgs P = win_args(C);
  P.kts = sts;
  P.khi = shi;
  P.klo = slo;
  P.perm = perm;
  P.W = W;
  P.ablate = 0;
  C.tm->begin(ST_WINDOW_G);
  hipLaunchKernelGGL(k_window_g, dim3(W), dim3(WG_NT), 0, st, P);
  HIP_TRY(hipGetLastError());
  C.tm->end(ST_WINDOW_G);
  return SMX_OK;
}

// The meta block comes back through a pinned staging buffer (one per host thread): a
// DMA, not the runtime's staged copy into pageable memory.
struct PinnedMeta {  // freed when its host thread exits (thread-pool callers)
  ComposeMeta* p = nullptr;
  ~PinnedMeta() {
    if (p) (void)hipHostFree(p);
  }
};
static int read_meta(const Ctx& C, ComposeMeta* hm) {
  static thread_local PinnedMeta holder;
  ComposeMeta*& pinned = holder.p;
  if (!pinned) HIP_TRY(hipHostMalloc((void**)&pinned, sizeof(ComposeMeta), hipHostMallocDefault));
  HIP_TRY(hipMemcpyAsync(pinned, C.ws<ComposeMeta>(B_META), sizeof(ComposeMeta), hipMemcpyDeviceToHost, C.st));
  HIP_TRY(stream_wait(C.st));
  std::memcpy(hm, pinned, sizeof(ComposeMeta));
  return SMX_OK;
}

static int check_args(const smx_ops* ops, const smx_compose_out* out, void* ws, size_t ws_bytes, Layout* L) {
  const i64 na = ops->n_a, nb = ops->n_b, n = na + nb, n_sym = ops->n_sym;
  if (na < 0 || nb < 0 || n_sym < 0) return set_err(SMX_E_ARG, "negative size");
  if (n >= (i64)0x7fffffff) return set_err(SMX_E_ARG, "n_a + n_b must be < 2^31");
  if (n_sym > (i64)SYM_MASK + 1) return set_err(SMX_E_ARG, "n_sym must be <= 2^30");
  if (!out || !out->counts) return set_err(SMX_E_ARG, "null output");
  if (n == 0) return SMX_OK;
  if (!ops->kind || !ops->ts || !ops->oid_hi || !ops->oid_lo || !ops->sym || !ops->v0 || !ops->v1 ||
      !out->order || !out->addr || !out->file || !out->ctx || (!out->conflicts && out->conflict_cap > 0))
    return set_err(SMX_E_ARG, "null input/output pointer");
  if (n_sym < 1) return set_err(SMX_E_ARG, "n_sym must be >= 1");
  if (ops->b_gap < 0) return set_err(SMX_E_ARG, "b_gap must be >= 0");
  *L = layout(na, nb, n_sym);
  if (!ws || ws_bytes < L->total)
    return set_err(SMX_E_WORKSPACE, "workspace too small: need " + std::to_string(L->total));
  return SMX_OK;
}

static int profiling_on() {
  std::lock_guard<std::mutex> g(g_prof_mu);
  return g_prof;
}

// T order of the merge (plan + window kernels): the presorted plan first, with
// the tail (walk, tables, emit) launched behind it when `tail` -- every tail kernel
// is a no-op if the window kernel flags the plan as failed; a window that overflows
// LDS (dense timestamp ties) retries with smaller windows; a log that is not
// timestamp-ordered goes to the generic plan when allowed.  hm: the meta after it.
// The plan the last compose on this thread used (smx_last_plan).
static thread_local int g_plan = SMX_PLAN_PRESORTED;

// After a presorted attempt with target window size tgt (hm: the meta it left):
// a window that overflows LDS (dense timestamp ties) retries with smaller windows;
// a log that is not timestamp-ordered goes to the generic plan when allowed.  The
// tail (walk, tables, emit) is launched behind each plan when `tail`.
// require_ordered (a sharded range slice): a slice whose timestamps decrease must fail
// loudly -- the radix plan would order it locally, not across the shards -- so it is
// refused when the window kernel (f_fail bit 0) or the segmented sort (SEG_DECREASE)
// saw a decrease.  (k_fpart's early verdict, F_LONG, can hide bit 0: then the wide
// windows or the segmented sort report the decrease themselves.)
static int order_fallbacks(const Ctx& C, bool allow_generic, bool tail, ComposeMeta* hm, i64 tgt,
                           bool require_ordered = false, int level = WL_NORMAL) {
  int rc;
  auto unordered = [&]() {
    return set_err(SMX_E_ARG, "sharded merge needs timestamp-ordered branch logs in every shard");
  };
  g_plan = SMX_PLAN_PRESORTED;
  if (level == WL_SMALL && hm->f_fail && !(hm->f_fail & 1) && !hm->bad_sym) {
    // small windows that do not hold the log's timestamp groups: the normal ones
    tgt = knob("SMX_WIN_TGT", WIN_TGT);
    if ((rc = hm->f_fail == F_LONG ? run_presorted_rewide(C, tgt, WL_NORMAL) : run_presorted(C, tgt))) return rc;
    if (tail && (rc = launch_tail(C))) return rc;
    if ((rc = read_meta(C, hm))) return rc;
  }
  while (hm->f_fail == 2 && !hm->bad_sym && tgt > WIN_TGT_MIN) {  // dense groups: smaller windows
    tgt = (tgt / 2) / CH * CH;
    if ((rc = run_presorted(C, tgt))) return rc;
    if (tail && (rc = launch_tail(C))) return rc;
    if ((rc = read_meta(C, hm))) return rc;
  }
  // ordered logs whose equal-timestamp groups no WF_CAP window holds (F_LONG or 6, or 2 at
  // the smallest windows): the wide windows, from their full capacity down (a window
  // holds its target plus the group its end snaps back over; at full capacity each of
  // config 5's windows is one 8192-op group, and no window is empty)
  for (i64 wt = WF_WIDE_CAP; hm->f_fail && !(hm->f_fail & 1) && !hm->bad_sym && wt >= WIN_TGT_MIN; wt /= 2) {
    g_plan = SMX_PLAN_PRESORTED_WIDE;
    if ((rc = hm->f_fail == F_LONG ? run_presorted_rewide(C, wt) : run_presorted(C, wt, nullptr, WL_WIDE))) return rc;
    if (tail && (rc = launch_tail(C))) return rc;
    if ((rc = read_meta(C, hm))) return rc;
    if (hm->f_fail != 2) break;  // held, or groups longer than a wide window (6), or unordered (1)
  }
  if (hm->f_fail && !hm->bad_sym && allow_generic) {
    if (C.ops->b_gap != 0)
      return set_err(SMX_E_ARG, "branch logs not timestamp-ordered: the generic plan needs b_gap = 0");
    if (require_ordered && (hm->f_fail & 1)) return unordered();
    if (!(hm->f_fail & 1)) {  // ordered, long groups: the segmented sort, tail behind it
      g_plan = SMX_PLAN_SEGMENTED;
      if ((rc = run_generic(C, GEN_SEG))) return rc;
      if (tail && (rc = launch_tail(C))) return rc;
      if ((rc = read_meta(C, hm))) return rc;
      if (!hm->seg_over) return SMX_OK;
      if (require_ordered && (hm->seg_over & SEG_DECREASE)) return unordered();
    }
    g_plan = SMX_PLAN_RADIX;
    if ((rc = run_generic(C, GEN_RADIX))) return rc;
    if ((rc = read_meta(C, hm))) return rc;
    if (hm->dup_key) {
      g_plan = SMX_PLAN_RADIX_LO;
      if ((rc = run_generic(C, GEN_RADIX_LO))) return rc;
    }
    if (tail && (rc = launch_tail(C))) return rc;
    if ((rc = read_meta(C, hm))) return rc;
  }
  return SMX_OK;
}

// T order of the merge (plan + window kernels): the presorted plan first, with the
// tail launched behind it when `tail` -- every tail kernel is a no-op if the window
// kernel flags the plan as failed -- then the fallbacks.  hm: the meta after it.
static int run_order(const Ctx& C, bool allow_generic, bool tail, ComposeMeta* hm) {
  const i64 tgt = knob("SMX_WIN_TGT", WIN_TGT);
  int rc = run_presorted(C, tgt);
  if (rc) return rc;
  if (tail && (rc = launch_tail(C))) return rc;
  if ((rc = read_meta(C, hm))) return rc;
  return order_fallbacks(C, allow_generic, tail, hm, tgt);
}

__global__ void k_counts(const ComposeMeta* meta, u64 n, i64* counts) {
  counts[0] = (i64)(n - meta->n_skip);
  counts[1] = (i64)meta->n_conf;
}

// Moves whose newAddress or newFile is None see the symbol's inclusive prefix of
// non-None values: moves grouped by symbol (radix sort), then a scan per symbol,
// seeded from the lower shards' values (mvpre) in a sharded merge.
static int run_mvprefix(const Ctx& C, const ComposeMeta& hm, const u64* mvpre) {
  hipStream_t st = C.st;
  const u64 nMv = hm.kcnt[KMOVE];
  if (hm.n_move_none == 0 || nMv == 0) return SMX_OK;
  const i64 n_sym = C.n_sym;
  u64* keys = C.ws<u64>(B_RKEY);
  u32* vals = C.ws<u32>(B_RVAL);
  RadixTemp rt{C.ws<u64>(B_RK2), C.ws<u32>(B_RV2), C.ws<u32>(B_RHIST), C.ws<u32>(B_PART)};
  int shifts[4], ns = 0;
  for (int dgt = 0; dgt < 4; ++dgt)
    if (((u64)(n_sym - 1) >> (8 * dgt)) != 0) shifts[ns++] = 8 * dgt;
  hipLaunchKernelGGL(k_mv_init, dim3(grid_for(nMv)), dim3(BLOCK), 0, st, C.ws<u32>(B_MSYM), nMv, keys, vals);
  if (ns) HIP_TRY(radix_sort_pairs(keys, vals, (i64)nMv, shifts, ns, rt, st));
  hipLaunchKernelGGL(k_mv_fix, dim3(grid_for(nMv)), dim3(BLOCK), 0, st, keys, vals, nMv, C.ws<u32>(B_MSYM), mvpre,
                     (u64)n_sym, C.out->addr, C.out->file);
  HIP_TRY(hipGetLastError());
  return SMX_OK;
}

// smx_compose_async: the presorted plan and its tail, enqueued without a host
// sync (hipGraph-capturable).  counts[0] < -1 afterwards asks for
// smx_compose_finish: -2 the plan failed, -3 moves with a None value need their
// prefix fix-up.
// Plan-failed counts without the tail: what k_emit4's first thread writes on a failed plan.
__global__ void k_counts_failed(const ComposeMeta* meta, i64* counts) {
  counts[0] = meta->bad_sym ? -1 : -2;
  counts[1] = meta->bad_sym ? -1 : (i64)meta->n_conf;
}

// The early-failure flag of this host thread on device dev (pinned, coherent).
static int early_fail_of(int dev, EarlyFail* e) {
  struct Slot {
    int dev = -1;
    EarlyFail e;
  };
  struct Slots {  // the pinned flags and events, freed when the host thread exits
    Slot s[4];
    ~Slots() {
      for (auto& x : s) {
        if (x.dev < 0) continue;
        int cur = 0;
        if (hipGetDevice(&cur) == hipSuccess && cur != x.dev) (void)hipSetDevice(x.dev);
        if (x.e.ev) (void)hipEventDestroy(x.e.ev);
        if (x.e.flag_host) (void)hipHostFree(x.e.flag_host);
        if (cur != x.dev) (void)hipSetDevice(cur);
      }
    }
  };
  static thread_local Slots holder;
  Slot* slots = holder.s;
  for (int i = 0; i < 4; ++i)
    if (Slot& s = slots[i]; s.dev == dev) {
      *e = s.e;
      return SMX_OK;
    }
  for (int i = 0; i < 4; ++i)
    if (Slot& s = slots[i]; s.dev < 0) {
      HIP_TRY(hipHostMalloc((void**)&s.e.flag_host, 64, hipHostMallocCoherent | hipHostMallocMapped));
      HIP_TRY(hipHostGetDevicePointer((void**)&s.e.flag_dev, s.e.flag_host, 0));
      // (no system-scope fence: k_khist / k_fpart store the flag itself at system scope,
      // and a missed flag only costs the tail launched behind a plan that then fails)
      HIP_TRY(hipEventCreateWithFlags(&s.e.ev, hipEventDisableTiming | (SMX_SIDE_SYSFENCE ? 0u : hipEventDisableSystemFence)));
      s.dev = dev;
      *e = s.e;
      return SMX_OK;
    }
  return SMX_E_HIP;  // (more than four devices per host thread: no early flag)
}

#ifndef SMX_SMALL
#define SMX_SMALL 1  // merges of at most SMALL_N ops: one workgroup, one launch (k_compose_small)
#endif

// Largest merge (ops) the one-workgroup path takes (smx_set_small_limit; 0: never).
static std::atomic<int64_t> g_small_max{SMX_SMALL ? SMALL_N : 0};
// (symbol ids index the small kernel's hash table with 0xffffffff as its empty mark)
static inline bool small_merge(const smx_ops* ops) {
  return ops->n_a + ops->n_b <= g_small_max.load(std::memory_order_relaxed) && ops->n_sym <= 0xffffffffll;
}

#ifndef SMX_EARLY_MIN
#define SMX_EARLY_MIN (1ll << 22)  // ops from which a synchronous merge waits for k_khist's verdict
#endif

// What the synchronous merge's host learned from k_khist before the windows ran.
struct EarlyVerdict {
  bool failed = false;  // the presorted plan fails for sure (f_fail F_LONG)
  bool bad = false;     // ... and k_khist saw an invalid kind
  // the merge's verdict word in mapped pinned host memory (synchronous calls): the
  // last kernel (k_compose_small, k_emit) stores seq << 1 | bit there, and finish reads
  // it after the stream wait instead of copying the meta block back (one copy packet
  // less per call).  bit: the small plan's invalid input; the large plan's "finish
  // has work left" (an error, a failed plan, None-value moves), which reads the meta.
  u64* hrec = nullptr;       // (device address)
  const u64* hrec_host = nullptr;
  u64 hseq = 0;
  bool rec_used = false;
  bool rec_small = false;
};

struct SmallRec {  // one per host thread, freed when the thread exits
  u64* h = nullptr;
  u64* d = nullptr;  // its device address as the device `dev` sees it
  int dev = -1;
  u64 seq = 0;
  ~SmallRec() {
    if (h) (void)hipHostFree(h);
  }
};
// The thread's verdict word: pinned, mapped, portable host memory.  Its device address is
// taken on the device current at the call and taken again when a later call runs on
// another device (no reliance on one address serving every device).
static SmallRec* small_rec() {
  static thread_local SmallRec r;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return nullptr;
  if (!r.h) {
    if (hipHostMalloc((void**)&r.h, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) !=
        hipSuccess) {
      r.h = nullptr;
      return nullptr;
    }
    *(volatile u64*)r.h = 0;
  }
  if (r.dev != cur) {
    if (hipHostGetDevicePointer((void**)&r.d, r.h, 0) != hipSuccess) {
      (void)hipGetLastError();
      r.d = nullptr;
      r.dev = -1;
      return nullptr;  // (the caller then reads the meta block instead)
    }
    r.dev = cur;
  }
  return &r;
}

static int enqueue_async(const smx_ops* ops, const smx_compose_out* out, void* ws, const Layout& L,
                         hipStream_t st, bool timed, bool early_ok = false, EarlyVerdict* verdict = nullptr) {
  const i64 na = ops->n_a, nb = ops->n_b, n = na + nb, n_sym = ops->n_sym;
  StageTimer tm(st, timed);
  Ctx C{ops, out, st, L, (char*)ws, na, nb, n, n_sym, 0, na, &tm};
  int rc;
  if (small_merge(ops)) {  // the whole merge in one workgroup (smx_small.h)
    tm.begin(ST_SMALL);
    u64* hrec = verdict ? verdict->hrec : nullptr;
    if (hrec) verdict->rec_used = verdict->rec_small = true;
    hipLaunchKernelGGL(k_compose_small, dim3(1), dim3(SMALL_NT), 0, st, *ops, *out, C.ws<ComposeMeta>(B_META), hrec,
                       hrec ? verdict->hseq : (u64)0);
    HIP_TRY(hipGetLastError());
    tm.end(ST_SMALL);
    tm.flush();
    return SMX_OK;
  }
  // A large synchronous merge (not captured): the host waits for k_khist's verdict while
  // k_fpart and the column scans run, then launches the normal or the wide windows and
  // the tail; on an invalid kind no window and no tail (smx_compose_finish reports it).
  EarlyFail early;
  bool use_early = false;
  if (early_ok && n >= SMX_EARLY_MIN) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    int dev = 0;
    HIP_TRY(hipStreamIsCapturing(st, &cs));
    HIP_TRY(hipGetDevice(&dev));
    use_early = cs == hipStreamCaptureStatusNone && early_fail_of(dev, &early) == SMX_OK;
    if (use_early) early.flag_host[0] = early.flag_host[1] = 0u;  // (the previous merge on this thread has synced)
  }
  Deferred dw;
  if ((rc = run_presorted(C, first_tgt(C), use_early ? &early : nullptr, first_level(C), &dw))) return rc;
  if (use_early) {
    HIP_TRY(hipEventSynchronize(early.ev));
    const bool lng = ((volatile u32*)early.flag_host)[0] != 0;
    if (dw.on && !((volatile u32*)early.flag_host)[1]) {
      // k_khist's verdict: the windows that hold the log's timestamp groups.  After
      // F_LONG k_fpart has placed the wide plan's boundaries and the scans its window
      // count (config 5: no doomed normal launch, no re-arm, no second k_fpart)
      if (lng) g_plan = SMX_PLAN_PRESORTED_WIDE;
      if ((rc = lng ? launch_presorted_windows(C, dw.W_w, dw.CM, WL_WIDE)
                    : launch_presorted_windows(C, dw.W, dw.CM, first_level(C))))
        return rc;
    } else if (lng || ((volatile u32*)early.flag_host)[1]) {
      const bool bad = ((volatile u32*)early.flag_host)[1] != 0;
      if (verdict) {
        verdict->failed = true;
        verdict->bad = bad;
      }
      if (!verdict || bad) {  // (smx_compose's finish runs the fallback plan next: it writes the counts)
        hipLaunchKernelGGL(k_counts_failed, dim3(1), dim3(1), 0, st, C.ws<ComposeMeta>(B_META), out->counts);
        HIP_TRY(hipGetLastError());
      }
      tm.flush();
      return SMX_OK;
    }
  }
  if (verdict && verdict->hrec) {  // k_emit publishes the verdict: finish skips the meta copy
    C.hrec = verdict->hrec;
    C.hseq = verdict->hseq;
    verdict->rec_used = true;
  }
  if (!knob("SMX_ABLATE", 0) && (rc = launch_tail(C))) return rc;  // SMX_ABLATE (diagnostic builds): window only
  tm.flush();
  return SMX_OK;
}

// The library once replayed a merge's ~25 launches as one cached HIP graph from the second
// merge of a (stream, buffers) key on.  On this ROCm the replay measured slower than
// enqueueing the launches (config 2 0.183 -> 0.160 ms, config 3 2.381 -> 2.352 ms without
// it, profiles/r05_x/graph_ab.txt: the graph's first kernel waits for the whole
// submission), so the cache was removed in round 6; a caller's own capture of
// smx_compose_async stays supported (tests/test_gpu_async.py).  smx_release_graphs is
// kept in the ABI and releases nothing.
extern "C" int smx_release_graphs(void* stream) {
  (void)stream;
  return SMX_OK;
}

// early_ok: the synchronous smx_compose (a host wait for k_khist's verdict is allowed)
static int compose_async_impl(const smx_ops* ops, const smx_compose_out* out, void* ws, size_t ws_bytes,
                              hipStream_t st, bool early_ok, EarlyVerdict* verdict = nullptr) {
  Layout L{};
  int rc = check_args(ops, out, ws, ws_bytes, &L);
  if (rc) return rc;
  const i64 n = ops->n_a + ops->n_b;
  const bool small = small_merge(ops);
  g_plan = small ? SMX_PLAN_SMALL : SMX_PLAN_PRESORTED;
  if (n == 0) {
    HIP_TRY(hipMemsetAsync(out->counts, 0, 2 * sizeof(int64_t), st));
    return SMX_OK;
  }
  const bool timed = profiling_on() != 0;
  EarlyVerdict ev;
  if (verdict) ev = *verdict;  // (the caller's verdict word, if any)
  if ((rc = enqueue_async(ops, out, ws, L, st, timed, early_ok, &ev))) return rc;
  if (verdict) *verdict = ev;
  return SMX_OK;
}

// smx_compose_finish: one host sync; runs whatever the asynchronous part left
// (the fallback plans, the None-value move prefix) and the final counts.
// known: the synchronous merge's early verdict (the plan failed): no meta read needed
// before the fallback plan -- k_khist was the last kernel to write the meta's flags
static int compose_finish_impl(const smx_ops* ops, const smx_compose_out* out, void* ws, size_t ws_bytes,
                               hipStream_t st, const EarlyVerdict* known = nullptr) {
  Layout L{};
  int rc = check_args(ops, out, ws, ws_bytes, &L);
  if (rc) return rc;
  const i64 na = ops->n_a, nb = ops->n_b, n = na + nb, n_sym = ops->n_sym;
  if (n == 0 || knob("SMX_ABLATE", 0)) return SMX_OK;
  StageTimer tm(st, profiling_on() != 0);
  Ctx C{ops, out, st, L, (char*)ws, na, nb, n, n_sym, 0, na, &tm};
  ComposeMeta hm;
  bool have = false;
  if (known && known->failed) {
    std::memset(&hm, 0, sizeof(hm));
    hm.f_fail = F_LONG;
    hm.bad_sym = known->bad ? 1 : 0;
    have = true;
  } else if (known && known->rec_used) {  // the verdict word: no meta copy when there is no work left
    HIP_TRY(stream_wait(st));
    const u64 v = *(volatile const u64*)known->hrec_host;
    if ((v >> 1) == known->hseq) {
      std::memset(&hm, 0, sizeof(hm));
      hm.bad_sym = v & 1;
      have = known->rec_small || !(v & 1);
    }
  }
  if (!have && (rc = read_meta(C, &hm))) {
    return rc;
  }
  if (hm.bad_sym) return set_err(SMX_E_ARG, "invalid input: sym[i] >= n_sym or kind[i] >= 18");
  if (hm.f_fail && (rc = order_fallbacks(C, true, true, &hm, first_tgt(C), false, first_level(C)))) return rc;
  if (hm.bad_sym) return set_err(SMX_E_ARG, "invalid input: sym[i] >= n_sym or kind[i] >= 18");
  if (hm.n_move_none && hm.kcnt[KMOVE]) {
    tm.begin(ST_MVPREFIX);
    if ((rc = run_mvprefix(C, hm, nullptr))) return rc;
    hipLaunchKernelGGL(k_counts, dim3(1), dim3(1), 0, st, C.ws<ComposeMeta>(B_META), (u64)n, out->counts);
    HIP_TRY(hipGetLastError());
    tm.end(ST_MVPREFIX);
  }
  tm.flush();
  return SMX_OK;
}

// ---------------------------------------------------------------------------
// sharded merge (include/smx.h smx_shard_step)

// summary[0..21]
__global__ void k_shard_summary(const ComposeMeta* meta, i64* summary) {
  for (int k = 0; k < SMX_N_KINDS; ++k) summary[k] = (i64)meta->kcnt[k];
  summary[18] = (i64)meta->n_ren_side[0];
  summary[19] = (i64)meta->n_ren_side[1];
  summary[20] = (i64)meta->n_move_none;
  summary[21] = (i64)((meta->f_fail & 1 ? 1 : 0) | (meta->bad_sym ? 2 : 0) | (meta->f_fail & 2 ? 4 : 0));
}

// An empty shard hands the incoming open region (device- or host-held) straight on.
__global__ void k_pass_region(const i64* in_dev, i64 in_ahead, i64 in_d, i64* summary) {
  if (in_dev) {
    in_ahead = in_dev[0];
    in_d = in_dev[1];
  }
  summary[22] = in_d > 0 ? 1 : 0;
  summary[23] = in_d > 0 ? in_ahead : 0;
  summary[24] = in_d > 0 ? in_d : 0;
  summary[25] = summary[26] = summary[27] = 0;
}

__global__ void k_shard_walk_sum(const ComposeMeta* meta, i64* summary) {
  summary[22] = (i64)meta->out_open;
  summary[23] = (i64)meta->out_ahead;
  summary[24] = (i64)meta->out_d;
  summary[25] = (i64)meta->n_conf;
  summary[26] = (i64)meta->n_skip;
  summary[27] = (i64)meta->halo_overflow;
}

__global__ void k_shard_tab_sum(const ComposeMeta* meta, i64* summary, int bucketed) {
  for (int i = 0; i < 3; ++i) summary[28 + i] = bucketed ? (i64)bit_width32(meta->vbits[i]) : 32;
  summary[31] = (i64)meta->tab_over;
}
__global__ void k_tab_over_reset(ComposeMeta* meta) { meta->tab_over = 0; }

// fin from the reduced partial tables: packed with the global widths when they
// fit in 64 bits (meta->vbits takes the global widths, for k_emit).
__global__ void k_fin_from_tab(const void* __restrict__ tabv, const i64* __restrict__ glob, i64 n_sym,
                               int tagbits, ComposeMeta* meta, int4* __restrict__ fin) {
  u32 w[3];
  const u64* tab = (const u64*)tabv;
  const u32* tab32 = (const u32*)tabv;
  for (int i = 0; i < 3; ++i)
    w[i] = (u32)min(max(tagbits ? (i64)(i32)tab32[3 * n_sym + i] : glob[i], (i64)0), (i64)32);
  const FinPack FP = fin_pack_make(w[0], w[1], w[2], true);
  if (blockIdx.x == 0 && threadIdx.x < 3)
    meta->vbits[threadIdx.x] = w[threadIdx.x] >= 32 ? ~0u : ((1u << w[threadIdx.x]) - 1u);
  for (i64 s = (i64)blockIdx.x * BLOCK + threadIdx.x; s < n_sym; s += (i64)gridDim.x * BLOCK) {
    int va, vf, vc;
    if (tagbits) {
      const u32 m = (1u << (31 - tagbits)) - 1u;
      const u32 a = tab32[s], f = tab32[n_sym + s], c = tab32[2 * n_sym + s];
      va = a ? (int)(a & m) - 1 : -1, vf = f ? (int)(f & m) - 1 : -1, vc = c ? (int)(c & m) - 1 : -1;
    } else {
      const u64 a = tab[s], f = tab[n_sym + s], c = tab[2 * n_sym + s];
      va = a ? (int)(u32)a - 1 : -1, vf = f ? (int)(u32)f - 1 : -1, vc = c ? (int)(u32)c - 1 : -1;
    }
    fin_put(FP, fin, (u32)s, va, vf, vc);
  }
}

// This shard's halo from the all-gather of every shard's ORDER outputs (smx_shard
// .order_gather): for each branch b, the first H renames of b on the following shards
// in shard order -- entry i is taken from the shard q whose cumulative count first
// exceeds i -- and halo_dev = (count, count, more, more).
__global__ void k_halo_gather(const i64* __restrict__ g, int W, int r, i64 H, u32* hs0, u32* hs1, i32* hc0, i32* hc1,
                              i32* hr0, i32* hr1, i64* halo_dev) {
  const i64 row = SMX_SHARD_SUMMARY + 3 * H;  // int64 words per shard
  for (int b = 0; b < 2; ++b) {
    u32* hs = b ? hs1 : hs0;
    i32* hc = b ? hc1 : hc0;
    i32* hr = b ? hr1 : hr0;
    i64 total = 0;
    for (int q = r + 1; q < W; ++q) total += max(g[q * row + 18 + b], (i64)0);
    const i64 got = min(total, H);
    for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < got; i += (i64)gridDim.x * BLOCK) {
      i64 cum = 0;
      int q = r + 1;
      for (; q < W; ++q) {
        const i64 c = min(max(g[q * row + 18 + b], (i64)0), H);
        if (i < cum + c) break;
        cum += c;
      }
      const i64 off = i - cum;
      const i32* X = reinterpret_cast<const i32*>(g + q * row + SMX_SHARD_SUMMARY);  // [3][2H] int32
      hs[i] = (u32)X[b * H + off];
      hc[i] = X[2 * H + b * H + off];
      hr[i] = X[4 * H + b * H + off];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      halo_dev[b] = got;
      halo_dev[2 + b] = total > got ? 1 : 0;
    }
  }
}

static int shard_impl(const smx_ops* ops, const smx_shard* sh, const smx_compose_out* out, void* ws,
                      size_t ws_bytes, hipStream_t st, int step) {
  if (!sh || !sh->summary) return set_err(SMX_E_ARG, "null shard / summary");
  Layout L{};
  int rc = check_args(ops, out, ws, ws_bytes, &L);
  if (rc) return rc;
  const i64 na = ops->n_a, nb = ops->n_b, n = na + nb, n_sym = ops->n_sym;
  StageTimer tm(st, profiling_on() != 0);
  Ctx C{ops, out, st, L, (char*)ws, na, nb, n, n_sym, sh->src_a, sh->src_b, &tm};
  C.src_map = sh->src_map;
  if (sh->src_map && ops->b_gap != 0) return set_err(SMX_E_ARG, "src_map needs b_gap = 0");
  if (n == 0) {  // an empty shard: neutral summaries and outputs
    if (step == SMX_SHARD_ORDER) HIP_TRY(hipMemsetAsync(sh->summary, 0, SMX_SHARD_SUMMARY * 8, st));
    if (step == SMX_SHARD_WALK) {
      // the open region passes through unchanged (or none comes in): always rewrite
      // the outgoing state, a previous round may have left another one
      hipLaunchKernelGGL(k_pass_region, dim3(1), dim3(1), 0, st, (const i64*)sh->in_state_dev,
                         (i64)sh->in_ahead, (i64)sh->in_d, sh->summary);
      HIP_TRY(hipGetLastError());
    }
    if (step == SMX_SHARD_TABLES && sh->part_tab)
      HIP_TRY(hipMemsetAsync(sh->part_tab, 0, (size_t)3 * n_sym * (sh->tab32 > 0 ? 4 : 8), st));
    if (step == SMX_SHARD_EMIT) HIP_TRY(hipMemsetAsync(out->counts, 0, 2 * sizeof(int64_t), st));
    return SMX_OK;
  }
  // The bucketed table records are consumed by SMX_SHARD_TABLES (k_tb_unskip kills the
  // walk's skipped renames in place): a second TABLES needs a SCATTER (or ORDER) first.
  // Tracked per workspace on the host, where the steps are issued in stream order.
  auto records_state = [&](int set) -> int {  // set: 1 scattered, 2 consumed; -1 query
    static std::mutex mu;
    static std::vector<std::pair<void*, int>> st_of;
    std::lock_guard<std::mutex> g(mu);
    for (auto& e : st_of)
      if (e.first == ws) {
        if (set >= 0) e.second = set;
        return e.second;
      }
    if (set >= 0) {
      if (st_of.size() >= 64) st_of.erase(st_of.begin());
      st_of.push_back({ws, set});
    }
    return set >= 0 ? set : 0;
  };
  auto order_outputs = [&]() -> int {
    hipLaunchKernelGGL(k_shard_summary, dim3(1), dim3(1), 0, st, C.ws<ComposeMeta>(B_META), sh->summary);
    if (sh->halo_cap > 0)
      hipLaunchKernelGGL(k_halo_export, dim3(1), dim3(EX_NT), 0, st, walk_args(C, nullptr), sh->export_sym,
                         sh->export_cls, sh->export_src, (u64)sh->halo_cap);
    HIP_TRY(hipGetLastError());
    // the table records, bucketed while the host exchanges the summaries and walks
    records_state(1);
    return launch_tb_prescatter(C);
  };
  switch (step) {
    case SMX_SHARD_ORDER:
    case SMX_SHARD_ORDER_FIX: {
      if (sh->halo_cap < 0 || (sh->halo_cap > 0 && (!sh->export_sym || !sh->export_cls || !sh->export_src)))
        return set_err(SMX_E_ARG, "bad export buffers");
      const i64 tgt = knob("SMX_WIN_TGT", WIN_TGT);
      if (step == SMX_SHARD_ORDER && !sh->src_map) {  // asynchronous: failures show in summary[21]
        g_plan = SMX_PLAN_PRESORTED;
        if ((rc = run_presorted(C, tgt))) return rc;
        return order_outputs();
      }
      ComposeMeta hm;
      if (step == SMX_SHARD_ORDER) {
        // a sample-sorted shard's branch logs are in any order: the generic plan
        if ((rc = run_order(C, true, false, &hm))) return rc;  // times its own stages
      } else {
        if ((rc = read_meta(C, &hm))) return rc;
        // a compacted shard (b_gap = 0) may take the generic plan
        if (hm.f_fail && (rc = order_fallbacks(C, ops->b_gap == 0, false, &hm, tgt, true))) return rc;
      }
      if ((rc = order_outputs())) return rc;
      if (hm.bad_sym) return set_err(SMX_E_ARG, "invalid input: sym[i] >= n_sym or kind[i] >= 18");
      if (hm.f_fail)
        return set_err(SMX_E_ARG, "sharded merge needs timestamp-ordered branch logs in every shard");
      break;
    }
    case SMX_SHARD_WALK: {
      tm.begin(ST_WALK);
      if (sh->order_gather && sh->halo_cap > 0) {
        if (!sh->halo_dev || !sh->halo_sym[0] || !sh->halo_sym[1] || !sh->halo_cls[0] || !sh->halo_cls[1] ||
            !sh->halo_src[0] || !sh->halo_src[1] || sh->world < 1 || sh->rank < 0 || sh->rank >= sh->world)
          return set_err(SMX_E_ARG, "order_gather needs writable halo buffers and halo_dev");
        hipLaunchKernelGGL(k_halo_gather, dim3(SMX_CEIL_DIV(sh->halo_cap, (i64)BLOCK)), dim3(BLOCK), 0, st,
                           sh->order_gather, (int)sh->world, (int)sh->rank, (i64)sh->halo_cap,
                           (u32*)sh->halo_sym[0], (u32*)sh->halo_sym[1], (i32*)sh->halo_cls[0],
                           (i32*)sh->halo_cls[1], (i32*)sh->halo_src[0], (i32*)sh->halo_src[1],
                           (i64*)sh->halo_dev);
        HIP_TRY(hipGetLastError());
      }
      if ((rc = launch_walk(C, sh))) return rc;
      hipLaunchKernelGGL(k_shard_walk_sum, dim3(1), dim3(1), 0, st, C.ws<ComposeMeta>(B_META), sh->summary);
      HIP_TRY(hipGetLastError());
      tm.end(ST_WALK);
      break;
    }
    case SMX_SHARD_TABLES: {
      if (!sh->part_tab) return set_err(SMX_E_ARG, "null part_tab");
      if (records_state(-1) != 1)
        return set_err(SMX_E_ARG, "SMX_SHARD_TABLES needs the records bucketed by SMX_SHARD_ORDER / "
                                  "ORDER_FIX / SCATTER since the last TABLES");
      records_state(2);
      tm.begin(ST_TABLES);
      bool bucketed = false;
      // (ORDER / ORDER_FIX / SCATTER bucketed the records)
      if (sh->tab32 < 0 || sh->tab32 > 8 || (sh->tab32 > 0 && ((u64)sh->rank + 1u) >> sh->tab32))
        return set_err(SMX_E_ARG, "tab32: the tag (rank + 1) must fit tab32 <= 8 bits");
      hipLaunchKernelGGL(k_tab_over_reset, dim3(1), dim3(1), 0, st, C.ws<ComposeMeta>(B_META));
      if ((rc = launch_tables(C, sh->part_tab, (u32)sh->rank + 1u, sh->tab32, &bucketed, true))) return rc;
      hipLaunchKernelGGL(k_shard_tab_sum, dim3(1), dim3(1), 0, st, C.ws<ComposeMeta>(B_META), sh->summary,
                         bucketed ? 1 : 0);
      HIP_TRY(hipGetLastError());
      tm.end(ST_TABLES);
      break;
    }
    case SMX_SHARD_SCATTER: {
      records_state(1);
      if ((rc = launch_tb_prescatter(C))) return rc;
      break;
    }
    case SMX_SHARD_EMIT: {
      if (!sh->fin_tab || (!sh->glob && sh->tab32 == 0)) return set_err(SMX_E_ARG, "null fin_tab / glob");
      if (sh->tab32 < 0 || sh->tab32 > 8) return set_err(SMX_E_ARG, "tab32 must be 0..8");
      tm.begin(ST_EMIT);
      hipLaunchKernelGGL(k_fin_from_tab, dim3(grid_for(n_sym)), dim3(BLOCK), 0, st, (const void*)sh->fin_tab,
                         sh->glob, n_sym, (int)sh->tab32, C.ws<ComposeMeta>(B_META), C.ws<int4>(B_FIN));
      if ((rc = launch_emit(C, true, sh))) return rc;
      tm.end(ST_EMIT);
      ComposeMeta hm;
      if (sh->summary_host) {  // what the move prefix needs, as the host gathered it
        hm.kcnt[KMOVE] = (u64)sh->summary_host[KMOVE];
        hm.n_move_none = (u64)sh->summary_host[20];
      } else if ((rc = read_meta(C, &hm))) {
        return rc;
      }
      tm.begin(ST_MVPREFIX);
      if ((rc = run_mvprefix(C, hm, sh->mv_prefix))) return rc;
      tm.end(ST_MVPREFIX);
      break;
    }
    default:
      return set_err(SMX_E_ARG, "unknown shard step");
  }
  tm.flush();
  return SMX_OK;
}

// smx_shard_range_info (include/smx.h): one block for the keys, then a grid over both
// slices for the order check (a violation stores 0; every writer stores the same).
__device__ __forceinline__ i64 rinfo_key(u64 v) { return (i64)(v ^ 0x8000000000000000ull); }
__global__ void k_range_info(const u64* __restrict__ ts, i64 off_a, i64 n_a, i64 off_b, i64 n_b, int rh,
                             int sa, int sb, i64* __restrict__ out) {
  const int t = threadIdx.x;
  if (t == 0) {
    out[0] = n_a;
    out[1] = n_b;
    out[2] = n_a ? rinfo_key(ts[off_a]) : 0;
    out[3] = n_a ? rinfo_key(ts[off_a + n_a - 1]) : 0;
    out[4] = n_b ? rinfo_key(ts[off_b]) : 0;
    out[5] = n_b ? rinfo_key(ts[off_b + n_b - 1]) : 0;
    out[6] = 1;
    out[7] = sa;
    out[8] = sb;
  }
  for (int i = t; i < 4 * rh; i += blockDim.x) {
    const int br = i / (2 * rh), j = i % (2 * rh);
    const i64 o = br ? off_b : off_a, n = br ? n_b : n_a;
    const i64 h = n < rh ? n : rh;
    i64 pos;
    if (n == 0) pos = -1;
    else if (j < rh) pos = j < h ? o + j : o;                         // head, padded
    else pos = j - rh < rh - h ? o : o + n - h + (j - rh - (rh - h));  // tail, right-aligned
    out[9 + i] = pos < 0 ? 0 : rinfo_key(ts[pos]);
  }
}
__global__ void k_range_order(const u64* __restrict__ ts, i64 off_a, i64 n_a, i64 off_b, i64 n_b,
                              i64* __restrict__ out) {
  bool bad = false;
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n_a + n_b; i += (i64)gridDim.x * blockDim.x) {
    const bool b = i >= n_a;
    const i64 k = b ? i - n_a : i;
    if (k == 0) continue;
    const i64 o = b ? off_b : off_a;
    bad |= ts[o + k] < ts[o + k - 1];
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) out[6] = 0;
}
extern "C" int smx_shard_range_info(const uint64_t* ts, int64_t off_a, int64_t n_a, int64_t off_b, int64_t n_b,
                                    int32_t rh, int32_t check_order, int32_t signed_a, int32_t signed_b, int64_t* out,
                                    void* stream) {
  if (!ts || !out || n_a < 0 || n_b < 0 || rh < 1 || off_a < 0 || off_b < 0)
    return set_err(SMX_E_ARG, "smx_shard_range_info: bad argument");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_range_info, dim3(1), dim3(BLOCK), 0, st, (const u64*)ts, off_a, n_a, off_b, n_b, rh,
                     signed_a, signed_b, (i64*)out);
  if (check_order && n_a + n_b > 1)
    hipLaunchKernelGGL(k_range_order, dim3(grid_for(n_a + n_b, BLOCK * 16)), dim3(BLOCK), 0, st, (const u64*)ts,
                       off_a, n_a, off_b, n_b, (i64*)out);
  HIP_TRY(hipGetLastError());
  return SMX_OK;
}

extern "C" int smx_shard_step(const smx_ops* ops, const smx_shard* shard, const smx_compose_out* out,
                              void* workspace, size_t workspace_bytes, void* stream, int step) {
  if (!ops) return set_err(SMX_E_ARG, "null ops");
  (void)hipGetLastError();  // an earlier call's error (any library's) is not this call's
  try {
    return shard_impl(ops, shard, out, workspace, workspace_bytes, (hipStream_t)stream, step);
  } catch (const std::exception& e) {
    return set_err(SMX_E_HIP, e.what());
  }
}

extern "C" int smx_compose_async(const smx_ops* ops, const smx_compose_out* out, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  if (!ops) return set_err(SMX_E_ARG, "null ops");
  (void)hipGetLastError();  // an earlier call's error (any library's) is not this call's
  try {
    return compose_async_impl(ops, out, workspace, workspace_bytes, (hipStream_t)stream, false);
  } catch (const std::exception& e) {
    return set_err(SMX_E_HIP, e.what());
  }
}

extern "C" int smx_compose_finish(const smx_ops* ops, const smx_compose_out* out, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (!ops) return set_err(SMX_E_ARG, "null ops");
  (void)hipGetLastError();  // an earlier call's error (any library's) is not this call's
  try {
    return compose_finish_impl(ops, out, workspace, workspace_bytes, (hipStream_t)stream);
  } catch (const std::exception& e) {
    return set_err(SMX_E_HIP, e.what());
  }
}

extern "C" int smx_compose(const smx_ops* ops, const smx_compose_out* out, void* workspace,
                           size_t workspace_bytes, void* stream) {
  if (!ops) return set_err(SMX_E_ARG, "null ops");
  (void)hipGetLastError();  // an earlier call's error (any library's) is not this call's
  int rc;
  try {
    EarlyVerdict ev;
    if (SmallRec* r = small_rec()) {
      ev.hrec = r->d;
      ev.hrec_host = r->h;
      ev.hseq = ++r->seq;
    }
    rc = compose_async_impl(ops, out, workspace, workspace_bytes, (hipStream_t)stream, true, &ev);
    if (!rc) rc = compose_finish_impl(ops, out, workspace, workspace_bytes, (hipStream_t)stream, &ev);
  } catch (const std::exception& e) {
    return set_err(SMX_E_HIP, e.what());
  }
  return rc;
}

extern "C" int smx_last_plan(void) { return g_plan; }

#ifdef SMALL_STAMPS
// diagnostic builds only: the small kernel's phase stamps of its last call (wall clock, 100 MHz)
extern "C" int smx_diag_small_stamps(uint64_t* host16) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_small_stamp), 16 * sizeof(u64)));
  return SMX_OK;
}
#endif

extern "C" int64_t smx_set_small_limit(int64_t n) {
  const int64_t v = n < 0 ? 0 : n > SMALL_N ? SMALL_N : n;
  return g_small_max.exchange(SMX_SMALL ? v : 0);
}

extern "C" int smx_set_profiling(int enabled) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  g_prof = enabled;
  return SMX_OK;
}

extern "C" int smx_set_profiling_stages(uint32_t mask) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  g_prof_mask = mask;
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

extern "C" const char* smx_version(void) { return "smx 0.2 gfx950"; }
