// smx_rga.hip — batched RGA replay on gfx950 (semmerge/crdt.py:23-57), C ABI in include/smx.h.
//
// Exact restatement of the sequential list:
//  * The list is always sorted by (key, creation index): insert places the new
//    element before the first strictly greater key (crdt.py:48-57), so equal
//    keys keep insertion order.
//  * An element's fate depends only on the events of its (list, value):
//    move pops the first live element of that value in list order (= the live
//    one with the smallest (key, index)) and always inserts a new element;
//    delete tombstones every present element of that value (crdt.py:33-43).
//  * materialize = live elements in (key, index) order (crdt.py:45-46).
// Pipeline: stable radix partition of 16-byte event records by list id (up to 65536
// lists: the high byte by a global pass, the low byte per high-byte bucket, which also
// gives the list starts; LDS-staged, coalesced) -> one wave per list (k_rga_wave,
// persistent, in LDS): value groups by hashing, one sequential replay per group,
// survivors ordered by (anchor, t, author, opid, index) -> compaction, each list's
// output offset summed by its own wave from per-chunk survivor sums.
#include <algorithm>
#include <chrono>
#include <string>

#include "smx_scan.h"

#define RGA_TRY(x)                                                                     \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess)                                                              \
      return smx_set_error(SMX_E_HIP, (std::string(#x) + ": " + hipGetErrorString(_e)).c_str()); \
  } while (0)

// Event record, 2 u64 words, grouped by list by the partition below:
//   w0 = anchor << 32 | t' >> 32   (t' = t with the sign bit flipped: order-preserving)
//   w1 = value << 32 | op << 30 | event index   (index = creation order)
// (anchor, t, author, opid, index) is the crdt.py:48-57 key order; w0 decides it
// unless two events share anchor and the top half of t, and only then are t, author
// and opid read from the input columns by event index (rga_key_lt).
#define RGA_REC 2
struct __attribute__((aligned(16))) R16 {  // one record (16-byte loads / stores)
  u64 a, b;
};
#define RGA_WV 1  // the value / op / index word
#define RGA_IDX_MASK 0x3fffffffu
#define RGA_TOMB_BIT 0x80000000u  // tmp_s: the element is tombstoned (list mode, smx_rga_out.out_tomb)

// Grouping the events by list: a stable radix partition of whole records on the list id,
// 8 bits per pass (one pass up to 256 lists; up to 65536 the high byte here and the low
// byte per bucket in k_rrec_local; beyond, LSD passes of this kernel).  The first
// pass reads the input columns and packs the records; each pass stages a tile in LDS
// in digit order and writes each digit's run of records contiguously, so every byte
// moves in full cache lines.  Stable: each list's events stay in stream order.
#ifndef RR_NT
#define RR_NT 512                         // scatter workgroup (persistent, one per CU)
#endif
#define RR_NW (RR_NT / WAVE)
#ifndef RR_PER_CU
#define RR_PER_CU 2  // persistent scatter workgroups per CU (LDS ~74 KB each)
#endif
#ifndef RREC_ITEMS
#define RREC_ITEMS 6
#endif
#define RREC_TILE (RR_NT * RREC_ITEMS)    // 3072 records (120 KB) per block and pass
#define RREC_SEG (RREC_TILE / RR_NW)      // contiguous records per wave
#define RGA_NDIG 256                      // digits per pass
#ifndef RR_HIST_OP
#define RR_HIST_OP 0  // 1: the histogram pass also reads the op column (to count bad ops as list 0)
#endif
#ifndef RR_W16
#define RR_W16 1  // runs written as 16-byte records (one store per record, not two)
#endif
static_assert(RREC_TILE % BLOCK == 0 && RREC_TILE <= 65535, "tile: k_rrec_hist blocks, u16 slots");

template <bool FIRST>
__global__ void __launch_bounds__(BLOCK) k_rrec_hist(smx_rga_ops o, const u32* __restrict__ keys, int shift,
                                                     u32* __restrict__ hist, i32* __restrict__ err) {
  __shared__ u32 h[RGA_NDIG];
  h[threadIdx.x] = 0;
  __syncthreads();
  const i64 base = (i64)blockIdx.x * RREC_TILE;
  constexpr int IT = RREC_TILE / BLOCK;
  u32 key[IT], bad = 0;  // all loads first: a conditional error store between them would
                         // order each iteration's loads after the previous check
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const i64 i = base + it * BLOCK + threadIdx.x;
    key[it] = 0;
    if (i < o.n_ops) {
      if constexpr (FIRST) {
        const u32 l = o.list[i];
        // a list id out of range counts as list 0, where k_rrec_scatter places it (an op
        // > 2 fails the call there; its record still goes to its list)
        const bool b = RR_HIST_OP ? l >= (u64)o.n_lists || o.op[i] > 2 : l >= (u64)o.n_lists;
        key[it] = b ? 0u : l;
        bad |= (u32)b;
      } else {
        key[it] = keys[i];
      }
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const i64 i = base + it * BLOCK + threadIdx.x;
    if (i < o.n_ops) atomicAdd(&h[(key[it] >> shift) & 255u], 1u);
  }
  if (bad) *err = 1;
  __syncthreads();
  hist[(i64)blockIdx.x * RGA_NDIG + threadIdx.x] = h[threadIdx.x];
}

// This thread's share of one tile, loaded into registers: pass 1 the input columns of
// its RREC_ITEMS events, pass 2+ their list ids and RREC_ITEMS * 5 consecutive record
// words of the previous pass (consecutive lanes, consecutive words).
template <bool FIRST>
struct RTile;
template <>
struct RTile<true> {
  u32 list[RREC_ITEMS], value[RREC_ITEMS], anchor[RREC_ITEMS];
  u32 op[RREC_ITEMS];
  i64 t[RREC_ITEMS];
};
#define RREC_V4 ((RREC_TILE * RGA_REC * 8 / 16 + RR_NT - 1) / RR_NT)  // 16-byte loads per thread
typedef u32 v4u32 __attribute__((ext_vector_type(4)));
template <>
struct RTile<false> {
  u32 key[RREC_ITEMS];
  v4u32 w[RREC_V4];
};

__device__ __forceinline__ i64 rrec_event(i64 base, u32 w, int it, u32 lane) {
  return base + (i64)w * RREC_SEG + it * WAVE + lane;
}

template <bool FIRST>
__device__ __forceinline__ void rrec_load(RTile<FIRST>& T, const smx_rga_ops& o, const u32* __restrict__ kin,
                                          const u64* __restrict__ rin, i64 base, u32 t, u32 w, u32 lane) {
  const i64 n = o.n_ops;
  if constexpr (FIRST) {
#pragma unroll
    for (int it = 0; it < RREC_ITEMS; ++it) {
      const i64 i = rrec_event(base, w, it, lane);
      const bool v = i < n;
      T.list[it] = v ? o.list[i] : 0u;
      T.op[it] = v ? o.op[i] : 0u;
      T.value[it] = v ? o.value[i] : 0u;
      T.anchor[it] = v ? o.anchor[i] : 0u;
      T.t[it] = v ? o.t[i] : 0;

    }
  } else {
#pragma unroll
    for (int it = 0; it < RREC_ITEMS; ++it) {
      const i64 i = rrec_event(base, w, it, lane);
      T.key[it] = i < n ? kin[i] : 0u;
    }
    // 16-byte chunks of the tile's words; an odd last word of the whole stream reads
    // 8 bytes of the buffer's (256-byte) padding with it
    const i64 cnt = n - base < RREC_TILE ? n - base : RREC_TILE;
    const i64 nv = (cnt * RGA_REC + 1) / 2;
    const v4u32* q = reinterpret_cast<const v4u32*>(rin + (u64)base * RGA_REC);
#pragma unroll
    for (int i = 0; i < RREC_V4; ++i) {
      const i64 x = (i64)t + (i64)i * RR_NT;
      T.w[i] = x < nv ? __builtin_nontemporal_load(&q[x]) : v4u32{0, 0, 0, 0};
    }
  }
}

// A persistent workgroup per CU walks the tiles; per tile: wave multisplit of the
// records by digit (ranks and per-wave digit counts), block scan of the digit totals,
// records staged in LDS in digit order, then every digit's run written contiguously
// (RREC_TILE / 256 records per run on average: whole cache lines).  The next tile's
// loads are issued before the current tile's runs are written, so the two overlap.
template <bool FIRST, typename KO = u32>
__global__ void __launch_bounds__(RR_NT) k_rrec_scatter(smx_rga_ops o, const u32* __restrict__ kin,
                                                        const u64* __restrict__ rin, KO* __restrict__ kout,
                                                        u64* __restrict__ rout, int shift,
                                                        const u32* __restrict__ offs, i32* __restrict__ err,
                                                        u32 ntiles) {
  __shared__ __attribute__((aligned(16))) u64 srec[RREC_TILE * RGA_REC];  // 48 KB
  __shared__ u32 skey[RREC_TILE];
  __shared__ u16 spos[RREC_TILE];            // tile record -> staged slot (pass 2+)
  __shared__ u16 wc[RR_NW][RGA_NDIG];        // per-wave digit counts, then offsets
  __shared__ u32 lstart[RGA_NDIG];
  __shared__ u32 gofs[RGA_NDIG];
  const u32 t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  const i64 n = o.n_ops;
  const u64 lt = lanemask_lt();
  RTile<FIRST> T;
  u32 tile = blockIdx.x;
  if (tile < ntiles) rrec_load<FIRST>(T, o, kin, rin, (i64)tile * RREC_TILE, t, w, lane);
  for (; tile < ntiles; tile += gridDim.x) {
    const i64 base = (i64)tile * RREC_TILE;
    const u32 cnt = (u32)(n - base < RREC_TILE ? n - base : RREC_TILE);
    for (int x = t; x < RR_NW * RGA_NDIG; x += RR_NT) (&wc[0][0])[x] = 0;
    if (t < RGA_NDIG) gofs[t] = offs[(i64)tile * RGA_NDIG + t];
    __syncthreads();
    u32 key[RREC_ITEMS], dr[RREC_ITEMS];
#pragma unroll
    for (int it = 0; it < RREC_ITEMS; ++it) {
      const bool valid = rrec_event(base, w, it, lane) < n;
      if constexpr (FIRST) {
        key[it] = T.list[it];
        const bool badl = key[it] >= (u64)o.n_lists, bado = T.op[it] > 2;
        if (valid && (badl || bado)) {
          *err = 1;
          if (badl || RR_HIST_OP) key[it] = 0;
        }
      } else {
        key[it] = T.key[it];
      }
      const u32 d = (key[it] >> shift) & 255u;
      const u64 peers = wave_peers<8>(d, valid);
      const u32 before = wc[w][d];
      dr[it] = d | ((before + (u32)__popcll(peers & lt)) << 8);
      if (valid && (peers >> lane) == 1ull) wc[w][d] = (u16)(before + (u32)__popcll(peers));
    }
    __syncthreads();
    if (t < RGA_NDIG) {
      u32 tot = 0;
#pragma unroll
      for (int q = 0; q < RR_NW; ++q) tot += wc[q][t];
      lstart[t] = tot;
    }
    __syncthreads();
    if (t < WAVE) {  // exclusive scan of the 256 digit totals, 4 per lane
      u32 x[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = lstart[4 * t + j];
        sum += x[j];
      }
      u32 run = wave_incl_sum(sum) - sum;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lstart[4 * t + j] = run;
        run += x[j];
      }
    }
    __syncthreads();
    if (t < RGA_NDIG) {
      u32 acc = lstart[t];
#pragma unroll
      for (int q = 0; q < RR_NW; ++q) {
        const u32 c = wc[q][t];
        wc[q][t] = (u16)acc;
        acc += c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < RREC_ITEMS; ++it) {
      const u32 li = (u32)(w * RREC_SEG + it * WAVE + lane);
      const i64 i = base + li;
      if (i >= n) continue;
      const u32 d = dr[it] & 255u, p = wc[w][d] + (dr[it] >> 8);
      skey[p] = key[it];
      if constexpr (FIRST) {
        u64* r = &srec[p * RGA_REC];
        const u64 tt = (u64)T.t[it] ^ 0x8000000000000000ull;
        r[0] = ((u64)T.anchor[it] << 32) | (tt >> 32);
        const u32 op = T.op[it] > 2 ? 0u : T.op[it];
        r[RGA_WV] = ((u64)T.value[it] << 32) | (op << 30) | (u32)i;
      } else {
        spos[li] = (u16)p;
      }
    }
    if constexpr (!FIRST) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < RREC_V4; ++i) {
        const u32 c = t + (u32)i * RR_NT;  // words 2c, 2c + 1
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u32 x = 2 * c + h;
          if (x < cnt * RGA_REC) {
            const u32 r = x / RGA_REC, k = x - r * RGA_REC;
            srec[spos[r] * RGA_REC + k] = h ? ((u64)T.w[i].w << 32 | T.w[i].z) : ((u64)T.w[i].y << 32 | T.w[i].x);
          }
        }
      }
    }
    __syncthreads();
    // the next tile's loads fly while this tile's runs are written
    if (tile + gridDim.x < ntiles) rrec_load<FIRST>(T, o, kin, rin, (i64)(tile + gridDim.x) * RREC_TILE, t, w, lane);
#if RR_W16
#pragma unroll 1
    for (u32 p = t; p < cnt; p += RR_NT) {  // record-wise: consecutive lanes, consecutive 16-byte records
      const u32 key = skey[p];
      const u32 d = (key >> shift) & 255u;
      const u32 dst = gofs[d] + p - lstart[d];
      kout[dst] = (KO)key;  // (u8: the low byte, for k_rrec_local)
      *reinterpret_cast<R16*>(rout + (u64)dst * RGA_REC) = reinterpret_cast<const R16*>(srec)[p];
    }
#else
#pragma unroll 1
    for (u32 p = t; p < cnt; p += RR_NT) {
      const u32 d = (skey[p] >> shift) & 255u;
      kout[gofs[d] + p - lstart[d]] = (KO)skey[p];  // (u8: the low byte, for k_rrec_local)
    }
#pragma unroll 1
    for (u32 x = t; x < cnt * RGA_REC; x += RR_NT) {  // word-wise: consecutive lanes, consecutive words
      const u32 p = x / RGA_REC, k = x - p * RGA_REC;
      const u32 d = (skey[p] >> shift) & 255u;
      rout[(u64)(gofs[d] + p - lstart[d]) * RGA_REC + k] = srec[x];
    }
#endif
    __syncthreads();  // LDS is rewritten by the next tile
  }
}

// lstart[l] = first sorted position of list l (an empty list starts where the next
// one does); one pass over the sorted list ids.
// Also zeroes the survivor sums of 256-list chunks (csum, RGA_CS_MAX words), which the
// list kernels fill and k_rga_out reads.
#define RGA_CS_LISTS 256                   // lists per survivor-sum chunk
#define RGA_CS_MAX 256                     // chunks (k_rga_out: one uint4 per lane)
#define RGA_FUSED_MAX (RGA_CS_LISTS * RGA_CS_MAX)  // lists up to which k_rga_out finds its own offsets
#ifndef RGA_OUT_PRE
#define RGA_OUT_PRE 2
#endif
#ifndef RGA_OUT_LPW
#define RGA_OUT_LPW 1  // lists per wave in k_rga_out_fused (4: 28.8 us either way, round 4)
#endif
// err word bits: RGA_E_INPUT a list id >= n_lists or an op > 2 (the call fails);
// RGA_E_UNGROUPED a call that said its events come grouped by list (SMX_RGA_GROUPED) has a
// list id that decreases: every list kernel leaves at once and the call is redone with
// the partition
#ifndef RGA_DIRECT
#define RGA_DIRECT 1  // grouped calls: the list kernels read the input columns (no record pass)
#endif
#define RGA_E_INPUT 1
#define RGA_E_UNGROUPED 2

// Events already grouped by list (non-decreasing list ids: what crdt.replay and RGA
// hand over, stream after stream): the records are packed in place of the partition --
// one coalesced pass, four consecutive events per thread -- and the list starts come
// from the steps of the list id.  Also zeroes the survivor chunk sums (k_rga_bounds' duty).
__global__ void __launch_bounds__(BLOCK) k_rga_pack(smx_rga_ops o, u64* __restrict__ rout, u32* __restrict__ lstart,
                                                    u32* __restrict__ csum, i32* __restrict__ err) {
  const i64 n = o.n_ops, nl = o.n_lists;
  if (blockIdx.x == 0 && threadIdx.x < RGA_CS_MAX) csum[threadIdx.x] = 0u;
  u32 bad = 0;
  // consecutive lanes, consecutive events: coalesced column loads, one 16-byte record store
  for (i64 i = (i64)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (i64)gridDim.x * BLOCK) {
    const u32 l = o.list[i], op = o.op[i], v = o.value[i], an = o.anchor[i];
    const i64 t = o.t[i];
    const u32 prev = i > 0 ? o.list[i - 1] : 0u;  // (the neighbour lane's load: an L1 hit)
    bad |= (l >= (u64)nl || op > 2) ? (u32)(RGA_E_INPUT | RGA_E_UNGROUPED) : 0u;
    bad |= i > 0 && l < prev ? (u32)RGA_E_UNGROUPED : 0u;
    const u64 tt = (u64)t ^ 0x8000000000000000ull;
    R16 r;
    r.a = ((u64)an << 32) | (tt >> 32);
    r.b = ((u64)v << 32) | ((op > 2 ? 0u : op) << 30) | (u32)i;
    *reinterpret_cast<R16*>(rout + (u64)i * RGA_REC) = r;
    // list starts: the lists in (prev, l] start here (from list 0 at the first event);
    // after the last event the rest start at n (ids clamped: one out of range fails the call)
    const u32 lo = i == 0 ? 0u : prev + 1u, hi = l < (u64)nl ? l : (u32)(nl - 1);
    for (u32 L = lo; L <= hi; ++L) lstart[L] = (u32)i;
    if (i == n - 1)
      for (i64 L = (i64)hi + 1; L < nl; ++L) lstart[L] = (u32)n;
  }
  if (bad) atomicOr(err, (i32)bad);
}

// Grouped events read in place by the list kernels (ColSrc): only the list starts, the
// checks and the chunk sums' zeroing of k_rga_pack, reading the list ids and ops.
__global__ void __launch_bounds__(BLOCK) k_rga_gbounds(smx_rga_ops o, u32* __restrict__ lstart,
                                                       u32* __restrict__ csum, i32* __restrict__ err) {
  const i64 n = o.n_ops, nl = o.n_lists;
  if (blockIdx.x == 0 && threadIdx.x < RGA_CS_MAX) csum[threadIdx.x] = 0u;
  u32 bad = 0;
  // four consecutive events per thread: one 16-byte list-id load and one 4-byte op load
  // when aligned (the columns are the caller's: checked, else event by event)
  const bool vec = ((reinterpret_cast<uintptr_t>(o.list) | reinterpret_cast<uintptr_t>(o.op)) & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(o.list) & 15) == 0;
  for (i64 i0 = ((i64)blockIdx.x * BLOCK + threadIdx.x) * 4; i0 < n; i0 += (i64)gridDim.x * BLOCK * 4) {
    u32 l4[4], op4[4];
    if (vec && i0 + 4 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(o.list + i0);
      const u32 ob = *reinterpret_cast<const u32*>(o.op + i0);
      l4[0] = v.x, l4[1] = v.y, l4[2] = v.z, l4[3] = v.w;
#pragma unroll
      for (int u = 0; u < 4; ++u) op4[u] = (ob >> (8 * u)) & 0xffu;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        l4[u] = i0 + u < n ? (u32)o.list[i0 + u] : 0u;
        op4[u] = i0 + u < n ? (u32)o.op[i0 + u] : 0u;
      }
    }
    u32 prev = i0 > 0 ? (u32)o.list[i0 - 1] : 0u;  // (the neighbour lane's line: an L1 hit)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const i64 i = i0 + u;
      if (i >= n) break;
      const u32 l = l4[u], op = op4[u];
      bad |= (l >= (u64)nl || op > 2) ? (u32)(RGA_E_INPUT | RGA_E_UNGROUPED) : 0u;
      bad |= i > 0 && l < prev ? (u32)RGA_E_UNGROUPED : 0u;
      const u32 lo = i == 0 ? 0u : prev + 1u, hi = l < (u64)nl ? l : (u32)(nl - 1);
      for (u32 L = lo; L <= hi; ++L) lstart[L] = (u32)i;
      if (i == n - 1)
        for (i64 L = (i64)hi + 1; L < nl; ++L) lstart[L] = (u32)n;
      prev = l;
    }
  }
  if (bad) atomicOr(err, (i32)bad);
}

__global__ void k_rga_bounds(const u32* __restrict__ keys, i64 n, i64 nl, u32* __restrict__ lstart,
                             u32* __restrict__ csum) {
  if (blockIdx.x == 0 && threadIdx.x < RGA_CS_MAX) csum[threadIdx.x] = 0u;
  for (i64 j = (i64)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (i64)gridDim.x * BLOCK) {
    const i64 l = keys[j];
    const i64 lp = j ? (i64)keys[j - 1] : -1;
    for (i64 L = lp + 1; L <= l; ++L) lstart[L] = (u32)j;
    if (j == n - 1)
      for (i64 L = l + 1; L < nl; ++L) lstart[L] = (u32)n;
  }
}

// Two-byte list ids (257..65536 lists): the first pass partitions by the HIGH byte
// (k_rrec_hist / k_rrec_scatter, stable), then one workgroup per high-byte bucket orders
// its records by the low byte on its own (k_rrec_local): a count, a scan in LDS and a
// stable scatter of tiles in stream order -- no global histogram, scan or bounds pass
// (the bucket's list starts come from its scan), and no list ids written (the list
// kernels read only the starts).  Bucket d is [dstart[d], dstart[d + 1]).
#ifndef RGA_MSD
#define RGA_MSD 1  // 0: LSD passes (k_rrec_hist / k_rrec_scatter twice, k_rga_bounds)
#endif
#define RL_NT 1024
#define RL_NW (RL_NT / WAVE)
#ifndef RL_ITEMS
#define RL_ITEMS 4
#endif
#define RL_TILE (RL_NT * RL_ITEMS)
#define RL_SEG (RL_TILE / RL_NW)  // contiguous records per wave and tile
#define RL_CU 8                   // count phase: keys in flight per lane
#ifndef RL_S
#define RL_S 2  // workgroups per bucket
#endif
#ifndef RL_PF
#define RL_PF 0  // 1: the next tile's loads issued once this one is staged (measured slower: 0.58 -> 0.605 ms)
#endif
__global__ void __launch_bounds__(RL_NT) k_rrec_local(const u8* __restrict__ kin, const u64* __restrict__ rin,
                                                      u64* __restrict__ rout,
                                                      const u32* __restrict__ dstart, i64 nl,
                                                      u32* __restrict__ lstart, u32* __restrict__ csum) {
  __shared__ u32 cnt[RGA_NDIG];
  __shared__ u32 run[RGA_NDIG];
  __shared__ u16 wc[RL_NW][RGA_NDIG];
  __shared__ u32 tstart[RGA_NDIG], wsum[RGA_NDIG / WAVE];
  const u32 t = threadIdx.x, lane = t & (WAVE - 1), w = t / WAVE;
  // RL_S workgroups per bucket (two fit a CU): workgroup h scatters the h-th part of the
  // bucket, after counting the whole bucket and the parts before its own
  const u32 d = blockIdx.x / RL_S, h = blockIdx.x - d * RL_S;
  if (blockIdx.x == 0 && t < RGA_CS_MAX) csum[t] = 0u;  // (k_rga_bounds' other duty)
  const u32 b0 = dstart[d], b1 = dstart[d + 1];
  const u32 seg = (b1 - b0 + RL_S - 1) / RL_S;
  const u32 sa = min(b0 + h * seg, b1), sb = min(sa + seg, b1);
  u32 kd[RL_ITEMS], dr[RL_ITEMS];
  R16 rv[RL_ITEMS];
  auto load_tile = [&](u32 base) {
#pragma unroll
    for (int it = 0; it < RL_ITEMS; ++it) {
      const u32 i = base + w * RL_SEG + it * WAVE + lane;
      const bool valid = i < sb;
      kd[it] = valid ? kin[i] : 0u;
      rv[it].a = valid ? rin[(u64)i * RGA_REC] : 0ull;
      rv[it].b = valid ? rin[(u64)i * RGA_REC + 1] : 0ull;
    }
  };
  if (RL_PF && sa < sb) load_tile(sa);  // (in flight during the count)
  if (t < RGA_NDIG) {
    cnt[t] = 0;
    tstart[t] = 0;  // (first: the counts of the parts before this workgroup's)
  }
  __syncthreads();
  {  // 4 low bytes per load (aligned words over [b0, b1); the buffer has room past n)
    const u32* kw = reinterpret_cast<const u32*>(kin);
    const u32 w0 = b0 >> 2, w1 = (b1 + 3) >> 2;
    for (u32 x0 = w0 + t; x0 < w1; x0 += RL_NT * RL_CU) {  // RL_CU loads in flight per lane
      u32 k[RL_CU];
#pragma unroll
      for (int j = 0; j < RL_CU; ++j) {
        const u32 x = x0 + j * RL_NT;
        k[j] = x < w1 ? kw[x] : 0u;
      }
#pragma unroll
      for (int j = 0; j < RL_CU; ++j) {
        const u32 x = x0 + j * RL_NT;
        if (x >= w1) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const u32 i = 4 * x + q;
          if (i >= b0 && i < b1) {
            const u32 dd = (k[j] >> (8 * q)) & 255u;
            atomicAdd(&cnt[dd], 1u);
            if (i < sa) atomicAdd(&tstart[dd], 1u);
          }
        }
      }
    }
  }
  __syncthreads();
  if (t < WAVE) {  // exclusive scan of the 256 low-byte counts, 4 per lane
    u32 x[4], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = cnt[4 * t + j];
      sum += x[j];
    }
    u32 r = wave_incl_sum(sum) - sum;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      run[4 * t + j] = b0 + r;
      r += x[j];
    }
  }
  __syncthreads();
  if (t < RGA_NDIG) {  // list starts (an empty list starts where the next one does)
    const i64 l = (i64)d * RGA_NDIG + t;
    if (h == 0 && l < nl) lstart[l] = run[t];
    run[t] += tstart[t];
  }
  __syncthreads();
  const u64 lt = lanemask_lt();
  // the tile's records staged in LDS in (low byte, stream) order, then written run by
  // run: consecutive lanes store consecutive 16-byte records of one list
  __shared__ R16 stg[RL_TILE];
  __shared__ u8 sdig[RL_TILE];
  for (u32 base = sa; base < sb; base += RL_TILE) {
    if (!RL_PF) load_tile(base);
    for (u32 x = t; x < RL_NW * RGA_NDIG; x += RL_NT) (&wc[0][0])[x] = 0;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < RL_ITEMS; ++it) {
      const u32 i = base + w * RL_SEG + it * WAVE + lane;
      const bool valid = i < sb;
      const u32 dd = kd[it] & 255u;
      const u64 peers = wave_peers<8>(dd, valid);
      const u32 before = wc[w][dd];
      dr[it] = dd | ((before + (u32)__popcll(peers & lt)) << 8);
      if (valid && (peers >> lane) == 1ull) wc[w][dd] = (u16)(before + (u32)__popcll(peers));
    }
    __syncthreads();
    u32 tc = 0, inc = 0;
    if (t < RGA_NDIG) {  // per-wave offsets inside the digit's share of the tile
#pragma unroll
      for (int q = 0; q < RL_NW; ++q) {
        const u32 c = wc[q][t];
        wc[q][t] = (u16)tc;
        tc += c;
      }
      inc = wave_incl_sum(tc);
      if (lane == WAVE - 1) wsum[w] = inc;
    }
    __syncthreads();
    if (t < RGA_NDIG) {
      u32 ex = inc - tc;
      for (u32 q = 0; q < w; ++q) ex += wsum[q];
      tstart[t] = ex;
      cnt[t] = tc;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < RL_ITEMS; ++it) {
      const u32 i = base + w * RL_SEG + it * WAVE + lane;
      if (i >= sb) continue;
      const u32 dd = dr[it] & 255u;
      const u32 slot = tstart[dd] + wc[w][dd] + (dr[it] >> 8);
      stg[slot] = rv[it];
      sdig[slot] = (u8)dd;
    }
    __syncthreads();
    if (RL_PF && base + RL_TILE < sb) load_tile(base + RL_TILE);  // in flight while this tile is written
    const u32 nv = min((u32)RL_TILE, sb - base);
    for (u32 j = t; j < nv; j += RL_NT) {
      const u32 dd = sdig[j];
      const u32 pos = run[dd] + (j - tstart[dd]);
      *(R16*)(rout + (u64)pos * RGA_REC) = stg[j];
    }
    __syncthreads();
    if (t < RGA_NDIG) run[t] += cnt[t];
  }
}

__device__ __forceinline__ u32 rga_lend(const u32* lstart, u32 l, i64 nl, i64 n) {
  return l + 1 < nl ? lstart[l + 1] : (u32)n;
}

// A list's survivor count, and its share of its chunk's sum: the RGA_CS_MAX chunk
// sums sit just before scnt (rga_layout); k_rga_out adds them up to its list's offset.
__device__ __forceinline__ void rga_put_count(u32* scnt, u32 l, u32 m) {
  scnt[l] = m;
  if (l < RGA_FUSED_MAX) atomicAdd(scnt - RGA_CS_MAX + (l / RGA_CS_LISTS), m);  // (more lists: scan_excl)
}

// Events ia, ib (stream indices) whose record words 0 are equal: the rest of the
// crdt.py:48-57 key -- t (signed), author, opid -- then the creation index.
__device__ __forceinline__ bool rga_key_lt(const smx_rga_ops& o, u32 ia, u32 ib) {
  const i64 ta = o.t[ia], tb = o.t[ib];
  if (ta != tb) return ta < tb;
  const u32 aa = o.author[ia], ab = o.author[ib];
  if (aa != ab) return aa < ab;
  const u64 ha = (u64)o.opid_hi[ia], hb = (u64)o.opid_hi[ib];
  if (ha != hb) return ha < hb;
  const u64 la = (u64)o.opid_lo[ia], lb = (u64)o.opid_lo[ib];
  if (la != lb) return la < lb;
  return ia < ib;
}

// record a before record b in (key, creation index) order
__device__ __forceinline__ bool rec_lt(const u64* a, const u64* b, const smx_rga_ops& o) {
  if (a[0] != b[0]) return a[0] < b[0];
  return rga_key_lt(o, (u32)a[RGA_WV] & RGA_IDX_MASK, (u32)b[RGA_WV] & RGA_IDX_MASK);
}

// ---------------------------------------------------------------------------
// Lists of at most RW_CAP events: one wave per list, no block barriers.  Lane x owns
// the list's events x, x + 64, ... (K = ceil(cnt / 64) of them; the partition keeps
// each list's events in stream order, so event position = creation order).
//  1. value groups by an LDS hash table (CAS insert, a member chain per group);
//  2. the lane that inserted a group's value replays the group in stream order
//     (crdt.py:29-43);
//  3. the survivors, compacted, ordered by key word 0 with an in-register bitonic
//     network (DPP / swizzle lane exchanges); runs of equal word 0 are re-sorted on
//     the rest of the key and the index (crdt.py:45-57).
#define RW_CAP 256   // k_rga_wave; the deferred lists' kernel takes up to 2 * RW_CAP
#define RW_WAVES 2   // lists per block
#ifndef RW_PER_CU
#define RW_PER_CU 16  // k_rga_wave workgroups per CU (persistent; 0: one wave per list)
#endif
#define RW_EMPTY 0xffffffffu
#define RW_NIL 0xffffu
#define RW_DEAD 0x400u
#define RW_MOP 12       // member entries: event | op << RW_MOP
#define RW_MEV 0xfffu
#ifndef RW_HT1
#define RW_HT1 1
#endif
#ifndef RW_H16
#define RW_H16 1  // 16-bit group counts / bases (a list has at most 2 * RW_CAP events): less LDS per wave
#endif
#if RW_H16
#define RW_HT u16
#else
#define RW_HT u32
#endif
#ifndef RW_OCC_W
#define RW_OCC_W 8  // k_rga_wave: registers for this many waves per SIMD (0: compiler's choice)
#endif
#if RW_OCC_W
#define RW_OCC __attribute__((amdgpu_waves_per_eu(RW_OCC_W, RW_OCC_W)))
#else
#define RW_OCC
#endif
#ifndef RW_LAUNDER
#define RW_LAUNDER 1
#endif
#ifndef RW_RREG
#define RW_RREG 0  // 1: groups of 2-4 events replayed in registers (list kernel 199 -> 204 us: off)
#endif
#ifndef RW_PINS_K
#define RW_PINS_K 16  // lists of K >= this: a lane's K hash inserts probed together (off: for
                      // k_rga_wave's K = 4 0.563 -> 0.576 ms; k_rga_wave2's K = 8 26.9 us either way)
#endif
#ifndef RW_W0R
#define RW_W0R 1  // word 0 of a lane's own events kept in registers for the survivors' keys
#endif
#ifndef RW_MGP_UNION
#define RW_MGP_UNION 1  // mem / gp share LDS: 9.5 KB per two-list workgroup, 16 per CU
#endif
#ifndef RW_W0G
#define RW_W0G 1  // key word 0 read from the list's records in L2, not held in LDS: 2 KB less per list, more lists per CU
#endif
#ifndef RW_ABL
#define RW_ABL 0  // timing ablations (wrong results): bit0 no replay, bit1 no grouping / replay,
                  // bit2 no key order, bit3 load only
#endif


#ifndef RW_XV
#define RW_XV 0  // 1: exchanges on the VALU only (DPP, permlane swaps): measured 0.560 -> 0.57 ms, off
#endif
// v from lane ^ lm (lm a constant after unrolling): DPP for 1, 2, 3, 7, 15, a swizzle
// within 32 lanes for 4, 8, 16, 31, a permute otherwise.
__device__ __forceinline__ u32 xor32_swap(u32 v) {  // lane ^ 32 (v_permlane32_swap: VALU)
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return __lane_id() < 32 ? r[1] : r[0];
}
__device__ __forceinline__ u32 xor16_swap(u32 v) {  // lane ^ 16 (v_permlane16_swap: VALU)
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return __lane_id() & 16 ? r[0] : r[1];
}

__device__ __forceinline__ u32 xshfl(u32 v, u32 lm) {
#if RW_XV  // every exchange on the VALU (DPP, permlane swaps): no LDS-unit round trips
  switch (lm) {
    case 1: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    case 2: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    case 3: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x1B, 0xF, 0xF, false);
    case 7: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    case 15: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    case 4: {  // ^7 (row half mirror) then ^3 (quad perm 3,2,1,0)
      const u32 x = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
      return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x1B, 0xF, 0xF, false);
    }
    case 8: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    case 16: return xor16_swap(v);
    case 31: return (u32)__builtin_amdgcn_update_dpp(0, (int)xor16_swap(v), 0x140, 0xF, 0xF, false);
    case 32: return xor32_swap(v);
    case 63: return (u32)__builtin_amdgcn_update_dpp(0, (int)xor16_swap(xor32_swap(v)), 0x140, 0xF, 0xF, false);
    default: return (u32)__shfl_xor((int)v, (int)lm);
  }
#endif
  switch (lm) {
    case 1: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    case 2: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    case 3: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x1B, 0xF, 0xF, false);
    case 7: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    case 15: return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    case 4: return (u32)__builtin_amdgcn_ds_swizzle((int)v, (4 << 10) | 0x1f);
    case 8: return (u32)__builtin_amdgcn_ds_swizzle((int)v, (8 << 10) | 0x1f);
    case 16: return (u32)__builtin_amdgcn_ds_swizzle((int)v, (16 << 10) | 0x1f);
    case 31: return (u32)__builtin_amdgcn_ds_swizzle((int)v, (31 << 10) | 0x1f);
    default: return (u32)__shfl_xor((int)v, (int)lm);
  }
}

// Ascending bitonic network (all-ascending form: the first step of each merge compares
// e with its mirror e ^ (kk - 1)) over 64 * K (key, payload) pairs, e = k * 64 + lane;
// the partner of (lane, k) under mask m is (lane ^ (m & 63), k ^ (m >> 6)).  Steps are
// template-expanded so every exchange pattern is a constant.
template <int K, u32 KK, u32 J>
__device__ __forceinline__ void wave_bitonic_step(u64 (&key)[8], u32 (&pay)[8], u32 lane) {
  constexpr u32 mask = J == (KK >> 1) ? KK - 1 : J;
  constexpr u32 lm = mask & 63u, sm = mask >> 6;
  u64 nk[K];
  u32 np[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int src = k ^ (int)sm;
    u64 ok = key[src];
    u32 op = pay[src];
    if (lm) {
      ok = ((u64)xshfl((u32)(ok >> 32), lm) << 32) | xshfl((u32)ok, lm);
      op = xshfl(op, lm);
    }
    const bool lower = (((u32)k * 64u + lane) & J) == 0;
    const bool take = lower ? ok < key[k] : key[k] < ok;
    nk[k] = take ? ok : key[k];
    np[k] = take ? op : pay[k];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    key[k] = nk[k];
    pay[k] = np[k];
  }
  if constexpr (J > 1) wave_bitonic_step<K, KK, (J >> 1)>(key, pay, lane);
}

template <int K, u32 KK = 2>
__device__ __forceinline__ void wave_bitonic(u64 (&key)[8], u32 (&pay)[8], u32 lane) {
  wave_bitonic_step<K, KK, (KK >> 1)>(key, pay, lane);
  if constexpr (KK < 64u * K) wave_bitonic<K, KK * 2>(key, pay, lane);
}

// The same network over 64 * K packed 32-bit keys (rank fields above the event bits).
template <int K, u32 KK, u32 J>
__device__ __forceinline__ void wave_bitonic32_step(u32 (&key)[8], u32 lane) {
  constexpr u32 mask = J == (KK >> 1) ? KK - 1 : J;
  constexpr u32 lm = mask & 63u, sm = mask >> 6;
  u32 nk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    u32 ok = key[k ^ (int)sm];
    if (lm) ok = xshfl(ok, lm);
    const bool lower = (((u32)k * 64u + lane) & J) == 0;
    nk[k] = lower ? min(ok, key[k]) : max(ok, key[k]);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) key[k] = nk[k];
  if constexpr (J > 1) wave_bitonic32_step<K, KK, (J >> 1)>(key, lane);
}

template <int K, u32 KK = 2>
__device__ __forceinline__ void wave_bitonic32(u32 (&key)[8], u32 lane) {
  wave_bitonic32_step<K, KK, (KK >> 1)>(key, lane);
  if constexpr (KK < 64u * K) wave_bitonic32<K, KK * 2>(key, lane);
}

#ifndef RW_PACK
#define RW_PACK 1  // survivors' keys packed to 32 bits when the list's ranges allow (see rw_order)
#endif

template <int CAP>
struct RwLds {
  static constexpr int cap = CAP;
  // hash slots: one per event for k_rga_wave's lists (RW_HT1: 7.4 KB of LDS per list, five
  // waves per SIMD; a full table still terminates, every value finds its slot), two
  // per event otherwise
  static constexpr int HT = (RW_HT1 && CAP == RW_CAP) ? CAP : 2 * CAP;
#if !RW_W0G
  u64 w0[CAP];          // key word 0 of each event (words 1-3 stay in global memory / L2)
#endif
  u64 wv[CAP];          // value << 32 | op << 30 | index (record word RGA_WV)
  union {
    struct {
      u32 hkey[HT];     // the slot's value, RW_EMPTY
      RW_HT hcnt[HT];   // members of the slot's group
      RW_HT hbase[HT];  // first member position (exclusive scan of hcnt)
    } h;
    u64 gs[CAP];        // step 3: survivors' word 0, sorted
  };
#if RW_MGP_UNION
  union {               // (mem is dead once the groups are replayed)
#else
  struct {
#endif
    u16 mem[CAP];       // group members, group by group, each in event order (| op << RW_MOP)
    u16 gp[CAP];        // step 3: survivors' events, sorted
  };
  u8 st[CAP];           // bit0 present, bit1 tombstoned
};

// Where a list kernel reads its events' record words (event e of the list at s0):
//  RecSrc  the partitioned 16-byte records
//  ColSrc  the input columns themselves (SMX_RGA_GROUPED: event s0 + e is the list's e-th
//          event, so word 0 = anchor << 32 | t' >> 32 and word 1 = value << 32 | op << 30 |
//          index are built at the load, no record pass)
struct RecSrc {
  const u64* p;  // the list's first record
  __device__ __forceinline__ u64 w0(u32 e) const { return p[(u64)e * RGA_REC]; }
  __device__ __forceinline__ u64 w1(u32 e) const { return p[(u64)e * RGA_REC + RGA_WV]; }
};
struct ColSrc {
  const u32* anchor;
  const i64* t;
  const u32* value;
  const u8* op;
  u32 s0;
  __device__ __forceinline__ u64 w0(u32 e) const {
    const u32 j = s0 + e;
    return ((u64)anchor[j] << 32) | (((u64)t[j] ^ 0x8000000000000000ull) >> 32);
  }
  __device__ __forceinline__ u64 w1(u32 e) const {
    const u32 j = s0 + e, op3 = op[j];
    return ((u64)value[j] << 32) | ((op3 > 2 ? 0u : op3) << 30) | j;
  }
};

// Event a before event b of one list in (key, index) order (crdt.py:48-57): word 0
// from LDS, the rest from the input columns by stream index (rare: equal word 0).
template <class LDS, class SRC>
__device__ __forceinline__ bool ev_lt(const LDS& S, const SRC& src, const smx_rga_ops& o, u32 a,
                                      u32 b) {
#if RW_W0G
  const u64 wa = src.w0(a), wb = src.w0(b);  // (the list's records or columns, L2-resident)
#else
  const u64 wa = S.w0[a], wb = S.w0[b];
#endif
  if (wa != wb) return wa < wb;
  return rga_key_lt(o, (u32)S.wv[a] & RGA_IDX_MASK, (u32)S.wv[b] & RGA_IDX_MASK);
}

// Step 3 over the survivors' (word 0, event) pairs held K2 per lane.
template <int K2, class LDS, class SRC>
__device__ __forceinline__ void rw_order(LDS& S, const SRC& src, const smx_rga_ops& o, u64 (&key)[8],
                                         u32 (&pay)[8], u32 m,
                                         u32 s0, u32 lane, u32* __restrict__ tmp_v, u32* __restrict__ tmp_s) {
  constexpr u32 N = 64u * K2;
  bool packed = false;
#if RW_PACK
  {  // word 0 = anchor << 32 | t's top half.  When the survivors' anchor and t ranges fit
     // beside the event bits in 31 bits, sort (anchor - min, t - min, event) as one u32:
     // one lane exchange and a min / max per step instead of three exchanges and selects.
     // Equal packed fields <=> equal word 0, so the tie runs below are the same.
    constexpr u32 PB = LDS::cap <= 256 ? 8 : 9;  // event bits
    u32 amx = 0, anx = 0, tmx = 0, tnx = 0;
#pragma unroll
    for (int k = 0; k < K2; ++k)
      if ((u32)k * 64u + lane < m) {
        const u32 a = (u32)(key[k] >> 32), t = (u32)key[k];
        amx = max(amx, a);
        anx = max(anx, ~a);
        tmx = max(tmx, t);
        tnx = max(tnx, ~t);
      }
    amx = (u32)__builtin_amdgcn_readlane((int)wave_incl_max_u32(amx), WAVE - 1);
    anx = (u32)__builtin_amdgcn_readlane((int)wave_incl_max_u32(anx), WAVE - 1);
    tmx = (u32)__builtin_amdgcn_readlane((int)wave_incl_max_u32(tmx), WAVE - 1);
    tnx = (u32)__builtin_amdgcn_readlane((int)wave_incl_max_u32(tnx), WAVE - 1);
    const u32 amin = ~anx, tmin = ~tnx;
    const u32 ba = 32u - (u32)__clz((int)(amx - amin)), bt = 32u - (u32)__clz((int)(tmx - tmin));
    if (m > 0 && ba + bt + PB <= 31u) {
      packed = true;
      u32 pk[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) pk[k] = ~0u;
#pragma unroll
      for (int k = 0; k < K2; ++k)
        if ((u32)k * 64u + lane < m)
          pk[k] = (((u32)(key[k] >> 32) - amin) << (bt + PB)) | (((u32)key[k] - tmin) << PB) | pay[k];
      wave_bitonic32<K2>(pk, lane);
#pragma unroll
      for (int k = 0; k < K2; ++k) {
        const bool v = (u32)k * 64u + lane < m;
        key[k] = v ? (u64)(pk[k] >> PB) : ~0ull;
        pay[k] = v ? pk[k] & ((1u << PB) - 1u) : RW_DEAD;
      }
    }
  }
#endif
  if (!packed) wave_bitonic<K2>(key, pay, lane);
#pragma unroll
  for (int k = 0; k < K2; ++k) {
    const u32 q = (u32)k * 64u + lane;
    S.gs[q] = key[k];
    S.gp[q] = (u16)pay[k];
  }
  wave_lds_sync();
  auto tail_lt = [&](u32 b, u32 a) {  // events b, a with equal word 0; dead ones last
    if ((a | b) & RW_DEAD) return (a & RW_DEAD) && !(b & RW_DEAD);
    return ev_lt(S, src, o, b, a);
  };
#pragma unroll
  for (int k = 0; k < K2; ++k) {
    const u32 q = (u32)k * 64u + lane;
    if (q < m && q + 1 < N && S.gs[q + 1] == key[k] && (q == 0 || S.gs[q - 1] != key[k])) {
      u32 e = q + 2;  // the run [q, e) of equal word 0: insertion sort on the rest
      while (e < N && S.gs[e] == key[k]) ++e;
      for (u32 x = q + 1; x < e; ++x) {
        const u32 v = S.gp[x];
        u32 y = x;
        while (y > q && tail_lt(v, S.gp[y - 1])) {
          S.gp[y] = S.gp[y - 1];
          --y;
        }
        S.gp[y] = (u16)v;
      }
    }
  }
  wave_lds_sync();
  for (u32 q = lane; q < m; q += WAVE) {
    const u32 e = S.gp[q] & (RW_DEAD - 1);
    const u64 w = S.wv[e];
    tmp_v[s0 + q] = (u32)(w >> 32);
    tmp_s[s0 + q] = ((u32)w & RGA_IDX_MASK) | (S.st[e] & 2 ? RGA_TOMB_BIT : 0u);
  }
}

// tomb: list mode (crdt.py RGA.list) -- the tombstoned elements stay, flagged
// Returns the list's survivor count (wave-uniform); scnt[l] is the caller's to write.
template <int K, int CAP, class SRC>
__device__ __forceinline__ u32 rga_wave_list(const smx_rga_ops& o, const SRC src, u32 l, u32 s0, u32 cnt,
                                              RwLds<CAP>& S, u32 lane, bool tomb,
                                              u32* __restrict__ tmp_v, u32* __restrict__ tmp_s,
                                              u32* __restrict__ scnt) {
  static_assert(RW_W0R, "the record words come through src.w0 / src.w1");
#if RW_W0R
  u64 w0r[K];  // word 0 of this lane's events k * 64 + lane, kept for step 3
  {  // every load in flight at once; word 1 of each event to LDS
    u64 wvr[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const u32 e = (u32)k * 64u + lane;
      w0r[k] = e < cnt ? src.w0(e) : ~0ull;
      wvr[k] = e < cnt ? src.w1(e) : 0ull;
    }
    for (u32 t = lane; t < RwLds<CAP>::HT; t += WAVE) {
      S.h.hkey[t] = RW_EMPTY;
      S.h.hcnt[t] = 0;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const u32 e = (u32)k * 64u + lane;
      if (e < cnt) S.wv[e] = wvr[k];
    }
  }
#else
  {  // every load in flight at once; words 0 and 4 of each event to LDS
    u64 v[RGA_REC * K];
#pragma unroll
    for (int i = 0; i < RGA_REC * K; ++i) {
      const u32 x = lane + (u32)i * WAVE;
      v[i] = x < cnt * RGA_REC ? (x % RGA_REC ? src.w1(x / RGA_REC) : src.w0(x / RGA_REC)) : 0ull;
    }
    for (u32 t = lane; t < RwLds<CAP>::HT; t += WAVE) {
      S.h.hkey[t] = RW_EMPTY;
      S.h.hcnt[t] = 0;
    }
#pragma unroll
    for (int i = 0; i < RGA_REC * K; ++i) {
      const u32 x = lane + (u32)i * WAVE;
      const u32 e = x / RGA_REC, wd = x - e * RGA_REC;
      if (x < cnt * RGA_REC) {
#if !RW_W0G
        if (wd == 0) S.w0[e] = v[i];
#endif
        if (wd == RGA_WV) S.wv[e] = v[i];
      }
    }
  }
#endif
  wave_lds_sync();
  if (RW_ABL & 8) return (u32)__builtin_amdgcn_readfirstlane((int)((u32)S.wv[lane] & 1u));
  const u64 lt = lane ? ~0ull >> (WAVE - lane) : 0ull;  // (from `lane`: see k_rga_wave)
  constexpr int HB = RwLds<CAP>::HT == 256 ? 8 : RwLds<CAP>::HT == 512 ? 9 : 10;  // log2 of the hash slots
  static_assert(RwLds<CAP>::HT == 1 << HB, "hash slots");
  u32 slot[8], rk[8], opk[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) slot[k] = rk[k] = opk[k] = 0;
  if (RW_ABL & 2) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const u32 e = (u32)k * 64u + lane;
      S.st[e] = e < cnt && ((u32)(S.wv[e] >> 30) & 3u) != 2;
    }
  } else {
    // 1. value groups: each event's value into the hash table (CAS), its rank among
    //    the group's events (match within the wave, running counts across slots),
    //    then the groups laid out contiguously, each in event order
    if constexpr (K >= RW_PINS_K) {
    {  // all K of a lane's events probe together: one round of K CASes in flight per
       // step instead of K dependent probe chains (the slot a group lands in does not
       // matter; its members' order comes from the ranks below)
      u32 v[K], pend = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const u32 e = (u32)k * 64u + lane;
        S.st[e] = 0;
        v[k] = 0;
        if (e < cnt) {
          const u64 wv = S.wv[e];
          v[k] = (u32)(wv >> 32);
          opk[k] = (u32)(wv >> 30) & 3u;
          slot[k] = (v[k] * 0x9E3779B1u) >> (32 - HB);
          pend |= 1u << k;
        }
      }
      while (__ballot(pend != 0)) {
        u32 old[K];
#pragma unroll
        for (int k = 0; k < K; ++k) old[k] = (pend >> k) & 1u ? atomicCAS(&S.h.hkey[slot[k]], RW_EMPTY, v[k]) : 0u;
#pragma unroll
        for (int k = 0; k < K; ++k)
          if ((pend >> k) & 1u) {
            if (old[k] == RW_EMPTY || old[k] == v[k])
              pend &= ~(1u << k);
            else
              slot[k] = (slot[k] + 1) & (RwLds<CAP>::HT - 1);
          }
      }
    }
    } else {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const u32 e = (u32)k * 64u + lane;
      S.st[e] = 0;
      if (e < cnt) {
        const u64 wv = S.wv[e];
        const u32 v = (u32)(wv >> 32);
        opk[k] = (u32)(wv >> 30) & 3u;
        u32 h = (v * 0x9E3779B1u) >> (32 - HB);
        for (;;) {
          const u32 old = atomicCAS(&S.h.hkey[h], RW_EMPTY, v);
          if (old == RW_EMPTY || old == v) break;
          h = (h + 1) & (RwLds<CAP>::HT - 1);
        }
        slot[k] = h;
      }
    }
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const u32 e = (u32)k * 64u + lane;
      const bool valid = e < cnt;
      const u64 peers = wave_peers<HB>(slot[k], valid);
      const u32 base = valid ? S.h.hcnt[slot[k]] : 0u;
      rk[k] = base + (u32)__popcll(peers & lt);
      wave_lds_sync();
      if (valid && (peers & lt) == 0) S.h.hcnt[slot[k]] = (RW_HT)(base + (u32)__popcll(peers));
      wave_lds_sync();
    }
    {  // exclusive scan of the group sizes, HT / 64 slots per lane
      constexpr int PL = RwLds<CAP>::HT / WAVE;
      u32 c[PL], tot = 0;
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        c[i] = S.h.hcnt[lane * PL + i];
        tot += c[i];
      }
      u32 run = wave_incl_sum(tot) - tot;
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        S.h.hbase[lane * PL + i] = (RW_HT)run;
        run += c[i];
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const u32 e = (u32)k * 64u + lane;
      if (e < cnt) S.mem[S.h.hbase[slot[k]] + rk[k]] = (u16)(e | opk[k] << RW_MOP);  // event, op
    }
    wave_lds_sync();
    // 2. the group's first event's lane replays the group in event order (crdt.py:29-43)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const u32 e = (u32)k * 64u + lane;
      if (e >= cnt || rk[k] != 0) continue;
      const u32 b = S.h.hbase[slot[k]], c = S.h.hcnt[slot[k]];
      if (c == 1 || (RW_ABL & 1)) {
        S.st[e] = opk[k] != 2;
        continue;
      }
#if RW_RREG
      if (c <= 4) {  // small groups (most of them) replayed in registers: the members'
                     // entries read at once, no chain of dependent LDS reads.  A move
                     // with two live candidates (their list order needs the keys) takes
                     // the general loop below instead.
        u32 xm[4], sv[4] = {0u, 0u, 0u, 0u};
        bool hard = false;
#pragma unroll
        for (int i = 0; i < 4; ++i) xm[i] = (u32)i < c ? S.mem[b + i] : 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if ((u32)i >= c) break;
          const u32 op = xm[i] >> RW_MOP;
          if (op == 2) {  // delete: every present element is tombstoned
#pragma unroll
            for (int j = 0; j < i; ++j) sv[j] |= (sv[j] & 1u) << 1;
            continue;
          }
          if (op == 1) {  // move: pops the live element (the only one here)
            u32 cand = 0;
#pragma unroll
            for (int j = 0; j < i; ++j) cand |= (u32)(sv[j] == 1u) << j;
            if (cand & (cand - 1)) {
              hard = true;
              break;
            }
#pragma unroll
            for (int j = 0; j < i; ++j)
              if ((cand >> j) & 1u) sv[j] = 0u;
          }
          sv[i] = 1u;
        }
        if (!hard) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if ((u32)i < c) S.st[xm[i] & RW_MEV] = (u8)sv[i];
          continue;
        }
      }
#endif
      for (u32 i = 0; i < c; ++i) {
        const u32 xm = S.mem[b + i];
        const u32 x = xm & RW_MEV, op = xm >> RW_MOP;
        if (op == 2) {  // delete: every present element is tombstoned; creates nothing
          for (u32 j = 0; j < i; ++j) {
            const u32 y = S.mem[b + j] & RW_MEV;
            if (S.st[y] & 1) S.st[y] |= 2;
          }
          continue;
        }
        if (op == 1) {  // move: pops the live element first in list order
          u32 best = RW_NIL;
#if RW_W0G
          u64 wb = 0;  // best's word 0: read when a second candidate shows up, then kept
          bool wbl = false;
          for (u32 j = 0; j < i; ++j) {
            const u32 y = S.mem[b + j] & RW_MEV;
            if (S.st[y] != 1) continue;
            if (best == RW_NIL) {
              best = y;
              continue;
            }
            if (!wbl) {
              wb = src.w0(best);
              wbl = true;
            }
            const u64 wy = src.w0(y);
            if (wy < wb ||
                (wy == wb && rga_key_lt(o, (u32)S.wv[y] & RGA_IDX_MASK, (u32)S.wv[best] & RGA_IDX_MASK))) {
              best = y;
              wb = wy;
            }
          }
#else
          for (u32 j = 0; j < i; ++j) {
            const u32 y = S.mem[b + j] & RW_MEV;
            if (S.st[y] == 1 && (best == RW_NIL || ev_lt(S, src, o, y, best))) best = y;
          }
#endif
          if (best != RW_NIL) S.st[best] = 0;
        }
        S.st[x] = 1;
      }
    }
  }
  wave_lds_sync();
  // 3. survivors (event order) -> K2 (word 0, event) pairs per lane, ordered by key
  u32 m = 0;
  u64 key[8];
  u32 pay[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    key[k] = ~0ull;
    pay[k] = RW_DEAD;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const u32 e = (u32)k * 64u + lane;
    const bool live = e < cnt && (tomb ? (S.st[e] & 1) != 0 : S.st[e] == 1);
    const u64 ball = __ballot(live);
    if (live) {
      const u32 q = m + (u32)__popcll(ball & lt);
      S.gp[q] = (u16)e;
#if RW_W0R
      S.gs[q] = w0r[k];  // (the hash table under gs is dead after step 2)
#endif
    }
    m += (u32)__popcll(ball);
  }
  wave_lds_sync();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const u32 a = (u32)k * 64u + lane;
    if (a < m) {
      pay[k] = S.gp[a];
#if RW_W0R
      key[k] = S.gs[a];
#elif RW_W0G
      key[k] = src.w0(pay[k]);
#else
      key[k] = S.w0[pay[k]];
#endif
    }
  }
  wave_lds_sync();  // gp / the hash table are rewritten below
  if (RW_ABL & 4) {
    for (u32 q = lane; q < m; q += WAVE) {
      const u64 w = S.wv[S.gp[q]];
      tmp_v[s0 + q] = (u32)(w >> 32);
      tmp_s[s0 + q] = (u32)w & RGA_IDX_MASK;
    }
  } else if (m <= 64) {
    rw_order<1>(S, src, o, key, pay, m, s0, lane, tmp_v, tmp_s);
  } else if (m <= 128) {
    rw_order<2>(S, src, o, key, pay, m, s0, lane, tmp_v, tmp_s);
  } else if (K <= 4 || m <= 256) {
    rw_order<(K <= 4 ? K : 4)>(S, src, o, key, pay, m, s0, lane, tmp_v, tmp_s);
  } else {
    rw_order<8>(S, src, o, key, pay, m, s0, lane, tmp_v, tmp_s);
  }
  return m;
}

template <bool DIRECT>
__global__ void __launch_bounds__(WAVE * RW_WAVES) RW_OCC k_rga_wave(smx_rga_ops o, const u64* __restrict__ R,
                                                             const u32* __restrict__ lstart,
                                                             i64 n, i64 nl, u32* __restrict__ tmp_v,
                                                             u32* __restrict__ tmp_s, u32* __restrict__ scnt,
                                                             int tomb, const i32* __restrict__ gate) {
  __shared__ RwLds<RW_CAP> lds[RW_WAVES];
  if (*gate & RGA_E_UNGROUPED) return;  // (a grouped call whose list ids decrease: redone partitioned)
  const u32 lane = threadIdx.x & (WAVE - 1);
  // the wave index as a scalar: the list index, its bounds and the slice base stay in
  // SGPRs (scalar loads of lstart; LDS member offsets fold into the instructions)
  const u32 w = (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
  // persistent (RW_PER_CU workgroups per CU): each wave takes a contiguous range of
  // lists and adds its survivors into the 256-list chunk sums once per chunk (one device
  // atomic per list on a shared chunk word serialized the waves, and the next list's
  // loads waited for it)
  const u32 nw = gridDim.x * RW_WAVES, wid = blockIdx.x * RW_WAVES + w;
  const u32 per = (u32)((nl + nw - 1) / nw);
  const u32 L0 = min((u64)wid * per, (u64)nl), L1 = min((u64)L0 + per, (u64)nl);
  u32 acc = 0;
  for (u32 l = L0; l < L1; ++l) {
    const u32 s0 = lstart[l], cnt = rga_lend(lstart, l, nl, n) - s0;
    if (cnt <= RW_CAP) {  // (longer lists: k_rga_wave2 / k_rga_big count themselves)
      // the lane id laundered per list: otherwise the compiler hoists every lane-derived
      // constant of the list code out of the loop and keeps it live
      u32 ln = lane;
      if (RW_LAUNDER) asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
      u32 m;
      auto run = [&](auto src) {
        if (cnt <= 64) return rga_wave_list<1>(o, src, l, s0, cnt, lds[w], ln, tomb != 0, tmp_v, tmp_s, scnt);
        if (cnt <= 128) return rga_wave_list<2>(o, src, l, s0, cnt, lds[w], ln, tomb != 0, tmp_v, tmp_s, scnt);
        return rga_wave_list<4>(o, src, l, s0, cnt, lds[w], ln, tomb != 0, tmp_v, tmp_s, scnt);
      };
      if constexpr (DIRECT) m = run(ColSrc{o.anchor, o.t, o.value, o.op, s0});
      else m = run(RecSrc{R + (u64)s0 * RGA_REC});
      if (lane == 0) scnt[l] = m;
      acc += m;
      wave_lds_sync();  // the next list reuses the slice
    }
    if ((l + 1) % RGA_CS_LISTS == 0 || l + 1 == L1) {
      if (lane == 0 && acc && l < RGA_FUSED_MAX) atomicAdd(scnt - RGA_CS_MAX + l / RGA_CS_LISTS, acc);
      acc = 0;
    }
  }
}

// Lists of RW_CAP + 1 .. 2 * RW_CAP events: the same wave per list with twice the
// slots; longer ones go on to k_rga_big.  Each wave sweeps 64 lists at a time for the
// long ones itself (k_rga_wave skips them; no hand-off list).
__global__ void __launch_bounds__(WAVE * RW_WAVES) k_rga_wave2(smx_rga_ops o, const u64* __restrict__ R,
                                                              const u32* __restrict__ lstart,
                                                              i64 n, i64 nl, u32* __restrict__ defer,
                                                              u32* __restrict__ ndefer, u32* __restrict__ tmp_v,
                                                              u32* __restrict__ tmp_s, u32* __restrict__ scnt,
                                                              int tomb, const i32* __restrict__ gate, int direct) {
  __shared__ RwLds<2 * RW_CAP> lds[RW_WAVES];
  if (*gate & RGA_E_UNGROUPED) return;
  const u32 lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  const u64 nw = (u64)gridDim.x * RW_WAVES;
  for (u64 l0 = ((u64)blockIdx.x * RW_WAVES + w) * WAVE; l0 < (u64)nl; l0 += nw * WAVE) {
    const u64 me = l0 + lane;
    const u32 c = me < (u64)nl ? rga_lend(lstart, (u32)me, nl, n) - lstart[me] : 0u;
    u64 todo = __ballot(c > RW_CAP);
    while (todo) {
      const u32 l = (u32)(l0 + (u64)(__ffsll((unsigned long long)todo) - 1));
      todo &= todo - 1;
      const u32 s0 = lstart[l], cnt = rga_lend(lstart, l, nl, n) - s0;
      if (direct) {  // grouped events, no partition: this long list's records from the columns
        const ColSrc cs{o.anchor, o.t, o.value, o.op, s0};
        u64* rw = const_cast<u64*>(R) + (u64)s0 * RGA_REC;
        for (u32 e = lane; e < cnt; e += WAVE) {
          R16 r;
          r.a = cs.w0(e);
          r.b = cs.w1(e);
          *reinterpret_cast<R16*>(rw + (u64)e * RGA_REC) = r;
        }
        __threadfence_block();  // (this wave reads them back; k_rga_big after this kernel)
      }
      if (cnt > 2 * RW_CAP) {
        if (lane == 0) defer[atomicAdd(ndefer, 1u)] = l;
        continue;
      }
      const u32 m = rga_wave_list<8>(o, RecSrc{R + (u64)s0 * RGA_REC}, l, s0, cnt, lds[w], lane, tomb != 0, tmp_v, tmp_s, scnt);
      if (lane == 0) rga_put_count(scnt, l, m);
      wave_lds_sync();  // the next list reuses the slice
    }
  }
}

// Block-wide sort of the record positions p[0..cnt) by `less`, in global memory:
// the bitonic network in its all-ascending form (first stage of each merge compares
// i with its mirror i ^ (k - 1)), so positions past cnt act as +infinity and are
// never touched.
template <typename Less>
__device__ void block_sort_positions(u32* p, u32 cnt, Less less) {
  u32 P = 1;
  while (P < cnt) P <<= 1;
  for (u32 k = 2; k <= P; k <<= 1) {
    for (u32 j = k >> 1; j > 0; j >>= 1) {
      const u32 mask = j == (k >> 1) ? k - 1 : j;
      for (u32 i = threadIdx.x; i < P; i += blockDim.x) {
        const u32 q = i ^ mask;
        if (q > i && q < cnt && less(p[q], p[i])) {
          const u32 x = p[i];
          p[i] = p[q];
          p[q] = x;
        }
      }
      __syncthreads();
    }
  }
}

// Lists longer than 2 * RW_CAP: the same replay from global memory, one block per list
// (such lists are rare — a whole file's history in one list).  Per list, in its
// record range: gp = positions sorted by (value, index), bst = state by that order;
// then the survivors' positions sorted by (key, index).
__device__ void rga_big_list(const smx_rga_ops& o, const u64* __restrict__ R, u32 l, const u32* __restrict__ lstart, i64 n, i64 nl,
                             u8* __restrict__ bst, u32* __restrict__ gp, u32* __restrict__ tmp_v,
                             u32* __restrict__ tmp_s, u32* __restrict__ scnt, bool tomb) {
  __shared__ u32 ns;
  const u32 t = threadIdx.x, NT = blockDim.x;
  const u32 s0 = lstart[l], cnt = rga_lend(lstart, l, nl, n) - s0;
  const u64* L = R + (u64)s0 * RGA_REC;
  u8* S = bst + s0;
  u32* G = gp + s0;
  auto gkey = [&](u32 x) { const u64 w = L[x * RGA_REC + RGA_WV]; return ((w >> 32) << 30) | (w & RGA_IDX_MASK); };
  for (u32 x = t; x < cnt; x += NT) {
    G[x] = x;
    S[x] = 0;
  }
  __syncthreads();
  block_sort_positions(G, cnt, [&](u32 a, u32 b) { return gkey(a) < gkey(b); });
  for (u32 j = t; j < cnt; j += NT) {
    const u64 v = gkey(G[j]) >> 30;
    if (j != 0 && (gkey(G[j - 1]) >> 30) == v) continue;
    u32 end = j + 1;
    while (end < cnt && (gkey(G[end]) >> 30) == v) ++end;
    for (u32 x = j; x < end; ++x) {
      const u32 op = (u32)(L[G[x] * RGA_REC + RGA_WV] >> 30) & 3u;
      if (op == 2) {
        for (u32 y = j; y < x; ++y)
          if (S[y] & 1) S[y] |= 2;
        continue;
      }
      if (op == 1) {
        int best = -1;
        for (u32 y = j; y < x; ++y)
          if (S[y] == 1 && (best < 0 || rec_lt(&L[G[y] * RGA_REC], &L[G[best] * RGA_REC], o))) best = (int)y;
        if (best >= 0) S[best] = 0;
      }
      S[x] = 1;
    }
  }
  __syncthreads();
  // survivors' positions to the front of G (their order is fixed by the sort below);
  // the tombstone flag rides in bit 31 (positions < 2^30)
  if (t == 0) {
    u32 w = 0;
    for (u32 j = 0; j < cnt; ++j)
      if (tomb ? (S[j] & 1) : S[j] == 1) G[w++] = G[j] | (S[j] & 2 ? RGA_TOMB_BIT : 0u);
    ns = w;
  }
  __syncthreads();
  const u32 m = ns;
  block_sort_positions(G, m, [&](u32 a, u32 b) {
    return rec_lt(&L[(a & ~RGA_TOMB_BIT) * RGA_REC], &L[(b & ~RGA_TOMB_BIT) * RGA_REC], o);
  });
  for (u32 j = t; j < m; j += NT) {
    const u64 w = L[(G[j] & ~RGA_TOMB_BIT) * RGA_REC + RGA_WV];
    tmp_v[s0 + j] = (u32)(w >> 32);
    tmp_s[s0 + j] = ((u32)w & RGA_IDX_MASK) | (G[j] & RGA_TOMB_BIT);
  }
  if (t == 0) rga_put_count(scnt, l, m);
}

#ifndef RGA_BIG_GRID
#define RGA_BIG_GRID 32  // workgroups of k_rga_big (lists of > 2 RW_CAP events, one per workgroup at a time;
                         // 256 cost ~5 us of launch on every call, most of which have none)
#endif
__global__ void __launch_bounds__(1024) k_rga_big(smx_rga_ops o, const u64* __restrict__ R,
                                                  const u32* __restrict__ lstart, i64 n,
                                                  i64 nl, const u32* __restrict__ todo, const u32* __restrict__ ntodo,
                                                  u8* __restrict__ bst, u32* __restrict__ gp,
                                                  u32* __restrict__ tmp_v, u32* __restrict__ tmp_s,
                                                  u32* __restrict__ scnt, int tomb, const i32* __restrict__ gate) {
  if (*gate & RGA_E_UNGROUPED) return;
  for (u32 item = blockIdx.x; item < *ntodo; item += gridDim.x) {
    __syncthreads();
    rga_big_list(o, R, todo[item], lstart, n, nl, bst, gp, tmp_v, tmp_s, scnt, tomb != 0);
  }
}

// Per list (one wave each): its output offset = the survivor sums of the earlier chunks
// + the counts of the chunk's earlier lists (one 16-byte read of each per lane, a wave
// sum), then its survivors, in list order, to their place in the output.  The last
// list's wave writes the total.  n_lists <= RGA_FUSED_MAX.
// RGA_OUT_LPW consecutive lists per wave (one 256-list chunk): one offset sum serves
// them all (the next list's offset is this one's plus its count), and all their first
// survivors are read before it is known.
__global__ void __launch_bounds__(BLOCK) k_rga_out_fused(const u32* __restrict__ tmp_v, const u32* __restrict__ tmp_s,
                                                        const u32* __restrict__ lstart, const u32* __restrict__ scnt,
                                                        i64 nl, smx_rga_out out, const i32* __restrict__ gate) {
  constexpr int LPW = RGA_OUT_LPW;
  if (*gate & RGA_E_UNGROUPED) return;
  static_assert(RGA_CS_LISTS % LPW == 0, "a wave's lists share a chunk");
  const u32 lane = threadIdx.x & (WAVE - 1);
  const i64 l0 = ((i64)blockIdx.x * (BLOCK / WAVE) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE))) * LPW;
  if (l0 >= nl) return;
  const u32 c = (u32)l0 / RGA_CS_LISTS, c0 = c * RGA_CS_LISTS;
  const uint4 cs = reinterpret_cast<const uint4*>(scnt - RGA_CS_MAX)[lane];
  const uint4 ls = reinterpret_cast<const uint4*>(scnt + c0)[lane];
  u32 s0[LPW], m[LPW];
#pragma unroll
  for (int j = 0; j < LPW; ++j) {
    const bool v = l0 + j < nl;
    s0[j] = v ? lstart[l0 + j] : 0u;
    m[j] = v ? scnt[l0 + j] : 0u;
  }
  u32 pv[LPW][RGA_OUT_PRE], ps[LPW][RGA_OUT_PRE];
#pragma unroll
  for (int j = 0; j < LPW; ++j)
#pragma unroll
    for (int i = 0; i < RGA_OUT_PRE; ++i) {
      const u32 x = lane + (u32)i * WAVE;
      pv[j][i] = x < m[j] ? __builtin_nontemporal_load(&tmp_v[s0[j] + x]) : 0u;
      ps[j][i] = x < m[j] ? __builtin_nontemporal_load(&tmp_s[s0[j] + x]) : 0u;
    }
  const u32 q = 4 * lane;
  u32 part = (q < c ? cs.x : 0u) + (q + 1 < c ? cs.y : 0u) + (q + 2 < c ? cs.z : 0u) + (q + 3 < c ? cs.w : 0u);
  const u32 r = (u32)l0 - c0;
  part += (q < r ? ls.x : 0u) + (q + 1 < r ? ls.y : 0u) + (q + 2 < r ? ls.z : 0u) + (q + 3 < r ? ls.w : 0u);
  u32 d = (u32)__builtin_amdgcn_readlane((int)wave_incl_sum_u32(part), WAVE - 1);
#pragma unroll
  for (int j = 0; j < LPW; ++j) {
    if (l0 + j >= nl) break;
#pragma unroll
    for (int i = 0; i < RGA_OUT_PRE; ++i) {
      const u32 x = lane + (u32)i * WAVE;
      if (x >= m[j]) break;
      out.out_value[d + x] = pv[j][i];
      out.out_src[d + x] = (i32)(ps[j][i] & ~RGA_TOMB_BIT);
      if (out.out_tomb) out.out_tomb[d + x] = ps[j][i] & RGA_TOMB_BIT ? 1 : 0;
    }
    for (u32 x = lane + RGA_OUT_PRE * WAVE; x < m[j]; x += WAVE) {
      out.out_value[d + x] = __builtin_nontemporal_load(&tmp_v[s0[j] + x]);
      const u32 sx = __builtin_nontemporal_load(&tmp_s[s0[j] + x]);
      out.out_src[d + x] = (i32)(sx & ~RGA_TOMB_BIT);
      if (out.out_tomb) out.out_tomb[d + x] = sx & RGA_TOMB_BIT ? 1 : 0;
    }
    if (lane == 0) {
      out.out_offsets[l0 + j] = d;
      if (l0 + j == nl - 1) {
        out.out_offsets[nl] = d + m[j];
        out.counts[0] = d + m[j];
      }
    }
    d += m[j];
  }
}

// Per list (one wave each): its survivors, in list order, to their place in the output.
// (k_rga_out_fused: RGA_OUT_PRE loads per lane issued with the offset's loads)
__global__ void __launch_bounds__(BLOCK) k_rga_out(const u32* __restrict__ tmp_v, const u32* __restrict__ tmp_s,
                                                  const u32* __restrict__ lstart, const u32* __restrict__ scnt,
                                                  const u32* __restrict__ soff, i64 nl, smx_rga_out out,
                                                  const i32* __restrict__ gate) {
  if (*gate & RGA_E_UNGROUPED) return;
  const u32 lane = threadIdx.x & (WAVE - 1);
  const i64 l = (i64)blockIdx.x * (BLOCK / WAVE) + threadIdx.x / WAVE;
  if (l >= nl) return;
  const u32 s0 = lstart[l], m = scnt[l], d = soff[l];
  for (u32 x = lane; x < m; x += WAVE) {
    out.out_value[d + x] = __builtin_nontemporal_load(&tmp_v[s0 + x]);
    const u32 sx = __builtin_nontemporal_load(&tmp_s[s0 + x]);
    out.out_src[d + x] = (i32)(sx & ~RGA_TOMB_BIT);
    if (out.out_tomb) out.out_tomb[d + x] = sx & RGA_TOMB_BIT ? 1 : 0;
  }
  if (lane == 0) out.out_offsets[l] = d;
}

__global__ void k_rga_fin(const u32* __restrict__ soff_total, i64 n_lists, smx_rga_out out, const i32* __restrict__ gate) {
  if (*gate & RGA_E_UNGROUPED) return;
  out.out_offsets[n_lists] = *soff_total;
  out.counts[0] = *soff_total;
}

static int g_rr_grid = 0;  // persistent scatter grid (RR_PER_CU per CU of the device)
static int g_cus = 256;

static bool o_ok(const smx_rga_ops* o) {
  return o->list && o->op && o->value && o->anchor && o->t && o->author && o->opid_hi && o->opid_lo;
}

struct RgaLayout {
  size_t off[16];
  size_t total;
};

enum { R_REC, R_REC2, R_KEYS, R_KEYS2, R_RHIST, R_TV, R_TS, R_BST, R_GP, R_DEF2, R_PART, R_LSTART, R_SCNT, R_SOFF, R_N };

static RgaLayout rga_layout(i64 n, i64 nl) {
  const i64 nn = n > 0 ? n : 1;
  size_t sz[R_N];
  sz[R_REC] = sz[R_REC2] = (size_t)nn * RGA_REC * 8;
  sz[R_KEYS] = sz[R_KEYS2] = sz[R_TV] = sz[R_TS] = sz[R_GP] = (size_t)nn * 4;
  {
    const i64 nblk = SMX_CEIL_DIV(nn, (i64)RREC_TILE);
    sz[R_RHIST] = (size_t)256 * nblk * 4 + hscan_tsum_bytes(nblk, 256) + 260 * 4;
  }
  sz[R_BST] = (size_t)nn;
  sz[R_PART] = SCAN_NB * 8 + 64;  // + error word + totals
  sz[R_LSTART] = sz[R_SOFF] = sz[R_DEF2] = (size_t)(nl + 1) * 4;
  // scnt: RGA_CS_MAX chunk sums, then the counts padded to whole 256-list chunks
  sz[R_SCNT] = (size_t)(RGA_CS_MAX + SMX_CEIL_DIV(nl + 1, (i64)RGA_CS_LISTS) * RGA_CS_LISTS) * 4;
  RgaLayout L;
  size_t acc = 0;
  for (int i = 0; i < R_N; ++i) {
    L.off[i] = acc;
    acc += (sz[i] + 255) & ~(size_t)255;
  }
  L.total = acc;
  return L;
}

extern "C" int smx_rga_workspace_bytes(int64_t n_ops, int64_t n_lists, size_t* bytes) {
  if (!bytes || n_ops < 0 || n_lists < 0) return SMX_E_ARG;
  *bytes = rga_layout(n_ops, n_lists).total;
  return SMX_OK;
}

// Host wait for a stream: a short spin on hipStreamQuery, then the blocking sync.  A call
// ends within a millisecond, and a blocking sync wakes the calling thread ~10-20 us after
// the stream's last packet: 10M events 0.520 -> 0.502 ms, grouped 0.297 -> 0.287 ms
// (profiles/r05_x/spin_ab.txt).  The spin is adaptive per calling thread: twice the
// previous call's wait, between RGA_SPIN_MIN_US and RGA_SPIN_US (a long batch, or many
// caller threads, no longer burn a core for a fixed 20 ms; RGA_SPIN_US 0: block at once).
#ifndef RGA_SPIN_US
#define RGA_SPIN_US 2000
#endif
#ifndef RGA_SPIN_MIN_US
#define RGA_SPIN_MIN_US 200
#endif
static hipError_t stream_wait(hipStream_t st) {
  static thread_local long long last_us = RGA_SPIN_US / 2;  // this thread's previous wait
  if (RGA_SPIN_US > 0) {
    const long long budget = std::min<long long>(RGA_SPIN_US, std::max<long long>(RGA_SPIN_MIN_US, 2 * last_us));
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipStreamQuery(st);
      const long long us =
          std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
      if (e != hipErrorNotReady) {
        last_us = us;
        return e;
      }
      if (us > budget) break;
    }
    const hipError_t e = hipStreamSynchronize(st);
    last_us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    return e;
  }
  return hipStreamSynchronize(st);
}

static int rga_impl(const smx_rga_ops* ops, const smx_rga_out* out, void* ws, size_t wsb, hipStream_t st,
                    bool grouped) {
  const i64 n = ops->n_ops, nl = ops->n_lists;
  if (n < 0 || nl < 0 || n > (i64)RGA_IDX_MASK || nl >= (i64)0x7fffffff)
    return smx_set_error(SMX_E_ARG, "bad sizes");
  if (!out || !out->out_offsets || !out->counts) return smx_set_error(SMX_E_ARG, "null output");
  if (n == 0) {
    RGA_TRY(hipMemsetAsync(out->out_offsets, 0, (size_t)(nl + 1) * 8, st));
    RGA_TRY(hipMemsetAsync(out->counts, 0, 8, st));
    return SMX_OK;
  }
  if (nl < 1) return smx_set_error(SMX_E_ARG, "n_lists must be >= 1");
  if (!o_ok(ops)) return smx_set_error(SMX_E_ARG, "null input pointer");
  const RgaLayout L = rga_layout(n, nl);
  if (!ws || wsb < L.total)
    return smx_set_error(SMX_E_WORKSPACE, ("workspace too small: need " + std::to_string(L.total)).c_str());
  char* b = (char*)ws;
  u64* rec = (u64*)(b + L.off[R_REC]);
  u64* rec2 = (u64*)(b + L.off[R_REC2]);
  u32* keys = (u32*)(b + L.off[R_KEYS]);
  u32* keys2 = (u32*)(b + L.off[R_KEYS2]);
  u32* rhist = (u32*)(b + L.off[R_RHIST]);
  u32* tmp_v = (u32*)(b + L.off[R_TV]);
  u32* tmp_s = (u32*)(b + L.off[R_TS]);
  u8* bst = (u8*)(b + L.off[R_BST]);
  u32* gp = (u32*)(b + L.off[R_GP]);
  u32* part = (u32*)(b + L.off[R_PART]);
  i32* err = (i32*)(b + L.off[R_PART] + SCAN_NB * 8);
  u32* totals = (u32*)(err + 2);
  u32* lstart = (u32*)(b + L.off[R_LSTART]);
  u32* scnt = (u32*)(b + L.off[R_SCNT]) + RGA_CS_MAX;  // (the chunk sums before it)
  u32* soff = (u32*)(b + L.off[R_SOFF]);
  u32* def2 = (u32*)(b + L.off[R_DEF2]);
  u32* ndef = (u32*)(err + 4);  // (ndef[1]: lists for k_rga_big)
  const smx_rga_ops o = *ops;
  const int grid = (int)(SMX_CEIL_DIV(n, (i64)BLOCK) < 8192 ? SMX_CEIL_DIV(n, (i64)BLOCK) : 8192);

  RGA_TRY(hipMemsetAsync(err, 0, 32, st));
  if (g_rr_grid == 0) {  // persistent scatter workgroups
    int dev = 0, cus = 0;
    RGA_TRY(hipGetDevice(&dev));
    RGA_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    g_cus = cus > 0 ? cus : 256;
    g_rr_grid = g_cus * RR_PER_CU;
  }
  const bool direct = grouped && RGA_DIRECT;  // the list kernels read the columns in place
  if (grouped) {  // the caller's events come list by list: no partition
    const int pgrid = (int)(SMX_CEIL_DIV(n, (i64)BLOCK) < 8192 ? SMX_CEIL_DIV(n, (i64)BLOCK) : 8192);
    if (direct)
      hipLaunchKernelGGL(k_rga_gbounds, dim3((int)SMX_CEIL_DIV((i64)pgrid, (i64)4)), dim3(BLOCK), 0, st, *ops, lstart,
                         scnt - RGA_CS_MAX, err);
    else
      hipLaunchKernelGGL(k_rga_pack, dim3(pgrid), dim3(BLOCK), 0, st, *ops, rec, lstart, scnt - RGA_CS_MAX, err);
  } else {  // records grouped by list: LSD passes over the list id, ping-pong into rec
    int npass = 1;
    while (npass < 4 && ((u64)(nl - 1) >> (8 * npass)) != 0) ++npass;
    const int nblk = (int)SMX_CEIL_DIV(n, (i64)RREC_TILE);
    u32* tsum = rhist + (size_t)256 * nblk;
    u32* dstart = tsum + hscan_tsum_bytes(nblk, 256) / 4;
    u64* rbuf[2] = {npass % 2 ? rec : rec2, npass % 2 ? rec2 : rec};
    u32* kbuf[2] = {keys, keys2};
    if (RGA_MSD && npass == 2) {  // high byte by the global pass, low byte per bucket
      hipLaunchKernelGGL(k_rrec_hist<true>, dim3(nblk), dim3(BLOCK), 0, st, o, nullptr, 8, rhist, err);
      // (one-launch column scan with the bucket starts from its last workgroup, on a
      // [digit][tile] histogram: 18.7 + 34.3 us against hscan's 22 + 28.8, profiles/r04_ac)
      hscan(rhist, nblk, 256u, tsum, dstart, st);
      const int sgrid = nblk < g_rr_grid ? nblk : g_rr_grid;
      hipLaunchKernelGGL((k_rrec_scatter<true, u8>), dim3(sgrid), dim3(RR_NT), 0, st, o, nullptr, nullptr, (u8*)keys2,
                         rec2, 8, rhist, err, (u32)nblk);
      hipLaunchKernelGGL(k_rrec_local, dim3(RGA_NDIG * RL_S), dim3(RL_NT), 0, st, (const u8*)keys2, rec2, rec, dstart, nl,
                         lstart, scnt - RGA_CS_MAX);
      npass = 0;  // (done: rec holds the list-ordered records, lstart their starts)
    }
    for (int p = 0; p < npass; ++p) {
      if (p == 0)
        hipLaunchKernelGGL(k_rrec_hist<true>, dim3(nblk), dim3(BLOCK), 0, st, o, nullptr, 0, rhist, err);
      else
        hipLaunchKernelGGL(k_rrec_hist<false>, dim3(nblk), dim3(BLOCK), 0, st, o, kbuf[(p - 1) & 1], 8 * p, rhist,
                           err);
      hscan(rhist, nblk, 256u, tsum, dstart, st);
      const int sgrid = nblk < g_rr_grid ? nblk : g_rr_grid;
      if (p == 0)
        hipLaunchKernelGGL(k_rrec_scatter<true>, dim3(sgrid), dim3(RR_NT), 0, st, o, nullptr, nullptr, kbuf[0],
                           rbuf[0], 0, rhist, err, (u32)nblk);
      else
        hipLaunchKernelGGL(k_rrec_scatter<false>, dim3(sgrid), dim3(RR_NT), 0, st, o, kbuf[(p - 1) & 1],
                           rbuf[(p - 1) & 1], kbuf[p & 1], rbuf[p & 1], 8 * p, rhist, err, (u32)nblk);
    }
    if (npass)
      hipLaunchKernelGGL(k_rga_bounds, dim3(grid), dim3(BLOCK), 0, st, kbuf[(npass - 1) & 1], n, nl, lstart,
                         scnt - RGA_CS_MAX);
  }
  const int tomb = out->out_tomb != nullptr;
  i64 wg = SMX_CEIL_DIV(nl, (i64)RW_WAVES);
  if (RW_PER_CU > 0 && wg > (i64)g_cus * RW_PER_CU) wg = (i64)g_cus * RW_PER_CU;
  const dim3 wgrid((u32)wg);
  if (direct)
    hipLaunchKernelGGL(k_rga_wave<true>, wgrid, dim3(WAVE * RW_WAVES), 0, st, o, rec, lstart, n, nl, tmp_v, tmp_s,
                       scnt, tomb, (const i32*)err);
  else
    hipLaunchKernelGGL(k_rga_wave<false>, wgrid, dim3(WAVE * RW_WAVES), 0, st, o, rec, lstart, n, nl, tmp_v, tmp_s,
                       scnt, tomb, (const i32*)err);
  // lists of more than RW_CAP events (a few, if any).  (On a second stream beside
  // k_rga_wave they measured no faster: their workgroups trail k_rga_wave's, and the
  // join costs ~14 us, round 4.)
  hipLaunchKernelGGL(k_rga_wave2, dim3(64), dim3(WAVE * RW_WAVES), 0, st, o, rec, lstart, n, nl, def2, ndef + 1,
                     tmp_v, tmp_s, scnt, tomb, (const i32*)err, (int)direct);
  hipLaunchKernelGGL(k_rga_big, dim3(RGA_BIG_GRID), dim3(1024), 0, st, o, rec, lstart, n, nl, def2, ndef + 1, bst, gp, tmp_v,
                     tmp_s, scnt, tomb, (const i32*)err);
  if (nl <= RGA_FUSED_MAX) {  // each list's wave finds its own offset
    hipLaunchKernelGGL(k_rga_out_fused, dim3(SMX_CEIL_DIV(nl, (i64)(BLOCK / WAVE * RGA_OUT_LPW))), dim3(BLOCK), 0, st, tmp_v,
                       tmp_s, lstart, scnt, nl, *out, (const i32*)err);
  } else {
    RGA_TRY((scan_excl<OpSum, u32, u32>(scnt, soff, nl, nullptr, part, totals, st)));
    hipLaunchKernelGGL(k_rga_out, dim3(SMX_CEIL_DIV(nl, (i64)(BLOCK / WAVE))), dim3(BLOCK), 0, st, tmp_v, tmp_s,
                       lstart, scnt, soff, nl, *out, (const i32*)err);
    hipLaunchKernelGGL(k_rga_fin, dim3(1), dim3(1), 0, st, totals, nl, *out, (const i32*)err);
  }
  RGA_TRY(hipGetLastError());
  i32 herr = 0;
  RGA_TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  RGA_TRY(stream_wait(st));
  if (herr & RGA_E_INPUT) return smx_set_error(SMX_E_ARG, "invalid input: list >= n_lists or op > 2");
  if (herr & RGA_E_UNGROUPED) return rga_impl(ops, out, ws, wsb, st, false);  // (not grouped after all)
  return SMX_OK;
}


extern "C" int smx_rga_replay_ex(const smx_rga_ops* ops, const smx_rga_out* out, void* ws, size_t wsb,
                                 uint32_t flags, void* stream) {
  if (!ops) return SMX_E_ARG;
  if (flags & ~(uint32_t)SMX_RGA_GROUPED) return smx_set_error(SMX_E_ARG, "unknown smx_rga_replay_ex flag");
  (void)hipGetLastError();  // an earlier call's error (any library's) is not this call's
  return rga_impl(ops, out, ws, wsb, (hipStream_t)stream, (flags & SMX_RGA_GROUPED) != 0);
}

extern "C" int smx_rga_replay(const smx_rga_ops* ops, const smx_rga_out* out, void* ws, size_t wsb,
                              void* stream) {
  return smx_rga_replay_ex(ops, out, ws, wsb, 0u, stream);
}
