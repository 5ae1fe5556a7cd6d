// smx_common.h — shared device helpers for libsmx (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smx.h"

// Diagnostic build (-DSMX_DIAG=1, tools/build_variants.sh): environment knobs and the
// window kernel's phase ablations.  The release library compiles them out.
#ifndef SMX_DIAG
#define SMX_DIAG 0
#endif

typedef uint64_t u64;
typedef uint32_t u32;
typedef int64_t i64;
typedef int32_t i32;
typedef uint16_t u16;
typedef uint8_t u8;

#define WAVE 64
#define BLOCK 256
#define NWAVES (BLOCK / WAVE)

// Device-side state of one smx_compose call (lives at the start of the workspace).
// Counters written by kernels; read by later kernels and (once) by the host.
#define SEG_FAIL_BIT 8ull
#define F_LONG 22ull  // f_fail from k_fpart's long-group check (bits 1, 2 and 4), before any window ran
#define F_WLONG 32ull // f_fail bit 5: after an early F_LONG (k_khist), a group no wide window holds either
#define SEG_DECREASE 2ull  // meta->seg_over: a timestamp decreases (the segmented sort)
struct ComposeMeta {
  u64 kcnt[SMX_N_KINDS];     // ops per precedence rank (stats kernel)
  u64 base[SMX_N_KINDS + 1]; // exclusive prefix of kcnt: T-order segment starts
  u64 nonmono[2];            // per side: 1 if timestamps decrease somewhere
  u64 n_move_none;           // moves with a None newAddress or newFile
  u64 f_fail;                // the plan failed: bit 0 logs not ordered, 1 a window too large, 2 one
                             // timestamp per window; bit 3 (SEG_FAIL_BIT) the segmented sort;
                             // F_LONG: k_fpart's verdict, before any window ran
  u64 bad_sym;               // sym >= n_sym seen
  u64 n_ren_side[2];         // renames per side
  u64 key_or[2][3];          // per side OR / AND of (ts, hi, lo): constant radix digits
  u64 key_and[2][3];
  u64 n_cand;                // DivergentRename candidate starts
  u64 n_conf;                // conflicts (real)
  u32 vbits[4];              // OR of (value + 1) over table values: addr, file, ctx (packing widths)
  u64 n_skip;                // skipped renames (2 per conflict on one GPU; see smx_walk.h)
  // sharded merge (smx_shard_step): the incoming open region's end and conflicts,
  // the outgoing open region's state, halo too short
  u64 q_in, nconf_in;
  u64 out_open, out_ahead, out_d;
  u64 halo_overflow;
  u64 tab_over;              // sharded TABLES, 32-bit entries: a value too wide for them
  u64 n_conf_loc;            // conflicts of this shard's own regions (scan total)
  u64 nskip_in;              // skipped renames of the incoming region (head of the skip list)
  u64 dup_key;               // generic plan: equal (ts, oid_hi) pair seen -> sort with oid_lo
  u64 seg_over;              // segmented plan: bit 0 a timestamp group too long, bit 1 a branch not ordered
  u64 n_win;                 // windows of the plan that ran
  u32 kmask[2];              // presorted plan: kinds present per branch (k_khist)
  u64 cs_done;               // k_cscan_mid blocks done (the last one writes base[])
  u32 wk_done[2];            // k_boundary / k_replay_q blocks done (fused walk steps:
                             // the last block runs the next single-block step, resets it)
};

// Per-symbol final states (addr, file, ctx).  When the bit widths of (value + 1)
// add up to <= 64 they are packed per symbol (a smaller gather footprint for
// k_emit, whose lookups are bound by L2 misses); otherwise int4 entries.
//   <= 48 bits: 6-byte entries, 21 per 128-byte line (6.1 MB at 2^20 symbols); one
//               4-byte-aligned 8-byte load per lookup, never crossing a line
//   <= 64 bits: 8-byte entries
#ifndef SMX_FIN48
#define SMX_FIN48 1
#endif
struct FinPack {
  u32 wa, wf;
  bool packed;  // 6- or 8-byte entries
  bool p48;     // 6-byte entries
};

__device__ __forceinline__ u32 bit_width32(u32 x) { return x ? 32u - (u32)__clz((int)x) : 0u; }

__device__ __forceinline__ FinPack fin_pack_make(u32 wa, u32 wf, u32 wc, bool allow) {
  const bool packed = allow && wa + wf + wc <= 64;
  return FinPack{wa, wf, packed, SMX_FIN48 && packed && wa + wf + wc <= 48};
}

__device__ __forceinline__ FinPack fin_pack_of(const u32* vbits, bool allow) {
  return fin_pack_make(bit_width32(vbits[0]), bit_width32(vbits[1]), bit_width32(vbits[2]), allow);
}

__device__ __forceinline__ u64 fin_encode(const FinPack& P, int a, int f, int c) {
  const u64 x = (u64)(u32)(a + 1) | ((u64)(u32)(f + 1) << P.wa);
  return P.wa + P.wf >= 64 ? x : x | ((u64)(u32)(c + 1) << (P.wa + P.wf));
}

// byte offset of symbol s's 6-byte entry
__device__ __forceinline__ u64 fin48_off(u32 s) {
  const u32 line = s / 21u;
  return (u64)line * 128u + (u64)(s - line * 21u) * 6u;
}
__device__ __forceinline__ void fin48_store(void* fin, u32 s, u64 x) {
  u16* p = reinterpret_cast<u16*>(reinterpret_cast<u8*>(fin) + fin48_off(s));
  p[0] = (u16)x;
  p[1] = (u16)(x >> 16);
  p[2] = (u16)(x >> 32);
}
typedef u64 __attribute__((aligned(4))) u64_a4;
__device__ __forceinline__ u64 fin48_load(const void* fin, u32 s) {
  const u64 o = fin48_off(s);
  const u64 w = *reinterpret_cast<const u64_a4*>(reinterpret_cast<const u8*>(fin) + (o & ~3ull));
  return (w >> ((o & 2) * 8)) & 0xffffffffffffull;
}
// the packed word of symbol s (P.packed)
__device__ __forceinline__ u64 fin_word(const FinPack& P, const void* fin, u32 s) {
  return P.p48 ? fin48_load(fin, s) : reinterpret_cast<const u64*>(fin)[s];
}
__device__ __forceinline__ void fin_put(const FinPack& P, void* fin, u32 s, int a, int f, int c) {
  if (P.p48) fin48_store(fin, s, fin_encode(P, a, f, c));
  else if (P.packed) reinterpret_cast<u64*>(fin)[s] = fin_encode(P, a, f, c);
  else reinterpret_cast<int4*>(fin)[s] = make_int4(a, f, c, 0);
}

__device__ __forceinline__ int4 fin_decode(const FinPack& P, u64 x) {
  const u64 ma = P.wa >= 64 ? ~0ull : ((1ull << P.wa) - 1), mf = P.wf >= 64 ? ~0ull : ((1ull << P.wf) - 1);
  const int a = (int)(u32)(x & ma) - 1;
  const int f = (int)(u32)((x >> P.wa) & mf) - 1;
  const u32 sc = P.wa + P.wf;
  const int c = sc >= 64 ? -1 : (int)(u32)(x >> sc) - 1;
  return make_int4(a, f, c, 0);
}

// Workgroup b of a grid of n -> the work item it processes, so that the workgroups
// the dispatcher deals to one XCD (b % 8 labels them; cdna_hip_programming.md T1)
// take consecutive items: neighbouring windows share their input lines in that XCD's
// L2.  Bijective for any n.  A speed choice only: any placement gives the same result.
__device__ __forceinline__ i64 xcd_item(i64 b, i64 n) {
  const i64 q = n / 8, r = n % 8, x = b % 8, i = b / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ __forceinline__ u64 lanemask_lt() {
  const int lane = threadIdx.x & (WAVE - 1);
  return (lane == 0) ? 0ull : (~0ull >> (WAVE - lane));
}

// The kernel's argument block read through an opaque pointer: field loads are issued
// where the pointer is taken, not hoisted to the kernel's start (where long-lived
// scalars end up spilled to VGPR lanes in large kernels).
template <class T>
__device__ __forceinline__ const T* kernarg_late() {
#if defined(__HIP_DEVICE_COMPILE__)
  const T* p = (const T*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
#else
  return nullptr;
#endif
}

__device__ __forceinline__ void wave_lds_sync() {  // LDS writes of this wave visible to its lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Lanes of this wave holding the same `nbits`-bit value `d` (among lanes with `valid`).
template <int NBITS>
__device__ __forceinline__ u64 wave_peers(u32 d, bool valid) {
  u64 m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < NBITS; ++b) {
    const bool bit = (d >> b) & 1u;
    const u64 x = __ballot(bit);
    m &= bit ? x : ~x;
  }
  return m;
}

// wave_peers over the low `nbits` bits (wave-uniform at run time)
__device__ __forceinline__ u64 wave_peers_n(u32 d, bool valid, int nbits) {
  u64 m = __ballot(valid);
  for (int b = 0; b < nbits; ++b) {
    const bool bit = (d >> b) & 1u;
    const u64 x = __ballot(bit);
    m &= bit ? x : ~x;
  }
  return m;
}

// Inclusive wave64 prefix scans on the DPP network (VALU only; __shfl_up would be
// a chain of six ds_bpermute LDS round trips): row_shr 1, 2, 4, 8 inside each
// 16-lane row, then row_bcast:15 and row_bcast:31 carry across rows.
template <int CTRL, int ROWS>
__device__ __forceinline__ u32 dpp_u32(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}

__device__ __forceinline__ u32 wave_incl_sum_u32(u32 v) {
  v += dpp_u32<0x111, 0xf>(v);  // row_shr:1
  v += dpp_u32<0x112, 0xf>(v);  // row_shr:2
  v += dpp_u32<0x114, 0xf>(v);  // row_shr:4
  v += dpp_u32<0x118, 0xf>(v);  // row_shr:8
  v += dpp_u32<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v += dpp_u32<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  return v;
}

__device__ __forceinline__ u32 wave_incl_max_u32(u32 v) {
  v = max(v, dpp_u32<0x111, 0xf>(v));
  v = max(v, dpp_u32<0x112, 0xf>(v));
  v = max(v, dpp_u32<0x114, 0xf>(v));
  v = max(v, dpp_u32<0x118, 0xf>(v));
  v = max(v, dpp_u32<0x142, 0xa>(v));
  v = max(v, dpp_u32<0x143, 0xc>(v));
  return v;
}

// OR over the wave, valid in lane 63 (DPP, VALU only).
__device__ __forceinline__ u32 wave_or_to_last(u32 v) {
  v |= dpp_u32<0x111, 0xf>(v);
  v |= dpp_u32<0x112, 0xf>(v);
  v |= dpp_u32<0x114, 0xf>(v);
  v |= dpp_u32<0x118, 0xf>(v);
  v |= dpp_u32<0x142, 0xa>(v);
  v |= dpp_u32<0x143, 0xc>(v);
  return v;
}

// Inclusive wave prefix sum (64 lanes).
template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  if constexpr (sizeof(T) == 4) {
    return (T)wave_incl_sum_u32((u32)v);
  } else {
    const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
      T y = __shfl_up(v, o, WAVE);
      if (lane >= o) v += y;
    }
    return v;
  }
}

template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
  if constexpr (sizeof(T) == 4 && (T)(-1) > (T)0) {
    return (T)wave_incl_max_u32((u32)v);
  } else {
    const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
      T y = __shfl_up(v, o, WAVE);
      if (lane >= o) v = v > y ? v : y;
    }
    return v;
  }
}

struct OpSum {
  template <typename T>
  __device__ __forceinline__ static T apply(T a, T b) { return a + b; }
  template <typename T>
  __device__ __forceinline__ static T identity() { return T(0); }
  template <typename T>
  __device__ __forceinline__ static T wave_incl(T v) { return wave_incl_sum(v); }
};

struct OpMax {
  template <typename T>
  __device__ __forceinline__ static T apply(T a, T b) { return a > b ? a : b; }
  template <typename T>
  __device__ __forceinline__ static T identity() { return T(0); }
  template <typename T>
  __device__ __forceinline__ static T wave_incl(T v) { return wave_incl_max(v); }
};

// Block-wide exclusive scan of one value per thread; returns the exclusive prefix,
// writes the block aggregate to *total.  `s` must hold NW+1 entries (NW = waves
// per block).
template <typename Op, typename T, int NW = NWAVES>
__device__ __forceinline__ T block_excl_scan(T v, T* s, T* total) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x / WAVE;
  T inc = Op::template wave_incl<T>(v);
  if (lane == WAVE - 1) s[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T acc = Op::template identity<T>();
    for (int i = 0; i < NW; ++i) {
      T x = s[i];
      s[i] = acc;
      acc = Op::apply(acc, x);
    }
    s[NW] = acc;
  }
  __syncthreads();
  T wpre = s[w];
  T excl_in_wave = __shfl_up(inc, 1, WAVE);
  if (lane == 0) excl_in_wave = Op::template identity<T>();
  T r = Op::apply(wpre, excl_in_wave);
  *total = s[NW];
  __syncthreads();
  return r;
}

#define SMX_CEIL_DIV(a, b) (((a) + (b)-1) / (b))

// Records the thread-local error message returned by smx_last_error(); returns code.
int smx_set_error(int code, const char* msg);
