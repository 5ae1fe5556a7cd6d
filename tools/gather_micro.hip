// gather_micro.hip — cost of one random table lookup per lane, by entry shape and table
// size (tools only; the shape of k_emit4's final-state gathers).
//
// Each lane reads 4 consecutive 32-bit indices (one 16-byte coalesced load), looks up
// 4 table entries and writes one 16-byte coalesced word (the sum of what it read, so
// nothing is dead).  Shapes:
//   0  no lookup (the streams alone)
//   1  4-byte entries (dword, aligned)
//   2  8-byte entries (dwordx2, 8-aligned)
//   3  6-byte entries, 21 per 128-byte line, read as an 8-byte load at a 4-aligned
//      address (k_emit4's packed format)
//   4  16-byte entries (dwordx4, aligned)
//   5  6-byte entries read as two aligned dword loads (4-aligned + 2 more bytes)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int64_t i64;
typedef uint32_t u32;
typedef uint64_t u64;
typedef u64 __attribute__((aligned(4))) u64_a4;
typedef u32 v4u __attribute__((ext_vector_type(4)));

#define NT 256

__device__ __forceinline__ u64 off48(u32 s) {
  const u32 line = s / 21u;
  return (u64)line * 128u + (u64)(s - line * 21u) * 6u;
}

template <int V>
__device__ __forceinline__ u32 look(const uint8_t* __restrict__ tab, u32 s) {
  if (V == 0) return s;
  if (V == 1) return reinterpret_cast<const u32*>(tab)[s];
  if (V == 2) {
    const u64 x = reinterpret_cast<const u64*>(tab)[s];
    return (u32)x ^ (u32)(x >> 32);
  }
  if (V == 3) {
    const u64 o = off48(s);
    const u64 w = *reinterpret_cast<const u64_a4*>(tab + (o & ~3ull));
    const u64 x = (w >> ((o & 2) * 8)) & 0xffffffffffffull;
    return (u32)x ^ (u32)(x >> 32);
  }
  if (V == 4) {
    const uint4 x = reinterpret_cast<const uint4*>(tab)[s];
    return x.x ^ x.y ^ x.z ^ x.w;
  }
  // V == 5: two aligned dwords covering the 6 bytes
  const u64 o = off48(s);
  const u32* p = reinterpret_cast<const u32*>(tab + (o & ~3ull));
  return p[0] ^ (p[1] & ((o & 2) ? 0xffffffffu : 0xffffu));
}

// Shapes 6..8: some of a lane's four 6-byte lookups through the SCALAR memory path
// (each lane's symbol broadcast with readlane, one uniform-address load per lane, the
// result put back into its lane): the scalar cache and its L2 requests instead of the
// texture path (TA / TD), which bounds the vector gathers.  6: one of four scalar,
// 7: two of four, 8: all four.
__device__ __forceinline__ u32 look_scalar(const uint8_t* __restrict__ tab, u32 s) {
  const int lane = threadIdx.x & 63;
  u32 res = 0;
#pragma unroll 16
  for (int l = 0; l < 64; ++l) {
    const u32 sl = __builtin_amdgcn_readlane(s, l);
    const u64 o = off48(sl);
    const u64 w = *reinterpret_cast<const u64_a4*>(tab + (o & ~3ull));
    const u64 x = (w >> ((o & 2) * 8)) & 0xffffffffffffull;
    const u32 r = (u32)x ^ (u32)(x >> 32);
    res = lane == l ? r : res;
  }
  return res;
}

template <int V>
__device__ __forceinline__ u32 look_u(const uint8_t* __restrict__ tab, u32 s, int u) {
  if (V == 6) return u == 3 ? look_scalar(tab, s) : look<3>(tab, s);
  if (V == 7) return u >= 2 ? look_scalar(tab, s) : look<3>(tab, s);
  if (V == 8) return look_scalar(tab, s);
  return look<V>(tab, s);
}

template <int V>
__global__ void __launch_bounds__(NT) k_gather(const v4u* __restrict__ idx, const uint8_t* __restrict__ tab,
                                               u32 smask, i64 nq, v4u* __restrict__ out) {
  constexpr int B = 4;  // quads per lane in flight
  const i64 q0 = ((i64)blockIdx.x * NT * B) + threadIdx.x;
  v4u s[B];
#pragma unroll
  for (int j = 0; j < B; ++j) {
    const i64 q = q0 + (i64)j * NT;
    s[j] = q < nq ? __builtin_nontemporal_load(&idx[q]) : v4u{0, 0, 0, 0};
  }
#pragma unroll
  for (int j = 0; j < B; ++j) {
    const i64 q = q0 + (i64)j * NT;
    const v4u r = v4u{look_u<V>(tab, s[j].x & smask, 0), look_u<V>(tab, s[j].y & smask, 1),
                      look_u<V>(tab, s[j].z & smask, 2), look_u<V>(tab, s[j].w & smask, 3)};
    if (q < nq) __builtin_nontemporal_store(r, &out[q]);
  }
}

extern "C" int gather_run(int v, const void* idx, const void* tab, u32 smask, i64 nq, void* out, void* stream) {
  const int blocks = (int)((nq + NT * 4 - 1) / (NT * 4));
  hipStream_t st = (hipStream_t)stream;
  const v4u* I = (const v4u*)idx;
  const uint8_t* T = (const uint8_t*)tab;
  v4u* O = (v4u*)out;
  switch (v) {
    case 0: hipLaunchKernelGGL(k_gather<0>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 1: hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 2: hipLaunchKernelGGL(k_gather<2>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 3: hipLaunchKernelGGL(k_gather<3>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 4: hipLaunchKernelGGL(k_gather<4>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 5: hipLaunchKernelGGL(k_gather<5>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 6: hipLaunchKernelGGL(k_gather<6>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 7: hipLaunchKernelGGL(k_gather<7>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    case 8: hipLaunchKernelGGL(k_gather<8>, dim3(blocks), dim3(NT), 0, st, I, T, smask, nq, O); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
