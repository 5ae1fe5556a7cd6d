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
    const v4u r = v4u{look<V>(tab, s[j].x & smask), look<V>(tab, s[j].y & smask),
                      look<V>(tab, s[j].z & smask), look<V>(tab, s[j].w & smask)};
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
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
