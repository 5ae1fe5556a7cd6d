// emit_micro.hip — microbenchmarks for the access pattern of k_emit (tools only).
//
// Each variant reads order[T], sym[T] for n positions, gathers a 16-byte record
// fin[sym] (optional) and writes the composed outputs, either as four i32
// arrays (SoA, the current ABI) or as one 16-byte record per op (AoS).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int64_t i64;
typedef uint32_t u32;

#define NT 256

template <int V>
__global__ void __launch_bounds__(NT) k_micro(const int* __restrict__ order, const u32* __restrict__ sym,
                                              const int4* __restrict__ fin, u32 smask, i64 n,
                                              int* __restrict__ o0, int* __restrict__ o1, int* __restrict__ o2,
                                              int* __restrict__ o3, int4* __restrict__ oa) {
  constexpr int B = 8;
  const i64 base = (i64)blockIdx.x * NT * B + threadIdx.x;
  if (V == 4) {  // 4 positions per lane, 16-byte loads, AoS writes
    const i64 q = (i64)blockIdx.x * NT + threadIdx.x;
    if (q * 4 >= n) return;
    const int4 s = reinterpret_cast<const int4*>(order)[q];
    const uint4 y = reinterpret_cast<const uint4*>(sym)[q];
    const int4 f0 = fin[y.x & smask], f1 = fin[y.y & smask], f2 = fin[y.z & smask], f3 = fin[y.w & smask];
    oa[q * 4 + 0] = make_int4(s.x, f0.x, f0.y, f0.z);
    oa[q * 4 + 1] = make_int4(s.y, f1.x, f1.y, f1.z);
    oa[q * 4 + 2] = make_int4(s.z, f2.x, f2.y, f2.z);
    oa[q * 4 + 3] = make_int4(s.w, f3.x, f3.y, f3.z);
    return;
  }
  int src[B];
  u32 sy[B];
#pragma unroll
  for (int j = 0; j < B; ++j) {
    const i64 T = base + (i64)j * NT;
    const i64 Tc = T < n ? T : n - 1;
    src[j] = order[Tc];
    sy[j] = sym[Tc] & smask;
  }
  int4 F[B];
  const unsigned long long* fin8 = reinterpret_cast<const unsigned long long*>(fin);
  const u32* fin4 = reinterpret_cast<const u32*>(fin);
#pragma unroll
  for (int j = 0; j < B; ++j) {
    if (V == 0) {
      F[j] = make_int4(sy[j], sy[j] + 1, sy[j] + 2, 0);
    } else if (V == 5) {  // 8-byte packed entries: 27 + 20 + 17 bits
      const unsigned long long x = fin8[sy[j]];
      F[j] = make_int4((int)(x & 0x7ffffff) - 1, (int)((x >> 27) & 0xfffff) - 1, (int)(x >> 47) - 1, 0);
    } else if (V == 6) {  // 4-byte entries
      const u32 x = fin4[sy[j]];
      F[j] = make_int4((int)(x & 0xffff), (int)(x >> 16), 0, 0);
    } else {
      F[j] = fin[sy[j]];
    }
  }
#pragma unroll
  for (int j = 0; j < B; ++j) {
    const i64 T = base + (i64)j * NT;
    if (T >= n) continue;
    if (V == 0 || V == 1 || V == 5 || V == 6) {
      o0[T] = src[j];
      o1[T] = F[j].x;
      o2[T] = F[j].y;
      o3[T] = F[j].z;
    } else if (V == 2) {
      oa[T] = make_int4(src[j], F[j].x, F[j].y, F[j].z);
    } else if (V == 3) {  // SoA, outputs shifted by one (unaligned compaction shift)
      o0[T + 1] = src[j];
      o1[T + 1] = F[j].x;
      o2[T + 1] = F[j].y;
      o3[T + 1] = F[j].z;
    }
  }
}

extern "C" int micro_run(int variant, const int* order, const u32* sym, const int4* fin, u32 smask, i64 n,
                         int* o0, int* o1, int* o2, int* o3, int4* oa, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const i64 blocks8 = (n + NT * 8 - 1) / (NT * 8);
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_micro<0>, dim3(blocks8), dim3(NT), 0, st, order, sym, fin, smask, n, o0, o1, o2, o3, oa); break;
    case 1: hipLaunchKernelGGL(k_micro<1>, dim3(blocks8), dim3(NT), 0, st, order, sym, fin, smask, n, o0, o1, o2, o3, oa); break;
    case 2: hipLaunchKernelGGL(k_micro<2>, dim3(blocks8), dim3(NT), 0, st, order, sym, fin, smask, n, o0, o1, o2, o3, oa); break;
    case 3: hipLaunchKernelGGL(k_micro<3>, dim3(blocks8), dim3(NT), 0, st, order, sym, fin, smask, n, o0, o1, o2, o3, oa); break;
    case 4: hipLaunchKernelGGL(k_micro<4>, dim3((n / 4 + NT - 1) / NT), dim3(NT), 0, st, order, sym, fin, smask, n, o0, o1, o2, o3, oa); break;
    case 5: hipLaunchKernelGGL(k_micro<5>, dim3(blocks8), dim3(NT), 0, st, order, sym, fin, smask, n, o0, o1, o2, o3, oa); break;
    case 6: hipLaunchKernelGGL(k_micro<6>, dim3(blocks8), dim3(NT), 0, st, order, sym, fin, smask, n, o0, o1, o2, o3, oa); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
