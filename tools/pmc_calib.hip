// tools/pmc_calib.hip — FETCH_SIZE / WRITE_SIZE calibration kernels (profiling aid only).
// MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of a 16 B/lane stream on
// gfx950 and other widths are uncalibrated.  These kernels stream a known number of
// bytes with the access widths libsmx's kernels use (1, 4, 8 and 16 B per lane) so a
// --pmc pass can convert counter values of the real kernels into bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <typename T>
__global__ void k_calib_read(const T* __restrict__ in, size_t n, unsigned long long* sink) {
  unsigned long long acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const unsigned char* p = (const unsigned char*)&in[i];
    acc += p[0];
  }
  if (acc == 0x1234567) *sink = acc;  // keeps the loads alive
}

template <typename T>
__global__ void k_calib_write(T* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = T{};
}

// Random 8-byte gathers (like k_emit's final-state lookups) from a table of
// `tbl` elements: element hash(i) % tbl, no index stream.  TAG names the table size
// in the kernel name: 0 = 8 MB (the fin table of config 3: L2 misses, MALL hits),
// 1 = 1 GB (HBM).
template <int TAG>
__global__ void k_calib_gather(const uint64_t* __restrict__ tbl, size_t n_tbl, size_t n,
                               unsigned long long* sink) {
  unsigned long long acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    acc += tbl[(h >> 17) % n_tbl];
  }
  if (acc == 0x1234567) *sink = acc;
}

extern "C" int smx_calib_run(void* buf, size_t bytes, void* sink, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(4096), b(256);
  hipLaunchKernelGGL(k_calib_read<uint8_t>, g, b, 0, st, (const uint8_t*)buf, bytes, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_read<uint32_t>, g, b, 0, st, (const uint32_t*)buf, bytes / 4, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_read<uint64_t>, g, b, 0, st, (const uint64_t*)buf, bytes / 8, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_read<uint4>, g, b, 0, st, (const uint4*)buf, bytes / 16, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_write<uint32_t>, g, b, 0, st, (uint32_t*)buf, bytes / 4);
  hipLaunchKernelGGL(k_calib_write<uint4>, g, b, 0, st, (uint4*)buf, bytes / 16);
  // 32M gathers = 256 MB of algorithmic bytes each
  hipLaunchKernelGGL(k_calib_gather<0>, g, b, 0, st, (const uint64_t*)buf, (size_t)(8 << 20) / 8, (size_t)1 << 25,
                     (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_gather<1>, g, b, 0, st, (const uint64_t*)buf, bytes / 8, (size_t)1 << 25,
                     (unsigned long long*)sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
