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

extern "C" int smx_calib_run(void* buf, size_t bytes, void* sink, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(4096), b(256);
  hipLaunchKernelGGL(k_calib_read<uint8_t>, g, b, 0, st, (const uint8_t*)buf, bytes, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_read<uint32_t>, g, b, 0, st, (const uint32_t*)buf, bytes / 4, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_read<uint64_t>, g, b, 0, st, (const uint64_t*)buf, bytes / 8, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_read<uint4>, g, b, 0, st, (const uint4*)buf, bytes / 16, (unsigned long long*)sink);
  hipLaunchKernelGGL(k_calib_write<uint32_t>, g, b, 0, st, (uint32_t*)buf, bytes / 4);
  hipLaunchKernelGGL(k_calib_write<uint4>, g, b, 0, st, (uint4*)buf, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
