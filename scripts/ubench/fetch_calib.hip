// fetch_calib.hip — calibrate rocprofv3 FETCH_SIZE for the access widths of
// the wide scoring kernel (MI355X_MICROARCH.md: "Other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Each kernel touches a known set of distinct 128-B lines of a 1 GiB buffer
// exactly once; FETCH_SIZE (KB) x 1024 / lines = bytes counted per line.
//   stream16   16 B per lane, consecutive (the guide's reference: counted at 1/2)
//   line_u16   one 2-B load per 128-B line (the tsongs gather at its sparsest)
//   line_u32   one 4-B load per 128-B line (nbr_v / toff)
//   line_u64   one 8-B load per 128-B line (nbr_q)
//   half_u16   one 2-B load per 64-B half line
//   seq_u16    consecutive 2-B loads (64 lanes -> one 128-B line per wave)
// Usage: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void stream16(const int4* __restrict__ p, size_t n, int* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  int s = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) { int4 v = p[i]; s += v.x ^ v.y ^ v.z ^ v.w; }
  if (s == 0x12345) out[0] = s;
}
template <typename T>
__global__ void strided(const unsigned char* __restrict__ base, size_t n, size_t stride, int* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  int s = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) s += (int)*reinterpret_cast<const T*>(base + i * stride);
  if (s == 0x12345) out[0] = s;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  unsigned char* buf;
  int* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  hipMemset(buf, 1, bytes);
  hipDeviceSynchronize();
  const dim3 g(4096), b(256);
  const size_t lines = bytes / 128;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream16, g, b, 0, 0, (const int4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(strided<unsigned short>, g, b, 0, 0, buf, lines, (size_t)128, out);
    hipLaunchKernelGGL(strided<unsigned>, g, b, 0, 0, buf, lines, (size_t)128, out);
    hipLaunchKernelGGL(strided<unsigned long long>, g, b, 0, 0, buf, lines, (size_t)128, out);
    hipLaunchKernelGGL(strided<unsigned short>, g, b, 0, 0, buf, lines * 2, (size_t)64, out);
    hipLaunchKernelGGL(strided<unsigned short>, g, b, 0, 0, buf, bytes / 2, (size_t)2, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("lines (128 B) per kernel: stream16 %zu, line_u16/u32/u64 %zu, half_u16 %zu lines (%zu half lines), "
         "seq_u16 %zu\n", lines, lines, lines, lines * 2, lines);
  return 0;
}
