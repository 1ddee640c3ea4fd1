// store_probe.hip -- HBM write throughput of store patterns K2 could use (dev aid, round 4).
// 6.37 GB (1024 x 1080p RGB) written as 69,632 "MCU rows" of 92,160 B (16 x 5,760 B):
//   k2like<LDS>: one 64-lane wave per row, 12 chunks of 7,680 B (a strip's bytes), dwordx4,
//                with LDS bytes per workgroup limiting residency like K2 (9,984 B: 16 per CU)
//   fill:        grid-stride dwordx4 over the buffer, 256 threads per workgroup
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int LDS>
__global__ __launch_bounds__(64) void k2like(uint4 *dst, uint32_t rows) {
  __shared__ uint4 pad[LDS / 16 > 0 ? LDS / 16 : 1];
  if (LDS > 0 && threadIdx.x == 0) pad[0] = make_uint4(1, 2, 3, 4);
  const uint32_t r = blockIdx.x;
  if (r >= rows) return;
  uint4 *base = dst + uint64_t(r) * (92160 / 16);
  for (uint32_t c = 0; c < 12; c++) {
    uint4 *p = base + c * 480;
    for (uint32_t k = threadIdx.x; k < 480; k += 64) p[k] = make_uint4(k, c, r, LDS > 0 ? pad[0].x : 0u);
  }
}

__global__ __launch_bounds__(256) void fill(uint4 *dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256ull)
    dst[i] = make_uint4(uint32_t(i), 1, 2, 3);
}

template <typename F>
double timeit(F f) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  f();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int i = 0; i < 10; i++) f();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms / 10.0;
}

int main() {
  const uint32_t rows = 69632;
  const uint64_t bytes = uint64_t(rows) * 92160;
  uint4 *d = nullptr;
  CHK(hipMalloc(&d, bytes));
  auto rep = [&](const char *name, double ms) { printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6); };
  rep("k2like LDS 9984 (16/CU)", timeit([&] { hipLaunchKernelGGL(k2like<9984>, dim3(rows), dim3(64), 0, 0, d, rows); }));
  rep("k2like LDS 4992 (32/CU)", timeit([&] { hipLaunchKernelGGL(k2like<4992>, dim3(rows), dim3(64), 0, 0, d, rows); }));
  rep("k2like LDS 0", timeit([&] { hipLaunchKernelGGL(k2like<0>, dim3(rows), dim3(64), 0, 0, d, rows); }));
  rep("fill 256 x 4096 WGs", timeit([&] { hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, d, bytes / 16); }));
  rep("fill 256 x 65536 WGs", timeit([&] { hipLaunchKernelGGL(fill, dim3(65536), dim3(256), 0, 0, d, bytes / 16); }));
  CHK(hipFree(d));
  return 0;
}
