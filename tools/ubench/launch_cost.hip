// Host cost of hipLaunchKernel on this pool (tools/README.md): an empty kernel launched 20000
// times back to back, on a plain stream, on a CU-masked stream (hipExtStreamCreateWithCUMask),
// and with a long kernel keeping the GPU busy on another stream; prints microseconds per launch.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1024) p[0] = 1;
}
__global__ void spin_kernel(int64_t cycles, int* p) {
  const int64_t t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (p && threadIdx.x == 1024) p[0] = 2;
}

static double per_launch_us(hipStream_t st, int n, int grid) {
  (void)hipStreamSynchronize(st);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, st, nullptr);
  const auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(st);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t plain, masked, busy;
  if (hipStreamCreateWithFlags(&plain, hipStreamNonBlocking) != hipSuccess) return 1;
  if (hipStreamCreateWithFlags(&busy, hipStreamNonBlocking) != hipSuccess) return 1;
  std::vector<uint32_t> mask(8, 0x0000ffffu);   // half of every 32-bit word's CUs
  if (hipExtStreamCreateWithCUMask(&masked, 8, mask.data()) != hipSuccess) return 1;
  const int n = 20000;
  per_launch_us(plain, 200, 1);   // warm-up
  std::printf("plain stream, 1 block:   %.2f us per launch\n", per_launch_us(plain, n, 1));
  std::printf("plain stream, 256 blocks: %.2f us per launch\n", per_launch_us(plain, n, 256));
  std::printf("masked stream, 1 block:  %.2f us per launch\n", per_launch_us(masked, n, 1));
  // the GPU busy on another stream (1 block spinning ~0.5 s)
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, busy, (int64_t)1000000000, nullptr);
  std::printf("plain stream, GPU busy elsewhere: %.2f us per launch\n", per_launch_us(plain, 5000, 1));
  (void)hipStreamSynchronize(busy);
  // a deep queue: launches behind a long kernel on the same stream
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, plain, (int64_t)1000000000, nullptr);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 5000; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, plain, nullptr);
  const auto t1 = std::chrono::steady_clock::now();
  std::printf("plain stream behind a long kernel: %.2f us per launch\n",
              std::chrono::duration<double, std::micro>(t1 - t0).count() / 5000);
  (void)hipStreamSynchronize(plain);
  std::printf("done\n");
  return 0;
}
