// Microbenchmark: issue cost of dependent fp64 FMA chains on gfx950.  C independent chains per
// lane (C = 1, 2, 4, 8), W waves per SIMD (1, 2, 4); prints SIMD cycles per v_fma_f64 at the
// measured clock, so a dependent-latency floor shows up as cycles/FMA > 4 at low C x W.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/dp_latency.hip -o tools/ubench/dp_latency
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ __launch_bounds__(256) void k(double* out, int iters, double a, double b) {
  double x[C];
#pragma unroll
  for (int c = 0; c < C; ++c) x[c] = threadIdx.x + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 64 / C; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c) x[c] = fma(x[c], a, b);
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += x[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int C>
float run(double* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k<C><<<blocks, 256>>>(out, iters, 1.0000001, 1e-9);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<C><<<blocks, 256>>>(out, iters, 1.0000001, 1e-9);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double* out;
  const int iters = 20000;
  hipMalloc(&out, sizeof(double) * 256 * 256 * 4);
  const double ghz = 2.3;   // nominal for the cycle figure; the ratio between rows is what matters
  for (int w : {1, 2, 4}) {
    const int blocks = 256 * w;   // 4 waves per block, one per SIMD
    float t[4] = {run<1>(out, blocks, iters), run<2>(out, blocks, iters),
                  run<4>(out, blocks, iters), run<8>(out, blocks, iters)};
    const int cs[4] = {1, 2, 4, 8};
    for (int i = 0; i < 4; ++i) {
      const double fmas_per_simd = (double)w * iters * 64;   // wave-instructions per SIMD
      printf("waves/SIMD=%d chains=%d: %.3f ms, %.2f cycles per fp64 FMA at %.1f GHz\n", w, cs[i],
             t[i], t[i] * 1e-3 * ghz * 1e9 / fmas_per_simd, ghz);
    }
  }
  hipFree(out);
  return 0;
}
