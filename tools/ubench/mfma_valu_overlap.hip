// Microbenchmark: do fp64 MFMA (v_mfma_f64_16x16x4) and fp64 VALU FMAs from the same wave /
// other waves overlap on gfx950?  Times NM MFMAs alone, NV VALU FMAs alone, and both interleaved.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>   // 1: MFMA only, 2: VALU only, 3: both
__global__ __launch_bounds__(256) void k(double* out, int iters, double a, double b) {
  d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  for (int i = 0; i < iters; ++i) {
    if (MODE & 1) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc3, 0, 0, 0);
    }
    if (MODE & 2) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {   // 64 independent-ish fp64 FMAs per iteration
        x0 = fma(x0, a, b); x1 = fma(x1, a, b); x2 = fma(x2, a, b); x3 = fma(x3, a, b);
        x4 = fma(x4, a, b); x5 = fma(x5, a, b); x6 = fma(x6, a, b); x7 = fma(x7, a, b);
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc0[0] + acc1[1] + acc2[2] + acc3[3] + x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

template <int MODE>
float run(double* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k<MODE><<<blocks, 256>>>(out, iters, 1.0000001, 1e-9);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<MODE><<<blocks, 256>>>(out, iters, 1.0000001, 1e-9);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double* out;
  const int iters = 20000;
  for (int blocks : {256 * 2, 256 * 4}) {
    hipMalloc(&out, sizeof(double) * 256 * blocks);
    float m = run<1>(out, blocks, iters), v = run<2>(out, blocks, iters), b = run<3>(out, blocks, iters);
    const double waves = blocks * 4.0;
    // per SIMD: waves/1024 waves each doing iters*(4 MFMA) / iters*64 VALU
    const double mfma_cyc = waves / 1024 * iters * 4 * 64, valu_cyc = waves / 1024 * iters * 64 * 4;
    printf("blocks=%d (waves/SIMD=%.0f): mfma %.3f ms  valu %.3f ms  both %.3f ms  (sum %.3f)  "
           "implied clock mfma %.2f GHz valu %.2f GHz\n", blocks, waves / 1024, m, v, b, m + v,
           mfma_cyc / (m * 1e6), valu_cyc / (v * 1e6));
    hipFree(out);
  }
  return 0;
}
