// Write pattern of the gains phase 3 (k_lgssm.hip gains_phase3): a thread per chunk of L = 256
// steps, and at each step every lane of a wave emits one 128-byte record.  Two layouts of the
// same bytes:
//   chunk-major (the library's): record (chain, k = chunk * 256 + s) at rec + (chain n + k) * 16,
//     so a wave-step writes 64 lines 32 KB apart;
//   chunk-interleaved: record (chain, group g of 64 chunks, s, lane) at
//     rec + (((chain * G + g) * 256 + s) * 64 + lane) * 16, so a wave-step writes 8 KB contiguous.
// Both store each record as 8 lanes x 16 bytes (the staging the kernel uses: RS / 2 lanes per
// record, 8 records per instruction).  A few dependent fp64 operations per step stand in for the
// recursion.  hipcc --offload-arch=gfx950 -O3 tools/ubench/rec_write.hip -o rec_write
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

constexpr int L = 256, RD = 16;   // steps per chunk, doubles per record

template <bool INTERLEAVED>
__global__ __launch_bounds__(256, 2) void rec_write(double* __restrict__ rec, int64_t nch, int work) {
  __shared__ double stage[4][64 * (RD + 1)];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t chunk = blockIdx.x * (int64_t)256 + threadIdx.x;
  const int chain = blockIdx.y;
  const int64_t n = nch * L;
  const int64_t G = nch / 64;
  const int64_t group = chunk >> 6;
  double x = 1.0 + 1e-3 * (double)chunk;
  double* sb = stage[wave];
  for (int s = 0; s < L; ++s) {
    for (int w = 0; w < work; ++w) x = fma(x, 0.999999, 1e-9);
    for (int e = 0; e < RD; ++e) sb[lane * (RD + 1) + e] = x + e;
    __builtin_amdgcn_wave_barrier();
    // 8 instructions: record r = 8 it + lane / 8, 16-byte piece lane % 8
    for (int it = 0; it < 8; ++it) {
      const int r = 8 * it + (lane >> 3), pc = lane & 7;
      const double a = sb[r * (RD + 1) + 2 * pc], b = sb[r * (RD + 1) + 2 * pc + 1];
      int64_t off;
      if constexpr (INTERLEAVED)
        off = ((((int64_t)chain * G + group) * L + s) * 64 + r) * RD;
      else
        off = ((int64_t)chain * n + (chunk - lane + r) * L + s) * RD;
      double2 v{a, b};
      *reinterpret_cast<double2*>(rec + off + 2 * pc) = v;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

int main(int argc, char** argv) {
  const int chains = argc > 1 ? std::atoi(argv[1]) : 62;
  const int work = argc > 2 ? std::atoi(argv[2]) : 0;
  const int64_t nch = 4096;                        // chunks per chain (1 048 576 steps)
  const size_t bytes = (size_t)chains * nch * L * RD * sizeof(double);
  double* rec = nullptr;
  CK(hipMalloc(&rec, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 grid((unsigned)(nch / 256), (unsigned)chains);
  for (int mode = 0; mode < 2; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(a, 0));
      if (mode == 0) rec_write<false><<<grid, 256>>>(rec, nch, work);
      else rec_write<true><<<grid, 256>>>(rec, nch, work);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      CK(hipGetLastError());
      float ms = 0.0f;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    std::printf("%s chains=%d work=%d: %.3f ms, %.2f TB/s\n", mode ? "interleaved " : "chunk-major ",
                chains, work, best, bytes / (best * 1e-3) / 1e12);
  }
  CK(hipFree(rec));
  return 0;
}
