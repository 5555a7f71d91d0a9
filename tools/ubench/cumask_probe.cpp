// cumask_probe: which hardware CUs (XCC, SE, CU) a stream created with a CU mask runs on.
// For each test mask, launches many short workgroups on the masked stream; every workgroup
// records its XCC_ID and HW_ID (s_getreg reads) with a vector store; the host prints the
// distinct (xcc, se, cu) triples hit.  Build: hipcc --offload-arch=gfx950 -O2 -o cumask_probe
// cumask_probe.cpp
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>
#include <set>
#include <tuple>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                         \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__global__ void where(uint32_t* out) {
  if (threadIdx.x != 0) return;
  // HW_REG_HW_ID (4): whole 32 bits; HW_REG_XCC_ID (20): low 4 bits
  const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
  const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));
  // keep the workgroup resident a little so the dispatcher spreads them
  uint64_t t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < 20000) {
  }
  out[2 * blockIdx.x] = hw;
  out[2 * blockIdx.x + 1] = xcc;
}

int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int ncu = pr.multiProcessorCount;
  std::printf("CUs %d\n", ncu);
  const int nwg = 8192;
  uint32_t* d;
  CK(hipMalloc(&d, nwg * 2 * sizeof(uint32_t)));
  std::vector<uint32_t> h(nwg * 2);
  const int words = (ncu + 31) / 32;
  struct T {
    const char* name;
    int kind;
  } tests[] = {{"bits 0..31", 0}, {"bits i%8==0", 1}, {"bits i%32<4", 2}, {"bit 0 only", 3},
               {"bits 0..7", 4}, {"all", 5}, {"bits 0..39", 6}, {"bits 40..255", 7}};
  for (auto& t : tests) {
    std::vector<uint32_t> mask(words, 0);
    for (int i = 0; i < ncu; ++i) {
      bool on = t.kind == 0 ? i < 32 : t.kind == 1 ? i % 8 == 0 : t.kind == 2 ? i % 32 < 4
                : t.kind == 3 ? i == 0 : t.kind == 4 ? i < 8 : t.kind == 6 ? i < 40 : t.kind == 7 ? i >= 40 : true;
      if (on) mask[i / 32] |= 1u << (i % 32);
    }
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, words, mask.data()));
    CK(hipMemsetAsync(d, 0xff, nwg * 2 * sizeof(uint32_t), s));
    where<<<nwg, 64, 0, s>>>(d);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d, nwg * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::set<std::tuple<int, int, int>> seen;
    std::set<int> xccs;
    for (int b = 0; b < nwg; ++b) {
      const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
      const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
      seen.insert({(int)xcc, se, cu + 16 * sh});
      xccs.insert((int)xcc);
    }
    std::printf("%-14s: %zu distinct CUs, XCCs:", t.name, seen.size());
    for (int x : xccs) std::printf(" %d", x);
    std::printf("\n   ");
    int k = 0;
    for (auto& e : seen) {
      if (k++ < 48) std::printf(" (%d,%d,%d)", std::get<0>(e), std::get<1>(e), std::get<2>(e));
    }
    std::printf("\n");
    CK(hipStreamDestroy(s));
  }
  CK(hipFree(d));
  return 0;
}
