// Accuracy of fp64 sqrt / exp building blocks on gfx950 (ulp error against host long double):
//   sqrt: x * v_rsq_f64(x) (raw seed), + one Goldschmidt step, + one Newton correction with the
//         unrefined half-reciprocal (6 VALU + rsq), and device_common.hpp's sqrt_pos;
//   exp(-x): device_common.hpp's exp_neg.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
#include "../../gpar-at-scale_amd/csrc/device_common.hpp"

__device__ __forceinline__ double exp_neg11(double x) {
  const double y = fmax(-x, -745.5);
  const double nf = rint(y * 1.4426950408889634074);
  double r = fma(-nf, 6.93147180369123816490e-01, y);
  r = fma(-nf, 1.90821492927058770002e-10, r);
  double p = 2.5110037605963777e-08;
  p = fma(p, r, 2.763263963904103e-07);
  p = fma(p, r, 2.755724091857897e-06);
  p = fma(p, r, 2.4801485482328494e-05);
  p = fma(p, r, 0.00019841269890047113);
  p = fma(p, r, 0.0013888888952314775);
  p = fma(p, r, 0.008333333333319601);
  p = fma(p, r, 0.0416666666664881);
  p = fma(p, r, 0.1666666666666668);
  p = fma(p, r, 0.5000000000000019);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)nf);
}

__global__ void k(const double* x, double* s1, double* s2, double* s3, double* s4, double* e1, double* e2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  const double y = __builtin_amdgcn_rsq(v);
  s1[i] = v * y;
  double g = v * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  s2[i] = g;
  const double d = fma(-g, g, v);
  s3[i] = fma(d, h, g);
  s4[i] = gpar::sqrt_pos(v);
  e1[i] = gpar::exp_neg(v * 1e-3 * (i % 1000));   // arguments 0 .. ~1e3 * |x|
  e2[i] = exp_neg11(v * 1e-3 * (i % 1000));
}

static double ulp_err(double got, long double ref) {
  const double r = (double)ref;
  if (r == 0.0) return got == 0.0 ? 0.0 : 1e300;
  const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
  return (double)(std::fabs((long double)got - ref) / u);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n);
  std::vector<std::vector<double>> o(6, std::vector<double>(n));
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> e(-12.0, 3.0), f(1.0, 10.0);
  for (int i = 0; i < n; ++i) x[i] = f(rng) * std::pow(10.0, e(rng));
  double* dx;
  double* d[6];
  (void)hipMalloc(&dx, n * 8);
  for (auto& p : d) (void)hipMalloc(&p, n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, d[0], d[1], d[2], d[3], d[4], d[5], n);
  for (int j = 0; j < 6; ++j) (void)hipMemcpy(o[j].data(), d[j], n * 8, hipMemcpyDeviceToHost);
  const char* names[6] = {"x*rsq(x)", "+Goldschmidt", "+Newton (6 VALU + rsq)", "sqrt_pos", "exp_neg", "exp_neg deg-11 minimax"};
  for (int j = 0; j < 6; ++j) {
    double mx = 0, s = 0;
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
      long double ref;
      if (j < 4) {
        ref = std::sqrt((long double)x[i]);
      } else {
        const double arg = x[i] * 1e-3 * (i % 1000);
        if (arg > 700) continue;
        ref = std::exp(-(long double)arg);
      }
      const double er = ulp_err(o[j][i], ref);
      mx = std::max(mx, er);
      s += er;
      ++cnt;
    }
    printf("%-26s max %.3g ulp, mean %.3g ulp (%d samples)\n", names[j], mx, s / cnt, cnt);
  }
  return 0;
}
