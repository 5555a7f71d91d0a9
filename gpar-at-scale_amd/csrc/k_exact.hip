// k_exact.hip -- dense exact GP / GPAR on gfx950.
//
// Replaces Stheno's dense path used by create_optim_gp / create_optim_gpar
// (src/gp/optimized.jl:19-59, 106-183) and the posterior marginals (optimized.jl:94,236;
// plot_examples.jl:106-122):
//   K(x, x') = s_t k_t(|x_0 - x'_0| / l_t) + s_o k_o(||x_{1:} - x'_{1:}|| / l_o)    (:132-144)
//   logpdf   = -1/2 [n log 2pi + logdet(K + s2 I) + y' (K + s2 I)^{-1} y]           (:152)
//   mean_*   = K_*' (K + s2 I)^{-1} y,  var_* = k_** - ||L^{-1} K_*||^2
// The n x n Cholesky / triangular solves reuse k_dense.hip; this file holds the covariance
// assembly and the reductions.  Distances are direct differences (Stheno's pairwise on 1-D
// time and on the masked output coordinates).
#include "device_common.hpp"

namespace gpar {

// K[i * ldk + j] = cov(x_i, x2_j) (+ diag on i == j).  x point k, dim q at x[k * ldx + q].
__global__ __launch_bounds__(256) void exact_cov_kernel(
    const double* __restrict__ x, int64_t ldx, int64_t n, const double* __restrict__ x2,
    int64_t ldx2, int64_t n2, int dx, int tk, int ok, double inv_lt, double st, double inv_lo,
    double so, double diag, double* __restrict__ K, int64_t ldk) {
  const int64_t j = (int64_t)blockIdx.x * 16 + (threadIdx.x & 15);
  const int64_t i = (int64_t)blockIdx.y * 16 + (threadIdx.x >> 4);
  if (i >= n || j >= n2) return;
  const double* a = x + i * ldx;
  const double* b = x2 + j * ldx2;
  double k = st * kappa_rt(tk, fabs(a[0] - b[0]) * inv_lt);
  if (dx > 1) {
    double d2 = 0.0;
    for (int q = 1; q < dx; ++q) {
      const double e = a[q] - b[q];
      d2 = fma(e, e, d2);
    }
    k += so * kappa_rt(ok, sqrt(d2) * inv_lo);
  }
  if (i == j) k += diag;
  K[i * ldk + j] = k;
}

// lml = -1/2 [n log 2pi + 2 sum log L_ii + |w|^2], w = L^{-1} y; NaN if the Cholesky failed.
__global__ __launch_bounds__(256) void exact_logpdf_finish(const double* __restrict__ L, int64_t ld,
                                                           int n, const double* __restrict__ w,
                                                           const int* __restrict__ status,
                                                           double* __restrict__ out) {
  __shared__ double red[2][4];
  double ld_ = 0.0, ww = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    ld_ += log(L[(int64_t)i * ld + i]);
    ww = fma(w[i], w[i], ww);
  }
  ld_ = wave_sum(ld_);
  ww = wave_sum(ww);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wave] = ld_;
    red[1][wave] = ww;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const double b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    *out = *status ? __builtin_nan("") : -0.5 * ((double)n * kLog2Pi + 2.0 * a + b);
  }
}

// W = L^{-1} K_* (n x n_star, row-major ld): mean_j = sum_i W_ij w_i, var_j = kss - sum_i W_ij^2.
__global__ __launch_bounds__(256) void exact_post_kernel(const double* __restrict__ W, int64_t ldw,
                                                         int n, int64_t n_star,
                                                         const double* __restrict__ w, double kss,
                                                         double* __restrict__ mean,
                                                         double* __restrict__ var) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n_star) return;
  double m = 0.0, s = 0.0;
  for (int i = 0; i < n; ++i) {
    const double v = W[(int64_t)i * ldw + j];
    m = fma(v, w[i], m);
    s = fma(v, v, s);
  }
  mean[j] = m;
  var[j] = kss - s;
}

void launch_exact_cov(hipStream_t st, const double* x, int64_t ldx, int64_t n, const double* x2,
                      int64_t ldx2, int64_t n2, int dx, int tk, int ok, double inv_lt, double s_t,
                      double inv_lo, double s_o, double diag, double* K, int64_t ldk) {
  dim3 grid((unsigned)((n2 + 15) / 16), (unsigned)((n + 15) / 16));
  exact_cov_kernel<<<grid, 256, 0, st>>>(x, ldx, n, x2, ldx2, n2, dx, tk, ok, inv_lt, s_t, inv_lo,
                                         s_o, diag, K, ldk);
}

void launch_exact_logpdf_finish(hipStream_t st, const double* L, int64_t ld, int n, const double* w,
                                const int* status, double* out) {
  exact_logpdf_finish<<<1, 256, 0, st>>>(L, ld, n, w, status, out);
}

void launch_exact_post(hipStream_t st, const double* W, int64_t ldw, int n, int64_t n_star,
                       const double* w, double kss, double* mean, double* var) {
  exact_post_kernel<<<(unsigned)((n_star + 255) / 256), 256, 0, st>>>(W, ldw, n, n_star, w, kss,
                                                                     mean, var);
}

}  // namespace gpar
