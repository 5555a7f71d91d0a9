// k_path.hip -- posterior path sampling on gfx950: TemporalGPs `posterior_rand` (called at
// src/gp/tmp.jl:161-167) and the path Monte Carlo estimator of the scaled-GPAR prediction that
// tmp.jl:119-167 builds on it.
//
// Draws come from the simulation smoother of Durbin & Koopman (2002), batched over S samples that
// share the chain's gains (oracle/gpar_oracle.py lgssm_posterior_rand restates it):
//   prior path   x~_0 = chol(s Pinf) eta_0,  x~_k = A_k x~_{k-1} + chol(Q_k) eta_k,
//                y~_k = x~_k[0] + sqrt(R_k) eps_k      (Q_k in closed form: sde_q_stable)
//   sample       f_s = x~[0] + E[f | y - y~]           (exactly a draw from p(f | y))
// E[f | v] = v - R Sigma^{-1} v is the smoother mean the prediction already computes through the
// whitening's adjoint (Sigma^{-1} = W^T W, k_lgssm.hip): S data columns, one shared gains record.
// Forward-filter backward-sample draws from the same posterior, but its backward coefficients
// J_k = P_k A^T (P^-_{k+1})^{-1} amplify rounding on the clustered merged grids of a prediction
// (the oracle measured Matern-5/2 draws moving by 1.6e-2 under 1e-13 relative perturbations of the
// model on a 700-point grid with dt down to 8e-5; this form moves them by 4e-13), so the device uses
// this form.  The prior path is an affine recurrence, time-chunked like the whitening: a local pass
// per (sample, chunk) from zero, a carry over chunks with Phi_j = prod A_k, a final pass from the
// true incoming state.  Threads are (sample, chunk) pairs, samples fastest.  Draws
// eta_{s,k,i} = counter_normal(path seed, s, k (D + 1) + i) (i < D), eps_{s,k} = the same at
// i = D (device_common.hpp), exported by gpar_path_normals with d = D + 1.
#include "device_common.hpp"

namespace gpar {

// ---------------------------------------------------------------------------- Cf*u from distances
// In place: r (Matern kernels) or r^2 (EQ) -> s_o kappa(r / l_o) for c < m, 0 on the padding
// (the same device functions as the whitening kernels' on-the-fly Kfu).
template <int OK>
__global__ __launch_bounds__(256) void kfu_from_dist(double* __restrict__ K, int64_t n, int64_t m,
                                                     int64_t mp, double inv_l, double s,
                                                     ExpNegConsts ec) {
  const int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (e >= n * mp) return;
  const int64_t c = e % mp;
  if (c >= m) {
    K[e] = 0.0;
    return;
  }
  const double v = K[e];
  if constexpr (OK == KEQ)
    K[e] = skappa_sq_k<KEQ>(v, inv_l, s, ec);
  else
    K[e] = skappa_r_k<OK>(v, inv_l, s, ec);
}

// ---------------------------------------------------------------------------- q(u) sample loadings
// Bm[s * ldb + c] = w[c] + sum_j W[j * ld + c] xi[s * ldxi + j]  (c < m; 0 up to mp): the
// pseudo-point sample U_u^{-1} (m_e + Lc xi_s) = w + W^T xi_s with W = Lc^T L_u^{-1}
// (mc_factor_kernel), w = U_u^{-1} m_e.
__global__ __launch_bounds__(256) void path_bmat(const double* __restrict__ W, int64_t ld,
                                                 const double* __restrict__ w,
                                                 const double* __restrict__ xi, int64_t ldxi,
                                                 int S, int m, int64_t mp, double* __restrict__ Bm,
                                                 int64_t ldb) {
  const int64_t c = blockIdx.x * (int64_t)256 + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= mp || s >= S) return;
  double acc = 0.0;
  if (c < m) {
    acc = w[c];
    const double* xs = xi + (int64_t)s * ldxi;
    for (int j = 0; j < m; ++j) acc = fma(W[(int64_t)j * ld + c], xs[j], acc);
  }
  Bm[(int64_t)s * ldb + c] = acc;
}

// ---------------------------------------------------------------------------- prior paths
template <int D>
__device__ __forceinline__ void chol_guarded(const double (&C)[D][D], double (&L)[D][D]) {
  mat_zero(L);
#pragma unroll
  for (int j = 0; j < D; ++j) {
    double t = C[j][j];
#pragma unroll
    for (int q = 0; q < j; ++q) t -= L[j][q] * L[j][q];
    L[j][j] = t > 0.0 ? sqrt(t) : 0.0;
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      double v = C[i][j];
#pragma unroll
      for (int q = 0; q < j; ++q) v -= L[i][q] * L[j][q];
      L[i][j] = L[j][j] > 0.0 ? v / L[j][j] : 0.0;
    }
  }
}

// Regularized lower incomplete gamma P(m1, x), integer m1 >= 1: the series
// e^{-x} sum_{k >= m1} x^k / k! for x < 4 (no cancellation for short steps), else
// 1 - e^{-x} sum_{k < m1} x^k / k!  (oracle/gpar_oracle.py _inc_gamma_p, the same loops)
__device__ double inc_gamma_p(int m1, double x) {
  if (x < 4.0) {
    double t = exp(-x);
    for (int k = 1; k <= m1; ++k) t *= x / k;
    double acc = 0.0;
    int k = m1;
    for (int it = 0; it < 80; ++it) {
      acc += t;
      ++k;
      t *= x / k;
      if (t < 1e-18 * acc) break;
    }
    return acc;
  }
  double term = 1.0, tot = 1.0;
  for (int k = 1; k < m1; ++k) {
    term *= x / k;
    tot += term;
  }
  return 1.0 - exp(-x) * tot;
}

// Q(tau) = s Pinf - A s Pinf A^T in closed form (oracle sde_q_stable): Q = q s int_0^tau a a^T with
// a(u) = exp(F u) e_D = e^{-lam u} sum_p al[i][p] u^p; the integrals int_0^tau u^m e^{-2 lam u} du =
// m! / (2 lam)^{m+1} P(m + 1, 2 lam tau).  Accurate for short steps, where the subtraction form
// loses the small eigenvalues' digits (the prior path factors it).
template <int D>
__device__ void sde_q_stable(double tau, double s, double (&Q)[D][D]) {
  double al[D][D], q, lam;
  if constexpr (D == 1) {
    lam = 1.0;
    al[0][0] = 1.0;
    q = 2.0;
  } else if constexpr (D == 2) {
    lam = kSqrt3;
    al[0][0] = 0.0; al[0][1] = 1.0;
    al[1][0] = 1.0; al[1][1] = -lam;
    q = 4.0 * lam * lam * lam;
  } else {
    lam = kSqrt5;
    al[0][0] = 0.0; al[0][1] = 0.0;        al[0][2] = 0.5;
    al[1][0] = 0.0; al[1][1] = 1.0;        al[1][2] = -0.5 * lam;
    al[2][0] = 1.0; al[2][1] = -2.0 * lam; al[2][2] = 0.5 * lam * lam;
    q = 16.0 * lam * lam * lam * lam * lam / 3.0;
  }
  double I[2 * D - 1];
  const double x = 2.0 * lam * tau;
  double fact = 1.0, pw = 2.0 * lam;   // m!, (2 lam)^{m+1}
  for (int m = 0; m < 2 * D - 1; ++m) {
    if (m > 0) {
      fact *= m;
      pw *= 2.0 * lam;
    }
    I[m] = fact / pw * inc_gamma_p(m + 1, x);
  }
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int r = 0; r < D; ++r) acc += al[i][p] * al[j][r] * I[p + r];
      Q[i][j] = q * s * acc;
    }
}

// lq[k] = chol(Q_k) (row-major D x D; Q_k of the step's scaled length (t_k - t_{k-1}) / l in closed
// form, so short steps keep their small eigenvalues), lq[0] = chol(s Pinf) (the stationary start)
template <int D>
__global__ __launch_bounds__(256) void dk_consts(const double* __restrict__ t, int64_t n,
                                                 double inv_l, double s, double* __restrict__ lq) {
  const int64_t k = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (k >= n) return;
  double Q[D][D], L[D][D];
  if (k == 0)
    sde_pinf<D>(s, Q);
  else
    sde_q_stable<D>((t[k] - t[k - 1]) * inv_l, s, Q);
  chol_guarded<D>(Q, L);
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) lq[k * D * D + i * D + q] = L[i][q];
}

// phia[j] = A_{k1-1} ... A_{k0} (the prior path's chunk transfer; step 0 starts afresh: A_0 = 0)
template <int D>
__global__ __launch_bounds__(256) void dk_phi(const double* __restrict__ rec, int64_t n, int L,
                                              int64_t nch, double* __restrict__ phia) {
  constexpr int RS = Rec<D>::size;
  const int64_t j = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (j >= nch) return;
  const int64_t k0 = j * L, k1 = (k0 + L < n) ? k0 + L : n;
  double Ph[D][D], A[D][D], X[D][D];
  mat_eye(Ph);
  for (int64_t k = k0; k < k1; ++k) {
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int q = 0; q < D; ++q) A[i][q] = k == 0 ? 0.0 : rec[k * RS + i * D + q];
    mat_mul(A, Ph, X);
    mat_copy(X, Ph);
  }
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int q = 0; q < D; ++q) phia[j * D * D + i * D + q] = Ph[i][q];
}

__device__ __forceinline__ double path_noise(const double* __restrict__ noise, int64_t k, double r) {
  if (!noise) return r;
  const double v = noise[k];
  return v < 0.0 ? r : v;
}

// Prior path of sample s over chunk j (thread = (s, j), s fastest).  cin null: local pass from
// zero, chunk end state -> send[(j * S + s) * 4 + i].  Else from the true incoming state:
// ft[k * S + s] = x~_k[0] and z[s * n + k] = ym[k] - fx[k * ldfx + s] - y~_k (fx null: no fx term),
// the data column whose smoother mean completes the draw.
template <int D>
__global__ __launch_bounds__(256) void dk_prior(const double* __restrict__ rec,
                                                const double* __restrict__ lq,
                                                const double* __restrict__ noise, double r,
                                                int64_t n, int L, int64_t nch, int S, uint64_t seed,
                                                const double* __restrict__ ym,
                                                const double* __restrict__ fx, int64_t ldfx,
                                                const double* __restrict__ cin,
                                                double* __restrict__ send,
                                                double* __restrict__ ft, double* __restrict__ z) {
  constexpr int RS = Rec<D>::size;
  const int64_t idx = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (idx >= (int64_t)S * nch) return;
  const int s = (int)(idx % S);
  const int64_t j = idx / S;
  const int64_t k0 = j * L, k1 = (k0 + L < n) ? k0 + L : n;
  double x[D];
#pragma unroll
  for (int i = 0; i < D; ++i) x[i] = cin ? cin[(j * S + s) * kSStride + i] : 0.0;
  for (int64_t k = k0; k < k1; ++k) {
    const double* a = rec + k * RS;
    const double* l = lq + k * D * D;
    double eta[D], nx[D];
#pragma unroll
    for (int i = 0; i < D; ++i) eta[i] = counter_normal(seed, (uint64_t)s, (uint64_t)(k * (D + 1) + i));
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = 0.0;
      if (k > 0) {
#pragma unroll
        for (int q = 0; q < D; ++q) acc = fma(a[i * D + q], x[q], acc);
      }
#pragma unroll
      for (int q = 0; q <= i; ++q) acc = fma(l[i * D + q], eta[q], acc);
      nx[i] = acc;
    }
#pragma unroll
    for (int i = 0; i < D; ++i) x[i] = nx[i];
    if (ft) {
      const double eps = counter_normal(seed, (uint64_t)s, (uint64_t)(k * (D + 1) + D));
      const double yt = fma(sqrt(path_noise(noise, k, r)), eps, x[0]);
      ft[k * S + s] = x[0];
      z[(int64_t)s * n + k] = (fx ? ym[k] - fx[k * ldfx + s] : ym[k]) - yt;
    }
  }
  if (send) {
#pragma unroll
    for (int i = 0; i < D; ++i) send[(j * S + s) * kSStride + i] = x[i];
  }
}

// f[k * S + s] += z[s * n + k] - R_k (u_{k,s} + h_k . chat[j][s]): the smoother mean of the
// column (v - R Sigma^{-1} v) added to the prior path (thread = (s, j), s fastest)
template <int D>
__global__ __launch_bounds__(256) void dk_finish(const double* __restrict__ X, int64_t ldx,
                                                 const double* __restrict__ h,
                                                 const double* __restrict__ chat,
                                                 const double* __restrict__ z,
                                                 const double* __restrict__ noise, double r,
                                                 int64_t n, int L, int64_t nch, int S,
                                                 double* __restrict__ f) {
  const int64_t idx = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (idx >= (int64_t)S * nch) return;
  const int s = (int)(idx % S);
  const int64_t j = idx / S;
  const int64_t k0 = j * L, k1 = (k0 + L < n) ? k0 + L : n;
  double ch[D];
#pragma unroll
  for (int i = 0; i < D; ++i) ch[i] = chat[(j * S + s) * kSStride + i];
  for (int64_t k = k0; k < k1; ++k) {
    double u = X[k * ldx + s];
#pragma unroll
    for (int i = 0; i < D; ++i) u = fma(h[k * kGStride + i], ch[i], u);
    f[k * S + s] += z[(int64_t)s * n + k] - path_noise(noise, k, r) * u;
  }
}

// ---------------------------------------------------------------------------- outputs
// Path Monte Carlo statistics at the test points (gpar_scaled_inference.jl:130-135 reduces its
// samples this way): one wave per test point i at merged row k = pos[i], samples v_s =
// fx[k * ldfx + s] + F[k * S + s]; mean and Bessel std over s.
__global__ __launch_bounds__(256) void path_stats(const double* __restrict__ fx, int64_t ldfx,
                                                  const double* __restrict__ F, int S,
                                                  const int64_t* __restrict__ pos, int64_t nstar,
                                                  double* __restrict__ mean,
                                                  double* __restrict__ std) {
  const int64_t i = blockIdx.x * (int64_t)4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= nstar) return;
  const int64_t k = pos[i];
  double a = 0.0;
  for (int s = lane; s < S; s += 64) a += fx[k * ldfx + s] + F[k * S + s];
  const double mu = wave_sum(a) / (double)S;
  double q = 0.0;
  for (int s = lane; s < S; s += 64) {
    const double v = fx[k * ldfx + s] + F[k * S + s] - mu;
    q = fma(v, v, q);
  }
  const double var = wave_sum(q) / (double)(S - 1);
  if (lane == 0) {
    mean[i] = mu;
    std[i] = sqrt(var);
  }
}

// out[s * n + k] = F[k * S + s] (the posterior_rand entry point's sample-major layout)
__global__ __launch_bounds__(256) void path_transpose(const double* __restrict__ F, int64_t n, int S,
                                                      double* __restrict__ out) {
  const int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (e >= n * S) return;
  const int64_t k = e % n, s = e / n;
  out[e] = F[k * S + s];
}

// ---------------------------------------------------------------------------- launchers
void launch_kfu_from_dist(hipStream_t st, int out_kind, double* K, int64_t n, int64_t m,
                          int64_t mp, double inv_l, double s) {
  const unsigned nb = (unsigned)((n * mp + 255) / 256);
  const ExpNegConsts ec = exp_neg_consts();
  switch (out_kind) {
    case KM12: kfu_from_dist<KM12><<<nb, 256, 0, st>>>(K, n, m, mp, inv_l, s, ec); break;
    case KM32: kfu_from_dist<KM32><<<nb, 256, 0, st>>>(K, n, m, mp, inv_l, s, ec); break;
    case KM52: kfu_from_dist<KM52><<<nb, 256, 0, st>>>(K, n, m, mp, inv_l, s, ec); break;
    default: kfu_from_dist<KEQ><<<nb, 256, 0, st>>>(K, n, m, mp, inv_l, s, ec); break;
  }
}

void launch_path_bmat(hipStream_t st, const double* W, int64_t ld, const double* w, const double* xi,
                      int64_t ldxi, int S, int m, int64_t mp, double* Bm, int64_t ldb) {
  dim3 grid((unsigned)((mp + 255) / 256), (unsigned)S);
  path_bmat<<<grid, 256, 0, st>>>(W, ld, w, xi, ldxi, S, m, mp, Bm, ldb);
}

#define GPAR_PATH_DISPATCH(sdim, call) \
  switch (sdim) {                      \
    case 1: { constexpr int D = 1; call; } break; \
    case 2: { constexpr int D = 2; call; } break; \
    default: { constexpr int D = 3; call; } break; \
  }

void launch_dk_consts(hipStream_t st, int sdim, const double* t, int64_t n, double inv_l, double s,
                      double* lq) {
  const unsigned nb = (unsigned)((n + 255) / 256);
  GPAR_PATH_DISPATCH(sdim, (dk_consts<D><<<nb, 256, 0, st>>>(t, n, inv_l, s, lq)));
}

void launch_dk_phi(hipStream_t st, int sdim, const double* rec, int64_t n, int L, int64_t nch,
                   double* phia) {
  const unsigned nb = (unsigned)((nch + 255) / 256);
  GPAR_PATH_DISPATCH(sdim, (dk_phi<D><<<nb, 256, 0, st>>>(rec, n, L, nch, phia)));
}

void launch_dk_prior(hipStream_t st, int sdim, const double* rec, const double* lq,
                     const double* noise, double r, int64_t n, int L, int64_t nch, int S,
                     uint64_t seed, const double* ym, const double* fx, int64_t ldfx,
                     const double* cin, double* send, double* ft, double* z) {
  const unsigned nb = (unsigned)(((int64_t)S * nch + 255) / 256);
  GPAR_PATH_DISPATCH(sdim, (dk_prior<D><<<nb, 256, 0, st>>>(rec, lq, noise, r, n, L, nch, S, seed,
                                                             ym, fx, ldfx, cin, send, ft, z)));
}

void launch_dk_finish(hipStream_t st, int sdim, const double* X, int64_t ldx, const double* h,
                      const double* chat, const double* z, const double* noise, double r,
                      int64_t n, int L, int64_t nch, int S, double* f) {
  const unsigned nb = (unsigned)(((int64_t)S * nch + 255) / 256);
  GPAR_PATH_DISPATCH(sdim, (dk_finish<D><<<nb, 256, 0, st>>>(X, ldx, h, chat, z, noise, r, n, L,
                                                              nch, S, f)));
}
#undef GPAR_PATH_DISPATCH

void launch_path_stats(hipStream_t st, const double* fx, int64_t ldfx, const double* F, int S,
                       const int64_t* pos, int64_t nstar, double* mean, double* std) {
  path_stats<<<(unsigned)((nstar + 3) / 4), 256, 0, st>>>(fx, ldfx, F, S, pos, nstar, mean, std);
}

void launch_path_transpose(hipStream_t st, const double* F, int64_t n, int S, double* out) {
  path_transpose<<<(unsigned)((n * S + 255) / 256), 256, 0, st>>>(F, n, S, out);
}

}  // namespace gpar
