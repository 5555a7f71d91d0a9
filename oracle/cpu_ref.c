/* cpu_ref.c -- C/OpenMP restatement of the reference's CPU hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Used only by tests/ (checked against the numpy oracle, oracle/gpar_oracle.py) and by the
 * cpu_baseline leg of bench.py, as the timed CPU baseline (SURVEY.md §8d "cpu_ref"):  the
 * reference's own Julia path cannot run in this image (no Julia).  The product
 * path (gpar-at-scale_amd/) never loads it.
 *
 * It follows the reference's operation order for the per-output DTC objective and the
 * prediction, with the numerically heavy, BLAS-free parts in C:
 *   gpar_cpu_pairwise      Stheno pairwise(kernel(k; l, s), V, Z)     dtc.jl:104,119;
 *                          gpar_scaled_inference.jl:89,156-157 (direct differences)
 *   gpar_cpu_gains         TemporalGPs to_sde + Riccati recursion      dtc.jl:101-102;
 *                          temporal_gp_inference.jl:28-38 (stationary start, tau_1 = 1)
 *   gpar_cpu_filter        decorrelate over the columns of X           dtc.jl:106,110-117;
 *                          gpar_scaled_inference.jl:175,183
 *   gpar_cpu_smooth_first  RTS smoother, first state component         temporal_gp_inference.jl:109;
 *                          gpar_scaled_inference.jl:117
 * The dense M x M / M x N algebra (cholesky, trsm, gemm: dtc.jl:119-125) is left to OpenBLAS
 * through numpy/scipy by oracle/cpu_ref.py, as the reference leaves it to Julia's OpenBLAS.
 *
 * Deliberately faster than a literal port: the reference runs one sequential Kalman sweep per
 * column (dtc.jl:110-117); here one pass over the steps advances a block of columns at once
 * (vectorised across columns, OpenMP over column blocks).  That makes the CPU baseline a
 * stronger, not weaker, comparison.
 *
 * Layouts: V is D x N column-major (point k, dim i at V[k*D + i], util.jl:16-31), Z is D x M,
 * X / out matrices are step-major: row k, column c at X[k*ldx + c].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { KM12 = 0, KM32 = 1, KM52 = 2, KEQ = 3 };

static double kappa(int kind, double r) {
  switch (kind) {
    case KM12: return exp(-r);
    case KM32: { const double x = sqrt(3.0) * r; return (1.0 + x) * exp(-x); }
    case KM52: { const double x = sqrt(5.0) * r; return (1.0 + x + x * x / 3.0) * exp(-x); }
    default: return exp(-0.5 * r * r);
  }
}

/* out[k*ldo + c] = s * kappa(||V[:,k] - Z[:,c]|| / l), k < n, c < m. */
void gpar_cpu_pairwise(int kind, const double* V, int64_t n, const double* Z, int64_t m, int64_t d,
                       double l, double s, double* out, int64_t ldo) {
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < n; ++k) {
    const double* v = V + k * d;
    double* o = out + k * ldo;
    for (int64_t c = 0; c < m; ++c) {
      const double* z = Z + c * d;
      double s2 = 0.0;
      for (int64_t i = 0; i < d; ++i) {
        const double df = v[i] - z[i];
        s2 += df * df;
      }
      o[c] = s * kappa(kind, sqrt(s2) / l);
    }
  }
}

static int sde_dim(int kind) { return kind == KM12 ? 1 : (kind == KM32 ? 2 : 3); }

static void sde_pinf(int kind, double s, double P[3][3]) {
  memset(P, 0, sizeof(double) * 9);
  if (kind == KM12) {
    P[0][0] = s;
  } else if (kind == KM32) {
    P[0][0] = s; P[1][1] = 3.0 * s;
  } else {
    P[0][0] = s; P[0][2] = -(5.0 / 3.0) * s; P[1][1] = (5.0 / 3.0) * s;
    P[2][0] = -(5.0 / 3.0) * s; P[2][2] = 25.0 * s;
  }
}

/* A = exp(F tau) = e^{-lam tau} (I + tau N + tau^2/2 N^2), N = F + lam I nilpotent. */
static void sde_transition(int kind, double tau, double A[3][3]) {
  memset(A, 0, sizeof(double) * 9);
  if (kind == KM12) {
    A[0][0] = exp(-tau);
    return;
  }
  if (kind == KM32) {
    const double lam = sqrt(3.0), e = exp(-lam * tau);
    /* N = [[lam, 1], [-lam^2, -lam]] */
    A[0][0] = e * (1.0 + tau * lam); A[0][1] = e * tau;
    A[1][0] = e * (-tau * lam * lam); A[1][1] = e * (1.0 - tau * lam);
    return;
  }
  const double lam = sqrt(5.0), e = exp(-lam * tau);
  const double Nm[3][3] = {{lam, 1.0, 0.0}, {0.0, lam, 1.0}, {-lam * lam * lam, -3.0 * lam * lam, -2.0 * lam}};
  double N2[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double a = 0.0;
      for (int q = 0; q < 3; ++q) a += Nm[i][q] * Nm[q][j];
      N2[i][j] = a;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      A[i][j] = e * ((i == j ? 1.0 : 0.0) + tau * Nm[i][j] + 0.5 * tau * tau * N2[i][j]);
}

/* Gains of the discretised time GP over t (ascending), per step k:
 *   rec[k*16 + 0..8] = A_k (row-major 3x3, padded), rec[k*16 + 9..11] = K_k, rec[k*16 + 12] = S_k,
 *   pf[k*9..]  = filtered covariance, pp[k*9..] = predicted covariance (either may be NULL).
 * R: per-step noise variance when rvec != NULL, else r.  Returns sum_k log S_k. */
double gpar_cpu_gains(int kind, const double* t, int64_t n, double l, double s, double r,
                      const double* rvec, double* rec, double* pf, double* pp) {
  const int d = sde_dim(kind);
  double pinf[3][3], P[3][3];
  sde_pinf(kind, s, pinf);
  memcpy(P, pinf, sizeof P);
  double logs = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const double tau = k == 0 ? 1.0 : (t[k] - t[k - 1]) / l;
    double A[3][3], AP[3][3], Pm[3][3], Q[3][3], Ap[3][3];
    sde_transition(kind, tau, A);
    /* Q = Pinf - A Pinf A^T */
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        double a = 0.0;
        for (int q = 0; q < d; ++q) a += A[i][q] * pinf[q][j];
        Ap[i][j] = a;
      }
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        double a = 0.0;
        for (int q = 0; q < d; ++q) a += Ap[i][q] * A[j][q];
        Q[i][j] = pinf[i][j] - a;
      }
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        double a = 0.0;
        for (int q = 0; q < d; ++q) a += A[i][q] * P[q][j];
        AP[i][j] = a;
      }
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        double a = 0.0;
        for (int q = 0; q < d; ++q) a += AP[i][q] * A[j][q];
        Pm[i][j] = a + Q[i][j];
      }
    const double Sk = Pm[0][0] + (rvec ? rvec[k] : r);
    double K[3];
    for (int i = 0; i < d; ++i) K[i] = Pm[i][0] / Sk;
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) P[i][j] = Pm[i][j] - K[i] * Pm[0][j];
    double* rk = rec + k * 16;
    memset(rk, 0, sizeof(double) * 16);
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) rk[i * 3 + j] = A[i][j];
    for (int i = 0; i < d; ++i) rk[9 + i] = K[i];
    rk[12] = Sk;
    if (pf)
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) pf[k * 9 + i * 3 + j] = (i < d && j < d) ? P[i][j] : 0.0;
    if (pp)
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) pp[k * 9 + i * 3 + j] = (i < d && j < d) ? Pm[i][j] : 0.0;
    logs += log(Sk);
  }
  return logs;
}

#define CB 64   /* columns advanced together */

/* Kalman filter (decorrelate) of every column of X: alpha[k*lda + c] = innovation / sqrt(S_k).
 * mf (optional): filtered state means, mf[(k*3 + i)*ldm + c]. */
void gpar_cpu_filter(int kind, const double* rec, int64_t n, const double* X, int64_t ldx,
                     int64_t ncol, double* alpha, int64_t lda, double* mf, int64_t ldm) {
  const int d = sde_dim(kind);
  const int64_t nb = (ncol + CB - 1) / CB;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t c0 = b * CB, cn = (c0 + CB <= ncol) ? CB : ncol - c0;
    double m0[CB], m1[CB], m2[CB];
    for (int c = 0; c < CB; ++c) m0[c] = m1[c] = m2[c] = 0.0;
    for (int64_t k = 0; k < n; ++k) {
      const double* rk = rec + k * 16;
      const double rs = 1.0 / sqrt(rk[12]);
      const double* x = X + k * ldx + c0;
      double* al = alpha + k * lda + c0;
      if (d == 3) {
        for (int c = 0; c < cn; ++c) {
          const double a0 = rk[0] * m0[c] + rk[1] * m1[c] + rk[2] * m2[c];
          const double a1 = rk[3] * m0[c] + rk[4] * m1[c] + rk[5] * m2[c];
          const double a2 = rk[6] * m0[c] + rk[7] * m1[c] + rk[8] * m2[c];
          const double e = x[c] - a0;
          al[c] = e * rs;
          m0[c] = a0 + rk[9] * e; m1[c] = a1 + rk[10] * e; m2[c] = a2 + rk[11] * e;
        }
      } else if (d == 2) {
        for (int c = 0; c < cn; ++c) {
          const double a0 = rk[0] * m0[c] + rk[1] * m1[c];
          const double a1 = rk[3] * m0[c] + rk[4] * m1[c];
          const double e = x[c] - a0;
          al[c] = e * rs;
          m0[c] = a0 + rk[9] * e; m1[c] = a1 + rk[10] * e;
        }
      } else {
        for (int c = 0; c < cn; ++c) {
          const double a0 = rk[0] * m0[c];
          const double e = x[c] - a0;
          al[c] = e * rs;
          m0[c] = a0 + rk[9] * e;
        }
      }
      if (mf) {
        double* f = mf + (k * 3) * ldm + c0;
        for (int c = 0; c < cn; ++c) {
          f[c] = m0[c];
          f[ldm + c] = m1[c];
          f[2 * ldm + c] = m2[c];
        }
      }
    }
  }
}

static void inv3(int d, const double M[3][3], double R[3][3]) {
  memset(R, 0, sizeof(double) * 9);
  if (d == 1) {
    R[0][0] = 1.0 / M[0][0];
  } else if (d == 2) {
    const double det = M[0][0] * M[1][1] - M[0][1] * M[1][0];
    R[0][0] = M[1][1] / det; R[0][1] = -M[0][1] / det;
    R[1][0] = -M[1][0] / det; R[1][1] = M[0][0] / det;
  } else {
    const double c00 = M[1][1] * M[2][2] - M[1][2] * M[2][1];
    const double c01 = M[1][2] * M[2][0] - M[1][0] * M[2][2];
    const double c02 = M[1][0] * M[2][1] - M[1][1] * M[2][0];
    const double det = M[0][0] * c00 + M[0][1] * c01 + M[0][2] * c02;
    R[0][0] = c00 / det;
    R[0][1] = (M[0][2] * M[2][1] - M[0][1] * M[2][2]) / det;
    R[0][2] = (M[0][1] * M[1][2] - M[0][2] * M[1][1]) / det;
    R[1][0] = c01 / det;
    R[1][1] = (M[0][0] * M[2][2] - M[0][2] * M[2][0]) / det;
    R[1][2] = (M[0][2] * M[1][0] - M[0][0] * M[1][2]) / det;
    R[2][0] = c02 / det;
    R[2][1] = (M[0][1] * M[2][0] - M[0][0] * M[2][1]) / det;
    R[2][2] = (M[0][0] * M[1][1] - M[0][1] * M[1][0]) / det;
  }
}

/* RTS smoother gain G_k = Pf_k A_{k+1}^T Pp_{k+1}^{-1} (3x3 row-major, zero-padded), k < n - 1. */
static void smoother_gain(int d, const double* rec, const double* pf, const double* pp, int64_t k,
                          double* G) {
  double Pf[3][3], A[3][3], Pp[3][3], Pi[3][3], T[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      Pf[i][j] = pf[k * 9 + i * 3 + j];
      A[i][j] = rec[(k + 1) * 16 + i * 3 + j];
      Pp[i][j] = pp[(k + 1) * 9 + i * 3 + j];
    }
  inv3(d, Pp, Pi);
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) {
      double a = 0.0;
      for (int q = 0; q < d; ++q) a += Pf[i][q] * A[j][q];
      T[i][j] = a;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double a = 0.0;
      if (i < d && j < d)
        for (int q = 0; q < d; ++q) a += T[i][q] * Pi[q][j];
      G[i * 3 + j] = a;
    }
}

/* RTS smoother over every column of X; out[k*ldo + c] = first component of the smoothed state
 * mean (the `.m[1]` the reference reads, gpar_scaled_inference.jl:117-127).
 * pf, pp: filtered / predicted covariances from gpar_cpu_gains.  Scratch: 3*n*ncol doubles. */
int gpar_cpu_smooth_first(int kind, const double* rec, const double* pf, const double* pp, int64_t n,
                          const double* X, int64_t ldx, int64_t ncol, double* out, int64_t ldo) {
  const int d = sde_dim(kind);
  double* mf = (double*)malloc(sizeof(double) * 3 * n * ncol);
  double* al = (double*)malloc(sizeof(double) * n * ncol);
  double* G = (double*)malloc(sizeof(double) * 9 * n);
  if (!mf || !al || !G) {
    free(mf); free(al); free(G);
    return 1;
  }
  gpar_cpu_filter(kind, rec, n, X, ldx, ncol, al, ncol, mf, ncol);
  for (int64_t k = 0; k + 1 < n; ++k) smoother_gain(d, rec, pf, pp, k, G + k * 9);
  const int64_t nb = (ncol + CB - 1) / CB;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t c0 = b * CB, cn = (c0 + CB <= ncol) ? CB : ncol - c0;
    double s0[CB], s1[CB], s2[CB];
    const double* f = mf + (n - 1) * 3 * ncol + c0;
    for (int c = 0; c < cn; ++c) {
      s0[c] = f[c]; s1[c] = f[ncol + c]; s2[c] = f[2 * ncol + c];
      out[(n - 1) * ldo + c0 + c] = s0[c];
    }
    for (int64_t k = n - 2; k >= 0; --k) {
      const double* A = rec + (k + 1) * 16;
      const double* g = G + k * 9;
      const double* fk = mf + k * 3 * ncol + c0;
      for (int c = 0; c < cn; ++c) {
        const double q0 = fk[c], q1 = fk[ncol + c], q2 = fk[2 * ncol + c];
        /* m_pred_{k+1} = A_{k+1} m_f_k */
        const double p0 = A[0] * q0 + A[1] * q1 + A[2] * q2;
        const double p1 = A[3] * q0 + A[4] * q1 + A[5] * q2;
        const double p2 = A[6] * q0 + A[7] * q1 + A[8] * q2;
        const double e0 = s0[c] - p0, e1 = s1[c] - p1, e2 = s2[c] - p2;
        s0[c] = q0 + g[0] * e0 + g[1] * e1 + g[2] * e2;
        s1[c] = q1 + g[3] * e0 + g[4] * e1 + g[5] * e2;
        s2[c] = q2 + g[6] * e0 + g[7] * e1 + g[8] * e2;
        out[k * ldo + c0 + c] = s0[c];
      }
    }
  }
  free(mf); free(al); free(G);
  return 0;
}

/* Smoothed marginal variance of the first state component (the `.P[1,1]` of TemporalGPs smooth,
 * temporal_gp_inference.jl:109-114): P^s_{n-1} = Pf_{n-1},
 * P^s_k = Pf_k + G_k (P^s_{k+1} - Pp_{k+1}) G_k^T.  Data-independent; var[k] = P^s_k[0][0]. */
void gpar_cpu_smooth_var(int kind, const double* rec, const double* pf, const double* pp, int64_t n,
                         double* var) {
  const int d = sde_dim(kind);
  double Ps[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Ps[i][j] = pf[(n - 1) * 9 + i * 3 + j];
  var[n - 1] = Ps[0][0];
  for (int64_t k = n - 2; k >= 0; --k) {
    double G[9], D[3][3], GD[3][3];
    smoother_gain(d, rec, pf, pp, k, G);
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) D[i][j] = Ps[i][j] - pp[(k + 1) * 9 + i * 3 + j];
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        double a = 0.0;
        for (int q = 0; q < d; ++q) a += G[i * 3 + q] * D[q][j];
        GD[i][j] = a;
      }
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < d; ++j) {
        double a = 0.0;
        for (int q = 0; q < d; ++q) a += GD[i][q] * G[j * 3 + q];
        Ps[i][j] = pf[k * 9 + i * 3 + j] + a;
      }
    var[k] = Ps[0][0];
  }
}

int gpar_cpu_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}
