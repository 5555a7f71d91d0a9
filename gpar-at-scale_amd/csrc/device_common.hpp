// device_common.hpp -- gfx950 device helpers shared by the GPAR kernels.
//
// Stationary kernels (Stheno Matern12/32/52, EQ) and the closed-form
// Matern-nu state-space discretisation (TemporalGPs `to_sde`).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

namespace gpar {

enum KernelKind : int { KM12 = 0, KM32 = 1, KM52 = 2, KEQ = 3 };

constexpr double kSqrt3 = 1.7320508075688772935;
constexpr double kSqrt5 = 2.2360679774997896964;
constexpr double kLog2Pi = 1.8378770664093454836;

// Per-step gains record: A (d x d, row-major) | K (d) | rs = 1/sqrt(S) ; padded.
template <int D> struct Rec { static constexpr int size = D == 3 ? 16 : (D == 2 ? 8 : 4); };
// compact gains record {K_k (D), rs_k, pad}: A_k is recomputed from the step's time difference by
// the one consumer that takes it (whiten_kfu_d2x2)
template <int D> struct CRec { static constexpr int size = D == 1 ? 2 : 4; };
// Per-step fix-up vector g_k (d), padded to 4 doubles.
constexpr int kGStride = 4;
// Carry / end-state vectors (d), padded to 4 doubles.
constexpr int kSStride = 4;

// f(std::integral_constant<int, i>) for i = 0 .. N-1 (compile-time indices for fmac_row's lane)
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// acc + row[E] * m, where each 16-lane DPP row of the wave holds the same 16-double step row (a
// gains record and its fix-up row, {A_k, K_k, rs_k, g_k}; lane i: element i) and row_newbcast:E
// hands element E to every lane of its row as the FMA's first source.  A step's 16 values then
// reach all 64 lanes from one ds_read_b64 (2 LDS cycles) instead of broadcast ds_read_b128 reads
// (4 LDS cycles per 2 doubles, ≈ 34 per step): the filter recursions that read a record per step
// were LDS-bound, 8-9 waves per CU sharing one LDS.  The source must not be written by a VALU in
// the two instructions before (DPP hazard): `row` comes straight from an LDS read.  Same operation
// order and rounding as fma(row[E], m, acc).
template <int E>
__device__ __forceinline__ double fmac_row(double acc, double row, double m) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(row), "v"(m), "n"(E));
  return acc;
}

// row[E] in every lane of its 16-lane row (a v_mov_b64 with the same DPP source)
template <int E>
__device__ __forceinline__ double bcast_row(double row) {
  return __builtin_amdgcn_update_dpp(0.0, row, 0x150 + E, 0xf, 0xf, false);
}

template <int KIND> struct Sde;
template <> struct Sde<KM12> { static constexpr int d = 1; };
template <> struct Sde<KM32> { static constexpr int d = 2; };
template <> struct Sde<KM52> { static constexpr int d = 3; };

// e^{-x} for x >= 0, branch-free (so independent evaluations interleave): Cody-Waite
// reduction with a split ln 2, then a degree-11 near-minimax polynomial for e^r on
// |r| <= ln2/2 (Chebyshev fit, approximation error 1.7e-17 relative with the coefficients
// rounded to fp64; two FMAs fewer than the degree-13 Taylor form it replaces), v_ldexp_f64; x
// beyond 745.5 underflows to 0.  Measured on gfx950: max 0.93 ulp, mean 0.25 ulp
// (tools/ubench/rsq_precision.hip).
__device__ __forceinline__ double exp_neg(double x) {
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

// exp_neg with its constants handed in by the caller: passed as a kernel argument they live in
// SGPRs and feed the FMAs directly (a 64-bit literal cannot be an f64 VALU operand, so the
// inline-constant form re-materialises each one with a v_mov_b64 per evaluation).
struct ExpNegConsts {
  double c[12];                 // degree-11 polynomial, highest first (exp_neg's coefficients)
  double log2e, ln2hi, ln2lo, lo;
};
inline ExpNegConsts exp_neg_consts() {
  return ExpNegConsts{{2.5110037605963777e-08, 2.763263963904103e-07, 2.755724091857897e-06,
                       2.4801485482328494e-05, 0.00019841269890047113, 0.0013888888952314775,
                       0.008333333333319601, 0.0416666666664881, 0.1666666666666668,
                       0.5000000000000019, 1.0, 1.0},
                      1.4426950408889634074, 6.93147180369123816490e-01,
                      1.90821492927058770002e-10, -745.5};
}
__device__ __forceinline__ double exp_neg_k(double x, const ExpNegConsts& k) {
  const double y = fmax(-x, k.lo);
  const double nf = rint(y * k.log2e);
  double r = fma(-nf, k.ln2hi, y);
  r = fma(-nf, k.ln2lo, r);
  double p = k.c[0];
#pragma unroll
  for (int i = 1; i < 12; ++i) p = fma(p, r, k.c[i]);
  return ldexp(p, (int)nf);
}

// s * kappa(sqrt(d2) / l) with the exp constants from the caller (see ExpNegConsts)
template <int KIND>
__device__ __forceinline__ double skappa_sq_k(double d2, double inv_l, double s,
                                              const ExpNegConsts& k);

// sqrt for x >= 0 (squared distances): v_rsq_f64 seed (~2^-24), one Goldschmidt step for
// g ~ sqrt(x) (~2^-47), one Newton correction g += (x - g^2) h with the unrefined half-reciprocal
// h = rsq/2 (its 2^-24 error enters only at second order).  No denormal rescaling or inf/nan
// class fix-ups (x is clamped to >= 1e-200, whose root 1e-100 is 0 for every kernel here).
// Measured on gfx950: max 0.5 ulp, the same as the 3-correction form (tools/ubench/
// rsq_precision.hip); 7 VALU ops + rsq instead of 18 for sqrt(double).
__device__ __forceinline__ double sqrt_pos(double x) {
  const double xs = fmax(x, 1e-200);
  const double y = __builtin_amdgcn_rsq(xs);
  double g = xs * y;
  const double h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  const double d = fma(-g, g, xs);
  return fma(d, h, g);
}

// Unit-variance, unit-length kernel of the distance r >= 0.
template <int KIND>
__device__ __forceinline__ double kappa(double r) {
  if constexpr (KIND == KM12) {
    return exp_neg(r);
  } else if constexpr (KIND == KM32) {
    const double x = kSqrt3 * r;
    return (1.0 + x) * exp_neg(x);
  } else if constexpr (KIND == KM52) {
    const double x = kSqrt5 * r;
    return (1.0 + x + x * x * (1.0 / 3.0)) * exp_neg(x);
  } else {
    return exp_neg(0.5 * r * r);
  }
}

// Kernel from a squared distance (EQ needs no sqrt).
template <int KIND>
__device__ __forceinline__ double kappa_sq(double d2, double inv_l) {
  if constexpr (KIND == KEQ) {
    return exp_neg(0.5 * d2 * inv_l * inv_l);
  } else {
    return kappa<KIND>(sqrt_pos(d2) * inv_l);
  }
}

// s * kappa from a squared distance, the variance folded into the Matern polynomial.
template <int KIND>
__device__ __forceinline__ double skappa_sq(double d2, double inv_l, double s) {
  if constexpr (KIND == KEQ) {
    return s * exp_neg(0.5 * d2 * inv_l * inv_l);
  } else if constexpr (KIND == KM12) {
    return s * exp_neg(sqrt_pos(d2) * inv_l);
  } else if constexpr (KIND == KM32) {
    const double x = kSqrt3 * inv_l * sqrt_pos(d2);
    return fma(s, x, s) * exp_neg(x);
  } else {
    const double x = kSqrt5 * inv_l * sqrt_pos(d2);
    return fma(x, fma(x, s * (1.0 / 3.0), s), s) * exp_neg(x);
  }
}

// s * kappa(r / l) from the distance r = sqrt_pos(d2) itself (the Matern forms; the fit's
// distance cache stores r, so the square root is taken once per fit, bit-identical to skappa_sq_k)
template <int KIND>
__device__ __forceinline__ double skappa_r_k(double r, double inv_l, double s,
                                             const ExpNegConsts& k) {
  if constexpr (KIND == KM12) {
    return s * exp_neg_k(r * inv_l, k);
  } else if constexpr (KIND == KM32) {
    const double x = kSqrt3 * inv_l * r;
    return fma(s, x, s) * exp_neg_k(x, k);
  } else {
    const double x = kSqrt5 * inv_l * r;
    return fma(x, fma(x, s * (1.0 / 3.0), s), s) * exp_neg_k(x, k);
  }
}

template <int KIND>
__device__ __forceinline__ double skappa_sq_k(double d2, double inv_l, double s,
                                              const ExpNegConsts& k) {
  if constexpr (KIND == KEQ) {
    return s * exp_neg_k(0.5 * d2 * inv_l * inv_l, k);
  } else if constexpr (KIND == KM12) {
    return s * exp_neg_k(sqrt_pos(d2) * inv_l, k);
  } else if constexpr (KIND == KM32) {
    const double x = kSqrt3 * inv_l * sqrt_pos(d2);
    return fma(s, x, s) * exp_neg_k(x, k);
  } else {
    const double x = kSqrt5 * inv_l * sqrt_pos(d2);
    return fma(x, fma(x, s * (1.0 / 3.0), s), s) * exp_neg_k(x, k);
  }
}

__device__ __forceinline__ double kappa_rt(int kind, double r) {
  switch (kind) {
    case KM12: return kappa<KM12>(r);
    case KM32: return kappa<KM32>(r);
    case KM52: return kappa<KM52>(r);
    default: return kappa<KEQ>(r);
  }
}

// Stationary covariance of the unit SDE (times s gives the scaled prior: H = e1 convention).
template <int D>
__device__ __forceinline__ void sde_pinf(double s, double (&P)[D][D]) {
  if constexpr (D == 1) {
    P[0][0] = s;
  } else if constexpr (D == 2) {
    P[0][0] = s; P[0][1] = 0.0; P[1][0] = 0.0; P[1][1] = 3.0 * s;
  } else {
    P[0][0] = s;             P[0][1] = 0.0;               P[0][2] = -(5.0 / 3.0) * s;
    P[1][0] = 0.0;           P[1][1] = (5.0 / 3.0) * s;   P[1][2] = 0.0;
    P[2][0] = -(5.0 / 3.0) * s; P[2][1] = 0.0;            P[2][2] = 25.0 * s;
  }
}

// A = exp(F tau): F + lambda I is nilpotent, so exp(F tau) = e^{-lambda tau} (I + tau N + tau^2/2 N^2).
template <int D>
__device__ __forceinline__ void sde_transition(double tau, double (&A)[D][D]) {
  if constexpr (D == 1) {
    A[0][0] = exp(-tau);
  } else if constexpr (D == 2) {
    const double lam = kSqrt3;
    const double e = exp(-lam * tau);
    A[0][0] = e * (1.0 + lam * tau);  A[0][1] = e * tau;
    A[1][0] = -e * (3.0 * tau);       A[1][1] = e * (1.0 - lam * tau);
  } else {
    const double lam = kSqrt5, l2 = 5.0, l3 = 5.0 * kSqrt5, l4 = 25.0;
    const double e = exp(-lam * tau);
    const double t2 = tau * tau;
    A[0][0] = e * (1.0 + lam * tau + 0.5 * l2 * t2);
    A[0][1] = e * (tau + lam * t2);
    A[0][2] = e * (0.5 * t2);
    A[1][0] = e * (-0.5 * l3 * t2);
    A[1][1] = e * (1.0 + lam * tau - l2 * t2);
    A[1][2] = e * (tau - 0.5 * lam * t2);
    A[2][0] = e * (-l3 * tau + 0.5 * l4 * t2);
    A[2][1] = e * (-3.0 * l2 * tau + l3 * t2);
    A[2][2] = e * (1.0 - 2.0 * lam * tau + 0.5 * l2 * t2);
  }
}

// ---- small dense helpers (fully unrolled, registers only)
template <int D>
__device__ __forceinline__ void mat_mul(const double (&X)[D][D], const double (&Y)[D][D],
                                        double (&Z)[D][D]) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) acc = fma(X[i][k], Y[k][j], acc);
      Z[i][j] = acc;
    }
}

// Z = X * Y^T
template <int D>
__device__ __forceinline__ void mat_mul_bt(const double (&X)[D][D], const double (&Y)[D][D],
                                           double (&Z)[D][D]) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) acc = fma(X[i][k], Y[j][k], acc);
      Z[i][j] = acc;
    }
}

// Z = X^T * Y
template <int D>
__device__ __forceinline__ void mat_mul_at(const double (&X)[D][D], const double (&Y)[D][D],
                                           double (&Z)[D][D]) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) acc = fma(X[k][i], Y[k][j], acc);
      Z[i][j] = acc;
    }
}

template <int D>
__device__ __forceinline__ void mat_copy(const double (&X)[D][D], double (&Z)[D][D]) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) Z[i][j] = X[i][j];
}

template <int D>
__device__ __forceinline__ void mat_eye(double (&Z)[D][D]) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) Z[i][j] = (i == j) ? 1.0 : 0.0;
}

template <int D>
__device__ __forceinline__ void mat_zero(double (&Z)[D][D]) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) Z[i][j] = 0.0;
}

// Inverse of a small general matrix (adjugate / determinant).
template <int D>
__device__ __forceinline__ void mat_inv(const double (&X)[D][D], double (&Z)[D][D]) {
  if constexpr (D == 1) {
    Z[0][0] = 1.0 / X[0][0];
  } else if constexpr (D == 2) {
    const double det = X[0][0] * X[1][1] - X[0][1] * X[1][0];
    const double id = 1.0 / det;
    Z[0][0] = X[1][1] * id;  Z[0][1] = -X[0][1] * id;
    Z[1][0] = -X[1][0] * id; Z[1][1] = X[0][0] * id;
  } else {
    const double c00 = X[1][1] * X[2][2] - X[1][2] * X[2][1];
    const double c01 = X[1][2] * X[2][0] - X[1][0] * X[2][2];
    const double c02 = X[1][0] * X[2][1] - X[1][1] * X[2][0];
    const double det = X[0][0] * c00 + X[0][1] * c01 + X[0][2] * c02;
    const double id = 1.0 / det;
    Z[0][0] = c00 * id;
    Z[1][0] = c01 * id;
    Z[2][0] = c02 * id;
    Z[0][1] = (X[0][2] * X[2][1] - X[0][1] * X[2][2]) * id;
    Z[1][1] = (X[0][0] * X[2][2] - X[0][2] * X[2][0]) * id;
    Z[2][1] = (X[0][1] * X[2][0] - X[0][0] * X[2][1]) * id;
    Z[0][2] = (X[0][1] * X[1][2] - X[0][2] * X[1][1]) * id;
    Z[1][2] = (X[0][2] * X[1][0] - X[0][0] * X[1][2]) * id;
    Z[2][2] = (X[0][0] * X[1][1] - X[0][1] * X[1][0]) * id;
  }
}

// Standard normal of the counter (seed, s, m), s < 2^32, m < 2^32: splitmix64 hashes + Box-Muller.
// Reproducible for a given seed, independent of launch geometry (gpar_mc_normals /
// gpar_path_normals export the same draws).
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ double counter_normal(uint64_t seed, uint64_t s, uint64_t m) {
  const uint64_t key = (s << 32) | m;
  const uint64_t a = splitmix64(seed ^ splitmix64(key * 2 + 1));
  const uint64_t b = splitmix64(a ^ 0xD1B54A32D192ED03ull);
  const double u1 = ((double)(a >> 11) + 0.5) * (1.0 / 9007199254740992.0);
  const double u2 = ((double)(b >> 11)) * (1.0 / 9007199254740992.0);
  return sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace gpar
