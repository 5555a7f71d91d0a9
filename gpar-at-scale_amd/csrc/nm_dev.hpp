// nm_dev.hpp -- the Nelder-Mead ask/tell machine of nelder_mead.hpp as a fixed-size record that
// a GPU thread steps: one record per chain, advanced by a kernel right after the evaluation round
// that produced its value, so a fit of many chains runs round after round with no host round trip
// (r06; the host loop paid a ~80 us boundary per round for the D2H value copy, the host step and
// the next round's parameter upload).
//
// The same decisions and the same floating-point operations, in the same order, as NelderMead
// (Optim.jl NelderMead(), dtc.jl:58-61 / temporal_gp_inference.jl:82): AffineSimplexer
// (a = 0.025, b = 0.5), AdaptiveParameters, g_tol on the simplex value spread, the iteration cap,
// the evaluation budget and after_while!'s centroid.  Not supported: the wall-clock time limit
// (callers with one keep the host machine).  FMA contraction is off, so a record stepped on the
// device and one stepped on the host take bit-identical steps given identical values
// (tests/test_nm_dev.py steps both side by side against NelderMead on the host).
#pragma once
#include <cmath>

#if defined(__HIPCC__)
#define GPAR_HD __host__ __device__
#else
#define GPAR_HD
#endif
#if defined(__clang__)
#define GPAR_NO_FMA _Pragma("clang fp contract(off)")
#else
#define GPAR_NO_FMA
#endif

namespace gpar {

template <int N>
struct NmDev {
  static constexpr int M = N + 1;
  enum : int { Init, Reflect, Expand, ContractOut, ContractIn, Shrink, Centroid, Done };
  double simplex[M][N];
  double fs[M];
  int order[M];
  double pending[N], cen[N], x_lo[N], x_ref[N], x_c[N], x_min[N];
  double f_lo, f_2hi, f_hi, f_ref, f_min;
  double alpha, beta, gamma, delta, g_tol;
  int m, hi, init_i, shrink_i, shrink_o, evals, iters, max_evals, max_iter, converged, st;
};

template <int N>
GPAR_HD inline bool nm_can_eval(const NmDev<N>& s) {
  GPAR_NO_FMA
  return s.max_evals <= 0 || s.evals < s.max_evals - 1;
}

template <int N>
GPAR_HD inline void nm_argsort(NmDev<N>& s) {
  GPAR_NO_FMA
  // stable insertion sort of fs[0..m) (std::stable_sort's order)
  for (int i = 0; i < s.m; ++i) s.order[i] = i;
  for (int i = 1; i < s.m; ++i) {
    const int k = s.order[i];
    int j = i - 1;
    while (j >= 0 && s.fs[k] < s.fs[s.order[j]]) {
      s.order[j + 1] = s.order[j];
      --j;
    }
    s.order[j + 1] = k;
  }
}

template <int N>
GPAR_HD inline double nm_obj(const NmDev<N>& s) {
  GPAR_NO_FMA
  double c = 0.0;
  for (int i = 0; i < s.m; ++i) c += s.fs[i];
  c /= (double)s.m;
  double q = 0.0;
  for (int i = 0; i < s.m; ++i) q += (s.fs[i] - c) * (s.fs[i] - c);
  return sqrt(q / (double)N);
}

template <int N>
GPAR_HD inline void nm_centroid_excluding(const NmDev<N>& s, int hi, double* c) {
  GPAR_NO_FMA
  for (int j = 0; j < N; ++j) c[j] = 0.0;
  for (int i = 0; i < s.m; ++i)
    if (i != hi)
      for (int j = 0; j < N; ++j) c[j] += s.simplex[i][j];
  for (int j = 0; j < N; ++j) c[j] /= (double)(s.m - 1);
}

template <int N>
GPAR_HD inline void nm_finish(NmDev<N>& s) {
  GPAR_NO_FMA
  nm_argsort(s);
  const int hi = s.order[s.m - 1];
  int imin = 0;
  for (int i = 1; i < s.m; ++i)
    if (s.fs[i] < s.fs[imin]) imin = i;
  for (int j = 0; j < N; ++j) s.x_min[j] = s.simplex[imin][j];
  s.f_min = s.fs[imin];
  if (s.m > 1) {
    nm_centroid_excluding(s, hi, s.pending);
    s.st = NmDev<N>::Centroid;
  } else {
    s.st = NmDev<N>::Done;
  }
}

template <int N>
GPAR_HD inline void nm_begin_iteration(NmDev<N>& s) {
  GPAR_NO_FMA
  if (s.converged || s.iters >= s.max_iter || s.m != N + 1) {
    nm_finish(s);
    return;
  }
  ++s.iters;
  s.hi = s.order[s.m - 1];
  nm_centroid_excluding(s, s.hi, s.cen);
  for (int j = 0; j < N; ++j) s.x_lo[j] = s.simplex[s.order[0]][j];
  s.f_lo = s.fs[s.order[0]];
  s.f_2hi = s.fs[s.order[N - 1]];
  s.f_hi = s.fs[s.hi];
  for (int j = 0; j < N; ++j) s.x_ref[j] = s.cen[j] + s.alpha * (s.cen[j] - s.simplex[s.hi][j]);
  if (!nm_can_eval(s)) {
    nm_finish(s);
    return;
  }
  for (int j = 0; j < N; ++j) s.pending[j] = s.x_ref[j];
  s.st = NmDev<N>::Reflect;
}

template <int N>
GPAR_HD inline void nm_end_iteration(NmDev<N>& s) {
  GPAR_NO_FMA
  s.converged = nm_obj(s) <= s.g_tol;
  nm_begin_iteration(s);
}

template <int N>
GPAR_HD inline void nm_accept(NmDev<N>& s, const double* x, double f) {
  GPAR_NO_FMA
  for (int j = 0; j < N; ++j) s.simplex[s.hi][j] = x[j];
  s.fs[s.hi] = f;
}

template <int N>
GPAR_HD inline void nm_next_shrink(NmDev<N>& s) {
  GPAR_NO_FMA
  if (s.shrink_i == s.m) {
    nm_argsort(s);
    nm_end_iteration(s);
    return;
  }
  s.shrink_o = s.order[s.shrink_i];
  double xs[N];
  for (int j = 0; j < N; ++j) xs[j] = s.x_lo[j] + s.delta * (s.simplex[s.shrink_o][j] - s.x_lo[j]);
  if (!nm_can_eval(s)) {
    nm_finish(s);
    return;
  }
  for (int j = 0; j < N; ++j) s.pending[j] = xs[j];
  s.st = NmDev<N>::Shrink;
}

template <int N>
GPAR_HD inline void nm_on_reflect(NmDev<N>& s, double f) {
  GPAR_NO_FMA
  s.f_ref = f;
  if (f < s.f_lo) {
    double xe[N];
    for (int j = 0; j < N; ++j) xe[j] = s.cen[j] + s.beta * (s.x_ref[j] - s.cen[j]);
    if (!nm_can_eval(s)) {
      nm_finish(s);
      return;
    }
    for (int j = 0; j < N; ++j) s.pending[j] = xe[j];
    s.st = NmDev<N>::Expand;
  } else if (f < s.f_2hi) {
    nm_accept(s, s.x_ref, f);
    nm_argsort(s);
    nm_end_iteration(s);
  } else {
    const bool outside = f < s.f_hi;
    for (int j = 0; j < N; ++j)
      s.x_c[j] = outside ? s.cen[j] + s.gamma * (s.x_ref[j] - s.cen[j])
                         : s.cen[j] - s.gamma * (s.x_ref[j] - s.cen[j]);
    if (!nm_can_eval(s)) {
      nm_finish(s);
      return;
    }
    for (int j = 0; j < N; ++j) s.pending[j] = s.x_c[j];
    s.st = outside ? NmDev<N>::ContractOut : NmDev<N>::ContractIn;
  }
}

template <int N>
GPAR_HD inline void nm_on_expand(NmDev<N>& s, double f) {
  GPAR_NO_FMA
  if (f < s.f_ref)
    nm_accept(s, s.pending, f);
  else
    nm_accept(s, s.x_ref, s.f_ref);
  int o[N + 1];
  o[0] = s.hi;
  for (int i = 1; i < s.m; ++i) o[i] = s.order[i - 1];
  for (int i = 0; i < s.m; ++i) s.order[i] = o[i];
  nm_end_iteration(s);
}

// NelderMead's constructor
template <int N>
GPAR_HD inline void nm_init(NmDev<N>& s, const double* x0, int max_evals, int max_iter, double g_tol) {
  GPAR_NO_FMA
  const double n = (double)N;
  s.alpha = 1.0;
  s.beta = 1.0 + 2.0 / n;
  s.gamma = 0.75 - 1.0 / (2.0 * n);
  s.delta = 1.0 - 1.0 / n;
  s.m = N + 1;
  for (int i = 0; i < s.m; ++i)
    for (int j = 0; j < N; ++j) s.simplex[i][j] = x0[j];
  for (int j = 0; j < N; ++j) s.simplex[j + 1][j] = (1.0 + 0.5) * s.simplex[j + 1][j] + 0.025;
  for (int i = 0; i < s.m; ++i) s.fs[i] = 0.0;
  for (int i = 0; i < s.m; ++i) s.order[i] = i;
  s.max_evals = max_evals;
  s.max_iter = max_iter;
  s.g_tol = g_tol;
  s.f_lo = s.f_2hi = s.f_hi = s.f_ref = 0.0;
  s.f_min = NAN;
  s.hi = s.init_i = s.shrink_i = s.shrink_o = s.evals = s.iters = 0;
  s.converged = 0;
  for (int j = 0; j < N; ++j) s.cen[j] = s.x_lo[j] = s.x_ref[j] = s.x_c[j] = 0.0;
  if (!nm_can_eval(s)) {
    for (int j = 0; j < N; ++j) s.x_min[j] = x0[j];
    for (int j = 0; j < N; ++j) s.pending[j] = x0[j];
    s.st = NmDev<N>::Done;
  } else {
    for (int j = 0; j < N; ++j) s.x_min[j] = x0[j];
    for (int j = 0; j < N; ++j) s.pending[j] = s.simplex[0][j];
    s.st = NmDev<N>::Init;
  }
}

// NelderMead::tell
template <int N>
GPAR_HD inline void nm_tell(NmDev<N>& s, double f) {
  GPAR_NO_FMA
  ++s.evals;
  switch (s.st) {
    case NmDev<N>::Init:
      s.fs[s.init_i] = f;
      ++s.init_i;
      if (s.init_i < s.m) {
        if (!nm_can_eval(s)) {
          s.m = s.init_i;
          nm_finish(s);
          return;
        }
        for (int j = 0; j < N; ++j) s.pending[j] = s.simplex[s.init_i][j];
        return;
      }
      nm_argsort(s);
      s.converged = nm_obj(s) <= s.g_tol;
      nm_begin_iteration(s);
      return;
    case NmDev<N>::Reflect: nm_on_reflect(s, f); return;
    case NmDev<N>::Expand: nm_on_expand(s, f); return;
    case NmDev<N>::ContractOut:
      if (f < s.f_ref) {
        nm_accept(s, s.x_c, f);
        nm_argsort(s);
        nm_end_iteration(s);
      } else {
        s.shrink_i = 1;
        nm_next_shrink(s);
      }
      return;
    case NmDev<N>::ContractIn:
      if (f < s.f_hi) {
        nm_accept(s, s.x_c, f);
        nm_argsort(s);
        nm_end_iteration(s);
      } else {
        s.shrink_i = 1;
        nm_next_shrink(s);
      }
      return;
    case NmDev<N>::Shrink:
      for (int j = 0; j < N; ++j) s.simplex[s.shrink_o][j] = s.pending[j];
      s.fs[s.shrink_o] = f;
      ++s.shrink_i;
      nm_next_shrink(s);
      return;
    case NmDev<N>::Centroid:
      if (f < s.f_min) {
        for (int j = 0; j < N; ++j) s.x_min[j] = s.pending[j];
        s.f_min = f;
      }
      s.st = NmDev<N>::Done;
      return;
    default: return;
  }
}

}  // namespace gpar
