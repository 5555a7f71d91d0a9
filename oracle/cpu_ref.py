"""C/OpenMP CPU restatement of the reference's per-output path (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` (checked against the numpy oracle, ``oracle/gpar_oracle.py``) and the
``cpu_baseline`` leg of ``bench.py`` use this module; the product path never does.

This is the CPU baseline SURVEY.md §8d calls ``cpu_ref``: the reference's own Julia CPU path
cannot run in this image, so the baseline follows the reference's operation order
with the per-element work in C (``oracle/cpu_ref.c``: kernel assembly, Kalman gains, the
per-column ``decorrelate`` sweeps, the RTS smoother) and the dense algebra in OpenBLAS through
numpy/scipy, as the reference leaves it to Julia's OpenBLAS:

* ``compute_gpar_dtc_objective``        src/gp/dtc.jl:83-128
* ``compute_q_u``                        src/gp/gpar_scaled_inference.jl:141-196
* ``get_gpar_scaled_predictions_fixed``  src/gp/gpar_scaled_inference.jl:20-136 (analytic mode)
* ``lgssm_logpdf`` / ``lgssm_smooth``     src/gp/temporal_gp_inference.jl:78,109-114 (one chain)

One stated deviation, shared with the oracle and the GPU path: logdet Sigma = sum_k log S_k
instead of the dense N x N LU of dtc.jl:96-99,123 (same quantity; the dense form is O(N^3)).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
from scipy.linalg import cho_factor, cho_solve, solve_triangular

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgpar_cpu.so")
KIND = {"matern12": 0, "matern32": 1, "matern52": 2, "eq": 3}
LOG2PI = float(np.log(2.0 * np.pi))
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = C.CDLL(LIB_PATH)
        P, I64, D, I = C.c_void_p, C.c_int64, C.c_double, C.c_int
        lib.gpar_cpu_pairwise.argtypes = [I, P, I64, P, I64, I64, D, D, P, I64]
        lib.gpar_cpu_gains.argtypes = [I, P, I64, D, D, D, P, P, P, P]
        lib.gpar_cpu_gains.restype = D
        lib.gpar_cpu_filter.argtypes = [I, P, I64, P, I64, I64, P, I64, P, I64]
        lib.gpar_cpu_smooth_first.argtypes = [I, P, P, P, I64, P, I64, I64, P, I64]
        lib.gpar_cpu_smooth_first.restype = I
        lib.gpar_cpu_smooth_var.argtypes = [I, P, P, P, I64, P]
        lib.gpar_cpu_smooth_var.restype = None
        lib.gpar_cpu_threads.restype = I
        _lib = lib
    return _lib


def threads():
    return int(load().gpar_cpu_threads())


def _p(a):
    return None if a is None else a.ctypes.data


def _colvecs(X):
    """D x N (util.jl:16-31) -> contiguous point-major rows for the C kernels."""
    return np.ascontiguousarray(np.atleast_2d(np.asarray(X, dtype=np.float64)).T)


def pairwise(kind, V, Z, l, s):
    """Stheno pairwise(kernel(k; l, s), V, Z): N x M (dtc.jl:104,119)."""
    Vr, Zr = _colvecs(V), _colvecs(Z)
    n, d = Vr.shape
    m = Zr.shape[0]
    out = np.empty((n, m))
    load().gpar_cpu_pairwise(KIND[kind], _p(Vr), n, _p(Zr), m, d, float(l), float(s), _p(out), m)
    return out


def gains(kind, t, l, s, r, rvec=None, covs=False):
    t = np.ascontiguousarray(t, dtype=np.float64)
    n = t.shape[0]
    if n > 1 and np.any(np.diff(t) < 0):
        raise ValueError("time locations must be ascending")
    rec = np.empty((n, 16))
    pf = np.empty((n, 9)) if covs else None
    pp = np.empty((n, 9)) if covs else None
    rv = None if rvec is None else np.ascontiguousarray(rvec, dtype=np.float64)
    logs = load().gpar_cpu_gains(KIND[kind], _p(t), n, float(l), float(s), float(r), _p(rv),
                                 _p(rec), _p(pf), _p(pp))
    return rec, logs, pf, pp


def decorrelate(kind, rec, X):
    """alpha = L_Sigma^{-1} X column by column (TemporalGPs decorrelate, dtc.jl:106,110-117)."""
    X2 = np.ascontiguousarray(X if X.ndim == 2 else X[:, None], dtype=np.float64)
    n, c = X2.shape
    out = np.empty((n, c))
    load().gpar_cpu_filter(KIND[kind], _p(rec), n, _p(X2), c, c, _p(out), c, None, 0)
    return out if X.ndim == 2 else out[:, 0]


def smooth_first(kind, rec, pf, pp, X):
    X2 = np.ascontiguousarray(X if X.ndim == 2 else X[:, None], dtype=np.float64)
    n, c = X2.shape
    out = np.empty((n, c))
    if load().gpar_cpu_smooth_first(KIND[kind], _p(rec), _p(pf), _p(pp), n, _p(X2), c, c, _p(out), c):
        raise MemoryError("gpar_cpu_smooth_first")
    return out if X.ndim == 2 else out[:, 0]


def lgssm_logpdf(kind, t, y, l, s, r):
    """TemporalGPs ``logpdf(lgssm, y)`` of one temporal-only chain (temporal_gp_inference.jl:78):
    -1/2 (n log 2 pi + sum_k log S_k + sum_k alpha_k^2).  s: process variance, r: noise variance."""
    y = np.ascontiguousarray(y, dtype=np.float64)
    rec, logs, _, _ = gains(kind, t, l, s, r)
    al = decorrelate(kind, rec, y)
    return -0.5 * (y.shape[0] * LOG2PI + logs + float(al @ al))


def lgssm_smooth(kind, t, y, l, s, r, rvec=None):
    """TemporalGPs ``smooth`` of one chain (temporal_gp_inference.jl:109-114): the smoothed mean
    and marginal variance of the first state component, (n,) each."""
    rec, _, pf, pp = gains(kind, t, l, s, r, rvec=rvec, covs=True)
    mean = smooth_first(kind, rec, pf, pp, np.ascontiguousarray(y, dtype=np.float64))
    var = np.empty(rec.shape[0])
    load().gpar_cpu_smooth_var(KIND[kind], _p(rec), _p(pf), _p(pp), rec.shape[0], _p(var))
    return mean, var


def compute_gpar_dtc_objective(V, Z, t, y, theta, out_kernel="matern52", time_kernel="matern52",
                               kuu_noise=True):
    """src/gp/dtc.jl:83-128 at theta = (l_t, time_var, l_o, out_var, sigma) -> (dtc, A)."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    y = np.asarray(y, dtype=np.float64)
    n = y.shape[0]
    Kfu = pairwise(out_kernel, V, Z, l_o, s_o)                     # cov(f, u)   dtc.jl:104
    Kuu = pairwise(out_kernel, Z, Z, l_o, s_o)                     # cov(u)      dtc.jl:119
    if kuu_noise:
        Kuu[np.diag_indices_from(Kuu)] += s2
    rec, logdet_sigma, _, _ = gains(time_kernel, t, l_t, s_t, s2)  # dtc.jl:101-102
    alpha = decorrelate(time_kernel, rec, y)                       # dtc.jl:106
    beta = decorrelate(time_kernel, rec, Kfu)                      # dtc.jl:110-117
    Lu = np.linalg.cholesky(Kuu)
    A = solve_triangular(Lu, beta.T, lower=True)                   # dtc.jl:119
    Lam = A @ A.T
    Lam[np.diag_indices_from(Lam)] += 1.0
    Llam = np.linalg.cholesky(Lam)                                 # dtc.jl:120
    w = solve_triangular(Llam, A @ alpha, lower=True)
    tmp = logdet_sigma + 2.0 * np.sum(np.log(np.diag(Llam))) + alpha @ alpha - w @ w
    return -(n * LOG2PI + tmp) / 2.0, A                            # dtc.jl:122-127


def compute_q_u(V, Z, t, y, theta, out_kernel="matern52", time_kernel="matern52", kuu_noise=False):
    """src/gp/gpar_scaled_inference.jl:141-196 -> (m_e, inv(D), U_u)."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    m = np.atleast_2d(Z).shape[1]
    Cfu = pairwise(out_kernel, V, Z, l_o, s_o)
    Cuu = pairwise(out_kernel, Z, Z, l_o, s_o)
    if kuu_noise:
        Cuu[np.diag_indices_from(Cuu)] += s2
    L_u = np.linalg.cholesky(Cuu)
    rec, _, _, _ = gains(time_kernel, t, l_t, s_t, s2)
    beta = decorrelate(time_kernel, rec, Cfu)
    B = solve_triangular(L_u, beta.T, lower=True)
    b_y = decorrelate(time_kernel, rec, np.asarray(y, dtype=np.float64))
    D = B @ B.T
    D[np.diag_indices_from(D)] += 1.0
    m_e = cho_solve(cho_factor(D, lower=True), B @ b_y)
    cov = np.linalg.inv(D)
    _ = m
    return m_e, 0.5 * (cov + cov.T), L_u.T


def get_gpar_scaled_predictions_fixed(V, Z, t, y, t_star, V_star, theta, out_kernel="matern52",
                                      time_kernel="matern52", qu_kuu_noise=False):
    """Prediction half of src/gp/gpar_scaled_inference.jl:20-136, analytic mode (the S -> inf
    limit of the 100-sample Monte Carlo, as in the oracle) -> (mean, std) at t_star."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    V, V_star = np.atleast_2d(V), np.atleast_2d(V_star)
    n, ns = len(t), len(t_star)
    m_e, cov, U_u = compute_q_u(V, Z, t, y, theta, out_kernel, time_kernel, qu_kuu_noise)
    tc = np.concatenate([np.asarray(t, float), np.asarray(t_star, float)])
    perm = np.argsort(tc, kind="stable")                           # :75-87
    Vc = np.hstack([V, V_star])[:, perm]
    yc = np.concatenate([np.asarray(y, float), np.zeros(ns)])[perm]
    Rc = np.concatenate([np.full(n, s2), np.full(ns, 1e10)])[perm]  # :100-107
    Kstar = pairwise(out_kernel, Vc, Z, l_o, s_o)                  # :89
    rec, _, pf, pp = gains(time_kernel, tc[perm], l_t, s_t, 0.0, rvec=Rc, covs=True)
    mu = Kstar @ solve_triangular(U_u, m_e, lower=False)
    mean_s = mu + smooth_first(time_kernel, rec, pf, pp, yc - mu)
    Y = Kstar @ solve_triangular(U_u, np.linalg.cholesky(cov), lower=False)
    W = Y - smooth_first(time_kernel, rec, pf, pp, Y)
    std_s = np.sqrt(np.sum(W * W, axis=1))
    inv = np.argsort(perm, kind="stable")
    return mean_s[inv][n:], std_s[inv][n:]
