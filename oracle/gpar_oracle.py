"""CPU oracle (fp64 numpy) for the GPAR-at-scale per-output GP hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
*checker*.  The product path (``gpar-at-scale_amd/``) never imports it and has no
CPU fallback.

What this is
------------
A plain restatement of the reference algorithm (TudorParas/GPAR-at-scale, Julia)
for the hot path, following the reference's own operation order:

* ``compute_gpar_dtc_objective``      src/gp/dtc.jl:83-128
* ``get_optim_scaled_gpar_params``    src/gp/dtc.jl:11-77
* ``compute_q_u``                     src/gp/gpar_scaled_inference.jl:141-196
* ``get_gpar_scaled_predictions``     src/gp/gpar_scaled_inference.jl:20-136
* ``create_lgssm`` / ``get_sde_predictions``  src/gp/temporal_gp_inference.jl:15-114
* exact GP / GPAR                     src/gp/optimized.jl:19-239
* ``unpack_gp[ar]``, masks, init      src/util.jl:36-169
* toy data                            src/data/toy_data.jl:9-98

The arithmetic the reference delegates to third-party Julia packages is restated
from their published algorithms:

* Stheno 0.6-era kernels / ``pairwise`` / FiniteGP ``cov`` (Kuu gets the FiniteGP
  noise on its diagonal, ``cov(f, u)`` does not),
* TemporalGPs 0.3-era ``to_sde`` / ``decorrelate`` / ``logpdf`` / ``smooth``
  (Matern-nu as a d-state SDE, stationary start, Kalman whitening, RTS),
* Optim.jl ``NelderMead`` (AffineSimplexer(a=0.025, b=0.5), AdaptiveParameters),

all of which are *absent* from this image (no Julia, no depot, versions unpinned in
Project.toml:3-17 with Manifest.toml git-ignored).

Pinning
-------
The reference ships no tests, fixtures or golden vectors and
Julia cannot run here, so this oracle is pinned by the reference's own cross-check
identity ``examples/dtc_example.jl:8-64`` (LGSSM-whitened DTC == dense-Sigma DTC),
made asserting in ``tests/test_oracle.py``, plus dense-linear-algebra identities
(Kalman whitening == L_Sigma^{-1} y, sum log S_k == logdet Sigma, DTC == dense
N(y; 0, Kfu Kuu'^{-1} Kuf + Sigma), SDE cross-covariance == kernel).  Agreement
with the *Julia* numerics themselves is **parity unpinned** (see DESIGN.md).

Conventions fixed here (documented in DESIGN.md):
* state-space scaling folds the time-kernel variance into the stationary covariance
  (P0 = s_t * Pinf, H = e1), so the first state component IS the latent f;
* the stationary start is a prepended step of length 1 (scaled time) from Pinf;
* distances are direct differences sqrt(sum (x-z)^2) / l.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
from scipy.linalg import cho_factor, cho_solve, solve_triangular

LOG2PI = math.log(2.0 * math.pi)

KERNELS = ("matern12", "matern32", "matern52", "eq")
KERNEL_ID = {k: i for i, k in enumerate(KERNELS)}


# ----------------------------------------------------------------------------- util.jl
def unpack_gp(params):
    """src/util.jl:36-43 -> (l, process_var, noise_sigma) = exp(p) + 1e-3."""
    p = np.asarray(params, dtype=np.float64)
    return tuple(float(np.exp(v) + 1e-3) for v in p[:3])


def unpack_gpar(params):
    """src/util.jl:45-55 -> (time_l, time_var, out_l, out_var, noise_sigma)."""
    p = np.asarray(params, dtype=np.float64)
    return tuple(float(np.exp(v) + 1e-3) for v in p[:5])


def get_time_mask(input_length):
    """src/util.jl:102-106."""
    m = np.zeros(input_length)
    m[0] = 1.0
    return m


def get_output_mask(input_length):
    """src/util.jl:111-123 (DomainError for input_length <= 1)."""
    if input_length <= 1:
        raise ValueError("Input length must be integer greater than 1")
    m = np.zeros((input_length - 1, input_length))
    for r in range(input_length - 1):
        m[r, r + 1] = 1.0
    return m


def parse_initial_params(vals, rng=None):
    """src/util.jl:141-169: missing initial log-params are drawn U(0,1) (rand())."""
    rng = rng if rng is not None else np.random.default_rng()
    return np.array([rng.random() if v is None else float(v) for v in vals])


def to_colvecs(inputs):
    """src/util.jl:16-31: list of 1-D arrays (one per input dim) -> D x N matrix."""
    if isinstance(inputs, np.ndarray):
        return np.atleast_2d(np.asarray(inputs, dtype=np.float64))
    return np.vstack([np.asarray(a, dtype=np.float64) for a in inputs])


# ----------------------------------------------------------------------------- kernels
def kappa(kind, r):
    """Unit-variance, unit-length stationary kernels as a function of distance r >= 0.

    Stheno Matern12/Matern32/Matern52/EQ (restated)."""
    r = np.asarray(r, dtype=np.float64)
    if kind == "matern12":
        return np.exp(-r)
    if kind == "matern32":
        x = math.sqrt(3.0) * r
        return (1.0 + x) * np.exp(-x)
    if kind == "matern52":
        x = math.sqrt(5.0) * r
        return (1.0 + x + x * x / 3.0) * np.exp(-x)
    if kind == "eq":
        return np.exp(-0.5 * r * r)
    raise ValueError(kind)


def sqdist(X, Z):
    """X: D x N, Z: D x M -> N x M squared Euclidean distances (direct differences)."""
    X = np.atleast_2d(X)
    Z = np.atleast_2d(Z)
    out = np.zeros((X.shape[1], Z.shape[1]))
    for d in range(X.shape[0]):
        diff = X[d][:, None] - Z[d][None, :]
        out += diff * diff
    return out


def pairwise(kind, X, Z, l, s):
    """s * kappa(||x - z|| / l): Stheno ``pairwise(kernel(k; l, s), X, Z)``
    (dtc.jl:31,104; gpar_scaled_inference.jl:89,156-157)."""
    return s * kappa(kind, np.sqrt(sqdist(X, Z)) / l)


# ----------------------------------------------------------------------------- SDE
_SDE_DIM = {"matern12": 1, "matern32": 2, "matern52": 3}


def sde_dim(kind):
    if kind not in _SDE_DIM:
        raise ValueError(f"kernel {kind!r} has no finite state-space form")
    return _SDE_DIM[kind]


def sde_pinf(kind):
    """Stationary covariance of the unit Matern-nu SDE (TemporalGPs ``to_sde``)."""
    if kind == "matern12":
        return np.array([[1.0]])
    if kind == "matern32":
        return np.diag([1.0, 3.0])
    if kind == "matern52":
        return np.array([[1.0, 0.0, -5.0 / 3.0], [0.0, 5.0 / 3.0, 0.0], [-5.0 / 3.0, 0.0, 25.0]])
    raise ValueError(kind)


def sde_lambda(kind):
    return {"matern12": 1.0, "matern32": math.sqrt(3.0), "matern52": math.sqrt(5.0)}[kind]


def sde_feedback(kind):
    lam = sde_lambda(kind)
    if kind == "matern12":
        return np.array([[-1.0]])
    if kind == "matern32":
        return np.array([[0.0, 1.0], [-lam**2, -2.0 * lam]])
    return np.array([[0.0, 1.0, 0.0], [0.0, 0.0, 1.0], [-lam**3, -3.0 * lam**2, -3.0 * lam]])


def sde_transition(kind, tau):
    """A = exp(F tau) in closed form: F + lam I is nilpotent (F has the single eigenvalue -lam)."""
    lam = sde_lambda(kind)
    d = sde_dim(kind)
    Nm = sde_feedback(kind) + lam * np.eye(d)
    e = math.exp(-lam * tau)
    if d == 1:
        return np.array([[e]])
    if d == 2:
        return e * (np.eye(2) + tau * Nm)
    return e * (np.eye(3) + tau * Nm + 0.5 * tau * tau * (Nm @ Nm))


def _inc_gamma_p(m1, x):
    """Regularized lower incomplete gamma P(m1, x) for an integer m1 >= 1: the series
    e^{-x} sum_{k >= m1} x^k / k! for x < 4 (no cancellation for short steps), else
    1 - e^{-x} sum_{k < m1} x^k / k!.  Same loop as the device's (k_path.hip)."""
    if x < 4.0:
        t = math.exp(-x)
        for k in range(1, m1 + 1):
            t *= x / k
        acc, k = 0.0, m1
        for _ in range(80):
            acc += t
            k += 1
            t *= x / k
            if t < 1e-18 * acc:
                break
        return acc
    term, tot = 1.0, 1.0
    for k in range(1, m1):
        term *= x / k
        tot += term
    return 1.0 - math.exp(-x) * tot


def sde_q_stable(kind, tau, s):
    """Process-noise covariance Q(tau) = s Pinf - A s Pinf A^T of a step of scaled length tau in
    closed form: the white noise drives the last state, so Q = q s int_0^tau a(u) a(u)^T du with
    a(u) = exp(F u) e_d = e^{-lam u} (polynomial in u) and q the spectral density that makes
    Q(inf) = s Pinf; the integrals are incomplete gamma functions.  Equal to the subtraction form
    to rounding, but accurate (and positive definite) for short steps, where the subtraction loses
    all digits of the small eigenvalues: the simulation smoother factors it (lgssm_posterior_rand)."""
    lam = sde_lambda(kind)
    if kind == "matern12":
        al, q = [[1.0]], 2.0
    elif kind == "matern32":
        al, q = [[0.0, 1.0], [1.0, -lam]], 4.0 * lam ** 3
    else:
        al = [[0.0, 0.0, 0.5], [0.0, 1.0, -0.5 * lam], [1.0, -2.0 * lam, 0.5 * lam * lam]]
        q = 16.0 * lam ** 5 / 3.0
    d = len(al)
    x = 2.0 * lam * tau
    I = [math.factorial(m) / (2.0 * lam) ** (m + 1) * _inc_gamma_p(m + 1, x) for m in range(2 * d - 1)]
    Q = np.zeros((d, d))
    for i in range(d):
        for j in range(d):
            acc = 0.0
            for pp in range(d):
                for r in range(d):
                    acc += al[i][pp] * al[j][r] * I[pp + r]
            Q[i, j] = q * s * acc
    return Q


@dataclass
class LGSSM:
    """Discretised time GP: per step k, x_k = A_k x_{k-1} + q_k, y_k = x_k[0] + eps_k.

    Built as ``to_sde(GP(kernel(k; l, s)))(t, R)`` (dtc.jl:101-102,
    temporal_gp_inference.jl:28-38, gpar_scaled_inference.jl:105-107)."""

    A: np.ndarray   # N x d x d
    Q: np.ndarray   # N x d x d
    R: np.ndarray   # N
    P0: np.ndarray  # d x d  (prior at the prepended start point)
    kind: str = ""
    tau: np.ndarray = None   # N scaled step lengths (tau_0 = 1: the stationary start)
    s: float = 1.0           # time-kernel variance


def build_lgssm(t, kind, l, s, R):
    """t ascending (the fit does not sort: dtc.jl:102); R scalar or per-step noise variance.

    Stationary start: a step of length 1 (scaled time) from x0 ~ N(0, s Pinf)
    (TemporalGPs prepends t_1 - 1)."""
    t = np.asarray(t, dtype=np.float64)
    n = t.shape[0]
    if n > 1 and np.any(np.diff(t) < 0):
        raise ValueError("time locations must be ascending")
    d = sde_dim(kind)
    pinf = s * sde_pinf(kind)
    ts = t / l
    dt = np.empty(n)
    dt[0] = 1.0
    dt[1:] = np.diff(ts)
    A = np.empty((n, d, d))
    Q = np.empty((n, d, d))
    for k in range(n):
        a = sde_transition(kind, dt[k])
        A[k] = a
        Q[k] = pinf - a @ pinf @ a.T
    R = np.broadcast_to(np.asarray(R, dtype=np.float64), (n,)).copy()
    return LGSSM(A=A, Q=Q, R=R, P0=pinf, kind=kind, tau=dt, s=s)


def riccati(lg):
    """Data-independent filter quantities: predicted/filtered covariances, S_k, gains."""
    n, d = lg.A.shape[0], lg.A.shape[1]
    Pp = np.empty((n, d, d))
    Pf = np.empty((n, d, d))
    S = np.empty(n)
    K = np.empty((n, d))
    P = lg.P0
    for k in range(n):
        A = lg.A[k]
        Pm = A @ P @ A.T + lg.Q[k]
        s = Pm[0, 0] + lg.R[k]
        g = Pm[:, 0] / s
        P = Pm - np.outer(g, Pm[0, :])
        Pp[k], Pf[k], S[k], K[k] = Pm, P, s, g
    return Pp, Pf, S, K


def kalman_filter(lg, X):
    """Kalman filter over the columns of X (N or N x C).

    Returns (alpha, logS, m_pred, m_filt): alpha = innovations / sqrt(S) (TemporalGPs
    ``decorrelate``, used at dtc.jl:106,115 and gpar_scaled_inference.jl:175,183)."""
    X = np.asarray(X, dtype=np.float64)
    vec = X.ndim == 1
    X2 = X[:, None] if vec else X
    n, c = X2.shape
    d = lg.A.shape[1]
    _, _, S, K = riccati(lg)
    m = np.zeros((d, c))
    alpha = np.empty((n, c))
    mp = np.empty((n, d, c))
    mf = np.empty((n, d, c))
    for k in range(n):
        mm = lg.A[k] @ m
        e = X2[k] - mm[0]
        alpha[k] = e / math.sqrt(S[k])
        m = mm + np.outer(K[k], e)
        mp[k], mf[k] = mm, m
    if vec:
        alpha, mp, mf = alpha[:, 0], mp[:, :, 0], mf[:, :, 0]
    return alpha, np.log(S), mp, mf


def decorrelate(lg, X):
    """(lml, alpha) with lml = sum_k log N(x_k; prediction, S_k) for vector X."""
    alpha, logS, _, _ = kalman_filter(lg, X)
    lml = -0.5 * (np.sum(logS) + np.sum(alpha * alpha, axis=0) + alpha.shape[0] * LOG2PI)
    return lml, alpha


def lgssm_logpdf(lg, y):
    """TemporalGPs ``logpdf(lgssm, y)`` (temporal_gp_inference.jl:78)."""
    return float(decorrelate(lg, y)[0])


def rts_smooth(lg, X):
    """RTS smoother (TemporalGPs ``smooth``, temporal_gp_inference.jl:109,
    gpar_scaled_inference.jl:117). Returns smoothed state means (N x d [x C]) and
    covariances (N x d x d)."""
    X = np.asarray(X, dtype=np.float64)
    vec = X.ndim == 1
    X2 = X[:, None] if vec else X
    n = X2.shape[0]
    Pp, Pf, _, _ = riccati(lg)
    _, _, mp, mf = kalman_filter(lg, X2)
    ms = np.empty_like(mf)
    Ps = np.empty_like(Pf)
    ms[-1], Ps[-1] = mf[-1], Pf[-1]
    for k in range(n - 2, -1, -1):
        G = Pf[k] @ lg.A[k + 1].T @ np.linalg.inv(Pp[k + 1])
        ms[k] = mf[k] + G @ (ms[k + 1] - mp[k + 1])
        Ps[k] = Pf[k] + G @ (Ps[k + 1] - Pp[k + 1]) @ G.T
    if vec:
        ms = ms[:, :, 0]
    return ms, Ps


def _chol_guarded(C):
    """Lower Cholesky factor of a small symmetric PSD matrix, negative pivots clamped to zero
    (the backward-sampling covariance C_k loses definiteness to rounding where it is nearly
    singular); written out so the device kernel (k_path.hip) follows the same operation order."""
    d = C.shape[0]
    L = np.zeros((d, d))
    for j in range(d):
        t = C[j, j] - sum(L[j, q] * L[j, q] for q in range(j))
        L[j, j] = math.sqrt(t) if t > 0.0 else 0.0
        for i in range(j + 1, d):
            v = C[i, j] - sum(L[i, q] * L[j, q] for q in range(j))
            L[i, j] = v / L[j, j] if L[j, j] > 0.0 else 0.0
    return L


def ffbs_constants(lg):
    """Data-independent coefficients of backward sampling from the LGSSM posterior (the
    forward-filter backward-sample algorithm behind TemporalGPs ``posterior_rand``, called at
    src/gp/tmp.jl:161-167; TemporalGPs itself is absent and unpinned, SURVEY §8c, so the algorithm
    is restated from Carter & Kohn 1994 / Fruhwirth-Schnatter 1994):
        x_{n-1} ~ N(m_{n-1}, P_{n-1}),
        x_k | x_{k+1} ~ N(m_k + J_k (x_{k+1} - A_{k+1} m_k), C_k),
        J_k = P_k A_{k+1}^T (A_{k+1} P_k A_{k+1}^T + Q_{k+1})^{-1},  C_k = P_k - J_k A_{k+1} P_k,
    with (m_k, P_k) the filtered moments.  Returns J, B = I - J_k A_{k+1} and L = chol(C_k)
    (n x d x d each; step n-1: J = 0, B = I, L = chol(P_{n-1})), so that a draw is
    x_k = J_k x_{k+1} + B_k m_k + L_k xi_k."""
    _, Pf, _, _ = riccati(lg)
    n, d = lg.A.shape[0], lg.A.shape[1]
    J = np.zeros((n, d, d))
    B = np.zeros((n, d, d))
    L = np.zeros((n, d, d))
    for k in range(n):
        P = Pf[k]
        if k == n - 1:
            B[k] = np.eye(d)
            C = P
        else:
            A = lg.A[k + 1]
            Pm = A @ P @ A.T + lg.Q[k + 1]
            PAt = P @ A.T
            J[k] = PAt @ np.linalg.inv(Pm)
            C = P - J[k] @ PAt.T
            B[k] = np.eye(d) - J[k] @ A
        L[k] = _chol_guarded(0.5 * (C + C.T))
    return J, B, L


def lgssm_posterior_rand_ffbs(lg, Y, xi):
    """Forward-filter backward-sample draws (ffbs_constants) of the latent f given Y (n, or n x S
    one column per sample); xi: S x n x d.  Returns S x n.  The textbook algorithm, kept as a
    cross-check of lgssm_posterior_rand's distribution: its backward coefficients amplify rounding
    on clustered grids (see lgssm_posterior_rand)."""
    xi = np.asarray(xi, dtype=np.float64)
    S, n, d = xi.shape
    Y = np.asarray(Y, dtype=np.float64)
    Y2 = np.repeat(Y[:, None], S, axis=1) if Y.ndim == 1 else Y
    _, _, _, mf = kalman_filter(lg, Y2)            # n x d x S
    J, B, L = ffbs_constants(lg)
    x = np.zeros((d, S))
    f = np.empty((S, n))
    for k in range(n - 1, -1, -1):
        x = J[k] @ x + B[k] @ mf[k] + L[k] @ xi[:, k, :].T
        f[:, k] = x[0]
    return f


def lgssm_posterior_rand(lg, Y, xi):
    """TemporalGPs ``posterior_rand(rng, lgssm, y)`` (src/gp/tmp.jl:161-167) with the draws given:
    joint samples of the latent f = x[0] from p(f | y).  TemporalGPs is absent and unpinned (SURVEY
    §8c); the draws here come from the simulation smoother of Durbin & Koopman (2002), exact
    posterior draws like forward-filter backward-sample (lgssm_posterior_rand_ffbs) but stable:
      prior path   x~_0 = chol(s Pinf) eta_0,  x~_k = A_k x~_{k-1} + chol(Q_k) eta_k,
                   y~_k = x~_k[0] + sqrt(R_k) eps_k   (Q_k in closed form: sde_q_stable),
      draw         f = x~[0] + E[f | y - y~]    (rts_smooth's mean of the latent f).
    (FFBS's J_k = P_k A^T (P^-_{k+1})^{-1} moves Matern-5/2 draws by 1.6e-2 under 1e-13 relative
    perturbations of A / Q on a 700-point grid with steps down to 8e-5; this form by 4e-13.)
    Y: n (one data vector for every sample) or n x S; xi: S x n x (d + 1), xi[s, k, :d] = eta,
    xi[s, k, d] = eps (gpar_path_normals' layout).  Returns S x n samples."""
    xi = np.asarray(xi, dtype=np.float64)
    S, n, d1 = xi.shape
    d = d1 - 1
    Y = np.asarray(Y, dtype=np.float64)
    Y2 = np.repeat(Y[:, None], S, axis=1) if Y.ndim == 1 else Y
    x = np.zeros((d, S))
    ft = np.empty((n, S))
    yt = np.empty((n, S))
    for k in range(n):
        if k == 0:
            x = _chol_guarded(lg.P0) @ xi[:, 0, :d].T
        else:
            Q = sde_q_stable(lg.kind, lg.tau[k], lg.s)
            x = lg.A[k] @ x + _chol_guarded(Q) @ xi[:, k, :d].T
        ft[k] = x[0]
        yt[k] = x[0] + math.sqrt(lg.R[k]) * xi[:, k, d]
    ms, _ = rts_smooth(lg, Y2 - yt)
    return (ft + ms[:, 0, :]).T


def dense_time_cov(t, kind, l, s):
    tt = np.asarray(t, dtype=np.float64)
    return s * kappa(kind, np.abs(tt[:, None] - tt[None, :]) / l)


# ----------------------------------------------------------------------------- DTC
def compute_gpar_dtc_objective(V, Z, t, y, theta, out_kernel="matern52",
                               time_kernel="matern52", kuu_noise=True,
                               dense_logdet=False, return_parts=False):
    """src/gp/dtc.jl:83-128, with theta = (time_l, time_var, out_l, out_var, noise_sigma)
    in natural units (unpack_gpar output).  Variances are squared (dtc.jl:31,37).

    logdet(noise_matrix) (dtc.jl:96-99,123) is evaluated as sum_k log S_k (identical
    math; the dense N x N LU is O(N^3)); pass dense_logdet=True for the dense form."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    V = to_colvecs(V)
    Z = to_colvecs(Z)
    y = np.asarray(y, dtype=np.float64)
    n = y.shape[0]
    m = Z.shape[1]
    Kfu = pairwise(out_kernel, V, Z, l_o, s_o)                      # cov(f, u)   dtc.jl:104
    Kuu = pairwise(out_kernel, Z, Z, l_o, s_o)                      # cov(u)      dtc.jl:119
    if kuu_noise:
        Kuu = Kuu + s2 * np.eye(m)
    lg = build_lgssm(t, time_kernel, l_t, s_t, s2)                  # dtc.jl:101-102
    alpha, logS, _, _ = kalman_filter(lg, y)                        # dtc.jl:106
    beta, _, _, _ = kalman_filter(lg, Kfu)                          # dtc.jl:110-117
    Lu = np.linalg.cholesky(Kuu)
    A = solve_triangular(Lu, beta.T, lower=True)                    # dtc.jl:119
    Lam = A @ A.T + np.eye(m)
    Llam = np.linalg.cholesky(Lam)                                  # dtc.jl:120
    if dense_logdet:
        logdet_sigma = np.linalg.slogdet(dense_time_cov(t, time_kernel, l_t, s_t) + s2 * np.eye(n))[1]
    else:
        logdet_sigma = float(np.sum(logS))
    w = solve_triangular(Llam, A @ alpha, lower=True)
    tmp = logdet_sigma + 2.0 * np.sum(np.log(np.diag(Llam))) + alpha @ alpha - w @ w
    dtc = -(n * LOG2PI + tmp) / 2.0                                 # dtc.jl:122-125
    if return_parts:
        G = beta.T @ beta
        r = beta.T @ alpha
        return dtc, dict(A=A, alpha=alpha, beta=beta, G=G, r=r, aa=float(alpha @ alpha),
                         logdet_sigma=logdet_sigma, Kuu=Kuu, Kfu=Kfu, Lam=Lam)
    return dtc, A


def dense_dtc_identity(V, Z, t, y, theta, out_kernel="matern52", time_kernel="matern52"):
    """examples/dtc_example.jl:10-23 ``_compute_intermediates``: the same DTC with a dense
    cholesky of the noise matrix, and the textbook form log N(y; 0, Kfu Kuu'^-1 Kuf + Sigma)."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    V, Z = to_colvecs(V), to_colvecs(Z)
    y = np.asarray(y, dtype=np.float64)
    n, m = y.shape[0], Z.shape[1]
    Sig = dense_time_cov(t, time_kernel, l_t, s_t) + s2 * np.eye(n)
    Ls = np.linalg.cholesky(Sig)
    Kfu = pairwise(out_kernel, V, Z, l_o, s_o)
    Kuu = pairwise(out_kernel, Z, Z, l_o, s_o) + s2 * np.eye(m)
    Lu = np.linalg.cholesky(Kuu)
    A = solve_triangular(Lu, solve_triangular(Ls, Kfu, lower=True).T, lower=True)
    Llam = np.linalg.cholesky(A @ A.T + np.eye(m))
    delta = solve_triangular(Ls, y, lower=True)
    w = solve_triangular(Llam, A @ delta, lower=True)
    tmp = 2 * np.sum(np.log(np.diag(Ls))) + 2 * np.sum(np.log(np.diag(Llam))) + delta @ delta - w @ w
    dtc = -(n * LOG2PI + tmp) / 2.0
    Cov = Kfu @ np.linalg.solve(Kuu, Kfu.T) + Sig
    c = cho_factor(Cov, lower=True)
    textbook = -0.5 * (n * LOG2PI + 2 * np.sum(np.log(np.diag(c[0]))) + y @ cho_solve(c, y))
    return dtc, A, textbook


# ----------------------------------------------------------------------------- Nelder-Mead
class NelderMead:
    """Optim.jl ``NelderMead()`` restated as an ask/tell state machine.

    AffineSimplexer(a=0.025, b=0.5); AdaptiveParameters: alpha=1, beta=1+2/n,
    gamma=0.75-1/(2n), delta=1-1/n; stop on g_tol (std of simplex values) or
    iterations; after the loop the centroid is evaluated and the better of centroid
    and best vertex is the minimizer (Optim ``after_while!``).

    ``max_evals`` (not an Optim option; the build's reproducible budget replacing the
    wall-clock ``time_limit`` of dtc.jl:59-61) caps the total number of objective
    evaluations *including* the final centroid evaluation; an iteration that would
    exceed it is abandoned with the simplex left consistent."""

    def __init__(self, x0, max_evals=None, g_tol=1e-8, iterations=1000, a=0.025, b=0.5):
        self.x0 = np.asarray(x0, dtype=np.float64).copy()
        self.n = self.x0.shape[0]
        n = self.n
        self.alpha, self.beta = 1.0, 1.0 + 2.0 / n
        self.gamma, self.delta = 0.75 - 1.0 / (2.0 * n), 1.0 - 1.0 / n
        self.a, self.b = a, b
        self.max_evals = max_evals
        self.g_tol = g_tol
        self.iterations = iterations
        self.evals = 0
        self.iters = 0
        self.trace = []
        self._gen = self._run()
        self._pending = next(self._gen)
        self.done = False
        self.x_min = None
        self.f_min = None

    def ask(self):
        return None if self.done else self._pending.copy()

    def tell(self, f):
        self.trace.append((self._pending.copy(), float(f)))
        self.evals += 1
        try:
            self._pending = self._gen.send(float(f))
        except StopIteration:
            self.done = True

    # budget: reserve one evaluation for the final centroid
    def _can_eval(self):
        return self.max_evals is None or self.evals < self.max_evals - 1

    def _run(self):
        n, m = self.n, self.n + 1
        simplex = [self.x0.copy() for _ in range(m)]
        for j in range(n):
            simplex[j + 1][j] = (1.0 + self.b) * simplex[j + 1][j] + self.a
        fs = np.empty(m)
        aborted = False
        for i in range(m):
            if not self._can_eval():
                aborted = True
                break
            fs[i] = yield simplex[i]
        if aborted:
            # degenerate budget: keep evaluated prefix only
            k = i
            simplex, fs, m = simplex[:k], fs[:k], k
            if k == 0:
                self.x_min, self.f_min = self.x0, float("nan")
                return
        order = list(np.argsort(fs, kind="stable"))
        converged = self._nm_obj(fs) <= self.g_tol
        while not converged and not aborted and self.iters < self.iterations and m == n + 1:
            self.iters += 1
            hi = order[m - 1]
            cen = np.mean([simplex[i] for i in range(m) if i != hi], axis=0)
            x_hi = simplex[hi].copy()
            x_lo = simplex[order[0]].copy()
            f_lo, f_2hi, f_hi = fs[order[0]], fs[order[n - 1]], fs[hi]
            x_ref = cen + self.alpha * (cen - x_hi)
            if not self._can_eval():
                break
            f_ref = yield x_ref
            shrink = False
            if f_ref < f_lo:
                x_exp = cen + self.beta * (x_ref - cen)
                if not self._can_eval():
                    break
                f_exp = yield x_exp
                if f_exp < f_ref:
                    simplex[hi], fs[hi] = x_exp, f_exp
                else:
                    simplex[hi], fs[hi] = x_ref, f_ref
                order = [hi] + order[:m - 1]
            elif f_ref < f_2hi:
                simplex[hi], fs[hi] = x_ref, f_ref
                order = list(np.argsort(fs, kind="stable"))
            else:
                if f_ref < f_hi:
                    x_c = cen + self.gamma * (x_ref - cen)
                    if not self._can_eval():
                        break
                    f_c = yield x_c
                    if f_c < f_ref:
                        simplex[hi], fs[hi] = x_c, f_c
                        order = list(np.argsort(fs, kind="stable"))
                    else:
                        shrink = True
                else:
                    x_c = cen - self.gamma * (x_ref - cen)
                    if not self._can_eval():
                        break
                    f_c = yield x_c
                    if f_c < f_hi:
                        simplex[hi], fs[hi] = x_c, f_c
                        order = list(np.argsort(fs, kind="stable"))
                    else:
                        shrink = True
            if shrink:
                for i in range(1, m):
                    o = order[i]
                    xs = x_lo + self.delta * (simplex[o] - x_lo)
                    if not self._can_eval():
                        aborted = True
                        break
                    fv = yield xs
                    simplex[o], fs[o] = xs, fv
                order = list(np.argsort(fs, kind="stable"))
            converged = self._nm_obj(fs) <= self.g_tol
        # after_while!
        order = list(np.argsort(fs, kind="stable"))
        hi = order[m - 1]
        i_min = int(np.argmin(fs))
        x_min, f_min = simplex[i_min].copy(), float(fs[i_min])
        if m > 1:
            cen = np.mean([simplex[i] for i in range(m) if i != hi], axis=0)
            f_cen = yield cen
            if f_cen < f_min:
                x_min, f_min = cen, f_cen
        self.x_min, self.f_min = x_min, f_min

    def _nm_obj(self, fs):
        c = np.mean(fs)
        return math.sqrt(np.sum((fs - c) ** 2) / self.n)


def nelder_mead(f, x0, **kw):
    nm = NelderMead(x0, **kw)
    while not nm.done:
        nm.tell(f(nm.ask()))
    return nm


# ----------------------------------------------------------------------------- fit / q(u) / predict
def get_optim_scaled_gpar_params(V, Z, t, y, out_kernel="matern52", time_kernel="matern52",
                                 log_theta0=None, max_evals=None, g_tol=1e-8, rng=None,
                                 return_nm=False):
    """src/gp/dtc.jl:11-77: NM over the 5 log-params minimising -dtc."""
    if log_theta0 is None:
        log_theta0 = [None] * 5
    p0 = parse_initial_params(log_theta0, rng)

    def nlml(p):
        return -compute_gpar_dtc_objective(V, Z, t, y, unpack_gpar(p), out_kernel, time_kernel)[0]

    nm = nelder_mead(nlml, p0, max_evals=max_evals, g_tol=g_tol)
    theta = unpack_gpar(nm.x_min)
    return (theta, nm) if return_nm else theta


def compute_q_u(V, Z, t, y, theta, out_kernel="matern52", time_kernel="matern52",
                qu_kuu_noise=False):
    """src/gp/gpar_scaled_inference.jl:141-196.  Cuu has NO noise (:157) unless qu_kuu_noise:
    then Cuu + sigma^2 I, the FiniteGP cov(u) the objective uses (dtc.jl:35) -- the build's
    opt-in for pseudo-input sets whose noise-free Cuu is numerically singular (the branch the
    north-star bench runs, gpar_problem.qu_kuu_noise).

    Returns (m_e, cov_e = inv(D), U_u upper, D)."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    V, Z = to_colvecs(V), to_colvecs(Z)
    m = Z.shape[1]
    Cfu = pairwise(out_kernel, V, Z, l_o, s_o)
    Cuu = pairwise(out_kernel, Z, Z, l_o, s_o)
    if qu_kuu_noise:
        Cuu = Cuu + s2 * np.eye(m)
    U_u = np.linalg.cholesky(Cuu).T
    L_u = U_u.T
    lg = build_lgssm(t, time_kernel, l_t, s_t, s2)
    beta, _, _, _ = kalman_filter(lg, Cfu)
    B = solve_triangular(L_u, beta.T, lower=True)
    b_y, _, _, _ = kalman_filter(lg, y)
    D = B @ B.T + np.eye(m)
    c = cho_factor(D, lower=True)
    m_e = cho_solve(c, B @ b_y)
    cov = np.linalg.inv(D)
    return m_e, 0.5 * (cov + cov.T), U_u, D


def merge_grid(t, t_star):
    """gpar_scaled_inference.jl:75-87: concat train+test and stable sortperm by time."""
    tc = np.concatenate([np.asarray(t, float), np.asarray(t_star, float)])
    perm = np.argsort(tc, kind="stable")
    return tc, perm


def get_gpar_scaled_predictions_fixed(V, Z, t, y, t_star, V_star, theta, out_kernel="matern52",
                                      time_kernel="matern52", mode="analytic", samples=100,
                                      rng=None, qu_kuu_noise=False, xi=None):
    """Prediction half of src/gp/gpar_scaled_inference.jl:20-136 at given theta.

    mode="mc": the reference's 100-sample Monte Carlo (:91-130) with Bessel std.
    mode="analytic": its S -> infinity limit: mean = (I-S) mu_x + S y*,
    var = diag((I-S) K* U_u^-1 D^-1 U_u^-T K*^T (I-S)^T) (latent f).
    qu_kuu_noise: q(u) with Cuu + sigma^2 I (see compute_q_u).  xi (M x S): the standard-normal
    draws of the MC mode, to replay a sampler's exact draws (else drawn from rng).
    Returns (mean, std) at the test points in input order."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    V, Z, V_star = to_colvecs(V), to_colvecs(Z), to_colvecs(V_star)
    n, ns = len(t), len(t_star)
    m_e, cov, U_u, D = compute_q_u(V, Z, t, y, theta, out_kernel, time_kernel, qu_kuu_noise)
    tc, perm = merge_grid(t, t_star)
    Vc = np.hstack([V, V_star])[:, perm]
    yc = np.concatenate([np.asarray(y, float), np.zeros(ns)])[perm]
    Rc = np.concatenate([np.full(n, s2), np.full(ns, 1e10)])[perm]
    Kstar = pairwise(out_kernel, Vc, Z, l_o, s_o)
    lg = build_lgssm(tc[perm], time_kernel, l_t, s_t, Rc)
    if mode == "mc":
        if xi is None:
            rng = rng if rng is not None else np.random.default_rng()
            xi = rng.standard_normal((len(m_e), samples))
        Lc = np.linalg.cholesky(cov)
        E = m_e[:, None] + Lc @ np.asarray(xi, dtype=np.float64)
        FX = Kstar @ solve_triangular(U_u, E, lower=False)
        ms, _ = rts_smooth(lg, yc[:, None] - FX)
        F = FX + ms[:, 0, :]
        mean_s, std_s = F.mean(axis=1), F.std(axis=1, ddof=1)
    else:
        w = solve_triangular(U_u, m_e, lower=False)
        mu = Kstar @ w
        ms, _ = rts_smooth(lg, yc - mu)
        mean_s = mu + ms[:, 0]
        Y = Kstar @ solve_triangular(U_u, np.linalg.cholesky(cov), lower=False)
        msY, _ = rts_smooth(lg, Y)
        W = Y - msY[:, 0, :]
        std_s = np.sqrt(np.sum(W * W, axis=1))
    inv = np.argsort(perm, kind="stable")
    return mean_s[inv][n:], std_s[inv][n:]


def get_gpar_scaled_predictions_path_fixed(V, Z, t, y, t_star, V_star, theta, xi_u, xi_path,
                                           out_kernel="matern52", time_kernel="matern52",
                                           qu_kuu_noise=False):
    """The Monte Carlo estimator of src/gp/tmp.jl:119-167 (the reference's scratch variant of
    get_gpar_scaled_predictions) with the draws given: per sample s,
      e_s = m_e + chol(inv(D)) xi_u[:, s]            (rand(q_u), :122-128 / gpar_scaled_inference.jl:103)
      fx_s = Cf*u U_u^{-1} e_s                          (generate_fx_sample, :121-129)
      f_t,s = posterior_rand(lgssm*, y* - fx_s)         (:161-167, FFBS: lgssm_posterior_rand)
      f*_s = fx_s + f_t,s,
    then the elementwise mean and Bessel std over the samples at the test points, as
    gpar_scaled_inference.jl:130-135 reduces its samples.  xi_u: M x S; xi_path: S x (n + n*) x
    (d + 1) (the merged grid in time order, lgssm_posterior_rand's layout).  Returns (mean, std) at the test points in input order."""
    l_t, sv_t, l_o, sv_o, sigma = (float(v) for v in theta)
    s_t, s_o, s2 = sv_t * sv_t, sv_o * sv_o, sigma * sigma
    V, Z, V_star = to_colvecs(V), to_colvecs(Z), to_colvecs(V_star)
    n, ns = len(t), len(t_star)
    m_e, cov, U_u, D = compute_q_u(V, Z, t, y, theta, out_kernel, time_kernel, qu_kuu_noise)
    tc, perm = merge_grid(t, t_star)
    Vc = np.hstack([V, V_star])[:, perm]
    yc = np.concatenate([np.asarray(y, float), np.zeros(ns)])[perm]
    Rc = np.concatenate([np.full(n, s2), np.full(ns, 1e10)])[perm]
    Kstar = pairwise(out_kernel, Vc, Z, l_o, s_o)
    lg = build_lgssm(tc[perm], time_kernel, l_t, s_t, Rc)
    E = m_e[:, None] + np.linalg.cholesky(cov) @ np.asarray(xi_u, dtype=np.float64)
    FX = Kstar @ solve_triangular(U_u, E, lower=False)            # (n + n*) x S
    Ft = lgssm_posterior_rand(lg, yc[:, None] - FX, xi_path)      # S x (n + n*)
    F = FX + Ft.T
    inv = np.argsort(perm, kind="stable")
    mean_s, std_s = F.mean(axis=1), F.std(axis=1, ddof=1)
    return mean_s[inv][n:], std_s[inv][n:]


def get_gpar_scaled_predictions(V, Z, t, y, t_star, V_star, out_kernel="matern52",
                                time_kernel="matern52", log_theta0=None, max_evals=None,
                                mode="analytic", samples=100, rng=None, g_tol=1e-8,
                                qu_kuu_noise=False):
    """src/gp/gpar_scaled_inference.jl:20-136 (fit, then predict).  Note the reference
    hard-codes Matern52 for the fit (:48-49)."""
    theta = get_optim_scaled_gpar_params(V, Z, t, y, "matern52", "matern52", log_theta0,
                                         max_evals, g_tol=g_tol, rng=rng)
    mean, std = get_gpar_scaled_predictions_fixed(V, Z, t, y, t_star, V_star, theta,
                                                  out_kernel, time_kernel, mode, samples, rng,
                                                  qu_kuu_noise=qu_kuu_noise)
    return mean, std, theta


# ----------------------------------------------------------------------------- temporal-only
def create_lgssm(t, l, process_var, noise_sigma, kind="matern52", noise_vector=None):
    """src/gp/temporal_gp_inference.jl:15-39 (kernel(k; l, s=process_var^2))."""
    R = noise_sigma ** 2 if noise_vector is None else np.asarray(noise_vector, float)
    return build_lgssm(t, kind, l, process_var ** 2, R)


def sde_predict_fixed(t, y, t_star, theta, kind="matern52"):
    """Smoothing half of get_sde_predictions (temporal_gp_inference.jl:93-113):
    marginals of f at t_star (mean, var), R = sigma^2 train / 1e10 test."""
    l, pv, ns = (float(v) for v in theta)
    n, nst = len(t), len(t_star)
    tc, perm = merge_grid(t, t_star)
    yc = np.concatenate([np.asarray(y, float), np.zeros(nst)])[perm]
    Rc = np.concatenate([np.full(n, ns * ns), np.full(nst, 1e10)])[perm]
    lg = create_lgssm(tc[perm], l, pv, ns, kind, noise_vector=Rc)
    ms, Ps = rts_smooth(lg, yc)
    inv = np.argsort(perm, kind="stable")
    return ms[:, 0][inv][n:], Ps[:, 0, 0][inv][n:]


def get_sde_predictions(t, y, t_star, kind="matern52", log_theta0=None, max_evals=None,
                        g_tol=1e-8, rng=None):
    """src/gp/temporal_gp_inference.jl:45-114: NM on -logpdf(lgssm, y) then smoothing."""
    if log_theta0 is None:
        log_theta0 = [None] * 3
    p0 = parse_initial_params(log_theta0, rng)

    def nlml(p):
        l, pv, ns = unpack_gp(p)
        return -lgssm_logpdf(create_lgssm(t, l, pv, ns, kind), y)

    nm = nelder_mead(nlml, p0, max_evals=max_evals, g_tol=g_tol)
    theta = unpack_gp(nm.x_min)
    mean, var = sde_predict_fixed(t, y, t_star, theta, kind)
    return theta, mean, var


# ----------------------------------------------------------------------------- exact GP / GPAR
def exact_gpar_kernel(X, X2, theta, time_kernel="eq", out_kernel="eq"):
    """optimized.jl:132-144: s_t k_t(mask_t x / l_t) + s_o k_o(Mask_o x / l_o); x = (t, y_1..)."""
    l_t, sv_t, l_o, sv_o = (float(v) for v in theta[:4])
    X, X2 = to_colvecs(X), to_colvecs(X2)
    K = pairwise(time_kernel, X[:1], X2[:1], l_t, sv_t * sv_t)
    if X.shape[0] > 1:
        K = K + pairwise(out_kernel, X[1:], X2[1:], l_o, sv_o * sv_o)
    return K


def exact_gp_kernel(x, x2, theta, kernel="eq"):
    """optimized.jl:28-36: process_var^2 * stretch(k, 1/l)."""
    l, pv = float(theta[0]), float(theta[1])
    return pairwise(kernel, to_colvecs(x), to_colvecs(x2), l, pv * pv)


def exact_logpdf(K, y, noise_sigma):
    """Stheno logpdf(f(x, sigma^2), y) via dense Cholesky (optimized.jl:34,152)."""
    y = np.asarray(y, float)
    c = cho_factor(K + noise_sigma ** 2 * np.eye(len(y)), lower=True)
    return -0.5 * (len(y) * LOG2PI + 2 * np.sum(np.log(np.diag(c[0]))) + y @ cho_solve(c, y))


def exact_posterior(K, Ks, kss_diag, y, noise_sigma):
    """Posterior marginals of f (optimized.jl:94,236; marginals at plot_examples.jl:106-122)."""
    c = cho_factor(K + noise_sigma ** 2 * np.eye(len(y)), lower=True)
    mean = Ks.T @ cho_solve(c, np.asarray(y, float))
    W = solve_triangular(c[0], Ks, lower=True)
    var = kss_diag - np.sum(W * W, axis=0)
    return mean, var


def create_optim_gp(x, y, kernel="eq", log_theta0=(None, None, None), max_evals=None, rng=None):
    """optimized.jl:19-59."""
    p0 = parse_initial_params(log_theta0, rng)

    def nlml(p):
        l, pv, ns = unpack_gp(p)
        return -exact_logpdf(exact_gp_kernel(x, x, (l, pv), kernel), y, ns)

    nm = nelder_mead(nlml, p0, max_evals=max_evals)
    return unpack_gp(nm.x_min)


def create_optim_gpar(X, y, time_kernel="eq", out_kernel="eq", log_theta0=(None,) * 5,
                      max_evals=None, rng=None):
    """optimized.jl:106-183 (multi_input=true)."""
    p0 = parse_initial_params(log_theta0, rng)

    def nlml(p):
        th = unpack_gpar(p)
        return -exact_logpdf(exact_gpar_kernel(X, X, th, time_kernel, out_kernel), y, th[4])

    nm = nelder_mead(nlml, p0, max_evals=max_evals)
    return unpack_gpar(nm.x_min)


# ----------------------------------------------------------------------------- data
START, STEP_SIZE = 0.0, 1.0 / 30.0


def f1_big(x):
    return 3.0 - np.sin(np.pi / 10.0 * (x + 1.0)) - np.power(x, 0.3)


def f2_big(x, y1):
    return np.cos(y1) ** 2 + np.sin(np.pi / 20.0 * x)


def f3_big(x, y1, y2):
    return y2 * y1 ** 2 + 0.1 * x


def f_ext(p, x, ys):
    """Build's extension for outputs p > 3: cos(y_{p-1})^2 + sin(pi t/(20+p)) + 0.1 y_{p-2}."""
    return np.cos(ys[p - 2]) ** 2 + np.sin(np.pi * x / (20.0 + p)) + 0.1 * ys[p - 3]


def nuke(x, nr_intervals, per_interval):
    """src/data/toy_data.jl:42-57."""
    if nr_intervals == 0:
        return x, 0
    kept = len(x) // (nr_intervals + 1)
    parts = [x[:kept]]
    for i in range(1, nr_intervals + 1):
        parts.append(x[i * kept + per_interval:(i + 1) * kept])
    nx = np.concatenate(parts)
    return nx, len(x) - len(nx)


def chained_outputs(x, P):
    ys = [f1_big(x)]
    if P > 1:
        ys.append(f2_big(x, ys[0]))
    if P > 2:
        ys.append(f3_big(x, ys[0], ys[1]))
    for p in range(4, P + 1):
        ys.append(f_ext(p, x, ys))
    return ys


def synthetic_gpar(n, P, seed=0, noise=0.8, gaps=0, gap_len=300):
    """toy_data.jl:76-98 shape (t = k/30, chained outputs, noise std = noise^2 quirk of
    toy_data.jl:29) generalised to P outputs.  Noise is added to each output before it is
    fed to the next, as in toy_data.jl:34-36.  Returns (t, Y n x P)."""
    rng = np.random.default_rng(seed)
    x = START + STEP_SIZE * np.arange(n, dtype=np.float64)
    x, _ = nuke(x, gaps, gap_len)
    ys = []
    std = noise * noise
    for p in range(1, P + 1):
        if p == 1:
            f = f1_big(x)
        elif p == 2:
            f = f2_big(x, ys[0])
        elif p == 3:
            f = f3_big(x, ys[0], ys[1])
        else:
            f = f_ext(p, x, ys)
        ys.append(f + rng.normal(0.0, std, size=x.shape[0]))
    return x, np.stack(ys, axis=1)


def pick_pseudo_inputs(V, M, seed):
    """Z_p = M rows of V_p sampled without replacement (seed p)."""
    V = to_colvecs(V)
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(V.shape[1], size=M, replace=False))
    return V[:, idx].copy()
