"""CPU: pin the oracle (oracle/gpar_oracle.py) before trusting it.

The reference has no tests or golden vectors; its only cross-check is
examples/dtc_example.jl:8-64 (LGSSM-whitened DTC == dense-Sigma DTC, printed).  Here that check
and the dense-linear-algebra identities behind every state-space shortcut are *asserting*:

* SDE cross-covariance == the stationary kernel                     (TemporalGPs to_sde)
* Kalman whitening alpha == L_Sigma^{-1} y, sum log S_k == logdet Sigma (TemporalGPs decorrelate)
* LGSSM logpdf == dense N(y; 0, K + s2 I)                            (temporal_gp_inference.jl:78)
* LGSSM DTC == dense-Sigma DTC == textbook N(y; 0, Kfu Kuu'^-1 Kuf + Sigma) (dtc_example.jl:10-23)
* RTS smoother marginals == dense GP posterior                       (TemporalGPs smooth)
* analytic prediction == its dense (I - S) K* q(u) + S y closed form (gpar_scaled_inference.jl:20-136)
* exact logpdf == scipy multivariate normal                          (optimized.jl:34,152)
* posterior_rand draws (simulation smoother, and FFBS) follow the dense posterior (tmp.jl:161-167)
plus the golden fixtures in tests/golden/ reproduce bit-for-bit-ish (regression guard).
"""
import dataclasses
import os

import numpy as np
import pytest
from scipy.linalg import solve_triangular
from scipy.stats import multivariate_normal

from oracle import gpar_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KINDS = ["matern12", "matern32", "matern52"]


def _gpar(n, P, M, seed, gaps=0, noise=0.3):
    t, Y = O.synthetic_gpar(n, P, seed=seed, noise=noise, gaps=gaps, gap_len=max(1, n // 20))
    V = Y[:, : P - 1].T.copy()
    return t, V, O.pick_pseudo_inputs(V, M, seed + 7), Y[:, P - 1].copy()


@pytest.mark.parametrize("kind", KINDS)
def test_sde_reproduces_kernel(kind):
    # cov(x(t+tau)[0], x(t)[0]) = e1' A(tau) s Pinf e1 must equal s k(tau / l)
    s = 1.7
    for tau in (0.0, 0.1, 0.7, 2.5):
        A = O.sde_transition(kind, tau)
        c = (A @ (s * O.sde_pinf(kind)))[0, 0]
        assert abs(c - s * O.kappa(kind, np.array(tau))) < 1e-13
    # stationarity: Q >= 0 and A Pinf A' + Q = Pinf
    A = O.sde_transition(kind, 0.3)
    Q = O.sde_pinf(kind) - A @ O.sde_pinf(kind) @ A.T
    assert np.linalg.eigvalsh(0.5 * (Q + Q.T)).min() > -1e-14


@pytest.mark.parametrize("kind", KINDS)
def test_kalman_whitening_is_cholesky_solve(kind):
    t, Y = O.synthetic_gpar(300, 1, seed=2, noise=0.4, gaps=2, gap_len=20)
    y = Y[:, 0]
    l, s, s2 = 0.9, 1.3, 0.2
    lg = O.build_lgssm(t, kind, l, s, s2)
    alpha, logS, _, _ = O.kalman_filter(lg, y)
    Sig = O.dense_time_cov(t, kind, l, s) + s2 * np.eye(len(t))
    Ls = np.linalg.cholesky(Sig)
    np.testing.assert_allclose(alpha, solve_triangular(Ls, y, lower=True), atol=1e-11)
    assert abs(np.sum(logS) - np.linalg.slogdet(Sig)[1]) < 1e-10
    ref = multivariate_normal(mean=np.zeros(len(t)), cov=Sig).logpdf(y)
    assert abs(O.lgssm_logpdf(lg, y) - ref) < 1e-9 * abs(ref)


@pytest.mark.parametrize("ok,tk", [("matern52", "matern52"), ("eq", "matern32"), ("matern12", "matern12")])
def test_dtc_identity_dtc_example(ok, tk):
    """examples/dtc_example.jl:8-64, made asserting."""
    t, V, Z, y = _gpar(300, 3, 40, 5, gaps=1)
    theta = (0.8, 1.2, 1.5, 0.9, 0.3)
    dtc, A = O.compute_gpar_dtc_objective(V, Z, t, y, theta, ok, tk)
    dtc_dense, A_dense, textbook = O.dense_dtc_identity(V, Z, t, y, theta, ok, tk)
    dtc_ld, _ = O.compute_gpar_dtc_objective(V, Z, t, y, theta, ok, tk, dense_logdet=True)
    assert abs(dtc - dtc_dense) < 1e-10 * abs(dtc)
    assert abs(dtc - textbook) < 1e-9 * abs(dtc)
    assert abs(dtc - dtc_ld) < 1e-10 * abs(dtc)
    np.testing.assert_allclose(A, A_dense, atol=1e-11)


@pytest.mark.parametrize("kind", KINDS)
def test_rts_smoother_is_dense_posterior(kind):
    t, Y = O.synthetic_gpar(250, 1, seed=4, noise=0.5)
    y = Y[:, 0]
    l, s, s2 = 1.1, 0.8, 0.3
    lg = O.build_lgssm(t, kind, l, s, s2)
    ms, Ps = O.rts_smooth(lg, y)
    K = O.dense_time_cov(t, kind, l, s)
    C = K + s2 * np.eye(len(t))
    mean = K @ np.linalg.solve(C, y)
    var = np.diag(K - K @ np.linalg.solve(C, K))
    np.testing.assert_allclose(ms[:, 0], mean, atol=1e-10)
    np.testing.assert_allclose(Ps[:, 0, 0], var, atol=1e-10)


def test_analytic_prediction_dense_form():
    """mean = (I - S) K* U^-1 m_e + S y, var = diag((I-S) K* U^-1 D^-1 U^-T K*' (I-S)'), with S the
    dense time-GP smoother over the merged grid (test points carry noise 1e10, :97-105)."""
    t, V, Z, y = _gpar(240, 3, 16, 6)
    theta = (1.2, 0.9, 1.4, 1.1, 0.25)
    ts = t[::5] + 0.011
    Vs = V[:, ::5] + 0.02
    mean, std = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, theta)
    l_t, sv_t, l_o, sv_o, sg = theta
    me, cov, U, _ = O.compute_q_u(V, Z, t, y, theta)
    Ks = O.pairwise("matern52", Vs, Z, l_o, sv_o ** 2)
    tc = np.concatenate([t, ts])
    Kt = O.dense_time_cov(tc, "matern52", l_t, sv_t ** 2)
    n = len(t)
    # smoother weights from the train block (test noise 1e10 -> contributes O(1e-10))
    S_ = Kt[n:, :n] @ np.linalg.inv(Kt[:n, :n] + sg ** 2 * np.eye(n))
    Ktr = O.pairwise("matern52", V, Z, l_o, sv_o ** 2)
    X = Ks @ solve_triangular(U, me, lower=False)
    Xtr = Ktr @ solve_triangular(U, me, lower=False)
    dense_mean = X + S_ @ (y - Xtr)
    B = solve_triangular(U, np.linalg.cholesky(cov), lower=False)
    W = Ks @ B - S_ @ (Ktr @ B)
    dense_std = np.sqrt(np.sum(W * W, axis=1))
    np.testing.assert_allclose(mean, dense_mean, rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(std, dense_std, rtol=1e-6, atol=1e-8)


def test_exact_logpdf_is_mvn():
    t, Y = O.synthetic_gpar(120, 2, seed=8, noise=0.3)
    X = np.vstack([t, Y[:, 0]])
    th = (1.5, 1.2, 2.0, 0.7, 0.25)
    K = O.exact_gpar_kernel(X, X, th)
    ref = multivariate_normal(mean=np.zeros(len(t)), cov=K + th[4] ** 2 * np.eye(len(t))).logpdf(Y[:, 1])
    assert abs(O.exact_logpdf(K, Y[:, 1], th[4]) - ref) < 1e-9 * abs(ref)


def test_unpack_and_masks():
    # util.jl:36-55: exp(log-param) + 1e-3; util.jl:102-123: masks select t / the outputs
    p = np.log([1.5, 2.0, 0.3, 0.7, 0.1])
    np.testing.assert_allclose(O.unpack_gpar(p), np.array([1.5, 2.0, 0.3, 0.7, 0.1]) + 1e-3)
    np.testing.assert_allclose(O.unpack_gp(p[:3]), np.array([1.5, 2.0, 0.3]) + 1e-3)
    tm, om = O.get_time_mask(4), O.get_output_mask(4)
    np.testing.assert_array_equal(tm, [1, 0, 0, 0])
    np.testing.assert_array_equal(om @ np.arange(4.0), [1, 2, 3])
    with pytest.raises(ValueError):
        O.get_output_mask(1)


def test_nelder_mead_quadratic_and_budget():
    f = lambda x: float(np.sum((x - np.array([1.0, -2.0, 0.5])) ** 2))  # noqa: E731
    nm = O.nelder_mead(f, np.zeros(3))
    np.testing.assert_allclose(nm.x_min, [1.0, -2.0, 0.5], atol=1e-3)
    nm = O.nelder_mead(f, np.zeros(3), max_evals=17)
    assert nm.evals <= 17


def test_nuke_matches_toy_data():
    # toy_data.jl:42-57: keep the first chunk, drop per_interval points at each later chunk start
    x = np.arange(100.0)
    nx, removed = O.nuke(x, 3, 5)
    assert removed == 15 and nx[0] == 0 and 25 not in nx and 30 in nx


# --------------------------------------------------------------------- golden fixtures
def _load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("name", ["dtc_m52_m52", "dtc_eq_m32_gaps", "dtc_m32_m12", "dtc_m12_m52"])
def test_oracle_reproduces_golden_dtc(name):
    g = _load(name)
    dtc, A = O.compute_gpar_dtc_objective(g["V"], g["Z"], g["t"], g["y"], g["theta"],
                                          str(g["out_kernel"]), str(g["time_kernel"]))
    assert abs(dtc - float(g["dtc"])) <= 1e-12 * abs(dtc)
    np.testing.assert_allclose(A[:, :128], g["A_head"], rtol=1e-12, atol=1e-14)


def test_oracle_reproduces_golden_temporal():
    g = _load("temporal")
    for kind in KINDS:
        lg = O.create_lgssm(g["t"], *g[f"theta_{kind}"], kind=kind)
        assert abs(O.lgssm_logpdf(lg, g["y"]) - float(g[f"logpdf_{kind}"])) < 1e-9
        m, v = O.sde_predict_fixed(g["t"], g["y"], g["t_star"], g[f"theta_{kind}"], kind)
        np.testing.assert_allclose(m, g[f"smooth_mean_{kind}"], rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(v, g[f"smooth_var_{kind}"], rtol=1e-12, atol=1e-13)


def test_oracle_reproduces_golden_nm():
    g = _load("nm_fit")

    def nlml(p):
        return -O.compute_gpar_dtc_objective(g["V"], g["Z"], g["t"], g["y"], O.unpack_gpar(p))[0]

    nm = O.nelder_mead(nlml, g["x0"], max_evals=int(g["max_evals"]))
    assert nm.evals == int(g["evals"])
    np.testing.assert_allclose(nm.x_min, g["x_min"], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("sampler", ["simulation_smoother", "ffbs"])
def test_posterior_rand_samples_follow_the_dense_posterior(sampler):
    """posterior_rand as restated (src/gp/tmp.jl:161-167): the simulation smoother the device
    runs, and forward-filter backward-sample, both draw from the dense GP posterior
    N(K Sigma^-1 y, K - K Sigma^-1 K): sample mean and joint covariance within sampling error
    (S = 20000)."""
    rng = np.random.default_rng(0)
    t = np.sort(rng.uniform(0, 10, 60))
    y = np.sin(t) + 0.1 * rng.standard_normal(60)
    lg = O.build_lgssm(t, "matern52", 1.3, 0.8, 0.05)
    S = 20000
    if sampler == "ffbs":
        f = O.lgssm_posterior_rand_ffbs(lg, y, rng.standard_normal((S, 60, 3)))
    else:
        f = O.lgssm_posterior_rand(lg, y, rng.standard_normal((S, 60, 4)))
    K = O.dense_time_cov(t, "matern52", 1.3, 0.8)
    Sig = K + 0.05 * np.eye(60)
    mu = K @ np.linalg.solve(Sig, y)
    post = K - K @ np.linalg.solve(Sig, K)
    sd = np.sqrt(np.diag(post))
    assert np.all(np.abs(f.mean(axis=0) - mu) <= 5 * sd / np.sqrt(S))
    C = np.cov(f.T)
    scale = np.sqrt(np.outer(np.diag(post), np.diag(post)))
    assert np.abs(C - post).max() <= 6 * np.sqrt(2.0 / S) * scale.max()


def test_simulation_smoother_is_stable_where_ffbs_is_not():
    """Why the device samples with the simulation smoother: on a clustered grid (random times,
    steps down to 1e-4) 1e-13 relative perturbations of the model move FFBS's Matern-5/2 draws by
    far more than rounding, the simulation smoother's by ~1e-12."""
    rng = np.random.default_rng(703)
    t = np.sort(rng.uniform(0.0, 40.0, 700))
    y = np.sin(0.7 * t) + 0.2 * rng.standard_normal(700)
    noise = np.full(700, 0.04)
    noise[rng.random(700) < 0.25] = 1e10
    lg = O.create_lgssm(t, 1.7, 0.9, 0.2, kind="matern52", noise_vector=noise)
    p = np.random.default_rng(9)
    lg2 = dataclasses.replace(lg, A=lg.A * (1 + 1e-13 * p.standard_normal(lg.A.shape)),
                              Q=lg.Q * (1 + 1e-13 * p.standard_normal(lg.Q.shape)),
                              tau=lg.tau * (1 + 1e-13 * p.standard_normal(lg.tau.shape)))
    xi = np.random.default_rng(5).standard_normal((4, 700, 4))
    dk = np.abs(O.lgssm_posterior_rand(lg2, y, xi) - O.lgssm_posterior_rand(lg, y, xi)).max()
    ff = np.abs(O.lgssm_posterior_rand_ffbs(lg2, y, xi[:, :, :3]) -
                O.lgssm_posterior_rand_ffbs(lg, y, xi[:, :, :3])).max()
    assert dk < 1e-10 and ff > 1e3 * dk, (dk, ff)
