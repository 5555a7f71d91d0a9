"""GPU parity of the exact GP / GPAR path (P=3, N=200) against the
golden fixture and the oracle (optimized.jl:19-239).  Tolerances fp64: logpdf rel <= 1e-10,
posterior marginals rtol 1e-8 (through (K + s2 I)^{-1}, cond ~1e4-1e6)."""
import os

import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_exact_golden():
    g = np.load(os.path.join(GOLDEN, "exact.npz"), allow_pickle=False)
    lml = G.exact_logpdf(g["X"], g["y"], g["theta"])
    assert abs(lml - float(g["logpdf"])) <= 1e-10 * abs(lml)
    m, v = G.exact_posterior(g["X"], g["y"], g["X_star"], g["theta"])
    np.testing.assert_allclose(m, g["post_mean"], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(v, g["post_var"], rtol=1e-8, atol=1e-10)
    lml1 = G.exact_logpdf(g["gp_t"], g["gp_y"], g["gp_theta"], time_kernel="matern32")
    assert abs(lml1 - float(g["gp_logpdf"])) <= 1e-10 * abs(lml1)
    m1, v1 = G.exact_posterior(g["gp_t"], g["gp_y"], g["gp_t_star"], g["gp_theta"], "matern32")
    np.testing.assert_allclose(m1, g["gp_mean"], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(v1, g["gp_var"], rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("tk,ok,n,P", [("eq", "eq", 200, 3), ("matern52", "matern32", 777, 4),
                                       ("matern12", "eq", 1500, 2)])
def test_exact_gpar_matches_oracle(tk, ok, n, P):
    t, Y = O.synthetic_gpar(n, P, seed=n, noise=0.3)
    X = np.vstack([t] + [Y[:, q] for q in range(P - 1)])
    theta = (1.1, 0.9, 1.7, 1.2, 0.35)
    K = O.exact_gpar_kernel(X, X, theta, tk, ok)
    ref = O.exact_logpdf(K, Y[:, P - 1], theta[4])
    assert abs(G.exact_logpdf(X, Y[:, P - 1], theta, tk, ok) - ref) <= 1e-10 * abs(ref)
    Xs = X[:, ::4] + 0.013
    Ks = O.exact_gpar_kernel(X, Xs, theta, tk, ok)
    kss = np.diag(O.exact_gpar_kernel(Xs, Xs, theta, tk, ok))
    rm, rv = O.exact_posterior(K, Ks, kss, Y[:, P - 1], theta[4])
    m, v = G.exact_posterior(X, Y[:, P - 1], Xs, theta, tk, ok)
    np.testing.assert_allclose(m, rm, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(v, rv, rtol=1e-8, atol=1e-10)


def test_create_optim_gpar_matches_oracle():
    """Config 1: the exact GPAR fit of output 3 (optimized.jl:106-183), 60 NM evaluations."""
    t, Y = O.synthetic_gpar(200, 3, seed=1, noise=0.3)
    X = np.vstack([t, Y[:, 0], Y[:, 1]])
    x0 = dict(i_log_time_l=0.0, i_log_time_var=0.0, i_log_out_l=0.0, i_log_out_var=0.0,
              i_log_noise_sigma=-1.0)
    ref = O.create_optim_gpar(X, Y[:, 2], log_theta0=tuple(x0.values()), max_evals=60)
    gp, th = G.create_optim_gpar(X, Y[:, 2], max_evals=60, **x0)
    np.testing.assert_allclose(th, ref, rtol=1e-6)
    m, v = gp.marginals(X[:, :5])
    assert np.all(v > 0) and np.all(np.isfinite(m))


def test_exact_not_pd_raises():
    t = np.repeat(np.linspace(0, 1, 20), 2)      # duplicated inputs, essentially no noise
    y = np.sin(t)
    with pytest.raises(G.PosDefException):
        G.exact_logpdf(t, y, (0.5, 1.0, 1e-12), time_kernel="eq")
