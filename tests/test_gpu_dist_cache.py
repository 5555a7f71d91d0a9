"""The fit's distance cache (gpar_ctx_set_dist_cache): the squared input distances are
theta-independent, so gpar_fit computes them once per call for outputs with D >= 17 and the
whitening reads them instead of rebuilding them in the fused kernel.  Same objective to rounding
(both use the centred Gram form, in a different summation order), so the same Nelder-Mead
trajectory: fitted theta rtol 1e-9, final -dtc rel 1e-12; and against the oracle's NM."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")

X0 = np.array([0.0, 0.0, 0.5, 0.0, -1.5])


def _batch(kernel="matern52"):
    t, Y = O.synthetic_gpar(1500, 71, seed=51, noise=0.3)
    probs, keep, data = [], [], []
    for D in (4, 20, 40, 70):              # 4: never cached; 70: distance path either way
        V = np.ascontiguousarray(Y[:, :D].T)
        Z = O.pick_pseudo_inputs(V, 90, D)
        pr, k = G.make_problem(V, Z, t, Y[:, D], kernel, "matern32")
        probs.append(pr)
        keep.append(k)
        data.append((V, Z, Y[:, D]))
    return t, probs, keep, data


@pytest.mark.parametrize("kernel", ["matern52", "eq", "matern12"])
def test_cache_on_off_same_fit(kernel):
    t, probs, keep, data = _batch(kernel)
    ctx = G.context(0)
    x0 = np.tile(X0, (len(probs), 1))
    try:
        ctx.set_dist_cache(0)
        off = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
        ctx.set_dist_cache(-1)
        on = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
        big = data[2]
        one = big[0].shape[1] * 128 * 8 + (1 << 20)       # room for one output of mp = 128
        ctx.set_dist_cache(one)
        part = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
    finally:
        ctx.set_dist_cache(-1)
    for r in (on, part):
        np.testing.assert_allclose(r.theta, off.theta, rtol=1e-9)
        np.testing.assert_allclose(r.nlml, off.nlml, rtol=1e-12)
    if kernel == "matern52":
        for i, (V, Z, y) in enumerate(data):
            th, _ = O.get_optim_scaled_gpar_params(V, Z, t, y, "matern52", "matern32", log_theta0=X0,
                                                   max_evals=30, g_tol=-1.0, return_nm=True)
            np.testing.assert_allclose(on.theta[i], th, rtol=1e-6)


def test_cache_budget_argument():
    ctx = G.context(0)
    with pytest.raises(G.DomainError):
        ctx.set_dist_cache(-2)
