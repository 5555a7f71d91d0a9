"""Posterior path sampling (VERDICT r02 missing #1): TemporalGPs posterior_rand
(src/gp/tmp.jl:161-167) on the GPU, batched over samples (k_path.hip: the Durbin-Koopman simulation
smoother, exact posterior draws; tests/test_oracle.py shows it and forward-filter backward-sample
both match the dense posterior, and why FFBS is not used), and the path Monte Carlo estimator
tmp.jl:119-167 builds on it (gpar_predict mode GPAR_PREDICT_PATH).

TemporalGPs is absent and unpinned, so the oracle restates the sampler with citations
(oracle/gpar_oracle.py lgssm_posterior_rand).  Checked here:
  * the device draws replayed through the oracle (gpar_path_normals / gpar_mc_normals export them):
    every sample at rtol 1e-7, over several chunks of the time recursion (n > 256) and every
    Matern order, with a merged-grid noise vector (1e10 at test points);
  * the sample moments against the RTS smoother's marginals (gpar_lgssm_smooth): mean within
    5 sigma / sqrt(S), variance within 6 sqrt(2 / S) relative;
  * gpar_fit_predict's path mode = gpar_predict's at the fitted theta (seed + i per output)."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")

DIM = {"matern12": 1, "matern32": 2, "matern52": 3}


def _grid(n, seed, test_frac=0.25):
    rng = np.random.default_rng(seed)
    t = np.sort(rng.uniform(0.0, 40.0, n))
    y = np.sin(0.7 * t) + 0.3 * np.cos(2.1 * t) + 0.2 * rng.standard_normal(n)
    noise = np.full(n, 0.04)
    test = rng.random(n) < test_frac
    noise[test] = 1e10                      # merged-grid test points (gpar_scaled_inference.jl:100-107)
    y[test] = 0.0
    return t, y, noise


@pytest.mark.parametrize("kernel", ["matern12", "matern32", "matern52"])
@pytest.mark.parametrize("n", [700, 3000])
def test_posterior_rand_replays_through_the_oracle(kernel, n):
    t, y, noise = _grid(n, 3 + n)
    theta = (1.7, 0.9, 0.2)
    S, seed = 5, 1234 + n
    got = G.posterior_rand(t, y, theta, kernel, samples=S, seed=seed, noise=noise)
    xi = G.path_normals(S, n, DIM[kernel] + 1, seed)
    lg = O.create_lgssm(t, *theta, kind=kernel, noise_vector=noise)
    ref = O.lgssm_posterior_rand(lg, y, xi)
    assert got.shape == (S, n)
    np.testing.assert_allclose(got, ref, rtol=1e-7, atol=1e-9 * np.abs(ref).max())


@pytest.mark.parametrize("kernel", ["matern32", "matern52"])
def test_posterior_rand_moments_match_the_smoother(kernel):
    t, y, noise = _grid(400, 17)
    theta = (2.3, 1.1, 0.2)
    S = 6000
    f = G.posterior_rand(t, y, theta, kernel, samples=S, seed=99, noise=noise)
    mean, var = G.lgssm_smooth_batch(t, y[None, :], np.array([theta]), kernel, noise=noise)
    mean, var = mean[0], var[0]
    sd = np.sqrt(var)
    assert np.all(np.abs(f.mean(axis=0) - mean) <= 5.0 * sd / np.sqrt(S) + 1e-12)
    rel = np.abs(f.var(axis=0, ddof=1) / var - 1.0)
    assert rel.max() <= 6.0 * np.sqrt(2.0 / S), rel.max()


def _gpar_case(kernel="matern52"):
    t, Y = O.synthetic_gpar(600, 3, seed=21, noise=0.3)
    V = np.ascontiguousarray(Y[:, :2].T)
    Z = O.pick_pseudo_inputs(V, 30, 5)
    y = Y[:, 2].copy()
    ts = np.sort(np.random.default_rng(4).uniform(t[0], t[-1], 150))
    Vs = np.vstack([np.interp(ts, t, V[q]) for q in range(2)])
    return V, Z, t, y, ts, Vs


@pytest.mark.parametrize("qu_noise,S", [(False, 8), (True, 8), (True, 200)])
def test_path_prediction_replays_through_the_oracle(qu_noise, S):
    """S = 200: more than one 128-column block of the f_x GEMM (its row-sum epilogue
    wrote past a buffer sized for one block)."""
    V, Z, t, y, ts, Vs = _gpar_case()
    theta = (1.3, 0.9, 0.8, 1.1, 0.2)
    seed = 77
    mean, std = G.predict_scaled(V, Z, t, y, theta, ts, Vs, mode="path", samples=S, seed=seed,
                                 qu_kuu_noise=qu_noise)
    xi_u = G.mc_normals(S, Z.shape[1], seed).T
    xi_p = G.path_normals(S, len(t) + len(ts), 4, seed)
    rm, rs = O.get_gpar_scaled_predictions_path_fixed(V, Z, t, y, ts, Vs, theta, xi_u, xi_p,
                                                      qu_kuu_noise=qu_noise)
    np.testing.assert_allclose(mean, rm, rtol=1e-7, atol=1e-9 * np.abs(rm).max())
    np.testing.assert_allclose(std, rs, rtol=1e-6, atol=1e-9 * np.abs(rs).max())
    # the path estimator's spread includes the time GP's posterior variance: at least the MC's
    mm, ms = G.predict_scaled(V, Z, t, y, theta, ts, Vs, mode="mc", samples=S, seed=seed,
                              qu_kuu_noise=qu_noise)
    assert np.median(std) > np.median(ms)


def test_fit_predict_path_mode_equals_predict():
    V, Z, t, y, ts, Vs = _gpar_case()
    V2, Z2 = V[:1].copy(), Z[:1].copy()
    probs, keep = [], []
    for VV, ZZ in ((V, Z), (V2, Z2)):
        pr, k = G.make_problem(VV, ZZ, t, y)
        probs.append(pr)
        keep.append(k)
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (2, 1))
    fr, means, stds = G.fit_predict_batch(probs, x0, ts, [Vs, Vs[:1]], max_evals=15, g_tol=-1.0,
                                          mode="path", samples=12, seed=5)
    for i, (VV, ZZ, VS) in enumerate(((V, Z, Vs), (V2, Z2, Vs[:1]))):
        m, s = G.predict_scaled(VV, ZZ, t, y, fr.theta[i], ts, VS, mode="path", samples=12,
                                seed=5 + i)
        np.testing.assert_allclose(means[i], m, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(stds[i], s, rtol=1e-12, atol=1e-14)


def test_path_arguments():
    t, y, noise = _grid(50, 1)
    with pytest.raises(G.DomainError):
        G.posterior_rand(t, y, (1.0, 1.0, 0.1), samples=0)
    with pytest.raises(G.DomainError):
        G.posterior_rand(t[::-1].copy(), y, (1.0, 1.0, 0.1), samples=2)
    with pytest.raises(G.Unsupported):
        G.posterior_rand(t, y, (1.0, 1.0, 0.1), kernel="eq", samples=2)
    # device inputs: lengths checked on the host (the C side cannot see them)
    import torch
    td, yd = torch.from_numpy(t).cuda(), torch.from_numpy(y).cuda()
    with pytest.raises(G.DomainError):
        G.posterior_rand(td, yd[:-1], (1.0, 1.0, 0.1), samples=2)
    with pytest.raises(G.DomainError):
        G.posterior_rand(td, yd, (1.0, 1.0, 0.1), samples=2, noise=yd[:10])
