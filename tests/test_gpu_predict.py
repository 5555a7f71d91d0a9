"""GPU parity of scaled-GPAR prediction (gpar_scaled_inference.jl:63-135) and of the
Nelder-Mead fit (dtc.jl:11-77) against the oracle."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")


def _data(n, P, M, seed, n_star, gaps=0):
    t, Y = O.synthetic_gpar(n, P, seed=seed, noise=0.3, gaps=gaps, gap_len=max(1, n // 25))
    V = Y[:, : P - 1].T
    y = Y[:, P - 1]
    Z = O.pick_pseudo_inputs(V, M, seed + 3)
    rng = np.random.default_rng(seed + 11)
    ts = np.sort(rng.uniform(t[0] - 1.0, t[-1] + 2.0, n_star))
    Vs = np.vstack([np.interp(ts, t, V[q]) for q in range(P - 1)])
    return t, V, Z, y, ts, Vs


# q(u) factors Cuu with no jitter (gpar_scaled_inference.jl:157-159), so agreement between
# any two fp64 implementations is limited by cond(Cuu) * eps; the cases below keep
# cond(Cuu) <= ~1e7 so the 1e-8 / 1e-7 tolerances are meaningful.
@pytest.mark.parametrize("n,P,M,kernels,l_o", [(400, 3, 30, ("matern52", "matern52"), 1.2),
                                               (700, 4, 140, ("eq", "matern32"), 0.25),
                                               (300, 2, 20, ("matern32", "matern12"), 0.3)])
def test_predict_analytic_matches_oracle(n, P, M, kernels, l_o):
    t, V, Z, y, ts, Vs = _data(n, P, M, 5, 150, gaps=2)
    theta = (1.4, 0.9, l_o, 1.1, 0.3)
    ok, tk = kernels
    m_ref, s_ref = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, theta, ok, tk, "analytic")
    m, s = G.predict_scaled(V, Z, t, y, theta, ts, Vs, ok, tk, mode="analytic")
    np.testing.assert_allclose(m, m_ref, rtol=1e-8, atol=1e-9 * np.abs(m_ref).max())
    np.testing.assert_allclose(s, s_ref, rtol=1e-7, atol=1e-9 * np.abs(s_ref).max())


def test_predict_unsorted_and_coincident_test_points():
    t, V, Z, y, ts, Vs = _data(350, 3, 25, 9, 120)
    ts = np.concatenate([ts, t[::37]])            # test times coinciding with train times
    Vs = np.hstack([Vs, V[:, ::37]])
    perm = np.random.default_rng(1).permutation(len(ts))
    ts, Vs = ts[perm], Vs[:, perm]
    theta = (0.9, 1.1, 0.8, 1.3, 0.25)
    m_ref, s_ref = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, theta, mode="analytic")
    m, s = G.predict_scaled(V, Z, t, y, theta, ts, Vs, mode="analytic")
    np.testing.assert_allclose(m, m_ref, rtol=1e-8, atol=1e-9 * np.abs(m_ref).max())
    np.testing.assert_allclose(s, s_ref, rtol=1e-7, atol=1e-9 * np.abs(s_ref).max())


def test_predict_mc_statistically_matches_analytic():
    """MC mode (reference-faithful, 100 samples): |mean_mc - mean| <= 5 std / sqrt(S)."""
    t, V, Z, y, ts, Vs = _data(500, 3, 40, 13, 200)
    theta = (1.2, 1.0, 1.0, 1.2, 0.3)
    m, s = G.predict_scaled(V, Z, t, y, theta, ts, Vs, mode="analytic")
    mm, sm = G.predict_scaled(V, Z, t, y, theta, ts, Vs, mode="mc", samples=100, seed=7)
    S = 100
    assert np.all(np.abs(mm - m) <= 5.0 * s / np.sqrt(S) + 1e-12)
    # sample std within chi-distribution tolerance of the analytic std
    ratio = sm / np.maximum(s, 1e-300)
    assert np.median(np.abs(ratio - 1.0)) < 0.15
    mm2, sm2 = G.predict_scaled(V, Z, t, y, theta, ts, Vs, mode="mc", samples=100, seed=7)
    np.testing.assert_array_equal(mm, mm2)    # seeded -> reproducible


def test_fit_matches_oracle_nelder_mead():
    """Same NM state machine on both sides: identical trajectories up to fp64 ties."""
    t, V, Z, y, _, _ = _data(300, 3, 25, 17, 1)
    x0 = [0.1, 0.2, 0.0, 0.1, -1.5]
    th_ref, nm = O.get_optim_scaled_gpar_params(V, Z, t, y, log_theta0=x0, max_evals=40,
                                                return_nm=True)
    th = G.get_optim_scaled_gpar_params(V, Z, t, y, i_log_time_l=x0[0], i_log_time_var=x0[1],
                                        i_log_out_l=x0[2], i_log_out_var=x0[3],
                                        i_log_noise_sigma=x0[4], max_evals=40,
                                        optimization_time_limit=0)
    np.testing.assert_allclose(th, th_ref, rtol=1e-6)


@pytest.mark.parametrize("kernel", ["matern12", "matern32", "matern52"])
def test_lgssm_smooth_matches_oracle(kernel):
    t, Y = O.synthetic_gpar(1200, 2, seed=4, noise=0.4, gaps=3, gap_len=80)
    th = [(0.7, 1.3, 0.2), (4.0, 0.8, 0.5)]
    rng = np.random.default_rng(3)
    noise = np.where(rng.random(len(t)) < 0.2, 1e10, -1.0)   # some 'test' points, rest chain sigma^2
    mean, var = G.lgssm_smooth_batch(t, Y.T, th, kernel, noise=noise)
    for c in range(2):
        R = np.where(noise < 0, th[c][2] ** 2, noise)
        lg = O.create_lgssm(t, *th[c], kind=kernel, noise_vector=R)
        ms, Ps = O.rts_smooth(lg, Y[:, c])
        np.testing.assert_allclose(mean[c], ms[:, 0], rtol=1e-9, atol=1e-10 * np.abs(ms[:, 0]).max())
        np.testing.assert_allclose(var[c], Ps[:, 0, 0], rtol=1e-8, atol=1e-12)


def test_sde_predictions_match_oracle():
    t, Y = O.synthetic_gpar(600, 2, seed=6, noise=0.4, gaps=2, gap_len=40)
    ts = np.sort(np.random.default_rng(2).uniform(-1, t[-1] + 1, 90))
    x0 = (-1.0, 0.2, -1.5)
    th_ref, m_ref, v_ref = O.get_sde_predictions(t, Y[:, 0], ts, "matern52", x0, max_evals=30)
    th, m, v = G.get_sde_predictions(t, Y[:, 0], ts, "matern52", *x0, max_evals=30)
    np.testing.assert_allclose(th, th_ref, rtol=1e-6)
    np.testing.assert_allclose(m, m_ref, rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(v, v_ref, rtol=1e-6, atol=1e-10)


@pytest.mark.parametrize("qu_noise", [True, False])
def test_fit_predict_equals_fit_then_predict(qu_noise):
    """gpar_fit_predict (get_gpar_scaled_predictions, gpar_scaled_inference.jl:20-136, batched
    over outputs) == gpar_fit followed by one gpar_predict per output at the fitted theta --
    bit for bit: with qu_kuu_noise q(u) reuses the fit's Gram at that theta, which is the same
    computation it would redo; without, q(u) recomputes it (from the fixed-up beta: reusing the
    fit's correction-form Gram for the noise-free Cuu measured 1.5e-7 off the oracle, r04a)."""
    import torch
    dev = torch.device("cuda", 0)
    t, Y = O.synthetic_gpar(900, 5, seed=23, noise=0.3)
    rng = np.random.default_rng(4)
    ts = np.sort(rng.uniform(t[0], t[-1], 200))
    Fs = np.column_stack([np.interp(ts, t, Y[:, q]) for q in range(5)])
    t_d, Y_d = torch.from_numpy(t).to(dev), torch.from_numpy(Y).to(dev)
    ts_d, Fs_d = torch.from_numpy(ts).to(dev), torch.from_numpy(Fs).to(dev)
    outs = [2, 4, 5]
    probs, keep, Zs = [], [], {}
    for p in outs:
        Zs[p] = torch.from_numpy(O.pick_pseudo_inputs(Y[:, : p - 1].T, 70, p).T.copy()).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Zs[p], t_d, Y_d[:, p - 1].contiguous(),
                               qu_kuu_noise=qu_noise)
        probs.append(pr)
        keep.append(k)
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(outs), 1))
    fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, [Fs_d[:, : p - 1] for p in outs],
                                          max_evals=30, g_tol=-1.0)
    fr2 = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
    np.testing.assert_array_equal(fr.theta, fr2.theta)
    for i, p in enumerate(outs):
        m2, s2 = G.predict_scaled(Y_d[:, : p - 1], Zs[p], t_d, Y_d[:, p - 1].contiguous(),
                                  fr.theta[i], ts_d, Fs_d[:, : p - 1], qu_kuu_noise=qu_noise)
        np.testing.assert_array_equal(means[i].cpu().numpy(), m2.cpu().numpy())
        np.testing.assert_array_equal(stds[i].cpu().numpy(), s2.cpu().numpy())


@pytest.mark.parametrize("M,n,n_star,tk", [(30, 3000, 333, "matern32"), (140, 3000, 333, "matern32"),
                                            (300, 3000, 333, "matern32"), (512, 3000, 333, "matern32"),
                                            (520, 3000, 333, "matern32"), (512, 2000, 6000, "matern32"),
                                            (140, 2000, 6000, "matern12"), (300, 1500, 5000, "matern52")])
def test_predict_fused_rows_variance_equals_unfused(M, n, n_star, tk):
    """predict_var (rows, mean and |Q_i V^T|^2 fused, m <= 512: NT = 2, 4, 6, 8 tile slots per
    wave; 520 takes the unfused path both ways) against predict_rows + gemm_nt on the same q(u):
    the same sums in another order.  N* = 333 leaves a ragged last 64-row panel and spreads a
    64-row panel over more than two chunks of the merged grid (the kernel's direct-load path);
    N* > N keeps most panels within two chunks (its LDS-DMA prefetching path)."""
    t, V, Z, y, ts, Vs = _data(n, 4, M, 21, n_star)
    theta = (1.3, 0.9, 0.9, 1.2, 0.3)
    ctx = G.context()
    try:
        ctx.set_predict_fused(False)
        m0, s0 = G.predict_scaled(V, Z, t, y, theta, ts, Vs, "matern52", tk, mode="analytic",
                                  qu_kuu_noise=True)
        ctx.set_predict_fused(True)
        m1, s1 = G.predict_scaled(V, Z, t, y, theta, ts, Vs, "matern52", tk, mode="analytic",
                                  qu_kuu_noise=True)
    finally:
        ctx.set_predict_fused(True)
    assert np.all(np.isfinite(m1)) and np.all(s1 > 0)
    np.testing.assert_allclose(m1, m0, rtol=1e-11, atol=1e-13 * np.abs(m0).max())
    np.testing.assert_allclose(s1, s0, rtol=1e-11, atol=1e-13 * np.abs(s0).max())
    # and the oracle directly: at an NT = 6 shape with masked high tiles (the direct-load path),
    # and every N* > N case (the LDS-DMA prefetching path the north bench's N* = N takes)
    if (M == 300 and n == 3000) or n_star > n:
        m_ref, s_ref = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, theta, "matern52",
                                                           tk, "analytic", qu_kuu_noise=True)
        np.testing.assert_allclose(m1, m_ref, rtol=1e-7, atol=1e-9 * np.abs(m_ref).max())
        np.testing.assert_allclose(s1, s_ref, rtol=1e-7, atol=1e-9 * np.abs(s_ref).max())
