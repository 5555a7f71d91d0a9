"""The per-output GPAR driver end to end against the oracle:

* get_gpar_scaled_predictions (gpar_scaled_inference.jl:20-136) over several outputs at once
  (gpar_fit_predict: batched NM fit with a fixed x0 and a fixed evaluation budget, then q(u) and
  the prediction at the fitted theta) against the oracle's per-output fit + prediction, for
  both q(u) conventions (noise-free Cuu as the reference, :157; Cuu + sigma^2 I as the bench);
* the MC estimator (:91-130) replayed with the device's own standard-normal draws
  (gpar_mc_normals) through the oracle's restatement, which maps them as Distributions'
  MvNormal does (m_e + chol(inv(D)).L xi);
* chained inference inputs (GPAR_scaled_examples.jl:172: y3's inference inputs are
  [test_y1, y2_out]) through gpar_fit_predict_chain, against the serial oracle chain.

Tolerances: theta rtol 1e-6 (same NM state machine, fp64 ties), predictions rtol
1e-7 (through inv(D), cond 1e6-1e8)."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")

X0 = np.array([0.0, 0.0, 0.0, 0.0, -2.0])


def _chain_data(n, P, seed, n_star):
    t, Y = O.synthetic_gpar(n, P, seed=seed, noise=0.3)
    rng = np.random.default_rng(seed + 1)
    ts = np.sort(rng.uniform(t[0], t[-1], n_star))
    F = np.column_stack([np.interp(ts, t, Y[:, q]) for q in range(P)])   # test inputs
    return t, Y, ts, F


def _close(got, ref, rtol):
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=rtol * 1e-2 * np.abs(ref).max())


@pytest.mark.parametrize("qu_noise", [False, True])
def test_fit_predict_batch_matches_oracle_driver(qu_noise):
    """Outputs with D = 1, 5, 20 in one gpar_fit_predict call, 40 evaluations each, g_tol off."""
    t, Y, ts, F = _chain_data(500, 21, 31, 120)
    outs = [2, 6, 21]
    probs, keep, Vs_list, refs = [], [], [], []
    for p in outs:
        V = np.ascontiguousarray(Y[:, : p - 1].T)
        Z = O.pick_pseudo_inputs(V, 24, p)
        pr, k = G.make_problem(V, Z, t, Y[:, p - 1], qu_kuu_noise=qu_noise)
        probs.append(pr)
        keep.append(k)
        Vs = np.ascontiguousarray(F[:, : p - 1].T)
        Vs_list.append(Vs)
        m, s, th = O.get_gpar_scaled_predictions(V, Z, t, Y[:, p - 1], ts, Vs, log_theta0=X0,
                                                 max_evals=40, g_tol=-1.0, qu_kuu_noise=qu_noise)
        refs.append((th, m, s))
    fr, means, stds = G.fit_predict_batch(probs, np.tile(X0, (len(outs), 1)), ts, Vs_list,
                                          max_evals=40, g_tol=-1.0)
    for i, (th, m, s) in enumerate(refs):
        np.testing.assert_allclose(fr.theta[i], th, rtol=1e-6)
        assert fr.evals[i] == 40
        _close(means[i], m, 1e-7)
        _close(stds[i], s, 1e-7)


@pytest.mark.parametrize("S", [100, 300])
def test_mc_replayed_draws_match_oracle(S):
    """MC mode with S draws (100 = the reference's count; 300 spans three 128-column tiles) equals
    the oracle's MC fed the same draws."""
    t, Y, ts, F = _chain_data(450, 4, 37, 150)
    V = np.ascontiguousarray(Y[:, :3].T)
    Z = O.pick_pseudo_inputs(V, 36, 5)
    Vs = np.ascontiguousarray(F[:, :3].T)
    theta = (1.2, 1.0, 1.1, 1.2, 0.3)
    seed = 1234
    xi = G.mc_normals(S, Z.shape[1], seed)
    assert xi.shape == (S, 36)
    m, s = G.predict_scaled(V, Z, t, Y[:, 3], theta, ts, Vs, mode="mc", samples=S, seed=seed)
    rm, rs = O.get_gpar_scaled_predictions_fixed(V, Z, t, Y[:, 3], ts, Vs, theta, mode="mc",
                                                 xi=xi.T)
    _close(m, rm, 1e-7)
    _close(s, rs, 1e-7)


def test_mc_normals_are_standard_normal_and_seeded():
    a = G.mc_normals(400, 256, 5)
    b = G.mc_normals(400, 256, 5)
    c = G.mc_normals(400, 256, 6)
    np.testing.assert_array_equal(a, b)
    assert not np.array_equal(a, c)
    # padding-independent: a prefix of the coordinates is the same draw
    np.testing.assert_array_equal(G.mc_normals(400, 100, 5), a[:, :100])
    z = a.ravel()
    assert abs(z.mean()) < 5.0 / np.sqrt(z.size)
    assert abs(z.std() - 1.0) < 5.0 / np.sqrt(2 * z.size)
    # third / fourth moments within 5 standard errors (var z^3 = 15, var z^4 = 96)
    assert abs(np.mean(z ** 3)) < 5.0 * np.sqrt(15.0 / z.size)
    assert abs(np.mean(z ** 4) - 3.0) < 5.0 * np.sqrt(96.0 / z.size)


def test_fit_predict_mc_uses_seed_plus_output_index():
    t, Y, ts, F = _chain_data(400, 5, 41, 100)
    outs = [3, 5]
    probs, keep, Vs_list, data = [], [], [], []
    for p in outs:
        V = np.ascontiguousarray(Y[:, : p - 1].T)
        Z = O.pick_pseudo_inputs(V, 28, p)
        pr, k = G.make_problem(V, Z, t, Y[:, p - 1], qu_kuu_noise=True)
        probs.append(pr)
        keep.append(k)
        Vs_list.append(np.ascontiguousarray(F[:, : p - 1].T))
        data.append((V, Z, Y[:, p - 1]))
    seed = 77
    fr, means, stds = G.fit_predict_batch(probs, np.tile(X0, (2, 1)), ts, Vs_list, max_evals=20,
                                          g_tol=-1.0, mode="mc", samples=100, seed=seed)
    for i, (V, Z, y) in enumerate(data):
        xi = G.mc_normals(100, Z.shape[1], seed + i)
        rm, rs = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs_list[i], fr.theta[i],
                                                     mode="mc", xi=xi.T, qu_kuu_noise=True)
        _close(means[i], rm, 1e-7)
        _close(stds[i], rs, 1e-7)


def _oracle_chain(t, Y, ts, F, outs, M, evals, qu_noise):
    """Serial reference chain: output p's inference inputs are [test_y1, pred_y2 .. pred_y(p-1)]."""
    chain = F[:, :1].copy()
    res = {}
    for p in outs:
        V = np.ascontiguousarray(Y[:, : p - 1].T)
        Z = O.pick_pseudo_inputs(V, M, p)
        Vs = np.ascontiguousarray(chain[:, : p - 1].T)
        m, s, th = O.get_gpar_scaled_predictions(V, Z, t, Y[:, p - 1], ts, Vs, log_theta0=X0,
                                                 max_evals=evals, g_tol=-1.0, qu_kuu_noise=qu_noise)
        chain = np.column_stack([chain, m])
        res[p] = (th, m, s)
    return res


@pytest.mark.parametrize("device", [False, True])
def test_chained_inference_inputs_match_serial_oracle(device):
    t, Y, ts, F = _chain_data(400, 5, 43, 90)
    outs, M, EV = [2, 3, 4, 5], 20, 25
    ref = _oracle_chain(t, Y, ts, F, outs, M, EV, True)
    chain = np.zeros((len(ts), 5))
    chain[:, 0] = F[:, 0]                         # test_y1: the true first output
    probs, keep = [], []
    if device:
        import torch
        dev = torch.device("cuda", 0)
        t_d, Y_d, ts_d = (torch.from_numpy(a).to(dev) for a in (t, Y, ts))
        chain_d = torch.from_numpy(chain).to(dev)
    for p in outs:
        Z = O.pick_pseudo_inputs(np.ascontiguousarray(Y[:, : p - 1].T), M, p)
        if device:
            pr, k = G.make_problem(Y_d[:, : p - 1], torch.from_numpy(Z.T.copy()).to(dev), t_d,
                                   Y_d[:, p - 1].contiguous(), qu_kuu_noise=True)
        else:
            pr, k = G.make_problem(np.ascontiguousarray(Y[:, : p - 1].T), Z, t, Y[:, p - 1],
                                   qu_kuu_noise=True)
        probs.append(pr)
        keep.append(k)
    fr, means, stds = G.fit_predict_batch(
        probs, np.tile(X0, (len(outs), 1)), ts_d if device else ts, [None] * len(outs),
        max_evals=EV, g_tol=-1.0, chain=chain_d if device else chain,
        chain_cols=[p - 1 for p in outs])
    got_chain = chain_d.cpu().numpy() if device else chain
    for i, p in enumerate(outs):
        th, m, s = ref[p]
        np.testing.assert_allclose(fr.theta[i], th, rtol=1e-6)
        mi = means[i].cpu().numpy() if device else means[i]
        si = stds[i].cpu().numpy() if device else stds[i]
        _close(mi, m, 1e-7)
        _close(si, s, 1e-7)
        np.testing.assert_array_equal(got_chain[:, p - 1], mi)
    np.testing.assert_array_equal(got_chain[:, 0], F[:, 0])
