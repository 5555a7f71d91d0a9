"""Posterior objects: get_gpar_scaled_predictions (gpar_scaled_inference.jl:
20-136) split where it first reads the inference inputs.  gpar_fit_posterior = the batched fit +
q(u) at the fitted theta (reusing the fit's Gram), kept on the device; gpar_posterior_predict = the
V*-dependent prediction.  The chained multi-rank sweep (GPAR_scaled_examples.jl:172, eeg.jl:249,274)
then runs only predictions inside its serial cross-rank order.

Checked: the posterior's predictions equal gpar_fit_predict's bit for bit (both q(u) conventions,
analytic and MC, device and host problems), and a chained sweep over posterior predictions equals
gpar_fit_predict_chain bit for bit."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")

X0 = np.array([0.0, 0.0, 0.0, 0.0, -2.0])


def _data(seed=23, n=900, P=5, n_star=200):
    t, Y = O.synthetic_gpar(n, P, seed=seed, noise=0.3)
    ts = np.sort(np.random.default_rng(seed + 1).uniform(t[0], t[-1], n_star))
    F = np.column_stack([np.interp(ts, t, Y[:, q]) for q in range(P)])
    return t, Y, ts, F


@pytest.mark.parametrize("qu_noise", [True, False])
@pytest.mark.parametrize("mode", ["analytic", "mc"])
def test_posterior_predict_equals_fit_predict_device(qu_noise, mode):
    import torch
    dev = torch.device("cuda", 0)
    t, Y, ts, F = _data()
    t_d, Y_d, ts_d, F_d = (torch.from_numpy(a).to(dev) for a in (t, Y, ts, F))
    outs = [2, 4, 5]
    probs, keep = [], []
    for p in outs:
        Z = torch.from_numpy(O.pick_pseudo_inputs(Y[:, : p - 1].T, 60, p).T.copy()).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(),
                               qu_kuu_noise=qu_noise)
        probs.append(pr)
        keep.append((k, Z))
    x0 = np.tile(X0, (len(outs), 1))
    Vs = [F_d[:, : p - 1] for p in outs]
    seed = 11
    fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, Vs, max_evals=25, g_tol=-1.0, mode=mode,
                                          samples=100, seed=seed)
    post = G.fit_posterior(probs, x0, max_evals=25, g_tol=-1.0, keep=keep)
    np.testing.assert_array_equal(post.theta, fr.theta)
    np.testing.assert_array_equal(post.fit.nlml, fr.nlml)
    for i in range(len(outs)):
        m, s = post.predict(i, ts_d, Vs[i], mode=mode, samples=100, seed=seed + i)
        np.testing.assert_array_equal(m.cpu().numpy(), means[i].cpu().numpy())
        np.testing.assert_array_equal(s.cpu().numpy(), stds[i].cpu().numpy())
    post.close()


def test_posterior_predict_host_problems():
    t, Y, ts, F = _data(seed=29, n=700, P=4, n_star=150)
    outs = [2, 4]
    probs, keep, Vs = [], [], []
    for p in outs:
        V = np.ascontiguousarray(Y[:, : p - 1].T)
        Z = O.pick_pseudo_inputs(V, 40, p)
        pr, k = G.make_problem(V, Z, t, Y[:, p - 1], qu_kuu_noise=True)
        probs.append(pr)
        keep.append(k)
        Vs.append(np.ascontiguousarray(F[:, : p - 1].T))
    x0 = np.tile(X0, (len(outs), 1))
    fr, means, stds = G.fit_predict_batch(probs, x0, ts, Vs, max_evals=20, g_tol=-1.0)
    post = G.fit_posterior(probs, x0, max_evals=20, g_tol=-1.0, keep=keep)
    del keep   # host inputs were copied: the posterior no longer needs them
    for i in range(len(outs)):
        # a call in between reuses the problem-upload workspace the posterior must not depend on
        G.compute_gpar_dtc_objective(Vs[i][:, :50], Vs[i][:, :10], ts[:50], ts[:50],
                                     (1.0, 1.0, 1.0, 1.0, 0.3))
        m, s = post.predict(i, ts, Vs[i])
        np.testing.assert_array_equal(m, means[i])
        np.testing.assert_array_equal(s, stds[i])
    with pytest.raises(G.DomainError):
        post.predict(5, ts, Vs[0])


def test_chained_sweep_over_posteriors_equals_fit_predict_chain():
    """The multi-rank chained path's arithmetic on one process: output p's inference inputs are
    [test_y1, predicted means of outputs 2 .. p-1] (GPAR_scaled_examples.jl:172)."""
    import torch
    dev = torch.device("cuda", 0)
    t, Y, ts, F = _data(seed=43, n=600, P=5, n_star=120)
    t_d, Y_d, ts_d = (torch.from_numpy(a).to(dev) for a in (t, Y, ts))
    outs = [2, 3, 4, 5]
    probs, keep = [], []
    for p in outs:
        Z = torch.from_numpy(O.pick_pseudo_inputs(Y[:, : p - 1].T, 24, p).T.copy()).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), qu_kuu_noise=True)
        probs.append(pr)
        keep.append((k, Z))
    x0 = np.tile(X0, (len(outs), 1))
    chain = torch.zeros((len(ts), 5), dtype=torch.float64, device=dev)
    chain[:, 0] = torch.from_numpy(F[:, 0]).to(dev)
    chain2 = chain.clone()
    fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, [None] * len(outs), max_evals=20,
                                          g_tol=-1.0, chain=chain, chain_cols=[p - 1 for p in outs])
    post = G.fit_posterior(probs, x0, max_evals=20, g_tol=-1.0, keep=keep)
    for i, p in enumerate(outs):
        m, s = post.predict(i, ts_d, chain2[:, : p - 1])
        chain2[:, p - 1] = m
        np.testing.assert_array_equal(m.cpu().numpy(), means[i].cpu().numpy())
        np.testing.assert_array_equal(s.cpu().numpy(), stds[i].cpu().numpy())
    np.testing.assert_array_equal(chain2.cpu().numpy(), chain.cpu().numpy())


def test_prepared_predictions_equal_in_line():
    """gpar_posterior_prepare: the merged grid's gains and adjoint fix-up rows queued ahead on the
    side stream give the same bits as computing them in line; a slot prepared for other test
    times, or overwritten by a third prepare, is not used."""
    import torch
    dev = torch.device("cuda", 0)
    t, Y, ts, F = _data(seed=31, n=800, P=5, n_star=170)
    t_d, Y_d, ts_d, F_d = (torch.from_numpy(a).to(dev) for a in (t, Y, ts, F))
    ts2_d = ts_d.clone()   # same values, another pointer: not the prepared slot
    outs = [2, 3, 4, 5]
    probs, keep = [], []
    for p in outs:
        Z = torch.from_numpy(O.pick_pseudo_inputs(Y[:, : p - 1].T, 40, p).T.copy()).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), qu_kuu_noise=True)
        probs.append(pr)
        keep.append((k, Z))
    post = G.fit_posterior(probs, np.tile(X0, (len(outs), 1)), max_evals=15, g_tol=-1.0, keep=keep)
    Vs = [F_d[:, : p - 1] for p in outs]
    ref = [post.predict(i, ts_d, Vs[i]) for i in range(len(outs))]
    # prepared one ahead, as the chained sweep does
    post.prepare(0, ts_d)
    for i in range(len(outs)):
        if i + 1 < len(outs):
            post.prepare(i + 1, ts_d)
        m, s = post.predict(i, ts_d, Vs[i])
        np.testing.assert_array_equal(m.cpu().numpy(), ref[i][0].cpu().numpy())
        np.testing.assert_array_equal(s.cpu().numpy(), ref[i][1].cpu().numpy())
    # three prepares: the first slot is reused by the third; every predict is still exact
    for i in (0, 1, 2):
        post.prepare(i, ts_d)
    for i in (0, 1, 2):
        m, s = post.predict(i, ts_d, Vs[i])
        np.testing.assert_array_equal(m.cpu().numpy(), ref[i][0].cpu().numpy())
        np.testing.assert_array_equal(s.cpu().numpy(), ref[i][1].cpu().numpy())
    # prepared for other test-time storage, and MC mode over a prepared slot
    post.prepare(3, ts2_d)
    m, s = post.predict(3, ts_d, Vs[3])
    np.testing.assert_array_equal(m.cpu().numpy(), ref[3][0].cpu().numpy())
    mc = post.predict(1, ts_d, Vs[1], mode="mc", samples=64, seed=5)
    post.prepare(1, ts_d)
    mc2 = post.predict(1, ts_d, Vs[1], mode="mc", samples=64, seed=5)
    np.testing.assert_array_equal(mc[0].cpu().numpy(), mc2[0].cpu().numpy())
    np.testing.assert_array_equal(mc[1].cpu().numpy(), mc2[1].cpu().numpy())
    post.close()


def test_chained_sweep_with_prepare_equals_fit_predict_chain():
    import torch
    from gparatscale import shard as S
    dev = torch.device("cuda", 0)
    t, Y, ts, F = _data(seed=47, n=600, P=5, n_star=120)
    t_d, Y_d, ts_d = (torch.from_numpy(a).to(dev) for a in (t, Y, ts))
    outs = [2, 3, 4, 5]
    probs, keep = [], []
    for p in outs:
        Z = torch.from_numpy(O.pick_pseudo_inputs(Y[:, : p - 1].T, 24, p).T.copy()).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), qu_kuu_noise=True)
        probs.append(pr)
        keep.append((k, Z))
    x0 = np.tile(X0, (len(outs), 1))
    chain = torch.zeros((len(ts), 5), dtype=torch.float64, device=dev)
    chain[:, 0] = torch.from_numpy(F[:, 0]).to(dev)
    chain2 = chain.clone()
    fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, [None] * len(outs), max_evals=20,
                                          g_tol=-1.0, chain=chain, chain_cols=[p - 1 for p in outs])
    post = G.fit_posterior(probs, x0, max_evals=20, g_tol=-1.0, keep=keep)
    idx = {p: i for i, p in enumerate(outs)}
    mine = S.chained_predictions(outs, {p: 0 for p in outs},
                                 lambda p, c: post.predict(idx[p], ts_d, c[:, : p - 1]), chain2,
                                 prepare_fn=lambda p: post.prepare(idx[p], ts_d))
    for i, p in enumerate(outs):
        np.testing.assert_array_equal(mine[p][0].cpu().numpy(), means[i].cpu().numpy())
        np.testing.assert_array_equal(mine[p][1].cpu().numpy(), stds[i].cpu().numpy())
    np.testing.assert_array_equal(chain2.cpu().numpy(), chain.cpu().numpy())
