"""Parity of the bench's headline schedule.

bench.py's north job runs the batched fit on the schedule that only engages on big problems: the
auto CU split (N Mp^2 >= 1e11, gpar_host.cpp split_active), the pipelined Gram stage and the
distance cache down to D = 1 (N >= 2^16 on the split), q(u) reusing the fit's Gram at the fitted
theta.  Here that schedule runs un-forced at N = 4e5, M = 512 (N Mp^2 = 1.05e11) over five outputs
with D = 1, 2, 8, 16, 32, HBM-resident inputs laid out as the bench lays them (V a column slice of
the N x P output matrix), and is compared with
  * the same call on the whole-chip, uncached schedule (gpar_ctx_set_cu_split(0),
    gpar_ctx_set_dist_cache(0)): fitted theta rtol 1e-9, -nlml rel 1e-12;
  * the C port (oracle/cpu_ref, pinned to the numpy oracle by tests/test_cpu_ref.py): each output's
    DTC objective (src/gp/dtc.jl:83-128) at its fitted theta rel <= 1e-9, and its analytic
    prediction (gpar_scaled_inference.jl:20-136, q(u) with Cuu + sigma^2 I as the bench) rtol 1e-7.
The cached distances themselves (dist2 at D = 1..16, the range the all-D cache added) are checked
against direct differences in test_gpu_dist_cache.py.

The bench predicts at N* = N test times interleaved with the training times, where predict_var's
64-row panels lie within two chunks of the merged grid and take its LDS-DMA prefetching path, and
the predictions alternate over two lanes.  That layout runs here too: N = N* =
4e5, two outputs (D = 8, 32) through fit_predict_batch on the headline schedule, each output's
objective and prediction against the C port.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

G = pytest.importorskip("gparatscale")
from gparatscale import data as D  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, M, NS, EV = 400_000, 512, 40_000, 10
OUTS = [2, 3, 9, 17, 33]            # D = p - 1 = 1, 2, 8, 16, 32


@pytest.fixture(scope="module")
def CR():
    if not os.path.exists(os.path.join(ROOT, "oracle", "libgpar_cpu.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    from oracle import cpu_ref
    cpu_ref.load()
    return cpu_ref


@pytest.fixture(scope="module")
def runs():
    import torch
    dev = torch.device("cuda", 0)
    ds = D.gpar_dataset(N, max(OUTS), seed=0, observation_noise=0.8, n_star=NS)
    Y_d = torch.from_numpy(ds["Y"]).to(dev)
    t_d = torch.from_numpy(ds["t"]).to(dev)
    ts_d = torch.from_numpy(ds["t_star"]).to(dev)
    Fs_d = torch.from_numpy(ds["F_star"]).to(dev)
    probs, keep, Zs = [], [], {}
    for p in OUTS:
        Zs[p] = D.pseudo_inputs(ds["Y"][:, : p - 1], M, seed=p)
        pr, k = G.make_problem(Y_d[:, : p - 1], torch.from_numpy(Zs[p]).to(dev), t_d,
                               Y_d[:, p - 1].contiguous(), "matern52", "matern52", qu_kuu_noise=True)
        probs.append(pr)
        keep.append(k)
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(OUTS), 1))
    Vs = [Fs_d[:, : p - 1] for p in OUTS]
    ctx = G.context(0)

    def run():
        fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, Vs, max_evals=EV, g_tol=-1.0)
        return fr, [m.cpu().numpy() for m in means], [s.cpu().numpy() for s in stds]

    try:
        ctx.set_cu_split(-1)          # the library default, gated by problem size as in the bench
        ctx.set_dist_cache(-1)
        assert ctx.cu_split() == 8
        head = run()
        cached = ctx.dist_cache_stats()[0]
        ctx.set_cu_split(0)
        ctx.set_dist_cache(0)
        whole = run()
    finally:
        ctx.set_cu_split(-1)
        ctx.set_dist_cache(-1)
    return dict(ds=ds, Zs=Zs, head=head, whole=whole, cached=cached)


def test_headline_schedule_engages(runs):
    # N Mp^2 = 4e5 * 512^2 >= 1e11 (split on by default) and N >= 2^16: every output cached
    assert N * 512 * 512 >= 1e11
    assert runs["cached"] == len(OUTS)


def test_headline_schedule_matches_whole_chip(runs):
    (a, am, asd), (b, bm, bsd) = runs["head"], runs["whole"]
    np.testing.assert_allclose(a.theta, b.theta, rtol=1e-9)
    np.testing.assert_allclose(a.nlml, b.nlml, rtol=1e-12)
    for i in range(len(OUTS)):
        np.testing.assert_allclose(am[i], bm[i], rtol=1e-8, atol=1e-10 * np.abs(bm[i]).max())
        np.testing.assert_allclose(asd[i], bsd[i], rtol=1e-8, atol=1e-10 * np.abs(bsd[i]).max())


@pytest.mark.timeout(600)
@pytest.mark.parametrize("i", range(len(OUTS)))
def test_headline_output_matches_cpu_port(runs, CR, i):
    p = OUTS[i]
    ds = runs["ds"]
    fr, means, stds = runs["head"]
    V = np.ascontiguousarray(ds["Y"][:, : p - 1].T)
    Z = np.ascontiguousarray(runs["Zs"][p].T)
    y = np.ascontiguousarray(ds["Y"][:, p - 1])
    theta = fr.theta[i]
    ref, _ = CR.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta)
    assert abs(-fr.nlml[i] - ref) <= 1e-9 * abs(ref), (p, -fr.nlml[i], ref)
    Vs = np.ascontiguousarray(ds["F_star"][:, : p - 1].T)
    rm, rs = CR.get_gpar_scaled_predictions_fixed(V, Z, ds["t"], y, ds["t_star"], Vs, theta,
                                                  qu_kuu_noise=True)
    np.testing.assert_allclose(means[i], rm, rtol=1e-7, atol=1e-8 * np.abs(rm).max())
    np.testing.assert_allclose(stds[i], rs, rtol=1e-7, atol=1e-8 * np.abs(rs).max())


NN_OUTS = [9, 33]                   # D = 8, 32


@pytest.fixture(scope="module")
def runs_nn():
    import torch
    dev = torch.device("cuda", 0)
    ds = D.gpar_dataset(N, max(NN_OUTS), seed=0, observation_noise=0.8)   # N* = N, interleaved
    assert len(ds["t_star"]) == N
    Y_d = torch.from_numpy(ds["Y"]).to(dev)
    t_d = torch.from_numpy(ds["t"]).to(dev)
    ts_d = torch.from_numpy(ds["t_star"]).to(dev)
    Fs_d = torch.from_numpy(ds["F_star"]).to(dev)
    probs, keep, Zs = [], [], {}
    for p in NN_OUTS:
        Zs[p] = D.pseudo_inputs(ds["Y"][:, : p - 1], M, seed=p)
        pr, k = G.make_problem(Y_d[:, : p - 1], torch.from_numpy(Zs[p]).to(dev), t_d,
                               Y_d[:, p - 1].contiguous(), "matern52", "matern52", qu_kuu_noise=True)
        probs.append(pr)
        keep.append(k)
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(NN_OUTS), 1))
    ctx = G.context(0)
    ctx.set_cu_split(-1)
    ctx.set_dist_cache(-1)
    fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, [Fs_d[:, : p - 1] for p in NN_OUTS],
                                          max_evals=EV, g_tol=-1.0)
    return dict(ds=ds, Zs=Zs, fr=fr, means=[m.cpu().numpy() for m in means],
                stds=[s.cpu().numpy() for s in stds])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("i", range(len(NN_OUTS)))
def test_headline_n_star_equals_n_matches_cpu_port(runs_nn, CR, i):
    p = NN_OUTS[i]
    ds, fr = runs_nn["ds"], runs_nn["fr"]
    V = np.ascontiguousarray(ds["Y"][:, : p - 1].T)
    Z = np.ascontiguousarray(runs_nn["Zs"][p].T)
    y = np.ascontiguousarray(ds["Y"][:, p - 1])
    theta = fr.theta[i]
    ref, _ = CR.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta)
    assert abs(-fr.nlml[i] - ref) <= 1e-9 * abs(ref), (p, -fr.nlml[i], ref)
    Vs = np.ascontiguousarray(ds["F_star"][:, : p - 1].T)
    rm, rs = CR.get_gpar_scaled_predictions_fixed(V, Z, ds["t"], y, ds["t_star"], Vs, theta,
                                                  qu_kuu_noise=True)
    np.testing.assert_allclose(runs_nn["means"][i], rm, rtol=1e-7, atol=1e-8 * np.abs(rm).max())
    np.testing.assert_allclose(runs_nn["stds"][i], rs, rtol=1e-7, atol=1e-8 * np.abs(rs).max())
