"""Inputs wider than 64 dimensions (BASELINE config 5: P = 256 outputs, so D = p - 1 up to 255).

The reference evaluates Kfu = pairwise(k_o, V, Z) for any D (dtc.jl:104, gpar_scaled_inference.jl:
89,156); the fused whitening keeps a pseudo-input in registers up to D = 64, wider inputs go through
the separate distance pass of k_dist.hip (fp64-MFMA Gram form for the smooth kernels, direct
differences for Matern-1/2) and the whitening from precomputed distances.  Checked against the
numpy oracle (direct differences) at small N: lml rel <= 1e-10, A rtol 1e-9,
q(u) / predictions rtol 1e-7; and at full size (N = 1e6, M = 1024, D = 255) against the C port,
lml rel <= 1e-9.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu

G = pytest.importorskip("gparatscale")
from gparatscale import data as Dd  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case(n, D, M, seed, noise=0.3):
    t, Y = O.synthetic_gpar(n, D + 1, seed=seed, noise=noise)
    V = np.ascontiguousarray(Y[:, :D].T)
    y = Y[:, D].copy()
    Z = O.pick_pseudo_inputs(V, M, seed + 7)
    return t, V, Z, y


WIDE = [
    # n, D, M, seed, (out kernel, time kernel), theta (l_o large enough that Kfu is not ~0)
    (600, 65, 40, 1, ("matern52", "matern52"), (1.3, 0.9, 6.0, 1.1, 0.2)),
    (700, 127, 300, 2, ("matern32", "matern12"), (0.8, 1.2, 8.0, 0.9, 0.3)),
    (500, 255, 130, 3, ("eq", "matern52"), (1.1, 1.0, 12.0, 1.2, 0.25)),
    (400, 255, 64, 4, ("matern12", "matern32"), (2.0, 0.7, 9.0, 1.0, 0.35)),
    (513, 100, 257, 5, ("matern52", "matern32"), (0.9, 1.1, 7.0, 0.8, 0.2)),
]


@pytest.mark.parametrize("case", WIDE, ids=[f"D{c[1]}_M{c[2]}_{c[4][0]}_{c[4][1]}" for c in WIDE])
def test_wide_objective_matches_oracle(case):
    n, D, M, seed, (ok, tk), theta = case
    t, V, Z, y = _case(n, D, M, seed)
    ref, _ = O.compute_gpar_dtc_objective(V, Z, t, y, theta, ok, tk)
    got = G.compute_gpar_dtc_objective(V, Z, t, y, theta, ok, tk)
    assert abs(got - ref) <= 1e-10 * max(1.0, abs(ref)), (got, ref)


def test_wide_objective_A():
    t, V, Z, y = _case(450, 90, 50, 11)
    theta = (0.8, 1.2, 6.0, 1.0, 0.25)
    ref, A_ref = O.compute_gpar_dtc_objective(V, Z, t, y, theta)
    got, A = G.compute_gpar_dtc_objective(V, Z, t, y, theta, return_A=True)
    assert abs(got - ref) <= 1e-10 * abs(ref)
    np.testing.assert_allclose(A, A_ref, rtol=1e-9, atol=1e-11 * np.abs(A_ref).max())


def test_mixed_width_batch():
    """One batched call whose outputs straddle the fused / distance-pass boundary (D = 8, 64, 65,
    200): each against the oracle."""
    t, Y = O.synthetic_gpar(600, 201, seed=21, noise=0.3)
    probs, keep, thetas, refs = [], [], [], []
    for i, D in enumerate([8, 64, 65, 200]):
        V = np.ascontiguousarray(Y[:, :D].T)
        Z = O.pick_pseudo_inputs(V, 48 + 16 * i, D)
        th = (1.0 + 0.1 * i, 0.9, 2.0 + 0.04 * D, 0.8 + 0.05 * i, 0.2)
        pr, k = G.make_problem(V, Z, t, Y[:, D])
        probs.append(pr)
        keep.append(k)
        thetas.append(th)
        refs.append(O.compute_gpar_dtc_objective(V, Z, t, Y[:, D], th)[0])
    got = G.dtc_objective_batch(probs, thetas)
    np.testing.assert_allclose(got, refs, rtol=1e-10)


def test_wide_q_u_and_prediction():
    t, V, Z, y = _case(500, 96, 40, 8)
    theta = (1.1, 0.8, 6.5, 1.2, 0.3)
    me_r, cov_r, U_r, _ = O.compute_q_u(V, Z, t, y, theta)
    me, cov, U = G.compute_q_u(V, Z, t, y, theta)
    np.testing.assert_allclose(U, U_r, rtol=1e-9, atol=1e-10 * np.abs(U_r).max())
    np.testing.assert_allclose(me, me_r, rtol=1e-7, atol=1e-9 * np.abs(me_r).max())
    np.testing.assert_allclose(cov, cov_r, rtol=1e-7, atol=1e-9 * np.abs(cov_r).max())
    ts, Vs = t[::7] + 0.013, V[:, ::7] + 0.01
    mean, std = G.predict_scaled(V, Z, t, y, theta, ts, Vs)
    rm, rs = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, theta)
    np.testing.assert_allclose(mean, rm, rtol=1e-7, atol=1e-9 * np.abs(rm).max())
    np.testing.assert_allclose(std, rs, rtol=1e-7, atol=1e-9 * np.abs(rs).max())


def test_wide_device_inputs_strided():
    """HBM-resident inputs with V a column slice of the N x P output matrix (ldv = P), as the
    bench passes them: equal to the host path (same kernels, same order -> bit-identical)."""
    torch = pytest.importorskip("torch")
    t, Y = O.synthetic_gpar(700, 151, seed=31, noise=0.3)
    D = 150
    V = np.ascontiguousarray(Y[:, :D].T)
    Z = O.pick_pseudo_inputs(V, 70, 3)
    theta = (1.0, 1.0, 7.0, 1.0, 0.2)
    host = G.compute_gpar_dtc_objective(V, Z, t, Y[:, D], theta)
    dev = torch.device("cuda", 0)
    Yd = torch.from_numpy(Y).to(dev)
    Zd = torch.from_numpy(np.ascontiguousarray(Z.T)).to(dev)
    td = torch.from_numpy(t).to(dev)
    got = G.compute_gpar_dtc_objective(Yd[:, :D], Zd, td, Yd[:, D], theta)
    assert got == host, (got, host)


def test_wide_fit_predict_batch():
    """gpar_fit_predict over outputs with D = 70 and 130 (fixed x0, 25 evaluations) against the
    oracle's NM + prediction per output (NM trajectory parity: theta rtol 1e-6)."""
    t, Y = O.synthetic_gpar(400, 131, seed=41, noise=0.3)
    ts = t[::5] + 0.011
    probs, keep, V_stars, refs = [], [], [], []
    x0 = np.array([0.0, 0.0, 1.8, 0.0, -1.5])
    for D in (70, 130):
        V = np.ascontiguousarray(Y[:, :D].T)
        Z = O.pick_pseudo_inputs(V, 32, D)
        pr, k = G.make_problem(V, Z, t, Y[:, D], qu_kuu_noise=True)
        probs.append(pr)
        keep.append(k)
        Vs = V[:, ::5] + 0.01
        V_stars.append(Vs)
        th, _ = O.get_optim_scaled_gpar_params(V, Z, t, Y[:, D], log_theta0=x0, max_evals=25,
                                               g_tol=-1.0, return_nm=True)
        rm, rs = O.get_gpar_scaled_predictions_fixed(V, Z, t, Y[:, D], ts, Vs, th,
                                                     qu_kuu_noise=True)
        refs.append((th, rm, rs))
    fr, means, stds = G.fit_predict_batch(probs, np.tile(x0, (2, 1)), ts, V_stars, max_evals=25,
                                          g_tol=-1.0)
    for i, (th, rm, rs) in enumerate(refs):
        np.testing.assert_allclose(fr.theta[i], th, rtol=1e-6)
        np.testing.assert_allclose(means[i], rm, rtol=1e-6, atol=1e-8 * np.abs(rm).max())
        np.testing.assert_allclose(stds[i], rs, rtol=1e-6, atol=1e-8 * np.abs(rs).max())


@pytest.fixture(scope="module")
def CR():
    if not os.path.exists(os.path.join(ROOT, "oracle", "libgpar_cpu.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    from oracle import cpu_ref
    cpu_ref.load()
    return cpu_ref


def test_config5_width_full_size(CR):
    """BASELINE config 5's widest output at N = 1e6 (of its 1e7), M = 1024, D = 255, against the
    C port: lml rel <= 1e-9 (1e6-term reductions in a different order, Gram-form distances)."""
    n, M, D = 1_000_000, 1024, 255
    ds = Dd.gpar_dataset(n, D + 1, seed=5, observation_noise=0.8)
    V = np.ascontiguousarray(ds["Y"][:, :D].T)
    y = ds["Y"][:, D].copy()
    Z = np.ascontiguousarray(Dd.pseudo_inputs(ds["Y"][:, :D], M, seed=D + 1).T)
    theta = (1.0, 1.0, 12.0, 1.0, 0.3)
    got = G.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta)
    ref, _ = CR.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta)
    assert abs(got - ref) <= 1e-9 * abs(ref), (got, ref)
