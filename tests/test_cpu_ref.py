"""The C/OpenMP CPU restatement (oracle/cpu_ref.{c,py}, bench.py's cpu_baseline) agrees with the
numpy oracle (oracle/gpar_oracle.py) -- both are test infrastructure; CPU only."""
import os
import subprocess

import numpy as np
import pytest

from oracle import gpar_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def CR():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    from oracle import cpu_ref
    cpu_ref.load()
    return cpu_ref


@pytest.fixture(scope="module")
def data():
    t, Y = O.synthetic_gpar(1500, 4, seed=3, noise=0.3)
    V, y = Y[:, :3].T.copy(), Y[:, 3].copy()
    Z = O.pick_pseudo_inputs(V, 40, 5)
    return t, V, y, Z


@pytest.mark.parametrize("ok", ["matern52", "matern32", "matern12", "eq"])
@pytest.mark.parametrize("tk", ["matern52", "matern32", "matern12"])
def test_objective_matches_oracle(CR, data, ok, tk):
    t, V, y, Z = data
    th = (1.3, 0.9, 0.7, 1.1, 0.2)
    a, Aa = O.compute_gpar_dtc_objective(V, Z, t, y, th, ok, tk)
    b, Ab = CR.compute_gpar_dtc_objective(V, Z, t, y, th, ok, tk)
    assert abs(a - b) <= 1e-10 * abs(a)
    np.testing.assert_allclose(Ab, Aa, rtol=1e-8, atol=1e-10)


def test_decorrelate_and_gains(CR, data):
    t, V, y, Z = data
    lg = O.build_lgssm(t, "matern52", 0.8, 1.7, 0.05)
    a_ref, logS, _, _ = O.kalman_filter(lg, y)
    rec, logs, _, _ = CR.gains("matern52", t, 0.8, 1.7, 0.05)
    assert abs(logs - logS.sum()) <= 1e-10 * abs(logS.sum())
    np.testing.assert_allclose(CR.decorrelate("matern52", rec, y), a_ref, rtol=1e-10, atol=1e-12)


def test_prediction_matches_oracle(CR, data):
    t, V, y, Z = data
    th = (1.3, 0.9, 0.7, 1.1, 0.2)
    ts, Vs = t[::7] + 0.013, V[:, ::7] + 0.01
    rm, rs = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, th)
    cm, cs = CR.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, th)
    np.testing.assert_allclose(cm, rm, rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(cs, rs, rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("ok", ["matern52", "eq"])
def test_qu_kuu_noise_branch_matches_oracle(CR, data, ok):
    """The branch the north-star bench runs (gpar_problem.qu_kuu_noise = 1: q(u) with Cuu +
    sigma^2 I): the C port and the numpy oracle agree on q(u) and on the prediction."""
    t, V, y, Z = data
    th = (1.3, 0.9, 0.7, 1.1, 0.2)
    me_r, cov_r, U_r, _ = O.compute_q_u(V, Z, t, y, th, ok, qu_kuu_noise=True)
    me_c, cov_c, U_c = CR.compute_q_u(V, Z, t, y, th, ok, kuu_noise=True)
    np.testing.assert_allclose(U_c, U_r, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(me_c, me_r, rtol=1e-9, atol=1e-11 * np.abs(me_r).max())
    np.testing.assert_allclose(cov_c, cov_r, rtol=1e-9, atol=1e-11 * np.abs(cov_r).max())
    # the jitter is not a no-op: the noise-free branch differs
    me_0, _, _, _ = O.compute_q_u(V, Z, t, y, th, ok)
    assert np.abs(me_0 - me_r).max() > 1e-6 * np.abs(me_r).max()
    ts, Vs = t[::7] + 0.013, V[:, ::7] + 0.01
    rm, rs = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, th, ok, qu_kuu_noise=True)
    cm, cs = CR.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, th, ok, qu_kuu_noise=True)
    np.testing.assert_allclose(cm, rm, rtol=1e-9, atol=1e-11 * np.abs(rm).max())
    np.testing.assert_allclose(cs, rs, rtol=1e-9, atol=1e-11 * np.abs(rs).max())


def test_rejects_unsorted_times(CR):
    with pytest.raises(ValueError):
        CR.gains("matern52", np.array([0.0, 2.0, 1.0]), 1.0, 1.0, 0.1)
