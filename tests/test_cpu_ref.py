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


@pytest.mark.parametrize("kind", ["matern12", "matern32", "matern52"])
def test_lgssm_logpdf_and_smooth_match_oracle(CR, data, kind):
    """The temporal-only chain (bench.py --config ssm's CPU baseline): logpdf and the RTS
    smoother's mean and marginal variance of the C port against the numpy oracle, with and
    without a per-step noise vector (get_sde_predictions' R = sigma^2 train / 1e10 test)."""
    t, V, y, Z = data
    l, pv, ns = 0.9, 1.4, 0.3
    lg = O.create_lgssm(t, l, pv, ns, kind)
    assert abs(CR.lgssm_logpdf(kind, t, y, l, pv * pv, ns * ns) - O.lgssm_logpdf(lg, y)) <= \
        1e-10 * abs(O.lgssm_logpdf(lg, y))
    ms, Ps = O.rts_smooth(lg, y)
    cm, cv = CR.lgssm_smooth(kind, t, y, l, pv * pv, ns * ns)
    np.testing.assert_allclose(cm, ms[:, 0], rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(cv, Ps[:, 0, 0], rtol=1e-9, atol=1e-12)
    R = np.where(np.arange(len(t)) % 4 == 0, 1e10, ns * ns)
    lgr = O.create_lgssm(t, l, pv, ns, kind, noise_vector=R)
    ms, Ps = O.rts_smooth(lgr, y)
    cm, cv = CR.lgssm_smooth(kind, t, y, l, pv * pv, ns * ns, rvec=R)
    np.testing.assert_allclose(cm, ms[:, 0], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(cv, Ps[:, 0, 0], rtol=1e-8, atol=1e-12)


def test_ssm_cpu_baseline_check_file(CR, tmp_path):
    """bench.py --config ssm's CPU baseline at a small N: the job figure and the self-check file
    (every chain's logpdf, chain 1's prediction at t*) agree with the numpy oracle."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))
    sys.path.insert(0, ROOT)
    import bench
    from gparatscale import data as D
    n, P = 3000, 3
    chk = tmp_path / "ssm.npz"
    r = bench.ssm_cpu_baseline(n, P, 5, "matern32", check_path=str(chk))
    assert r["value"] > 0 and r["kind"] == "port" and r["cores"] >= 1
    assert abs(r["job_seconds"] - (5 * r["round_seconds"] + r["smooth_seconds"])) < 1e-9
    ref = np.load(chk)
    ds = D.gpar_dataset(n, P, seed=0, observation_noise=0.8)
    l, pv, ns = bench.SSM_CHECK_THETA
    for p in range(P):
        lo = O.lgssm_logpdf(O.create_lgssm(ds["t"], l, pv, ns, "matern32"), ds["Y"][:, p])
        assert abs(ref["lml"][p] - lo) <= 1e-10 * abs(lo)
    m, v = O.sde_predict_fixed(ds["t"], ds["Y"][:, 0], ds["t_star"], (l, pv, ns), "matern32")
    np.testing.assert_allclose(ref["mean"], m, rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(ref["var"], v, rtol=1e-8, atol=1e-12)
