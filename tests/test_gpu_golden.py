"""GPU vs the committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py
from the oracle after it passed tests/test_oracle.py).  Everything runs through the C-ABI
(libgparhip.so) on gfx950; the oracle is not called here.

Tolerances (fp64): lml rel <= 1e-10; A, smoother marginals rtol 1e-9; q(u) and
predictions rtol 1e-7 (they go through inv(D) / Cuu^-1 with cond ~1e6-1e8); NM-fitted values
rtol 1e-6 (a 1e-12 objective difference can move a simplex vertex by that much)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DTC = ["dtc_m52_m52", "dtc_eq_m32_gaps", "dtc_m32_m12", "dtc_m12_m52"]


def _load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("name", DTC)
def test_dtc_golden(name):
    g = _load(name)
    ok, tk = str(g["out_kernel"]), str(g["time_kernel"])
    got, A = G.compute_gpar_dtc_objective(g["V"], g["Z"], g["t"], g["y"], g["theta"], ok, tk,
                                          return_A=True)
    ref = float(g["dtc"])
    assert abs(got - ref) <= 1e-10 * abs(ref), (got, ref)
    np.testing.assert_allclose(A[:, :128], g["A_head"], rtol=1e-9, atol=1e-11 * np.abs(g["A_head"]).max())
    np.testing.assert_allclose(np.sum(A * A, axis=0), g["A_colsq"], rtol=1e-9)


def test_q_u_and_predict_golden():
    g = _load("dtc_m52_m52")
    me, cov, U = G.compute_q_u(g["V"], g["Z"], g["t"], g["y"], g["theta"])
    np.testing.assert_allclose(U, g["U_u"], rtol=1e-9, atol=1e-10 * np.abs(g["U_u"]).max())
    np.testing.assert_allclose(me, g["m_e"], rtol=1e-7, atol=1e-9 * np.abs(g["m_e"]).max())
    np.testing.assert_allclose(cov, g["cov_e"], rtol=1e-7, atol=1e-9 * np.abs(g["cov_e"]).max())
    mean, std = G.predict_scaled(g["V"], g["Z"], g["t"], g["y"], g["theta"], g["t_star"], g["V_star"])
    np.testing.assert_allclose(mean, g["pred_mean"], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(std, g["pred_std"], rtol=1e-7, atol=1e-9)


def test_temporal_golden():
    g = _load("temporal")
    for kind in ("matern12", "matern32", "matern52"):
        th = g[f"theta_{kind}"]
        lml = G.logpdf(G.create_lgssm(g["t"], *th, kernel_structure=kind), g["y"])
        assert abs(lml - float(g[f"logpdf_{kind}"])) <= 1e-10 * abs(lml)
        # smoothing on the merged grid, test points with noise 1e10 (temporal_gp_inference.jl:93-109)
        t, ts = g["t"], g["t_star"]
        tc = np.concatenate([t, ts])
        perm = np.argsort(tc, kind="stable")
        yc = np.concatenate([g["y"], np.zeros(len(ts))])[perm]
        rc = np.concatenate([np.full(len(t), th[2] ** 2), np.full(len(ts), 1e10)])[perm]
        m, v = G.lgssm_smooth_batch(tc[perm], yc[None, :], th[None, :], kind, noise=rc)
        inv = np.argsort(perm, kind="stable")[len(t):]
        np.testing.assert_allclose(m[0][inv], g[f"smooth_mean_{kind}"], rtol=1e-9, atol=1e-11)
        np.testing.assert_allclose(v[0][inv], g[f"smooth_var_{kind}"], rtol=1e-9, atol=1e-11)
    th, mean, var = G.get_sde_predictions(g["t"], g["y"], g["t_star"], "matern52", 0.0, 0.0, -2.0,
                                          max_evals=60)
    np.testing.assert_allclose(th, g["sde_fit_theta"], rtol=1e-6)
    np.testing.assert_allclose(mean, g["sde_fit_mean"], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(var, g["sde_fit_var"], rtol=1e-6, atol=1e-10)


def test_nm_fit_golden():
    g = _load("nm_fit")
    th = G.get_optim_scaled_gpar_params(g["V"], g["Z"], g["t"], g["y"], "matern52", "matern52",
                                        *g["x0"], max_evals=int(g["max_evals"]))
    np.testing.assert_allclose(th, G.unpack_gpar(g["x_min"]), rtol=1e-6)
