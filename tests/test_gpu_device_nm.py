"""The chains fit with its Nelder-Mead machines on the device (schedule knob "device_nm", the
default; nm_dev.hpp, stepped by chain_carry_lml in k_lgssm.hip) against the same fit stepped on
the host (device_nm 0): the same rounds, the same values, the same steps.  The one difference allowed is the device's exp() in the
chain parameters of rounds after the first (the host loop uses the C library's), which could move
a value in its last bit -- the comparisons are at rtol 1e-12 on theta and the outputs.  Cases: the
evaluation budget (every machine ends on it), g_tol convergence with no budget (the host reads the
running count a batch behind, so the last batches are evaluated and discarded), budgets of 1 and 2
(no round, one round), and the oracle's own fit."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")


def _fit(t, Y, ts, kind, x0, device_nm, **kw):
    ctx = G.context(0)
    ctx.set_schedule("device_nm", device_nm)
    try:
        return G.get_sde_predictions(t, Y, ts, kind, *x0, **kw)
    finally:
        ctx.set_schedule("device_nm", 1)


@pytest.fixture(scope="module")
def chains():
    t, Y = O.synthetic_gpar(3000, 6, seed=11, noise=0.3, gaps=2, gap_len=60)
    ts = np.sort(np.random.default_rng(5).uniform(t[0] - 1, t[-1] + 1, 150))
    return t, np.ascontiguousarray(Y.T), ts


@pytest.mark.parametrize("kind,kw", [
    ("matern32", dict(max_evals=40, g_tol=-1.0)),
    ("matern52", dict(max_evals=0, g_tol=1e-4)),
    ("matern12", dict(max_evals=25, g_tol=1e-8)),
    ("matern32", dict(max_evals=1, g_tol=-1.0)),
    ("matern32", dict(max_evals=2, g_tol=-1.0)),
])
def test_device_nm_equals_host_nm(chains, kind, kw):
    t, Y, ts = chains
    x0 = (-0.5, 0.1, -1.5)
    th_d, m_d, v_d = _fit(t, Y, ts, kind, x0, 1, **kw)
    th_h, m_h, v_h = _fit(t, Y, ts, kind, x0, 0, **kw)
    np.testing.assert_allclose(th_d, th_h, rtol=1e-12)
    np.testing.assert_allclose(m_d, m_h, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(v_d, v_h, rtol=1e-12, atol=1e-16)


def test_device_nm_fit_matches_oracle():
    t, Y = O.synthetic_gpar(600, 2, seed=6, noise=0.4, gaps=2, gap_len=40)
    ts = np.sort(np.random.default_rng(2).uniform(-1, t[-1] + 1, 90))
    x0 = (-1.0, 0.2, -1.5)
    th_ref, m_ref, v_ref = O.get_sde_predictions(t, Y[:, 0], ts, "matern52", x0, max_evals=30)
    assert G.context(0).schedule("device_nm") == 1
    th, m, v = G.get_sde_predictions(t, Y[:, 0], ts, "matern52", *x0, max_evals=30)
    np.testing.assert_allclose(th, th_ref, rtol=1e-6)
    np.testing.assert_allclose(m, m_ref, rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(v, v_ref, rtol=1e-6, atol=1e-10)
