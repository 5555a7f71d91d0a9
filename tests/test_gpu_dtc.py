"""GPU parity of the DTC objective, (dtc, A), q(u) and LGSSM logpdf against the oracle.

The oracle (oracle/gpar_oracle.py) restates dtc.jl:83-128, gpar_scaled_inference.jl:141-196 and
temporal_gp_inference.jl:286-296; tolerances are fp64: lml rel <= 1e-10."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu

G = pytest.importorskip("gparatscale")


def _case(n, P, M, seed, gaps=0, noise=0.3):
    t, Y = O.synthetic_gpar(n, P, seed=seed, noise=noise, gaps=gaps, gap_len=max(1, n // 20))
    V = Y[:, : P - 1].T
    y = Y[:, P - 1]
    Z = O.pick_pseudo_inputs(V, M, seed + 7)
    return t, V, Z, y


CASES = [
    # n, P, M, seed, kernels, theta
    (300, 3, 40, 1, ("matern52", "matern52"), (1.3, 0.9, 0.7, 1.1, 0.2)),
    (700, 2, 130, 2, ("matern52", "matern52"), (0.4, 1.7, 1.5, 0.6, 0.35)),
    (1000, 6, 64, 3, ("eq", "matern32"), (2.0, 1.1, 2.5, 0.8, 0.15)),
    (513, 4, 200, 4, ("matern32", "matern12"), (0.9, 0.5, 1.2, 1.4, 0.5)),
    (257, 9, 17, 5, ("matern12", "matern52"), (3.0, 2.0, 4.0, 0.9, 0.05)),
]


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}_P{c[1]}_M{c[2]}_{c[4][0]}_{c[4][1]}" for c in CASES])
def test_dtc_objective_matches_oracle(case):
    n, P, M, seed, (ok, tk), theta = case
    t, V, Z, y = _case(n, P, M, seed)
    ref, parts = O.compute_gpar_dtc_objective(V, Z, t, y, theta, ok, tk, return_parts=True)
    got = G.compute_gpar_dtc_objective(V, Z, t, y, theta, ok, tk)
    assert abs(got - ref) <= 1e-10 * max(1.0, abs(ref)), (got, ref)


def test_dtc_with_gaps_and_A():
    t, V, Z, y = _case(900, 3, 50, 11, gaps=3)
    theta = (0.8, 1.2, 0.9, 1.0, 0.25)
    ref, A_ref = O.compute_gpar_dtc_objective(V, Z, t, y, theta)
    got, A = G.compute_gpar_dtc_objective(V, Z, t, y, theta, return_A=True)
    assert abs(got - ref) <= 1e-10 * max(1.0, abs(ref))
    assert A.shape == A_ref.shape
    np.testing.assert_allclose(A, A_ref, rtol=1e-9, atol=1e-11 * np.abs(A_ref).max())


def test_dtc_batch_matches_individual():
    probs, thetas, refs = [], [], []
    keep = []
    t, Y = O.synthetic_gpar(600, 5, seed=21, noise=0.3)
    for p in range(2, 6):
        V = Y[:, : p - 1].T
        Z = O.pick_pseudo_inputs(V, 48, p)
        th = (1.0 + 0.1 * p, 0.9, 1.1, 0.8 + 0.05 * p, 0.2)
        pr, k = G.make_problem(V, Z, t, Y[:, p - 1])
        probs.append(pr); keep.append(k); thetas.append(th)
        refs.append(O.compute_gpar_dtc_objective(V, Z, t, Y[:, p - 1], th)[0])
    got = G.dtc_objective_batch(probs, thetas)
    np.testing.assert_allclose(got, refs, rtol=1e-10)


def test_q_u_matches_oracle():
    t, V, Z, y = _case(500, 3, 30, 8)
    theta = (1.1, 0.8, 1.3, 1.2, 0.3)
    me_r, cov_r, U_r, _ = O.compute_q_u(V, Z, t, y, theta)
    me, cov, U = G.compute_q_u(V, Z, t, y, theta)
    np.testing.assert_allclose(U, U_r, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(me, me_r, rtol=1e-7, atol=1e-9 * np.abs(me_r).max())
    np.testing.assert_allclose(cov, cov_r, rtol=1e-7, atol=1e-9 * np.abs(cov_r).max())


@pytest.mark.parametrize("kernel", ["matern12", "matern32", "matern52"])
def test_lgssm_logpdf_matches_oracle(kernel):
    t, Y = O.synthetic_gpar(1500, 3, seed=3, noise=0.4, gaps=2, gap_len=100)
    th = [(0.5, 1.3, 0.2), (2.0, 0.7, 0.6), (10.0, 2.0, 0.05)]
    got = G.lgssm_logpdf_batch(t, Y.T, th, kernel)
    for c in range(3):
        ref = O.lgssm_logpdf(O.create_lgssm(t, *th[c], kind=kernel), Y[:, c])
        assert abs(got[c] - ref) <= 1e-10 * max(1.0, abs(ref)), (c, got[c], ref)


def test_not_pd_raises_posdef():
    # duplicated pseudo-inputs with no jitter: q(u)'s cholesky(Cuu) must fail like the reference
    t, V, Z, y = _case(300, 2, 20, 9)
    Z = np.concatenate([Z, Z[:, :1]], axis=1)
    with pytest.raises(G.PosDefException):
        G.compute_q_u(V, Z, t, y, (1.0, 1.0, 1.0, 1.0, 0.2))
