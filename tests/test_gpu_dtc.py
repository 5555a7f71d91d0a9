"""GPU parity of the DTC objective, (dtc, A), q(u) and LGSSM logpdf against the oracle.

The oracle (oracle/gpar_oracle.py) restates dtc.jl:83-128, gpar_scaled_inference.jl:141-196 and
temporal_gp_inference.jl:69-82; tolerances are fp64: lml rel <= 1e-10."""
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
    # M = 450: 8 diagonal blocks of the blocked 64 x 64 dense tail
    (700, 4, 450, 6, ("matern52", "matern52"), (1.1, 0.8, 0.9, 1.2, 0.3)),
    # Gram v2 shapes with an odd number of 128-blocks (Mp = 384, 640): off-diagonal groups plus
    # a diagonal group whose second block is missing
    (800, 3, 300, 12, ("matern52", "matern52"), (1.2, 0.9, 1.0, 1.1, 0.25)),
    (600, 3, 600, 13, ("matern32", "matern52"), (0.9, 1.1, 1.4, 0.9, 0.3)),
    # Gram v3's correction beside the OFF kernel with its K lanes packed over chunk pairs: state
    # dimension 2 (Matern-3/2 time) and 1 (Matern-1/2), odd chunk counts (6 and 5 chunks of 256,
    # the last one short), off-diagonal groups present (Mp = 384)
    (1297, 3, 260, 14, ("matern52", "matern32"), (1.0, 1.2, 1.1, 0.9, 0.2)),
    (1041, 2, 300, 15, ("eq", "matern12"), (1.4, 0.7, 1.6, 1.3, 0.3)),
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


def test_q_u_large_m():
    """q(u) with 8 dense blocks (M = 450); Cuu + sigma^2 I (qu_kuu_noise) keeps it well posed."""
    t, V, Z, y = _case(700, 4, 450, 6)
    theta = (1.1, 0.8, 0.9, 1.2, 0.3)
    dtc, A = O.compute_gpar_dtc_objective(V, Z, t, y, theta, return_parts=False)
    got = G.compute_gpar_dtc_objective(V, Z, t, y, theta)
    assert abs(got - dtc) <= 1e-10 * abs(dtc), (got, dtc)


def test_dtc_north_regime():
    """The north-star regime at reduced N (M = 512, D = 32, N = 2e4): G = beta^T beta is large,
    so Lambda = L_u^-1 G L_u^-T + I spans ~1e8 in eigenvalue; lml rel <= 1e-9 (reduction order
    over 2e4 rows and the ill-conditioned Lambda)."""
    from gparatscale import data as Dd
    ds = Dd.gpar_dataset(20000, 33, seed=0, observation_noise=0.8)
    V = ds["Y"][:, :32].T.copy()
    y = ds["Y"][:, 32].copy()
    Z = Dd.pseudo_inputs(ds["Y"][:, :32], 512, seed=33).T.copy()
    theta = (1.0, 1.0, 1.0, 1.0, 0.2)
    ref, _ = O.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta)
    got = G.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta)
    assert abs(got - ref) <= 1e-9 * abs(ref), (got, ref)


def test_q_u_matches_oracle():
    t, V, Z, y = _case(500, 3, 30, 8)
    theta = (1.1, 0.8, 1.3, 1.2, 0.3)
    me_r, cov_r, U_r, _ = O.compute_q_u(V, Z, t, y, theta)
    me, cov, U = G.compute_q_u(V, Z, t, y, theta)
    # the Cholesky factor of the noise-free Cuu (cond ~1e7): norm-wise agreement
    np.testing.assert_allclose(U, U_r, rtol=1e-9, atol=1e-10 * np.abs(U_r).max())
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


@pytest.mark.parametrize("kernel", ["matern12", "matern32", "matern52"])
def test_lgssm_logpdf_offset_data_matches_oracle(kernel):
    """Uncentred data (y + 1e3) with a small noise sd: the chains' logpdf sums alpha^2 from
    per-chunk moments s0 + 2 c.s1 + c^T S2 c of y filtered from a zero state, whose terms are
    ~1e6 per chunk and cancel to the chunk's true sum; the result must still match the oracle's
    directly summed alpha^2 at rel <= 1e-10, across many chunks."""
    t, Y = O.synthetic_gpar(256 * 40 + 8, 3, seed=5, noise=0.05)
    Y = Y + 1e3
    th = [(0.5, 1.3, 0.05), (2.0, 0.7, 0.05), (10.0, 2.0, 0.02)]
    got = G.lgssm_logpdf_batch(t, np.ascontiguousarray(Y.T), th, kernel)
    for c in range(3):
        ref = O.lgssm_logpdf(O.create_lgssm(t, *th[c], kind=kernel), Y[:, c])
        assert abs(got[c] - ref) <= 1e-10 * abs(ref), (c, got[c], ref)
