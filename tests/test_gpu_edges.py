"""GPU edge cases against the oracle: chunk / K-step / panel boundaries, tiny and odd sizes,
repeated time stamps, mixed-size batches, single-point and out-of-range predictions, many
temporal chains (config 3's shape), argument errors.  fp64 tolerances as in test_gpu_dtc."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")


def _case(n, D, M, seed, gaps=0, noise=0.3):
    t, Y = O.synthetic_gpar(n, D + 1, seed=seed, noise=noise, gaps=gaps, gap_len=max(1, n // 20))
    V = Y[:, :D].T.copy()
    y = Y[:, D].copy()
    Z = O.pick_pseudo_inputs(V, min(M, n), seed + 7) if M <= n else \
        np.random.default_rng(seed).normal(size=(D, M)) + V.mean(axis=1, keepdims=True)
    return t, V, Z, y


SIZES = [  # n, D, M: chunk (256) and K-step (16) boundaries, panel (64/128) boundaries, D buckets
    (1, 1, 1), (5, 2, 3), (17, 1, 16), (255, 3, 64), (256, 3, 65), (257, 4, 127), (513, 2, 128),
    (300, 17, 129), (400, 63, 40), (1000, 1, 200),
]


@pytest.mark.parametrize("n,D,M", SIZES, ids=[f"n{a}_D{b}_M{c}" for a, b, c in SIZES])
def test_dtc_sizes(n, D, M):
    t, V, Z, y = _case(n, D, M, seed=n + D + M)
    theta = (1.2, 0.9, 1.0 + 0.1 * D ** 0.5, 1.1, 0.3)
    ref, _ = O.compute_gpar_dtc_objective(V, Z, t, y, theta)
    got = G.compute_gpar_dtc_objective(V, Z, t, y, theta)
    assert abs(got - ref) <= 1e-10 * max(1.0, abs(ref)), (got, ref)


def test_repeated_time_stamps():
    t, V, Z, y = _case(400, 3, 30, 5)
    t = np.repeat(t[::2], 2)[: len(t)]          # every time twice: steps of length 0
    theta = (0.9, 1.1, 1.3, 0.8, 0.4)
    ref, _ = O.compute_gpar_dtc_objective(V, Z, t, y, theta)
    got = G.compute_gpar_dtc_objective(V, Z, t, y, theta)
    assert abs(got - ref) <= 1e-10 * abs(ref)


def test_unsorted_times_rejected():
    t, V, Z, y = _case(100, 2, 10, 6)
    t = t.copy()
    t[[10, 20]] = t[[20, 10]]
    with pytest.raises(G.DomainError):
        G.compute_gpar_dtc_objective(V, Z, t, y, (1.0, 1.0, 1.0, 1.0, 0.3))


def test_bad_theta_rejected():
    t, V, Z, y = _case(100, 2, 10, 6)
    with pytest.raises(G.DomainError):
        G.compute_gpar_dtc_objective(V, Z, t, y, (1.0, -1.0, 1.0, 1.0, 0.3))


def test_mixed_batch_sizes():
    """One batched call over outputs with different M and D (G padded to the widest)."""
    t, Y = O.synthetic_gpar(700, 5, seed=9, noise=0.3)
    probs, keep, thetas, refs = [], [], [], []
    for p, M in zip(range(2, 6), (20, 150, 64, 300)):
        V = Y[:, : p - 1].T.copy()
        Z = O.pick_pseudo_inputs(V, M, p)
        th = (1.0, 0.9, 1.0 + 0.2 * p, 1.1, 0.25)
        pr, k = G.make_problem(V, Z, t, Y[:, p - 1])
        probs.append(pr); keep.append(k); thetas.append(th)
        refs.append(O.compute_gpar_dtc_objective(V, Z, t, Y[:, p - 1], th)[0])
    got = G.dtc_objective_batch(probs, thetas)
    np.testing.assert_allclose(got, refs, rtol=1e-10)


def test_predict_single_and_out_of_range_points():
    t, V, Z, y = _case(600, 2, 25, 11)
    theta = (1.0, 1.0, 1.5, 1.0, 0.3)
    ts = np.array([t[0] - 1.0, t[-1] + 2.0, t[300]])
    Vs = V[:, [0, -1, 300]] + 0.05
    for k in (1, 3):
        mean, std = G.predict_scaled(V, Z, t, y, theta, ts[:k], Vs[:, :k])
        rm, rs = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts[:k], Vs[:, :k], theta)
        np.testing.assert_allclose(mean, rm, rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(std, rs, rtol=1e-7, atol=1e-9)


def test_many_temporal_chains_matern32():
    """Config 3's shape at small N: 16 Matern-3/2 chains sharing t (temporal_gp_inference.jl)."""
    t, Y = O.synthetic_gpar(3000, 16, seed=12, noise=0.4, gaps=2, gap_len=100)
    th = np.column_stack([np.linspace(0.3, 3.0, 16), np.linspace(0.5, 2.0, 16), np.full(16, 0.3)])
    got = G.lgssm_logpdf_batch(t, Y.T.copy(), th, "matern32")
    ref = [O.lgssm_logpdf(O.create_lgssm(t, *th[i], kind="matern32"), Y[:, i]) for i in range(16)]
    np.testing.assert_allclose(got, ref, rtol=1e-10)


def test_lgssm_single_step():
    t = np.array([0.5])
    y = np.array([0.7])
    got = G.lgssm_logpdf_batch(t, y[None, :], [[1.0, 1.2, 0.3]], "matern52")[0]
    ref = O.lgssm_logpdf(O.create_lgssm(t, 1.0, 1.2, 0.3), y)
    assert abs(got - ref) <= 1e-12 * abs(ref)


@pytest.mark.parametrize("sigma", [0.05, 0.01, 0.002])
def test_dtc_small_noise_ill_conditioned_kuu(sigma):
    """Small noise: cond(Kuu + s2 I) reaches ~3e7 (EQ, M = 200, sigma = 0.002).  The build forms
    Lambda = L_u^-1 (beta^T beta) L_u^-T; the reference forms A = L_u^-1 beta^T, then A A^T
    (dtc.jl:119-120).  The two associations differ by ~cond * eps in exact-data fp64 (numpy with
    triangular solves throughout: 8.6e-8 relative at sigma = 0.002), so the bound scales with
    the conditioning: rel <= max(1e-10, 1e-14 * cond)."""
    t, V, Z, y = _case(800, 3, 200, 21)
    theta = (1.0, 1.0, 1.5, 1.0, sigma)
    ref, parts = O.compute_gpar_dtc_objective(V, Z, t, y, theta, "eq", "matern52", return_parts=True)
    got = G.compute_gpar_dtc_objective(V, Z, t, y, theta, "eq", "matern52")
    tol = max(1e-10, 1e-14 * np.linalg.cond(parts["Kuu"]))
    assert abs(got - ref) <= tol * abs(ref), (got, ref, abs(got - ref) / abs(ref), tol)


def test_device_size_checks():
    """HBM inputs: the C side cannot see buffer lengths, so mismatches must raise before launch."""
    import torch
    dev = torch.device("cuda", 0)
    t, Y = O.synthetic_gpar(300, 3, seed=2, noise=0.3)
    Yd, td = torch.from_numpy(Y).to(dev), torch.from_numpy(t).to(dev)
    Zd = Yd[:20, :2].contiguous()
    with pytest.raises(G.DomainError):
        G.make_problem(Yd[:, :2], Zd, td[:-1], Yd[:, 2].contiguous())
    ts = td[:40] + 0.01
    with pytest.raises(G.DomainError):
        G.predict_scaled(Yd[:, :2], Zd, td, Yd[:, 2].contiguous(), (1.0, 1.0, 1.0, 1.0, 0.2), ts,
                         Yd[:39, :2])
    pr, k = G.make_problem(Yd[:, :2], Zd, td, Yd[:, 2].contiguous())
    with pytest.raises(G.DomainError):
        G.fit_predict_batch([pr], np.zeros((1, 5)), ts, [Yd[:41, :2]], max_evals=3)


def test_fresh_noncontiguous_device_inputs():
    """Inputs written by torch kernels just before the call, passed as strided views (the
    binding's .contiguous() copies run on torch's stream; the library orders itself after it):
    the same objective as from host memory."""
    import torch
    dev = torch.device("cuda", 0)
    t, Y = O.synthetic_gpar(4000, 4, seed=3, noise=0.3)
    V = np.ascontiguousarray(Y[:, :3].T)
    Z = O.pick_pseudo_inputs(V, 40, 1)
    theta = (1.1, 0.9, 1.2, 1.0, 0.25)
    host = G.compute_gpar_dtc_objective(V, Z, t, Y[:, 3], theta)
    for _ in range(3):
        base = torch.from_numpy(np.ascontiguousarray(Y.T)).to(dev) * 2.0   # fresh, 4 x N
        Yt = (base * 0.5).T                                                  # N x 4, strided
        Zt = torch.from_numpy(np.ascontiguousarray(Z)).to(dev).T             # M x 3, strided
        tt = torch.from_numpy(t).to(dev) + 0.0
        got = G.compute_gpar_dtc_objective(Yt[:, :3], Zt, tt, Yt[:, 3], theta)
        assert abs(got - host) <= 1e-12 * abs(host), (got, host)


@pytest.mark.parametrize("kind", ["matern12", "matern32", "matern52"])
def test_gains_fast_path_bit_identical_to_general(kind, monkeypatch):
    """The gains' phase-3 fast path (LDS-DMA staged inputs; its masked last block re-runs stale
    inputs past each chunk's end) against the general kernel (GPAR_GAINS_FAST=0): chain logpdfs
    (the moments form), smoothing with a noise vector, and a DTC objective are bit-identical, at
    chunk counts inside one block and across blocks, with short last chunks, large time gaps
    (negative stale steps) and short length scales."""
    rng = np.random.default_rng(11)
    # 256 * 300 + 8: an even n, so every chain's row of Y (ldy = n) is 16-byte aligned and the
    # multi-block case really takes the fast kernel with data (an odd n misaligns row 1 and the
    # library falls back to the general kernel for both settings)
    for n in (1300, 256 * 300 + 8):
        t = np.cumsum(rng.exponential(0.05, n) + np.where(rng.random(n) < 0.01, 3.0, 0.0))
        Y = np.ascontiguousarray(rng.normal(size=(3, n)))
        th = np.array([[0.05, 1.3, 0.2], [0.5, 0.7, 0.6], [4.0, 2.0, 0.05]])
        noise = np.where(np.arange(n) % 5 == 0, 1e10, -1.0)
        out = {}
        for fast in ("1", "0"):
            monkeypatch.setenv("GPAR_GAINS_FAST", fast)
            f0 = G.debug_counter("gains_fast")
            lml = np.asarray(G.lgssm_logpdf_batch(t, Y, th, kind))
            m, v = G.lgssm_smooth_batch(t, Y, th, kind, noise=noise)
            out[fast] = (lml, np.asarray(m), np.asarray(v))
            took = G.debug_counter("gains_fast") - f0
            assert (took >= 1) if fast == "1" else (took == 0), (n, fast, took)
        for a, b in zip(out["1"], out["0"]):
            assert np.all(np.isfinite(a))
            assert np.array_equal(a, b)
    # DTC objectives (the shared gains with data, HAS_Y): inside one block and across blocks
    for n in (1300, 256 * 300 + 8):
        t, V, Z, y = _case(n, 3, 40, 3)
        vals = []
        for fast in ("1", "0"):
            monkeypatch.setenv("GPAR_GAINS_FAST", fast)
            f0 = G.debug_counter("gains_fast")
            vals.append(G.compute_gpar_dtc_objective(V, Z, t, y, (1.2, 0.9, 1.1, 1.1, 0.3),
                                                     time_kernel=kind))
            took = G.debug_counter("gains_fast") - f0
            assert (took >= 1) if fast == "1" else (took == 0), (n, fast, took)
        assert np.isfinite(vals[0]) and vals[0] == vals[1], (n, vals)
