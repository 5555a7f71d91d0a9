"""The batched fit's CU split (gpar_ctx_set_cu_split): each output's whitening on CU-masked streams
beside the previous output's Gram, a share of the Gram's diagonal-block items on the whitening
CUs.  Forced on (an explicit width) at small sizes, so the split schedule itself is checked here:
the batched objective against the oracle (dtc.jl:83-128) and against the whole-chip schedule, fits
against the whole-chip fits, mixed Mp in one batch, and the setter's argument checks."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu

G = pytest.importorskip("gparatscale")


@pytest.fixture
def ctx():
    c = G.context(0)
    yield c
    c.set_cu_split(-1)   # back to the library default for the other tests


def _batch(n, outs, Ms, seed, kernels=("matern52", "matern52")):
    t, Y = O.synthetic_gpar(n, max(outs), seed=seed, noise=0.3)
    probs, keep, ref = [], [], []
    for p, M in zip(outs, Ms):
        V = np.ascontiguousarray(Y[:, : p - 1].T)
        Z = O.pick_pseudo_inputs(V, M, seed + p)
        pr, k = G.make_problem(V, Z, t, Y[:, p - 1], kernels[0], kernels[1])
        probs.append(pr)
        keep.append(k)
        ref.append((V, Z, t, Y[:, p - 1]))
    return probs, keep, ref


THETAS = np.array([[1.1, 0.9, 1.3, 0.8, 0.25], [0.7, 1.2, 0.9, 1.1, 0.3], [1.5, 1.0, 2.0, 0.9, 0.2],
                   [0.9, 0.8, 1.1, 1.2, 0.35], [1.2, 1.1, 0.8, 1.0, 0.15]])


@pytest.mark.parametrize("w", [4, 8, 12])
def test_split_objective_matches_oracle_and_whole_chip(ctx, w):
    # five outputs (the pipeline's buffer reuse and the last output's DG share), Mp = 128 / 256 / 384
    outs, Ms = [2, 3, 5, 6, 4], [60, 200, 300, 130, 90]
    probs, keep, ref = _batch(1300, outs, Ms, 41)
    ctx.set_cu_split(0)
    whole = G.dtc_objective_batch(probs, THETAS)
    ctx.set_cu_split(w)
    assert ctx.cu_split() == w
    split = G.dtc_objective_batch(probs, THETAS)
    again = G.dtc_objective_batch(probs, THETAS)
    np.testing.assert_array_equal(split, again)            # deterministic for a given width
    np.testing.assert_allclose(split, whole, rtol=1e-12)
    for i, (V, Z, t, y) in enumerate(ref):
        o, _ = O.compute_gpar_dtc_objective(V, Z, t, y, THETAS[i])
        assert abs(split[i] - o) <= 1e-10 * max(1.0, abs(o)), (i, split[i], o)


def test_split_with_offdiagonal_groups(ctx):
    # Mp = 512: six OFF groups beside the whitening, DG items shared; chunks of 256 over N = 2e4
    probs, keep, _ = _batch(20000, [3, 8, 17], [512, 512, 500], 43, ("matern52", "matern32"))
    th = THETAS[:3]
    ctx.set_cu_split(0)
    whole = G.dtc_objective_batch(probs, th)
    ctx.set_cu_split(8)
    split = G.dtc_objective_batch(probs, th)
    np.testing.assert_allclose(split, whole, rtol=1e-11)


def test_split_fit_matches_whole_chip_fit(ctx):
    probs, keep, _ = _batch(900, [2, 4, 6], [40, 70, 50], 47)
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (3, 1))
    ctx.set_cu_split(0)
    a = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
    ctx.set_cu_split(8)
    b = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
    np.testing.assert_allclose(b.theta, a.theta, rtol=1e-6)
    np.testing.assert_allclose(b.nlml, a.nlml, rtol=1e-10)


def test_set_cu_split_rejects_bad_widths(ctx):
    for bad in (6, 32, -2, 3):
        with pytest.raises((G.DomainError, G.GparError)):
            ctx.set_cu_split(bad)
    ctx.set_cu_split(8)
    assert ctx.cu_split() == 8
    ctx.set_cu_split(-1)
    assert ctx.cu_split() == 8    # the default width (applied to large enough Grams)


def test_overlapped_rounds_equal_round_by_round(ctx):
    """fit_overlapped (two groups of outputs taking turns, no drain between Nelder-Mead rounds)
    evaluates the same points with the same per-problem arithmetic as the round-by-round fit:
    bit-identical theta / -nlml, here with mixed Mp (padded Gram slots), an odd output count,
    outputs converging at different rounds (g_tol on) and the kept Grams of fit_predict."""
    outs, Ms = [2, 3, 5, 6, 4], [60, 200, 300, 130, 90]
    probs, keep, ref = _batch(2500, outs, Ms, 61)
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(outs), 1))
    ctx.set_cu_split(8)
    # a fixed DG plan: dg_rows_w's auto value differs between the two fits (a summation grouping)
    ctx.set_schedule("dg_rows_w", 10)
    res = {}
    try:
        for on in (False, True):
            ctx.set_fit_overlap(on)
            a = G.fit_batch(probs, x0, max_evals=20, g_tol=-1.0)
            b = G.fit_batch(probs, x0, max_evals=400, g_tol=0.05)
            t = ref[0][2]
            ts = np.linspace(t[0], t[-1], 700) + 1e-3
            Vs = [np.vstack([np.interp(ts, t, V[q]) for q in range(V.shape[0])]) for V, _, _, _ in ref]
            c, cm, cs = G.fit_predict_batch(probs, x0, ts, Vs, max_evals=16, g_tol=-1.0)
            res[on] = (a, b, c, cm, cs)
    finally:
        ctx.set_fit_overlap(True)
        ctx.set_cu_split(-1)
        ctx.set_schedule("dg_rows_w", -100)
    (a0, b0, c0, cm0, cs0), (a1, b1, c1, cm1, cs1) = res[False], res[True]
    assert len(set(b0.evals)) > 1          # the groups shrink at different rounds
    for x, y in ((a0, a1), (b0, b1), (c0, c1)):
        np.testing.assert_array_equal(x.theta, y.theta)
        np.testing.assert_array_equal(x.nlml, y.nlml)
        np.testing.assert_array_equal(x.evals, y.evals)
    for x, y in zip(cm0 + cs0, cm1 + cs1):
        np.testing.assert_array_equal(x, y)
