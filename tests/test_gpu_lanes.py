"""Two stream lanes (gpar_ctx_set_lanes(ctx, 2)): a batch's outputs alternate between two HIP
streams, and the Gram runs one workgroup per CU (its own split plan, fragments pipelined in
registers) so the other lane's whitening runs beside it.  Same objective as one lane up to the
Gram's summation order (rel <= 1e-12), against the oracle at rel <= 1e-10, and the same fit."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")


def _batch(n=20000, M=200):
    t, Y = O.synthetic_gpar(n, 41, seed=61, noise=0.4)
    probs, keep, data = [], [], []
    for D in (3, 12, 20, 33, 40):
        V = np.ascontiguousarray(Y[:, :D].T)
        Z = O.pick_pseudo_inputs(V, M, D)
        pr, k = G.make_problem(V, Z, t, Y[:, D])
        probs.append(pr)
        keep.append(k)
        data.append((V, Z, Y[:, D]))
    return t, probs, keep, data


def test_two_lanes_objective_and_fit():
    t, probs, keep, data = _batch()
    thetas = np.array([(1.0 + 0.1 * i, 1.0, 2.0 + 0.3 * i, 1.1, 0.3) for i in range(len(probs))])
    ctx = G.context(0)
    x0 = np.tile([0.0, 0.0, 0.5, 0.0, -1.5], (len(probs), 1))
    try:
        ctx.set_lanes(1)
        one = G.dtc_objective_batch(probs, thetas)
        f1 = G.fit_batch(probs, x0, max_evals=15, g_tol=-1.0)
        ctx.set_lanes(2)
        two = G.dtc_objective_batch(probs, thetas)
        f2 = G.fit_batch(probs, x0, max_evals=15, g_tol=-1.0)
    finally:
        ctx.set_lanes(1)
    np.testing.assert_allclose(two, one, rtol=1e-12)
    np.testing.assert_allclose(f2.theta, f1.theta, rtol=1e-9)
    for i, (V, Z, y) in enumerate(data[:2]):
        ref, _ = O.compute_gpar_dtc_objective(V, Z, t, y, thetas[i])
        assert abs(two[i] - ref) <= 1e-10 * abs(ref), (two[i], ref)
