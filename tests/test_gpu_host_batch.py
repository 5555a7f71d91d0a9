"""The C-ABI's host-memory batch path.

GPAR's outputs read column prefixes of one matrix of earlier outputs, so a host-memory batch
passes that matrix once (v = Y, ldv = P for every output: the Julia shim's matrix-form driver and
its Python mirror get_gpar_scaled_predictions_batch).  The library uploads the shared time grid and
input matrix once (prepare_batch), the shared test-input matrix once after the fit, runs the
predictions on device buffers with both lanes, and downloads the means / stds at the end.  The
arithmetic is the device-resident path's: results equal the device-memory call bit for bit, with
ascending and with shuffled test times."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")

P, N, NS, M, EV = 6, 3000, 700, 40, 20


def _data():
    t, Y = O.synthetic_gpar(N, P, seed=61, noise=0.3)
    ts = np.sort(np.random.default_rng(3).uniform(t[0], t[-1], NS))
    F = np.column_stack([np.interp(ts, t, Y[:, q]) for q in range(P)])
    Zs = [O.pick_pseudo_inputs(np.ascontiguousarray(Y[:, : p - 1].T), M, p) for p in range(2, P + 1)]
    return t, Y, ts, F, Zs


def _device_run(t, Y, ts, F, Zs, chained):
    import torch
    dev = torch.device("cuda", 0)
    t_d, Y_d, ts_d, F_d = (torch.from_numpy(a).to(dev) for a in (t, Y, ts, F))
    probs, keep = [], []
    for p in range(2, P + 1):
        Z = torch.from_numpy(np.ascontiguousarray(Zs[p - 2].T)).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), qu_kuu_noise=True)
        probs.append(pr)
        keep.append((k, Z))
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (P - 1, 1))
    if chained:
        chain = F_d.clone()
        fr, m, s = G.fit_predict_batch(probs, x0, ts_d, [None] * (P - 1), max_evals=EV, g_tol=-1.0,
                                       chain=chain, chain_cols=list(range(1, P)))
    else:
        fr, m, s = G.fit_predict_batch(probs, x0, ts_d, [F_d[:, : p - 1] for p in range(2, P + 1)],
                                       max_evals=EV, g_tol=-1.0)
    return fr, [a.cpu().numpy() for a in m], [a.cpu().numpy() for a in s]


@pytest.mark.parametrize("chained", [False, True])
def test_host_matrix_batch_equals_device(chained):
    t, Y, ts, F, Zs = _data()
    fr0, m0, s0 = _device_run(t, Y, ts, F, Zs, chained)
    fr, m, s = G.get_gpar_scaled_predictions_batch(Y, Zs, t, ts, F, chained=chained, max_evals=EV,
                                                   g_tol=-1.0, qu_kuu_noise=True)
    np.testing.assert_array_equal(fr.theta, fr0.theta)
    np.testing.assert_array_equal(fr.nlml, fr0.nlml)
    for i in range(P - 1):
        np.testing.assert_array_equal(m[i], m0[i])
        np.testing.assert_array_equal(s[i], s0[i])


def test_host_matrix_batch_shuffled_test_times():
    t, Y, ts, F, Zs = _data()
    fr0, m0, s0 = _device_run(t, Y, ts, F, Zs, False)
    perm = np.random.default_rng(9).permutation(NS)
    fr, m, s = G.get_gpar_scaled_predictions_batch(Y, Zs, t, ts[perm], F[perm], max_evals=EV,
                                                   g_tol=-1.0, qu_kuu_noise=True)
    np.testing.assert_array_equal(fr.theta, fr0.theta)
    for i in range(P - 1):
        np.testing.assert_array_equal(m[i], m0[i][perm])
        np.testing.assert_array_equal(s[i], s0[i][perm])
