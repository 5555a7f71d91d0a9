"""The unsplit round overlap (host_fit.cpp fit_overlapped_unsplit): batched fits below the CU
split's size (the dtc / eeg configs, a rank's eeg shard) deal their outputs into groups whose
rounds run on streams and workspaces of their own, one group's round boundary under another's
grouped Gram.

* Against its serialized twin (every group on the main stream, issue order): bit for bit -- any
  missing dependency between a group's launches, or a buffer two groups share, shows up here.
* Against the round-by-round fit (overlap 0: one group, one grouped Gram per round): the same
  simplex points per output with the same kernels; only the grouped-Gram plan, sized for the
  group's outputs, sums G in another grouping -- within rounding.
* fit_predict (the kept Grams of the best points feed q(u)) through the overlap.
Sizes: N = 2e4, M = 512 (N Mp^2 = 5e9: grouped Gram, no CU split; the overlap's default takes
Mp >= 512), six GPAR outputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

G = pytest.importorskip("gparatscale")
from gparatscale import data as D  # noqa: E402

N, M, NS, EV = 20_000, 512, 2_000, 12
OUTS = [2, 3, 4, 5, 6, 7]
KNOBS = {"overlap": 1, "overlap_group": 0, "serialize": 0}


@pytest.fixture(scope="module")
def job():
    import torch
    dev = torch.device("cuda", 0)
    ds = D.gpar_dataset(N, max(OUTS), seed=3, observation_noise=0.8, n_star=NS)
    Y_d = torch.from_numpy(ds["Y"]).to(dev)
    t_d = torch.from_numpy(ds["t"]).to(dev)
    ts_d = torch.from_numpy(ds["t_star"]).to(dev)
    Fs_d = torch.from_numpy(ds["F_star"]).to(dev)
    probs, keep = [], []
    for p in OUTS:
        Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, : p - 1], M, seed=p)).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), "matern52",
                               "matern52", qu_kuu_noise=True)
        probs.append(pr)
        keep.append((k, Z))
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(OUTS), 1))
    ctx = G.context(0)

    def run(knobs, predict=False):
        for k, v in KNOBS.items():
            ctx.set_schedule(k, v)
        try:
            for k, v in knobs.items():
                ctx.set_schedule(k, v)
            if predict:
                fr, means, stds = G.fit_predict_batch(probs, x0, ts_d,
                                                      [Fs_d[:, : p - 1] for p in OUTS],
                                                      max_evals=EV, g_tol=-1.0)
                return fr, [m.cpu().numpy() for m in means], [s.cpu().numpy() for s in stds]
            return G.fit_batch(probs, x0, max_evals=EV, g_tol=-1.0), None, None
        finally:
            for k, v in KNOBS.items():
                ctx.set_schedule(k, v)

    return run, keep


@pytest.mark.parametrize("knobs", [{}, {"overlap_group": 2}], ids=["two_groups", "three_groups"])
def test_overlap_unsplit_equals_its_serialized_twin(job, knobs):
    run, _ = job
    fa, _, _ = run(knobs)
    fb, _, _ = run({**knobs, "serialize": 1})
    np.testing.assert_array_equal(fa.theta, fb.theta)
    np.testing.assert_array_equal(fa.nlml, fb.nlml)
    np.testing.assert_array_equal(fa.evals, fb.evals)


def test_overlap_unsplit_matches_round_by_round(job):
    run, _ = job
    fa, _, _ = run({})
    fb, _, _ = run({"overlap": 0})
    np.testing.assert_array_equal(fa.evals, fb.evals)
    np.testing.assert_allclose(fa.nlml, fb.nlml, rtol=1e-9)
    np.testing.assert_allclose(fa.theta, fb.theta, rtol=1e-6)


def test_overlap_unsplit_fit_predict(job):
    run, _ = job
    fa, ma, sa = run({}, predict=True)
    fs, ms, ss = run({"serialize": 1}, predict=True)
    fb, mb, sb = run({"overlap": 0}, predict=True)
    np.testing.assert_array_equal(fa.theta, fs.theta)
    for i in range(len(OUTS)):
        np.testing.assert_array_equal(ma[i], ms[i])
        np.testing.assert_array_equal(sa[i], ss[i])
        np.testing.assert_allclose(ma[i], mb[i], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(sa[i], sb[i], rtol=1e-6, atol=1e-9)
