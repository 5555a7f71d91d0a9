"""The concurrent schedules against their serialized twin.

The headline schedule runs a batched fit on several CU-masked streams with hand-placed events: the
whitening of output i + 1 beside the Gram of output i, the Gram's chunk correction on a third
stream, a share of its diagonal-block items on the whitening CUs, the round-overlapping groups'
dense tails and gains on a fourth, and the predictions over two lanes.  Three stream-ordering races
were found in rounds 2-3 (a DG share overwriting partial slots, a first-round dense prefix not
waiting for the context stream, a q(u) Gram on the wrong lane).

gpar_ctx_set_schedule("serialize", 1) routes every launch of the same schedule to the context's one
stream, in issue order, with the same Gram plans, CU shares of work items and workspaces: an
order-free reference.  Any missing dependency in the concurrent schedule shows up as a difference.
Every other schedule knob (round overlap and its number of output groups, the dense prefix, the
short chains' CUs, compact gains records, batched q(u), prediction lanes) only reorders or
re-places the same launches, so it must give bit-identical results too.  (Round 5 deleted the
A/B-only knobs -- split round head variants, DG share, the round overlap's tail CUs, the dense
prefix on its own stream, the prediction's distance-pass whitening -- and their cases here.)  Sizes: the headline test's (N = 4e5, M = 512: the auto CU split, the pipelined Gram
stage, the distance cache down to D = 1, five outputs: the round overlap).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

G = pytest.importorskip("gparatscale")
from gparatscale import data as D  # noqa: E402

N, M, NS, EV = 400_000, 512, 40_000, 6
OUTS = [2, 3, 9, 17, 33]

SETTINGS = [
    {"serialize": 1},
    {"overlap": 0},
    {"overlap_group": 2},                # three groups (2, 2, 1 outputs) take turns
    {"overlap_group": 1},                # five groups of one
    {"overlap": 0, "serialize": 1},
    {"overlap": 0, "dense_early": 0},
    {"post_gram": 0},
    {"post_gram": 1, "overlap": 0},
    {"compact_rec": 0},
    {"compact_rec": 1, "overlap": 0},
    {"qu_batch": 0},
    {"predict_lanes": 1},
]
# dg_rows_w (a plan: G's summation grouping) is pinned for the comparisons: its auto value differs
# between the round-by-round fit (+40 %) and the round overlap (+20 %), which the settings switch
PLAN = {"dg_rows_w": 10}
DEFAULTS = {"serialize": 0, "overlap": 1, "overlap_group": 0, "dense_early": 1, "post_gram": -1,
            "compact_rec": -1, "dg_rows_w": -100, "qu_batch": 1, "predict_lanes": 2,
            "predict_fused": 1, "gram_group": -1, "fit_chunks": -1,
            "device_nm": 1}
DELETED = ["split_head", "dg_share", "tail_cus", "predict_d2"]


@pytest.fixture(scope="module")
def job():
    import torch
    dev = torch.device("cuda", 0)
    ds = D.gpar_dataset(N, max(OUTS), seed=0, observation_noise=0.8, n_star=NS)
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
    ctx.set_cu_split(-1)
    ctx.set_dist_cache(-1)
    assert ctx.cu_split() == 8

    def run(knobs):
        for k, v in {**DEFAULTS, **PLAN}.items():
            ctx.set_schedule(k, v)
        try:
            for k, v in knobs.items():
                ctx.set_schedule(k, v)
            fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, [Fs_d[:, : p - 1] for p in OUTS],
                                                  max_evals=EV, g_tol=-1.0)
            return fr, [m.cpu().numpy() for m in means], [s.cpu().numpy() for s in stds]
        finally:
            for k, v in DEFAULTS.items():
                ctx.set_schedule(k, v)

    base = run({})
    return run, base, keep


def test_schedule_knobs_round_trip():
    ctx = G.context(0)
    for k, v in DEFAULTS.items():
        assert ctx.schedule(k) == v
    ctx.set_schedule("serialize", 1)
    assert ctx.schedule("serialize") == 1
    ctx.set_schedule("serialize", 0)
    with pytest.raises(G.DomainError):
        ctx.set_schedule("no_such_knob", 1)
    with pytest.raises(G.DomainError):
        ctx.set_schedule("predict_lanes", 3)
    with pytest.raises(G.DomainError):
        ctx.set_schedule("dense_early", 2)
    with pytest.raises(G.DomainError):
        ctx.set_schedule("gram_group", 65)
    for k in DELETED:
        with pytest.raises(G.DomainError):
            ctx.set_schedule(k, 0)


@pytest.mark.parametrize("knobs", SETTINGS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_schedule_is_bit_identical(job, knobs):
    run, (fr0, m0, s0), _ = job
    fr, m, s = run(knobs)
    np.testing.assert_array_equal(fr.theta, fr0.theta)
    np.testing.assert_array_equal(fr.nlml, fr0.nlml)
    np.testing.assert_array_equal(fr.evals, fr0.evals)
    for i in range(len(OUTS)):
        np.testing.assert_array_equal(m[i], m0[i])
        np.testing.assert_array_equal(s[i], s0[i])


def test_dg_rows_w_is_a_plan_not_a_schedule(job):
    """dg_rows_w re-sizes the DG time splits (a different summation grouping of G): bit-identical to
    its own serialized twin, within rounding of the default plan."""
    run, (fr0, m0, s0), _ = job
    fa, ma, sa = run({"dg_rows_w": 0})
    fb, mb, sb = run({"dg_rows_w": 0, "serialize": 1})
    np.testing.assert_array_equal(fa.theta, fb.theta)
    np.testing.assert_array_equal(fa.nlml, fb.nlml)
    for i in range(len(OUTS)):
        np.testing.assert_array_equal(ma[i], mb[i])
        np.testing.assert_array_equal(sa[i], sb[i])
    # the objective's tolerance against the checkers (rel 1e-9): output 3's fit is ill-conditioned
    # (-nlml 1.7e9), and six simplex steps carry the last-bit difference of G to 1.7e-11
    np.testing.assert_allclose(fa.nlml, fr0.nlml, rtol=1e-9)
    np.testing.assert_allclose(fa.theta, fr0.theta, rtol=1e-6)


def test_grouped_gram_is_a_plan_not_a_schedule():
    """gram_group: an unsplit batched fit of small problems (here N = 3e4, M = 128, five outputs of
    one Mp) whitens every output of a group into buffers of its own over two streams and runs one
    grouped set of Gram launches for the group, with 1/g of the time splits per output.  A plan (G
    summed in another grouping): bit-identical to its serialized twin, for the auto groups (one
    group of five) and groups of two (2 + 2 + 1), and within rounding of the per-output Grams."""
    import torch
    dev = torch.device("cuda", 0)
    n, m, outs = 30_000, 128, [2, 3, 5, 9, 17]
    ds = D.gpar_dataset(n, max(outs), seed=3, observation_noise=0.8, n_star=4_000)
    Y_d = torch.from_numpy(ds["Y"]).to(dev)
    t_d = torch.from_numpy(ds["t"]).to(dev)
    ts_d = torch.from_numpy(ds["t_star"]).to(dev)
    Fs_d = torch.from_numpy(ds["F_star"]).to(dev)
    probs, keep = [], []
    for p in outs:
        Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, : p - 1], m, seed=p)).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), "eq",
                               "matern52", qu_kuu_noise=True)
        probs.append(pr)
        keep.append((k, Z))
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(outs), 1))
    ctx = G.context(0)
    ctx.set_cu_split(-1)
    assert ctx.cu_split() == 0 or n * 128 * 128 < 1e11   # the auto split stays off at this size
    th = np.tile([[1.1, 0.9, 1.3, 0.8, 0.3]], (len(outs), 1))

    def run(knobs):
        try:
            for k, v in knobs.items():
                ctx.set_schedule(k, v)
            vals = G.dtc_objective_batch(probs, th)
            fr, means, stds = G.fit_predict_batch(probs, x0, ts_d, [Fs_d[:, : p - 1] for p in outs],
                                                  max_evals=8, g_tol=-1.0)
            return np.asarray(vals), fr, [a.cpu().numpy() for a in means], [a.cpu().numpy() for a in stds]
        finally:
            for k, v in DEFAULTS.items():
                ctx.set_schedule(k, v)

    off = run({"gram_group": 0})
    for g in (-1, 2):
        a = run({"gram_group": g})
        b = run({"gram_group": g, "serialize": 1})
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1].theta, b[1].theta)
        np.testing.assert_array_equal(a[1].nlml, b[1].nlml)
        for i in range(len(outs)):
            np.testing.assert_array_equal(a[2][i], b[2][i])
            np.testing.assert_array_equal(a[3][i], b[3][i])
        np.testing.assert_allclose(a[0], off[0], rtol=1e-10)
        np.testing.assert_allclose(a[1].nlml, off[1].nlml, rtol=1e-9)
        np.testing.assert_allclose(a[1].theta, off[1].theta, rtol=1e-6)
        for i in range(len(outs)):
            np.testing.assert_allclose(a[2][i], off[2][i], rtol=1e-7, atol=1e-9)
            np.testing.assert_allclose(a[3][i], off[3][i], rtol=1e-7, atol=1e-9)


def test_grouped_gram_mixed_time_kernels_match_per_output():
    """A batch of small problems with the same N and Mp but different time kernels (Matern-1/2
    and Matern-5/2: different state dimension, so a different chunk correction in the Gram): the
    grouped plan must not run them under one group's correction.  Auto grouping equals the
    per-output Grams (gram_group = 0) within rounding, output by output."""
    import torch
    dev = torch.device("cuda", 0)
    n, m, outs = 30_000, 128, [2, 3, 5, 9]
    ds = D.gpar_dataset(n, max(outs), seed=4, observation_noise=0.8)
    Y_d = torch.from_numpy(ds["Y"]).to(dev)
    t_d = torch.from_numpy(ds["t"]).to(dev)
    probs, keep = [], []
    for i, p in enumerate(outs):
        Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, : p - 1], m, seed=p)).to(dev)
        tk = "matern12" if i % 2 else "matern52"
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), "matern52",
                               tk, qu_kuu_noise=True)
        probs.append(pr)
        keep.append((k, Z))
    ctx = G.context(0)
    ctx.set_cu_split(-1)
    th = np.tile([[1.1, 0.9, 1.3, 0.8, 0.3]], (len(outs), 1))
    vals = {}
    try:
        for g in (0, -1, 2):
            ctx.set_schedule("gram_group", g)
            vals[g] = np.asarray(G.dtc_objective_batch(probs, th))
    finally:
        for k, v in DEFAULTS.items():
            ctx.set_schedule(k, v)
    singles = np.array([G.dtc_objective_batch([pr], th[i:i + 1])[0] for i, pr in enumerate(probs)])
    for g in (0, -1, 2):
        np.testing.assert_allclose(vals[g], singles, rtol=1e-10)
