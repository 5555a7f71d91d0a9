"""The fit's distance cache (gpar_ctx_set_dist_cache): the input distances are
theta-independent, so gpar_fit computes them once per call for outputs with D >= 17 and the
whitening reads them instead of rebuilding them in the fused kernel.  Same objective to rounding
(both use the centred Gram form, in a different summation order), so the same Nelder-Mead
trajectory: fitted theta rtol 1e-9, final -dtc rel 1e-12; and against the oracle's NM."""
import numpy as np
import pytest

from oracle import gpar_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")

X0 = np.array([0.0, 0.0, 0.5, 0.0, -1.5])


def _batch(kernel="matern52"):
    t, Y = O.synthetic_gpar(1500, 71, seed=51, noise=0.3)
    probs, keep, data = [], [], []
    for D in (4, 20, 40, 70):              # 4: never cached; 70: distance path either way
        V = np.ascontiguousarray(Y[:, :D].T)
        Z = O.pick_pseudo_inputs(V, 90, D)
        pr, k = G.make_problem(V, Z, t, Y[:, D], kernel, "matern32")
        probs.append(pr)
        keep.append(k)
        data.append((V, Z, Y[:, D]))
    return t, probs, keep, data


@pytest.mark.parametrize("kernel", ["matern52", "eq", "matern12"])
def test_cache_on_off_same_fit(kernel):
    t, probs, keep, data = _batch(kernel)
    ctx = G.context(0)
    x0 = np.tile(X0, (len(probs), 1))
    try:
        ctx.set_dist_cache(0)
        off = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
        ctx.set_dist_cache(-1)
        on = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
        big = data[2]
        one = big[0].shape[1] * 128 * 8 + (1 << 20)       # room for one output of mp = 128
        ctx.set_dist_cache(one)
        part = G.fit_batch(probs, x0, max_evals=30, g_tol=-1.0)
    finally:
        ctx.set_dist_cache(-1)
    for r in (on, part):
        np.testing.assert_allclose(r.theta, off.theta, rtol=1e-9)
        np.testing.assert_allclose(r.nlml, off.nlml, rtol=1e-12)
    if kernel == "matern52":
        for i, (V, Z, y) in enumerate(data):
            th, _ = O.get_optim_scaled_gpar_params(V, Z, t, y, "matern52", "matern32", log_theta0=X0,
                                                   max_evals=30, g_tol=-1.0, return_nm=True)
            np.testing.assert_allclose(on.theta[i], th, rtol=1e-6)


def test_cache_budget_argument():
    ctx = G.context(0)
    with pytest.raises(G.DomainError):
        ctx.set_dist_cache(-2)


# ---------------------------------------------------------------- the all-D cache of split fits
def _split_batch(kernel, n=70_000, m=64, dims=(1, 4, 16)):
    t, Y = O.synthetic_gpar(n, max(dims) + 1, seed=53, noise=0.3)
    probs, keep, data = [], [], []
    for d in dims:
        V = np.ascontiguousarray(Y[:, :d].T)
        Z = O.pick_pseudo_inputs(V, m, 100 + d)
        pr, k = G.make_problem(V, Z, t, Y[:, d], kernel, "matern52")
        probs.append(pr)
        keep.append(k)
        data.append((V, Z, Y[:, d]))
    return t, probs, keep, data


@pytest.mark.parametrize("kernel", ["matern52", "eq", "matern12"])
def test_split_fit_caches_every_output(kernel):
    """With the CU split on and N >= 2^16 the fit caches outputs down to D = 1 (gpar_host.cpp
    attach_dist_cache): the small-D cached path (group-centred Gram-form distances, or direct
    differences for Matern-1/2) against the same split fit without the cache, and one output's
    objective at the fitted theta against the C port (dtc.jl:83-128)."""
    from oracle import cpu_ref as CR
    CR.load()
    t, probs, keep, data = _split_batch(kernel)
    ctx = G.context(0)
    x0 = np.tile(X0, (len(probs), 1))
    try:
        ctx.set_cu_split(8)
        ctx.set_dist_cache(-1)
        on = G.fit_batch(probs, x0, max_evals=25, g_tol=-1.0)
        assert ctx.dist_cache_stats()[0] == len(probs)
        assert ctx.dist_cache_stats()[2] == 0          # released when the fit returned
        ctx.set_dist_cache(0)
        off = G.fit_batch(probs, x0, max_evals=25, g_tol=-1.0)
        assert ctx.dist_cache_stats()[0] == 0
    finally:
        ctx.set_cu_split(-1)
        ctx.set_dist_cache(-1)
    np.testing.assert_allclose(on.theta, off.theta, rtol=1e-9)
    np.testing.assert_allclose(on.nlml, off.nlml, rtol=1e-12)
    V, Z, y = data[0]                                   # D = 1
    ref, _ = CR.compute_gpar_dtc_objective(V, Z, t, y, on.theta[0], kernel, "matern52")
    assert abs(-on.nlml[0] - ref) <= 1e-9 * abs(ref), (-on.nlml[0], ref)


@pytest.mark.parametrize("kernel", ["matern52", "eq", "matern12"])
def test_cached_distances_match_direct_differences(kernel):
    """gpar_pairwise_distances = the cache's kernel (dist2) at D = 1..16 against direct
    differences.  The Gram form |v - c|^2 + |z - c|^2 - 2 (v - c).(z - c) about per-256-column
    centres c loses |r^2| to cancellation by ~eps (|v - c|^2 + |z - c|^2); so r^2 is checked to
    32 eps of that scale everywhere, and r to rel 1e-12 wherever r^2 >= 1e-3 of it."""
    t, Y = O.synthetic_gpar(20_000, 17, seed=57, noise=0.3)
    eps = np.finfo(np.float64).eps
    for d in range(1, 17):
        V = np.ascontiguousarray(Y[:, :d].T)
        Z = O.pick_pseudo_inputs(V, 300, 200 + d)          # Mp = 384: two centre groups
        got = G.pairwise_distances(V, Z, kernel)
        diff = V.T[:, None, :] - Z.T[None, :, :]
        r2 = np.einsum("kcd,kcd->kc", diff, diff)
        if kernel == "matern12":                            # direct differences on the device too
            # (sqrt_pos floors r at 1e-100 where v = z: kappa(1e-100 / l) = 1 exactly)
            np.testing.assert_allclose(got, np.sqrt(r2), rtol=1e-14, atol=2e-100)
            continue
        g2 = got if kernel == "eq" else got * got
        scale = (np.einsum("dk,dk->k", V, V).max() + np.einsum("dc,dc->c", Z, Z).max())
        assert np.abs(g2 - r2).max() <= 32 * eps * scale, (d, np.abs(g2 - r2).max(), scale)
        big = r2 >= 1e-3 * scale
        assert big.mean() > 0.5
        r_got = np.sqrt(g2[big])
        np.testing.assert_allclose(r_got, np.sqrt(r2[big]), rtol=1e-12)


def test_cache_survives_memory_pressure():
    """A full device: the distance cache holds every slot (kept from an earlier call), a blocker
    tensor takes the rest, and the next call's predictions need more workspace (more test points):
    those allocations run out of memory, evict cache slots (ws_bytes) and retry, and
    gpar_fit_predict completes with the unconstrained run's results."""
    import torch
    n, m = 200_000, 256
    t, probs, keep, data = _split_batch("matern52", n=n, m=m, dims=(2, 8, 20, 40))
    ts_small = np.linspace(t[0], t[-1], 5000) + 1e-3
    ts = np.linspace(t[0], t[-1], 60000) + 1e-3

    def test_inputs(tt):
        return [np.vstack([np.interp(tt, t, V[q]) for q in range(V.shape[0])]) for V, _, _ in data]
    x0 = np.tile(X0, (len(probs), 1))
    ctx = G.context(0)
    blocker = None
    try:
        ctx.set_cu_split(8)
        ctx.set_dist_cache(0)
        ctx.trim()
        ref, rm, rs = G.fit_predict_batch(probs, x0, ts, test_inputs(ts), max_evals=12, g_tol=-1.0)
        ctx.trim()
        # every output cached and kept, with the workspace of the smaller call
        ctx.set_dist_cache(1 << 40)
        ctx.set_dist_cache_keep(True)
        G.fit_predict_batch(probs, x0, ts_small, test_inputs(ts_small), max_evals=12, g_tol=-1.0)
        held0 = ctx.dist_cache_stats()[2]
        torch.cuda.empty_cache()
        free = torch.cuda.mem_get_info(0)[0]
        blocker = torch.empty(free - (64 << 20), dtype=torch.uint8, device="cuda:0")
        ev0 = ctx.dist_cache_stats()[1]
        got, gm, gs = G.fit_predict_batch(probs, x0, ts, test_inputs(ts), max_evals=12, g_tol=-1.0)
        cached, ev1, held = ctx.dist_cache_stats()
    finally:
        del blocker
        torch.cuda.empty_cache()
        ctx.set_dist_cache_keep(False)
        ctx.set_cu_split(-1)
        ctx.set_dist_cache(-1)
        ctx.trim()
    assert held0 == len(probs) * n * m * 8, held0
    assert cached == len(probs), cached
    assert ev1 > ev0, (ev0, ev1)
    assert held < held0, (held, held0)
    np.testing.assert_allclose(got.theta, ref.theta, rtol=1e-9)
    np.testing.assert_allclose(got.nlml, ref.nlml, rtol=1e-12)
    for a, b in zip(gm + gs, rm + rs):
        np.testing.assert_allclose(a, b, rtol=1e-8, atol=1e-10 * np.abs(b).max())


def test_cache_auto_budget_under_memory_pressure():
    """The auto budget reads the free memory net of the workspace the call still needs: with
    room for the workspace, the 1 % reserve and about two slots, the fit caches what fits, needs no
    eviction, and matches the uncached run."""
    import torch
    n, m = 200_000, 256
    t, probs, keep, data = _split_batch("matern52", n=n, m=m, dims=(2, 8, 20, 40))
    x0 = np.tile(X0, (len(probs), 1))
    ctx = G.context(0)
    cache_bytes = n * m * 8
    blocker = None
    try:
        ctx.set_cu_split(8)
        ctx.set_dist_cache(0)
        ctx.trim()
        ref = G.fit_batch(probs, x0, max_evals=12, g_tol=-1.0)
        work = ctx.workspace_bytes()                  # the fit's workspace without the cache
        ctx.trim()
        torch.cuda.empty_cache()
        free, total = torch.cuda.mem_get_info(0)
        reserve = max(1 << 30, total // 100)
        leave = reserve + work + int(2.5 * cache_bytes)
        blocker = torch.empty(free - leave, dtype=torch.uint8, device="cuda:0")
        ctx.set_dist_cache(-1)
        ev0 = ctx.dist_cache_stats()[1]
        got = G.fit_batch(probs, x0, max_evals=12, g_tol=-1.0)
        cached, ev1, _ = ctx.dist_cache_stats()
    finally:
        del blocker
        torch.cuda.empty_cache()
        ctx.set_cu_split(-1)
        ctx.set_dist_cache(-1)
        ctx.trim()
    assert 1 <= cached < len(probs), cached
    assert ev1 == ev0
    np.testing.assert_allclose(got.theta, ref.theta, rtol=1e-9)
    np.testing.assert_allclose(got.nlml, ref.nlml, rtol=1e-12)


def test_fit_chunks_equal_one_fully_cached_batch():
    """fit_chunks (cache-resident sub-batches, the stress config's schedule): the outputs fitted in
    consecutive sub-batches of k, each computing its distances once, equal one batch with every
    output cached, bit for bit (per-output Grams: gram_group 0, whose grouping would otherwise
    follow the batch size); the auto rule leaves this pipelined fit as one batch."""
    t, Y = O.synthetic_gpar(20_000, 25, seed=52, noise=0.3)
    probs, keep = [], []
    for D in (17, 19, 21, 24, 18):
        V = np.ascontiguousarray(Y[:, :D].T)
        Z = O.pick_pseudo_inputs(V, 64, D)
        pr, k = G.make_problem(V, Z, t, Y[:, D], "matern52", "matern52")
        probs.append(pr)
        keep.append(k)
    ctx = G.context(0)
    x0 = np.tile(X0, (len(probs), 1))
    res = {}
    try:
        ctx.set_schedule("gram_group", 0)
        for k in (0, 2, 1, -1):
            ctx.set_schedule("fit_chunks", k)
            res[k] = G.fit_batch(probs, x0, max_evals=14, g_tol=-1.0)
            # outputs the last fit call (the last sub-batch) cached: 5 = 2 + 2 + 1 = 1 + ... + 1
            assert ctx.dist_cache_stats()[0] == {0: 5, -1: 5, 2: 1, 1: 1}[k]
    finally:
        ctx.set_schedule("fit_chunks", -1)
        ctx.set_schedule("gram_group", -1)
    for k in (2, 1, -1):
        np.testing.assert_array_equal(res[k].theta, res[0].theta)
        np.testing.assert_array_equal(res[k].nlml, res[0].nlml)
        np.testing.assert_array_equal(res[k].evals, res[0].evals)


def test_fit_chunks_auto_keeps_narrow_outputs_apart():
    """The auto rule where the fit is not pipelined (here: two lanes; in the stress config: an
    82 GB beta) and the cache budget holds fewer wide outputs than the batch has: the outputs
    with D < 17 (never cached) run as one sub-batch, the cacheable ones two at a time (the budget),
    and the fit equals one batch with every wide output cached, bit for bit."""
    t, Y = O.synthetic_gpar(12_000, 45, seed=53, noise=0.3)
    probs, keep = [], []
    dims = (4, 20, 40, 9, 18, 30)
    for D in dims:
        V = np.ascontiguousarray(Y[:, :D].T)
        Z = O.pick_pseudo_inputs(V, 64, D)
        pr, k = G.make_problem(V, Z, t, Y[:, D], "matern52", "matern52")
        probs.append(pr)
        keep.append(k)
    ctx = G.context(0)
    x0 = np.tile(X0, (len(probs), 1))
    two = 2 * 12_000 * 128 * 8 + (1 << 20)          # the distances of two outputs of Mp = 128
    try:
        ctx.set_lanes(2)
        ctx.set_schedule("fit_chunks", 0)
        whole = G.fit_batch(probs, x0, max_evals=12, g_tol=-1.0)
        assert ctx.dist_cache_stats()[0] == 4
        ctx.set_schedule("fit_chunks", -1)
        ctx.set_dist_cache(two)
        auto = G.fit_batch(probs, x0, max_evals=12, g_tol=-1.0)
        assert ctx.dist_cache_stats()[0] == 2          # the last sub-batch: two wide outputs
    finally:
        ctx.set_lanes(1)
        ctx.set_dist_cache(-1)
        ctx.set_schedule("fit_chunks", -1)
    np.testing.assert_array_equal(auto.theta, whole.theta)
    np.testing.assert_array_equal(auto.nlml, whole.nlml)
