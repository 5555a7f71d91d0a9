"""Python mirror of the reference's Julia API for the hot path (same names, argument
meaning and error behaviour), on top of the C-ABI in include/gpar_hip.h.

Reference functions mirrored (TudorParas/GPAR-at-scale):
  compute_gpar_dtc_objective     src/gp/dtc.jl:83-128
  get_optim_scaled_gpar_params   src/gp/dtc.jl:11-77
  compute_q_u                    src/gp/gpar_scaled_inference.jl:141-196
  get_gpar_scaled_predictions    src/gp/gpar_scaled_inference.jl:20-136
  create_lgssm / logpdf          src/gp/temporal_gp_inference.jl:15-39, :286-296
  get_sde_predictions            src/gp/temporal_gp_inference.jl:45-114
  create_optim_gp[_post] / create_optim_gpar[_post] logpdf / marginals  src/gp/optimized.jl

Inputs follow the reference's conventions: V / Z are ColVecs-like D x N matrices (or a list of
D length-N vectors, util.jl:16-31); theta in natural units (unpack_gpar, util.jl:45-55);
initial values are log-params (i_log_*), missing ones drawn U(0,1) like util.jl:128-134.
Host numpy arrays go through GPAR_MEM_HOST; torch CUDA tensors (rows = points) through
GPAR_MEM_DEVICE without host copies.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import GparFitOptions, GparProblem, KERNEL_ID, context

DEFAULT_TIME_LIMIT = 1000.0  # dtc.jl:21


# ----------------------------------------------------------------------------- util.jl
def unpack_gp(params):
    """util.jl:36-43."""
    return tuple(float(np.exp(p) + 1e-3) for p in list(params)[:3])


def unpack_gpar(params):
    """util.jl:45-55."""
    return tuple(float(np.exp(p) + 1e-3) for p in list(params)[:5])


def get_time_mask(input_length):
    """util.jl:102-106."""
    m = np.zeros(input_length)
    m[0] = 1.0
    return m


def get_output_mask(input_length):
    """util.jl:111-123; DomainError for input_length <= 1."""
    if input_length <= 1:
        raise _lib.DomainError(_lib.GPAR_ERR_ARG, "Input length must be integer greater than 1")
    m = np.zeros((input_length - 1, input_length))
    for r in range(input_length - 1):
        m[r, r + 1] = 1.0
    return m


def parse_initial_params(vals, rng=None):
    """util.jl:141-169: missing initial log-params are U(0,1) draws."""
    rng = rng if rng is not None else np.random.default_rng()
    return np.array([rng.random() if v is None else float(v) for v in vals], dtype=np.float64)


def parse_initial_gp_params(i_log_l, i_log_process_var, i_log_noise_sigma, rng=None):
    """util.jl:141-147."""
    return parse_initial_params([i_log_l, i_log_process_var, i_log_noise_sigma], rng)


def parse_initial_gpar_params(i_log_time_l, i_log_time_var, i_log_out_l, i_log_out_var,
                              i_log_noise_sigma, rng=None):
    """util.jl:154-169."""
    return parse_initial_params([i_log_time_l, i_log_time_var, i_log_out_l, i_log_out_var,
                                 i_log_noise_sigma], rng)


def to_colvecs(inputs):
    """util.jl:16-31: list of per-dimension vectors -> D x N."""
    if _is_torch(inputs):
        return inputs
    if isinstance(inputs, np.ndarray):
        return np.atleast_2d(np.asarray(inputs, dtype=np.float64))
    return np.vstack([np.asarray(a, dtype=np.float64) for a in inputs])


# ----------------------------------------------------------------------------- marshalling
def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _kernel_id(k):
    if isinstance(k, int):
        return k
    return KERNEL_ID[str(k).lower()]


class _Keep(list):
    pass


def _host_vec(x, keep):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).ravel())
    keep.append(a)
    return a.ctypes.data


def _host_points(X, keep):
    """D x N (ColVecs) -> point-major N x D contiguous; returns (ptr, ld, n, d)."""
    X = to_colvecs(X)
    P = np.ascontiguousarray(X.T)
    keep.append(P)
    return P.ctypes.data, P.shape[1], P.shape[0], P.shape[1]


def _dev_points(X, keep):
    """torch CUDA tensor with rows = points (N x D, unit column stride)."""
    if X.dim() == 1:
        X = X.reshape(-1, 1)
    assert X.dtype.is_floating_point and X.element_size() == 8, "float64 tensors required"
    if X.stride(1) != 1:
        X = X.contiguous()
    keep.append(X)
    return X.data_ptr(), X.stride(0), X.shape[0], X.shape[1]


def _dev_vec(x, keep):
    x = x.contiguous()
    keep.append(x)
    return x.data_ptr()


@contextlib.contextmanager
def _after_torch(ctx, on=True):
    """Device inputs are produced on torch's current stream (a .contiguous() copy above may still
    be in flight): for the calls inside the block the library's streams wait for it, device side,
    before their kernels.  The stream is forgotten again on exit, so no later call (host-memory
    ones included) touches a handle torch may since have freed."""
    if not on:
        yield
        return
    import torch
    ctx.follow_stream(torch.cuda.current_stream(ctx.device).cuda_stream)
    try:
        yield
    finally:
        ctx.follow_stream(0, enable=False)


_MODES = {"analytic": _lib.GPAR_PREDICT_ANALYTIC, "mc": _lib.GPAR_PREDICT_MC,
          "path": _lib.GPAR_PREDICT_PATH}


def _mode_id(mode):
    """Prediction mode: "analytic" (the MC estimator's S -> infinity limit), "mc" (the reference's
    estimator, gpar_scaled_inference.jl:110-130) or "path" (tmp.jl:119-167: posterior_rand paths)."""
    if mode not in _MODES:
        raise _arg_error(f"mode must be one of {sorted(_MODES)}")
    return _MODES[mode]


def _arg_error(msg):
    return _lib.DomainError(_lib.GPAR_ERR_ARG, msg)


def make_problem(V, Z, t, y, out_kernel="matern52", time_kernel="matern52", kuu_noise=True,
                 keep=None, qu_kuu_noise=False):
    """Build a gpar_problem.  Host: V, Z as D x N / D x M (ColVecs).  Device: torch tensors
    with rows = points (N x D, M x D)."""
    keep = keep if keep is not None else _Keep()
    p = GparProblem()
    dev = _is_torch(t)
    if dev:
        p.v, p.ldv, n, d = _dev_points(V, keep)
        p.z, p.ldz, m, dz = _dev_points(Z, keep)
        p.t = _dev_vec(t, keep)
        p.y = _dev_vec(y, keep)
        p.mem = _lib.GPAR_MEM_DEVICE
        # the C side cannot see device buffer lengths: check them here
        if t.numel() != n or y.numel() != n:
            raise _arg_error("t, y and V must have the same length")
    else:
        p.v, p.ldv, n, d = _host_points(V, keep)
        p.z, p.ldz, m, dz = _host_points(Z, keep)
        p.t = _host_vec(t, keep)
        p.y = _host_vec(y, keep)
        p.mem = _lib.GPAR_MEM_HOST
        if len(np.asarray(t)) != n or len(np.asarray(y)) != n:
            raise _arg_error("t, y and V must have the same length")
    if d != dz:
        raise _lib.DomainError(_lib.GPAR_ERR_ARG, "V and Z must have the same dimension")
    p.n, p.m, p.d = n, m, d
    p.out_kernel = _kernel_id(out_kernel)
    p.time_kernel = _kernel_id(time_kernel)
    p.kuu_noise = 1 if kuu_noise else 0
    p.qu_kuu_noise = 1 if qu_kuu_noise else 0
    return p, keep


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


# ----------------------------------------------------------------------------- DTC objective
def compute_gpar_dtc_objective(V, Z, t, y, theta, out_kernel="matern52", time_kernel="matern52",
                               kuu_noise=True, return_A=False, device=0):
    """dtc.jl:83-128.  theta = (time_l, time_var, out_l, out_var, noise_sigma), natural units.

    Returns the DTC log marginal likelihood; with return_A=True returns (dtc, A) like the
    reference (A = chol(cov(u)).U' \\ beta', M x N)."""
    ctx = context(device)
    lib = _lib.load()
    p, keep = make_problem(V, Z, t, y, out_kernel, time_kernel, kuu_noise)
    th = np.ascontiguousarray(np.asarray(theta, dtype=np.float64).reshape(5))
    out = np.zeros(1)
    with _after_torch(ctx, p.mem == _lib.GPAR_MEM_DEVICE):
        if return_A:
            A = np.zeros((p.n, p.m))  # column-major M x N == row-major N x M
            ctx.check(lib.gpar_dtc_objective_A(ctx.h, C.byref(p), _ptr(th), _ptr(out), _ptr(A)))
            return float(out[0]), A.T.copy()
        ctx.check(lib.gpar_dtc_objective(ctx.h, C.byref(p), 1, _ptr(th), _ptr(out)))
    return float(out[0])


def dtc_objective_batch(problems, thetas, device=0):
    """Batched objective over independent outputs (one GPU round)."""
    ctx = context(device)
    lib = _lib.load()
    arr = (GparProblem * len(problems))(*problems)
    th = np.ascontiguousarray(np.asarray(thetas, dtype=np.float64).reshape(len(problems), 5))
    out = np.zeros(len(problems))
    with _after_torch(ctx, problems[0].mem == _lib.GPAR_MEM_DEVICE):
        ctx.check(lib.gpar_dtc_objective(ctx.h, arr, len(problems), _ptr(th), _ptr(out)))
    return out


def pairwise_distances(V, Z, out_kernel="matern52", device=0):
    """The distances Kfu = pairwise(k_o, V, Z) is built from (dtc.jl:104), as the fit's distance
    cache holds them (gpar_pairwise_distances): |v_k - z_c| for the Matern kernels, squared for
    EQ; N x M.  Host V / Z (D x N / D x M ColVecs) or device tensors (rows = points)."""
    ctx, lib = context(device), _lib.load()
    if _is_torch(V):
        import torch
        n = V.shape[0]
        t = torch.arange(n, dtype=torch.float64, device=V.device)
        p, keep = make_problem(V, Z, t, torch.zeros_like(t), out_kernel)
        out = torch.empty((n, p.m), dtype=torch.float64, device=V.device)
        with _after_torch(ctx):
            ctx.check(lib.gpar_pairwise_distances(ctx.h, C.byref(p), C.c_void_p(out.data_ptr())))
        return out
    n = to_colvecs(V).shape[1]
    p, keep = make_problem(V, Z, np.arange(n, dtype=np.float64), np.zeros(n), out_kernel)
    out = np.zeros((n, p.m))
    ctx.check(lib.gpar_pairwise_distances(ctx.h, C.byref(p), _ptr(out)))
    return out


# ----------------------------------------------------------------------------- fit
@dataclass
class FitResult:
    theta: np.ndarray      # P x 5 natural units
    nlml: np.ndarray       # P
    evals: np.ndarray      # P


def fit_batch(problems, log_theta0, max_evals=0, max_iterations=1000, g_tol=1e-8,
              time_limit=0.0, device=0):
    """Batched NelderMead over outputs (gpar_fit)."""
    ctx = context(device)
    lib = _lib.load()
    P = len(problems)
    arr = (GparProblem * P)(*problems)
    x0 = np.ascontiguousarray(np.asarray(log_theta0, dtype=np.float64).reshape(P, 5))
    opts = GparFitOptions(int(max_evals), int(max_iterations), float(g_tol), float(time_limit))
    theta = np.zeros((P, 5))
    nlml = np.zeros(P)
    evals = np.zeros(P, dtype=np.int32)
    with _after_torch(ctx, problems[0].mem == _lib.GPAR_MEM_DEVICE):
        ctx.check(lib.gpar_fit(ctx.h, arr, P, _ptr(x0), C.byref(opts), _ptr(theta), _ptr(nlml),
                               _ptr(evals)))
    return FitResult(theta, nlml, evals)


def fit_predict_batch(problems, log_theta0, t_star, V_stars, max_evals=0, max_iterations=1000,
                      g_tol=1e-8, time_limit=0.0, mode="analytic", samples=100, seed=0, device=0,
                      keep=None, chain=None, chain_cols=None):
    """get_gpar_scaled_predictions (gpar_scaled_inference.jl:20-136) for a batch of outputs
    (gpar_fit_predict): the batched fit, then each output's prediction at its fitted theta,
    reusing the fit's Gram at that theta for q(u) when the problem has qu_kuu_noise.

    Device problems (make_problem on torch tensors): t_star a device vector, V_stars[i] output
    i's test inputs (N* x D_i tensor, rows = points); returns (FitResult, means, stds) with
    means/stds lists of device tensors.  Host problems: numpy t_star and D_i x N* ColVecs.

    Chained inference inputs (gpar_fit_predict_chain; GPAR_scaled_examples.jl:172 feeds y2's
    predicted means to y3): `chain` is an N* x K matrix (numpy C-order array for host problems, a
    device tensor with unit column stride otherwise), `chain_cols[i]` the column output i's
    predicted mean is written to after its prediction (-1: none).  V_stars[i] = None reads output
    i's inputs from chain's first D_i columns, as they stand when its prediction runs (columns of
    earlier outputs hold their predicted means, the others what the caller put there)."""
    P = len(problems)
    keep = keep if keep is not None else _Keep()
    if chain is not None:
        if chain_cols is None or len(chain_cols) != P:
            raise _arg_error("chain_cols needs one entry per problem")
        K = chain.shape[1]
        if any(c >= K for c in chain_cols):
            raise _arg_error("chain_cols entries must be < chain.shape[1]")
        if _is_torch(chain):
            if chain.stride(1) != 1 or chain.dtype != __import__("torch").float64:
                raise _arg_error("chain must be a float64 tensor with unit column stride")
            chain_ptr, ld_chain = chain.data_ptr(), chain.stride(0)
        else:
            if not (isinstance(chain, np.ndarray) and chain.dtype == np.float64 and chain.flags.c_contiguous):
                raise _arg_error("chain must be a C-contiguous float64 numpy array")
            chain_ptr, ld_chain = chain.ctypes.data, K
    elif any(v is None for v in V_stars):
        raise _arg_error("V_stars[i] = None needs a chain")
    arr = (GparProblem * P)(*problems)
    x0 = np.ascontiguousarray(np.asarray(log_theta0, dtype=np.float64).reshape(P, 5))
    opts = GparFitOptions(int(max_evals), int(max_iterations), float(g_tol), float(time_limit))
    theta = np.zeros((P, 5))
    nlml = np.zeros(P)
    evals = np.zeros(P, dtype=np.int32)
    dev = problems[0].mem == _lib.GPAR_MEM_DEVICE
    vptr, ldvs, means, stds = [], [], [], []
    if len(V_stars) != P:
        raise _arg_error("one V_star per problem")
    n_star = t_star.numel() if dev else len(np.asarray(t_star))
    if dev:
        import torch
        tsp = _dev_vec(t_star, keep)
        for i, Vs in enumerate(V_stars):
            if Vs is None:
                Vs = chain[:, : problems[i].d]
            p_, ld_, ns, ds = _dev_points(Vs, keep)
            if ns != n_star or ds != problems[i].d:
                raise _arg_error(f"V_stars[{i}] must be N* x D = {n_star} x {problems[i].d}")
            vptr.append(p_)
            ldvs.append(ld_)
            means.append(torch.empty(ns, dtype=torch.float64, device=t_star.device))
            stds.append(torch.empty(ns, dtype=torch.float64, device=t_star.device))
        mp_ = [m.data_ptr() for m in means]
        sp_ = [x.data_ptr() for x in stds]
    else:
        tsp = _host_vec(t_star, keep)
        for i, Vs in enumerate(V_stars):
            if Vs is None:   # read in place from the chain (aliasing is the point)
                if problems[i].d > chain.shape[1] or chain.shape[0] != n_star:
                    raise _arg_error(f"chain must be N* x K with K >= D_{i}")
                p_, ld_, ns, ds = chain.ctypes.data, chain.shape[1], chain.shape[0], problems[i].d
            else:
                p_, ld_, ns, ds = _host_points(Vs, keep)
            if ns != n_star or ds != problems[i].d:
                raise _arg_error(f"V_stars[{i}] must be D x N* = {problems[i].d} x {n_star}")
            vptr.append(p_)
            ldvs.append(ld_)
            means.append(np.zeros(ns))
            stds.append(np.zeros(ns))
        mp_ = [m.ctypes.data for m in means]
        sp_ = [x.ctypes.data for x in stds]
    ns = n_star
    ctx, lib = context(device), _lib.load()
    VP = (C.c_void_p * P)(*vptr)
    LD = (C.c_int64 * P)(*ldvs)
    MP = (C.c_void_p * P)(*mp_)
    SP = (C.c_void_p * P)(*sp_)
    md = _mode_id(mode)
    if chain is not None and dev and chain.shape[0] != n_star:
        raise _arg_error("chain must have N* rows")
    with _after_torch(ctx, dev):
        if chain is None:
            ctx.check(lib.gpar_fit_predict(ctx.h, arr, P, _ptr(x0), C.byref(opts), ns, tsp, VP, LD,
                                           md, int(samples), int(seed), _ptr(theta), _ptr(nlml),
                                           _ptr(evals), MP, SP))
        else:
            CC = (C.c_int32 * P)(*[int(c) for c in chain_cols])
            ctx.check(lib.gpar_fit_predict_chain(ctx.h, arr, P, _ptr(x0), C.byref(opts), ns, tsp, VP,
                                                 LD, md, int(samples), int(seed),
                                                 C.c_void_p(chain_ptr), int(ld_chain), CC,
                                                 _ptr(theta), _ptr(nlml), _ptr(evals), MP, SP))
    return FitResult(theta, nlml, evals), means, stds


def get_gpar_scaled_predictions_batch(Y, pseudo_input_locations, time_loc, inference_time_loc, F,
                                      chained=False, log_theta0=(0.0, 0.0, 0.0, 0.0, -2.0),
                                      max_evals=0, g_tol=1e-8, time_limit=0.0, mode="analytic",
                                      samples=100, seed=0, qu_kuu_noise=False, device=0):
    """The Julia shim's matrix-form batch driver (julia/GPARatScaleHIP.jl): GPAR's per-output loop
    (GPAR_scaled_examples.jl:132-175) for outputs 2..P of the host matrix Y (N x P, column i =
    output i; output i's inputs are columns 1..i-1), ONE matrix passed for every output's inputs
    (ldv = P; the library uploads it once) and one for the inference inputs F (N* x P; output i
    reads its first i - 1 columns, given or -- chained -- F's column 1 then predicted means).
    pseudo_input_locations[i - 2]: output i's D x M pseudo-inputs.  Returns (FitResult, means,
    stds) for outputs 2..P.

    Defaults differ from the Julia method on purpose, so that a call is reproducible: here
    mode="analytic" (Julia: mode=:mc, the reference's estimator), seed=0 (Julia: rand(UInt64)), a
    fixed log_theta0 (Julia: parse_initial_gpar_params, U(0,1) draws for missing values, util.jl:
    128-134) and no time limit (Julia: optimization_time_limit=1000.0, dtc.jl:21).  Pass
    mode="mc", a seed, log_theta0 and time_limit to reproduce a Julia call."""
    Y = np.ascontiguousarray(np.asarray(Y, dtype=np.float64))
    F = np.ascontiguousarray(np.array(F, dtype=np.float64))   # a copy: the chain writes into it
    n, P = Y.shape
    ns = F.shape[0]
    t = np.ascontiguousarray(np.asarray(time_loc, dtype=np.float64))
    ts = np.ascontiguousarray(np.asarray(inference_time_loc, dtype=np.float64))
    if P < 2 or F.shape[1] != P or len(t) != n or len(ts) != ns:
        raise _arg_error("Y (N x P), F (N* x P), time_loc (N), inference_time_loc (N*) disagree")
    if len(pseudo_input_locations) != P - 1:
        raise _arg_error("one pseudo-input set per output 2..P")
    keep = _Keep([Y, F, t, ts])
    probs = []
    for i in range(2, P + 1):
        p = GparProblem()
        p.z, p.ldz, m, dz = _host_points(pseudo_input_locations[i - 2], keep)
        if dz != i - 1:
            raise _arg_error(f"output {i}'s pseudo-inputs must have {i - 1} rows")
        p.n, p.m, p.d = n, m, i - 1
        p.t, p.v, p.ldv = t.ctypes.data, Y.ctypes.data, P
        p.y = _host_vec(Y[:, i - 1], keep)
        p.out_kernel = p.time_kernel = KERNEL_ID["matern52"]
        p.kuu_noise, p.mem, p.qu_kuu_noise = 1, _lib.GPAR_MEM_HOST, 1 if qu_kuu_noise else 0
        probs.append(p)
    Q = P - 1
    arr = (GparProblem * Q)(*probs)
    x0 = np.ascontiguousarray(np.tile(np.asarray(log_theta0, dtype=np.float64), (Q, 1)))
    opts = GparFitOptions(int(max_evals), 1000, float(g_tol), float(time_limit))
    theta, nlml, evals = np.zeros((Q, 5)), np.zeros(Q), np.zeros(Q, dtype=np.int32)
    means = [np.zeros(ns) for _ in range(Q)]
    stds = [np.zeros(ns) for _ in range(Q)]
    VP = (C.c_void_p * Q)(*([F.ctypes.data] * Q))
    LD = (C.c_int64 * Q)(*([P] * Q))
    MP = (C.c_void_p * Q)(*[a.ctypes.data for a in means])
    SP = (C.c_void_p * Q)(*[a.ctypes.data for a in stds])
    ctx, lib = context(device), _lib.load()
    md = _mode_id(mode)
    if chained:
        CC = (C.c_int32 * Q)(*range(1, P))
        ctx.check(lib.gpar_fit_predict_chain(ctx.h, arr, Q, _ptr(x0), C.byref(opts), ns,
                                             ts.ctypes.data, VP, LD, md, int(samples), int(seed),
                                             C.c_void_p(F.ctypes.data), P, CC, _ptr(theta),
                                             _ptr(nlml), _ptr(evals), MP, SP))
    else:
        ctx.check(lib.gpar_fit_predict(ctx.h, arr, Q, _ptr(x0), C.byref(opts), ns, ts.ctypes.data,
                                       VP, LD, md, int(samples), int(seed), _ptr(theta), _ptr(nlml),
                                       _ptr(evals), MP, SP))
    return FitResult(theta, nlml, evals), means, stds


class Posterior:
    """gpar_fit_posterior's result: the fitted theta of every output and its q(u), kept on the
    device, so that predictions whose inference inputs arrive later (the chained sweep of
    GPAR_scaled_examples.jl:172 / eeg.jl:249,274) run only the V*-dependent half of
    get_gpar_scaled_predictions (gpar_posterior_predict).  Holds the problems' buffers (`keep`)
    alive: device problems' inputs are borrowed by the posterior."""

    def __init__(self, handle, fit, problems, keep, device):
        self.h, self.fit, self.device = handle, fit, device
        self._problems, self._keep = list(problems), keep
        self._prepared = {}   # output -> the t_star tensor a pending prepare reads

    @property
    def theta(self):
        return self.fit.theta

    def predict(self, i, t_star, V_star, mode="analytic", samples=100, seed=0):
        """Output i's (mean, std) at (t_star, V_star): device tensors (V_star N* x D, rows =
        points) for device problems, numpy (D x N* ColVecs) for host ones."""
        if not 0 <= int(i) < len(self._problems):
            raise _arg_error(f"output index {i} out of range (0..{len(self._problems) - 1})")
        p = self._problems[i]
        keep = _Keep()
        ctx, lib = context(self.device), _lib.load()
        md = _mode_id(mode)
        if p.mem == _lib.GPAR_MEM_DEVICE:
            import torch
            vsp, ldvs, ns, ds = _dev_points(V_star, keep)
            tsp = _dev_vec(t_star, keep)
            if ns != t_star.numel() or ds != p.d:
                raise _arg_error("inference inputs must be N* x D with N* = len(t_star)")
            mean = torch.empty(ns, dtype=torch.float64, device=t_star.device)
            std = torch.empty(ns, dtype=torch.float64, device=t_star.device)
            with _after_torch(ctx):
                ctx.check(lib.gpar_posterior_predict(ctx.h, self.h, int(i), ns, tsp, vsp, ldvs, md,
                                                     int(samples), int(seed), mean.data_ptr(),
                                                     std.data_ptr()))
            # the prepared slot is consumed (stream-ordered before any later use of the memory)
            self._prepared.pop(int(i), None)
            return mean, std
        vsp, ldvs, ns, ds = _host_points(V_star, keep)
        if ds != p.d or ns != len(np.asarray(t_star)):
            raise _arg_error("inference inputs must be D x N* with N* = len(t_star)")
        mean, std = np.zeros(ns), np.zeros(ns)
        ctx.check(lib.gpar_posterior_predict(ctx.h, self.h, int(i), ns, _host_vec(t_star, keep), vsp,
                                             ldvs, md, int(samples), int(seed), _ptr(mean), _ptr(std)))
        return mean, std

    def prepare(self, i, t_star):
        """Queue output i's inference-input-independent prediction work for device test times
        t_star (gpar_posterior_prepare) on the context's side stream; the next predict(i, t_star,
        ...) with the same tensor uses it.  Device problems only.  The queued kernels read t_star
        asynchronously, so it must be contiguous (no temporary copy) and must not be freed or
        written until that predict has run: the Posterior holds a reference to it until then."""
        if not 0 <= int(i) < len(self._problems):
            raise _arg_error(f"output index {i} out of range (0..{len(self._problems) - 1})")
        if self._problems[i].mem != _lib.GPAR_MEM_DEVICE:
            raise _arg_error("prepare: device-memory posteriors only")
        if not t_star.is_contiguous():
            raise _arg_error("prepare: t_star must be a contiguous device tensor (the prepared "
                             "kernels read it after this call returns)")
        ctx, lib = context(self.device), _lib.load()
        with _after_torch(ctx):
            ctx.check(lib.gpar_posterior_prepare(ctx.h, self.h, int(i), t_star.numel(),
                                                 t_star.data_ptr()))
        # alive until the matching predict (two slots per context: at most two pending)
        self._prepared[int(i)] = t_star
        while len(self._prepared) > 2:
            self._prepared.pop(next(iter(self._prepared)))

    def close(self):
        if getattr(self, "h", None):
            _lib.load().gpar_posterior_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fit_posterior(problems, log_theta0, max_evals=0, max_iterations=1000, g_tol=1e-8,
                  time_limit=0.0, device=0, keep=None):
    """The fit and q(u) of get_gpar_scaled_predictions for a batch of outputs, kept on the device
    for later predictions (gpar_fit_posterior) -> Posterior.

    Device problems' buffers are borrowed by the posterior until it is closed, so their `keep`
    (the second value make_problem returns: the contiguous copies and columns the problems point
    at) is required and held by the Posterior.  Host problems are copied to the device."""
    ctx, lib = context(device), _lib.load()
    P = len(problems)
    if keep is None and any(p.mem == _lib.GPAR_MEM_DEVICE for p in problems):
        raise _arg_error("fit_posterior: device problems need their keep (make_problem's second "
                         "value): the posterior reads those buffers until it is closed")
    arr = (GparProblem * P)(*problems)
    x0 = np.ascontiguousarray(np.asarray(log_theta0, dtype=np.float64).reshape(P, 5))
    opts = GparFitOptions(int(max_evals), int(max_iterations), float(g_tol), float(time_limit))
    theta, nlml, evals = np.zeros((P, 5)), np.zeros(P), np.zeros(P, dtype=np.int32)
    h = C.c_void_p()
    with _after_torch(ctx, problems[0].mem == _lib.GPAR_MEM_DEVICE):
        ctx.check(lib.gpar_fit_posterior(ctx.h, arr, P, _ptr(x0), C.byref(opts), _ptr(theta),
                                         _ptr(nlml), _ptr(evals), C.byref(h)))
    return Posterior(h, FitResult(theta, nlml, evals), problems, keep, device)


def mc_normals(samples, m, seed, device=0):
    """The standard-normal draws MC-mode prediction uses for (samples, m, seed), samples x m
    (gpar_mc_normals): draw s maps to the pseudo-point sample m_e + chol(inv(D)).L xi_s
    (gpar_scaled_inference.jl:103,185).  fit_predict_batch draws output i with seed + i."""
    ctx = context(device)
    xi = np.zeros((int(samples), int(m)))
    ctx.check(_lib.load().gpar_mc_normals(ctx.h, int(samples), int(m), int(seed), _ptr(xi)))
    return xi


def path_normals(samples, n, d, seed, device=0):
    """The backward-sampling draws of posterior_rand / mode="path" for (samples, n, d, seed):
    samples x n x d (gpar_path_normals)."""
    ctx = context(device)
    xi = np.zeros((int(samples), int(n), int(d)))
    ctx.check(_lib.load().gpar_path_normals(ctx.h, int(samples), int(n), int(d), int(seed), _ptr(xi)))
    return xi


def posterior_rand(t, y, theta, kernel="matern52", samples=1, seed=0, noise=None, device=0):
    """TemporalGPs posterior_rand(rng, create_lgssm(t, l, pv, sigma, k; noise_vector), y, samples)
    (called at src/gp/tmp.jl:161-167): joint draws of the latent f over t from its posterior given
    y, by the Durbin-Koopman simulation smoother (gpar_lgssm_posterior_rand).  theta = (l,
    process_var, noise_sigma); noise: per-step observation variance (None: sigma^2).  Host arrays
    -> samples x n numpy array; torch CUDA tensors -> samples x n device tensor."""
    ctx, lib = context(device), _lib.load()
    th = np.ascontiguousarray(np.asarray(theta, dtype=np.float64).reshape(3))
    keep = _Keep()
    if _is_torch(t):
        import torch
        n = t.numel()
        # the C side cannot see device buffer lengths (as make_problem checks for the GPAR inputs)
        if y.numel() != n or (noise is not None and noise.numel() != n):
            raise _arg_error("t, y (and noise) must have the same length")
        out = torch.empty((int(samples), n), dtype=torch.float64, device=t.device)
        tp, yp = _dev_vec(t, keep), _dev_vec(y, keep)
        npp = _dev_vec(noise, keep) if noise is not None else None
        with _after_torch(ctx):
            ctx.check(lib.gpar_lgssm_posterior_rand(ctx.h, n, tp, yp, npp, _kernel_id(kernel),
                                                    _ptr(th), int(samples), int(seed),
                                                    _lib.GPAR_MEM_DEVICE, out.data_ptr()))
        return out
    n = len(np.asarray(t))
    if len(np.asarray(y)) != n or (noise is not None and len(np.asarray(noise)) != n):
        raise _arg_error("t, y (and noise) must have the same length")
    out = np.zeros((int(samples), n))
    ctx.check(lib.gpar_lgssm_posterior_rand(ctx.h, n, _host_vec(t, keep), _host_vec(y, keep),
                                            _host_vec(noise, keep) if noise is not None else None,
                                            _kernel_id(kernel), _ptr(th), int(samples), int(seed),
                                            _lib.GPAR_MEM_HOST, _ptr(out)))
    return out


def get_optim_scaled_gpar_params(input_locations, pseudo_input_locations, time_loc, outputs,
                                 out_kernel="matern52", time_kernel="matern52",
                                 i_log_time_l=None, i_log_time_var=None, i_log_out_l=None,
                                 i_log_out_var=None, i_log_noise_sigma=None,
                                 optimization_time_limit=DEFAULT_TIME_LIMIT, max_evals=0,
                                 g_tol=1e-8, rng=None, device=0):
    """dtc.jl:11-77: returns the optimised (time_l, time_var, out_l, out_var, noise_sigma)."""
    p, keep = make_problem(input_locations, pseudo_input_locations, time_loc, outputs,
                           out_kernel, time_kernel)
    x0 = parse_initial_params([i_log_time_l, i_log_time_var, i_log_out_l, i_log_out_var,
                               i_log_noise_sigma], rng)
    r = fit_batch([p], x0[None, :], max_evals=max_evals, g_tol=g_tol,
                  time_limit=optimization_time_limit or 0.0, device=device)
    return tuple(float(v) for v in r.theta[0])


# ----------------------------------------------------------------------------- q(u)
def compute_q_u(input_locations, pseudo_input_locations, time_loc, outputs, theta,
                out_kernel="matern52", time_kernel="matern52", device=0, qu_kuu_noise=False):
    """gpar_scaled_inference.jl:141-196 -> (m_e, cov_e = inv(D), U_u upper).  qu_kuu_noise:
    Cuu + sigma^2 I instead of the reference's noise-free Cuu (:157), as gpar_problem documents."""
    ctx = context(device)
    lib = _lib.load()
    p, keep = make_problem(input_locations, pseudo_input_locations, time_loc, outputs,
                           out_kernel, time_kernel, qu_kuu_noise=qu_kuu_noise)
    th = np.ascontiguousarray(np.asarray(theta, dtype=np.float64).reshape(5))
    m = p.m
    me = np.zeros(m)
    cov = np.zeros((m, m))
    U = np.zeros((m, m))  # column-major -> read as transposed
    with _after_torch(ctx, p.mem == _lib.GPAR_MEM_DEVICE):
        ctx.check(lib.gpar_q_u(ctx.h, C.byref(p), _ptr(th), _ptr(me), _ptr(cov), _ptr(U)))
    return me, cov, U.T.copy()


# ----------------------------------------------------------------------------- temporal-only
@dataclass
class LGSSMSpec:
    """create_lgssm(t, l, process_var, noise_sigma, k) (temporal_gp_inference.jl:15-39)."""
    t: np.ndarray
    l: float
    process_var: float
    noise_sigma: float
    kernel: str = "matern52"


def create_lgssm(latent_locations, l, process_var, noise_sigma, kernel_structure="matern52"):
    return LGSSMSpec(np.asarray(latent_locations, dtype=np.float64), float(l), float(process_var),
                     float(noise_sigma), kernel_structure)


def logpdf(lgssm: LGSSMSpec, y, device=0):
    """logpdf(lgssm, y) (temporal_gp_inference.jl:78)."""
    return float(lgssm_logpdf_batch(lgssm.t, np.asarray(y, dtype=np.float64)[None, :],
                                    [[lgssm.l, lgssm.process_var, lgssm.noise_sigma]],
                                    lgssm.kernel, device)[0])


def lgssm_logpdf_batch(t, Y, theta, kernel="matern52", device=0):
    """Chains sharing t: Y is nchains x n; theta nchains x 3 natural (l, pv, sigma)."""
    ctx = context(device)
    lib = _lib.load()
    keep = _Keep()
    Y = np.ascontiguousarray(np.asarray(Y, dtype=np.float64))
    nch, n = Y.shape
    th = np.ascontiguousarray(np.asarray(theta, dtype=np.float64).reshape(nch, 3))
    tp = _host_vec(t, keep)
    out = np.zeros(nch)
    ctx.check(lib.gpar_lgssm_logpdf(ctx.h, nch, n, tp, _ptr(Y), n, _kernel_id(kernel), _ptr(th),
                                    _lib.GPAR_MEM_HOST, _ptr(out)))
    return out


# ----------------------------------------------------------------------------- prediction
def predict_scaled(input_locations, pseudo_input_locations, time_loc, outputs, theta,
                   inference_time_loc, inference_input_locations, out_kernel="matern52",
                   time_kernel="matern52", mode="analytic", samples=100, seed=0, device=0,
                   qu_kuu_noise=False):
    """Prediction half of get_gpar_scaled_predictions (gpar_scaled_inference.jl:63-135) at a
    given theta.  Returns (mean, std) at the inference locations, in their input order.
    mode="mc" reproduces the reference's 100-sample Monte Carlo estimator; "analytic" is its
    S -> infinity limit."""
    p, keep = make_problem(input_locations, pseudo_input_locations, time_loc, outputs,
                           out_kernel, time_kernel, qu_kuu_noise=qu_kuu_noise)
    th = np.ascontiguousarray(np.asarray(theta, dtype=np.float64).reshape(5))
    md = _mode_id(mode)
    if p.mem == _lib.GPAR_MEM_DEVICE:
        import torch
        vsp, ldvs, ns, ds = _dev_points(inference_input_locations, keep)
        tsp = _dev_vec(inference_time_loc, keep)
        if ns != inference_time_loc.numel() or ds != p.d:
            raise _arg_error("inference inputs must be N* x D with N* = len(inference_time_loc)")
        ctx, lib = context(device), _lib.load()
        mean = torch.empty(ns, dtype=torch.float64, device=inference_time_loc.device)
        std = torch.empty(ns, dtype=torch.float64, device=inference_time_loc.device)
        with _after_torch(ctx):
            ctx.check(lib.gpar_predict(ctx.h, C.byref(p), _ptr(th), ns, tsp, vsp, ldvs, md,
                                       int(samples), int(seed), mean.data_ptr(), std.data_ptr()))
        return mean, std
    vsp, ldvs, ns, ds = _host_points(inference_input_locations, keep)
    tsp = _host_vec(inference_time_loc, keep)
    if ds != p.d or ns != len(np.asarray(inference_time_loc)):
        raise _arg_error("inference inputs must have the training dimension and one point per "
                         "inference time")
    ctx, lib = context(device), _lib.load()
    mean = np.zeros(ns)
    std = np.zeros(ns)
    ctx.check(lib.gpar_predict(ctx.h, C.byref(p), _ptr(th), ns, tsp, vsp, ldvs, md, int(samples),
                               int(seed), _ptr(mean), _ptr(std)))
    return mean, std


def get_gpar_scaled_predictions(input_locations, pseudo_input_locations, time_loc, outputs,
                                inference_time_loc, inference_input_locations,
                                out_kernel_structure="matern52", time_kernel_structure="matern52",
                                i_log_time_l=None, i_log_time_var=None, i_log_out_l=None,
                                i_log_out_var=None, i_log_noise_sigma=None,
                                optimization_time_limit=DEFAULT_TIME_LIMIT, max_evals=0,
                                mode="mc", samples=100, seed=0, rng=None, device=0):
    """gpar_scaled_inference.jl:20-136: fit theta (Matern52 hard-coded for the fit, :48-49),
    then predict; returns (mean, std) like the reference."""
    theta = get_optim_scaled_gpar_params(
        input_locations, pseudo_input_locations, time_loc, outputs, "matern52", "matern52",
        i_log_time_l, i_log_time_var, i_log_out_l, i_log_out_var, i_log_noise_sigma,
        optimization_time_limit, max_evals, rng=rng, device=device)
    return predict_scaled(input_locations, pseudo_input_locations, time_loc, outputs, theta,
                          inference_time_loc, inference_input_locations, out_kernel_structure,
                          time_kernel_structure, mode, samples, seed, device)


def lgssm_smooth_batch(t, Y, theta, kernel="matern52", noise=None, device=0):
    """smooth(create_lgssm(...; noise_vector), y) marginals of f for chains sharing t
    (temporal_gp_inference.jl:109): returns (mean, var), nchains x n."""
    ctx = context(device)
    lib = _lib.load()
    keep = _Keep()
    Y = np.ascontiguousarray(np.atleast_2d(np.asarray(Y, dtype=np.float64)))
    nch, n = Y.shape
    th = np.ascontiguousarray(np.asarray(theta, dtype=np.float64).reshape(nch, 3))
    tp = _host_vec(t, keep)
    npp = _host_vec(noise, keep) if noise is not None else None
    mean = np.zeros((nch, n))
    var = np.zeros((nch, n))
    ctx.check(lib.gpar_lgssm_smooth(ctx.h, nch, n, tp, _ptr(Y), n, npp, _kernel_id(kernel),
                                    _ptr(th), _lib.GPAR_MEM_HOST, _ptr(mean), _ptr(var)))
    return mean, var


def get_sde_predictions(data_locations, data_outputs, output_locations,
                        kernel_structure="matern52", i_log_time_l=None, i_log_time_var=None,
                        i_log_noise_sigma=None, max_evals=0, g_tol=1e-8, time_limit=0.0,
                        rng=None, device=0):
    """temporal_gp_inference.jl:45-114 for one or several chains sharing the time grid.

    data_outputs: n (one chain) or nchains x n.  Returns (theta, mean, var) with the
    marginals of f at output_locations (the reference returns their Gaussians; its
    `.m[1]` / `.P[1]` are mean / variance)."""
    ctx = context(device)
    lib = _lib.load()
    keep = _Keep()
    Y = np.ascontiguousarray(np.atleast_2d(np.asarray(data_outputs, dtype=np.float64)))
    nch, n = Y.shape
    x0 = np.vstack([parse_initial_params([i_log_time_l, i_log_time_var, i_log_noise_sigma], rng)
                    for _ in range(nch)])
    x0 = np.ascontiguousarray(x0)
    ts = np.asarray(output_locations, dtype=np.float64)
    tp = _host_vec(data_locations, keep)
    tsp = _host_vec(ts, keep)
    opts = GparFitOptions(int(max_evals), 1000, float(g_tol), float(time_limit))
    theta = np.zeros((nch, 3))
    mean = np.zeros((nch, len(ts)))
    var = np.zeros((nch, len(ts)))
    ctx.check(lib.gpar_sde_predictions(ctx.h, nch, n, tp, _ptr(Y), n, len(ts), tsp,
                                       _kernel_id(kernel_structure), _ptr(x0), C.byref(opts),
                                       _lib.GPAR_MEM_HOST, _ptr(theta), _ptr(mean), _ptr(var)))
    if nch == 1:
        return tuple(theta[0]), mean[0], var[0]
    return theta, mean, var


def get_sde_predictions_device(t, Y, t_star, kernel_structure="matern52", log_theta0=(0.0, 0.0, -2.0),
                               max_evals=0, g_tol=-1.0, time_limit=0.0, device=0):
    """get_sde_predictions with HBM-resident torch inputs: t (n), Y (n) or (nchains x n,
    contiguous rows), t_star (n_star, ascending).  Returns (theta, mean, var) on the device."""
    import torch
    ctx = context(device)
    lib = _lib.load()
    keep = _Keep()
    Y2 = Y.reshape(1, -1) if Y.dim() == 1 else Y
    Y2 = Y2.contiguous()
    nch, n = Y2.shape
    x0 = np.ascontiguousarray(np.tile(np.asarray(log_theta0, dtype=np.float64), (nch, 1)))
    opts = GparFitOptions(int(max_evals), 1000, float(g_tol), float(time_limit))
    theta = np.zeros((nch, 3))
    ns = t_star.shape[0]
    mean = torch.empty((nch, ns), dtype=torch.float64, device=t.device)
    var = torch.empty((nch, ns), dtype=torch.float64, device=t.device)
    if t.numel() != n:
        raise _arg_error("t and Y must have the same length")
    ts_ = _dev_vec(t_star, keep)
    tt_ = _dev_vec(t, keep)
    with _after_torch(ctx):
        ctx.check(lib.gpar_sde_predictions(ctx.h, nch, n, tt_, Y2.data_ptr(), n, ns,
                                           ts_, _kernel_id(kernel_structure),
                                           _ptr(x0), C.byref(opts), _lib.GPAR_MEM_DEVICE,
                                           _ptr(theta), mean.data_ptr(), var.data_ptr()))
    if nch == 1:
        return tuple(theta[0]), mean[0], var[0]
    return theta, mean, var


# ----------------------------------------------------------------------------- exact GP / GPAR
def _theta5(theta, dx):
    th = np.asarray(theta, dtype=np.float64).ravel()
    if dx == 1 and th.shape[0] == 3:        # unpack_gp order (l, process_var, noise_sigma)
        th = np.array([th[0], th[1], 1.0, 1.0, th[2]])
    return np.ascontiguousarray(th.reshape(5))


def exact_logpdf(X, y, theta, time_kernel="eq", out_kernel="eq", device=0):
    """logpdf(f(x, sigma^2), y) of the exact GP (dx == 1, optimized.jl:28-36, theta =
    (l, process_var, noise_sigma)) or GPAR (optimized.jl:132-154, theta = unpack_gpar order).
    X: 1-D times or ColVecs dx x n with row 0 = time."""
    ctx = context(device)
    keep = _Keep()
    xp, ldx, n, dx = _host_points(X, keep)
    th = _theta5(theta, dx)
    out = np.zeros(1)
    ctx.check(_lib.load().gpar_exact_logpdf(ctx.h, n, dx, xp, ldx, _host_vec(y, keep),
                                            _kernel_id(time_kernel), _kernel_id(out_kernel),
                                            _ptr(th), _lib.GPAR_MEM_HOST, _ptr(out)))
    return float(out[0])


def exact_posterior(X, y, X_star, theta, time_kernel="eq", out_kernel="eq", device=0):
    """Marginals (mean, var) of f at X_star under the exact posterior
    gp | (gp(x, sigma^2) <- y)  (optimized.jl:94,236)."""
    ctx = context(device)
    keep = _Keep()
    xp, ldx, n, dx = _host_points(X, keep)
    sp, ldxs, ns, dxs = _host_points(X_star, keep)
    if dxs != dx:
        raise _lib.DomainError(_lib.GPAR_ERR_ARG, "X_star must have the dimension of X")
    th = _theta5(theta, dx)
    mean = np.zeros(ns)
    var = np.zeros(ns)
    ctx.check(_lib.load().gpar_exact_posterior(ctx.h, n, dx, xp, ldx, _host_vec(y, keep), ns, sp,
                                               ldxs, _kernel_id(time_kernel), _kernel_id(out_kernel),
                                               _ptr(th), _lib.GPAR_MEM_HOST, _ptr(mean), _ptr(var)))
    return mean, var


@dataclass
class ExactGP:
    """Result of create_optim_gp[ar]: the fitted kernel (the reference returns the Stheno GP
    and opt_params)."""
    X: np.ndarray
    y: np.ndarray
    theta: tuple
    time_kernel: str
    out_kernel: str
    device: int = 0

    def logpdf(self):
        return exact_logpdf(self.X, self.y, self.theta, self.time_kernel, self.out_kernel, self.device)

    def marginals(self, X_star):
        """Posterior marginals (mean, var) at X_star: the create_optim_gp[ar]_post posterior."""
        return exact_posterior(self.X, self.y, X_star, self.theta, self.time_kernel,
                               self.out_kernel, self.device)


def _nm_fit(nlml, x0, max_evals):
    nm = _lib.NelderMead(x0, max_evals=max_evals)
    while (x := nm.ask()) is not None:
        try:
            f = nlml(x)
        except _lib.PosDefException:
            f = np.inf
        nm.tell(f)
    return nm.result()[0]


def create_optim_gp(input_locations, outputs, kernel_structure="eq", i_log_l=None,
                    i_log_process_var=None, i_log_noise_sigma=None, max_evals=0, rng=None, device=0):
    """optimized.jl:19-59: NelderMead on -logpdf over (l, process_var, noise_sigma);
    returns (ExactGP, opt_params)."""
    x = np.asarray(input_locations, dtype=np.float64).ravel()
    y = np.asarray(outputs, dtype=np.float64)
    x0 = parse_initial_params([i_log_l, i_log_process_var, i_log_noise_sigma], rng)
    xm = _nm_fit(lambda p: -exact_logpdf(x, y, unpack_gp(p), kernel_structure, device=device),
                 x0, max_evals)
    th = unpack_gp(xm)
    return ExactGP(x, y, th, kernel_structure, kernel_structure, device), th


def create_optim_gpar(input_locations, outputs, time_kernel="eq", out_kernel="eq",
                      i_log_time_l=None, i_log_time_var=None, i_log_out_l=None,
                      i_log_out_var=None, i_log_noise_sigma=None, multi_input=True, max_evals=0,
                      rng=None, device=0):
    """optimized.jl:106-183 (multi_input=False falls back to create_optim_gp, :118-127)."""
    if not multi_input:
        return create_optim_gp(input_locations, outputs, time_kernel, i_log_time_l, i_log_time_var,
                               i_log_noise_sigma, max_evals, rng, device)
    X = to_colvecs(input_locations)
    y = np.asarray(outputs, dtype=np.float64)
    x0 = parse_initial_params([i_log_time_l, i_log_time_var, i_log_out_l, i_log_out_var,
                               i_log_noise_sigma], rng)
    xm = _nm_fit(lambda p: -exact_logpdf(X, y, unpack_gpar(p), time_kernel, out_kernel, device),
                 x0, max_evals)
    th = unpack_gpar(xm)
    return ExactGP(X, y, th, time_kernel, out_kernel, device), th


def create_optim_gp_post(input_locations, outputs, kernel_structure="eq", **kw):
    """optimized.jl:76-97: the fitted GP conditioned on the data (use .marginals(x_star))."""
    return create_optim_gp(input_locations, outputs, kernel_structure, **kw)[0]


def create_optim_gpar_post(input_locations, outputs, time_kernel="eq", out_kernel="eq", **kw):
    """optimized.jl:201-239."""
    return create_optim_gpar(input_locations, outputs, time_kernel, out_kernel, **kw)[0]
