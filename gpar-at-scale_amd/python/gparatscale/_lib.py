"""ctypes binding of include/gpar_hip.h (libgparhip.so, built in-tree for gfx950).

The product path: every numeric result comes from the gfx950 kernels behind this C-ABI.
If the shared library is missing or no GPU is visible, calls raise -- there is no CPU
fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "libgparhip.so"))

GPAR_OK, GPAR_ERR_ARG, GPAR_ERR_NOT_PD, GPAR_ERR_HIP, GPAR_ERR_OOM, GPAR_ERR_UNSUPPORTED, GPAR_ERR_STATE = range(7)
GPAR_MEM_HOST, GPAR_MEM_DEVICE = 0, 1
GPAR_PREDICT_ANALYTIC, GPAR_PREDICT_MC, GPAR_PREDICT_PATH = 0, 1, 2
KERNEL_ID = {"matern12": 0, "matern32": 1, "matern52": 2, "eq": 3}

# Every entry point include/gpar_hip.h declares (tests check the library exports them all).
EXPORTED = (
    "gpar_abi_version", "gpar_ctx_create", "gpar_ctx_destroy", "gpar_last_error",
    "gpar_ctx_workspace_bytes", "gpar_ctx_trim", "gpar_dtc_objective", "gpar_dtc_objective_A",
    "gpar_fit", "gpar_fit_predict", "gpar_fit_predict_chain", "gpar_mc_normals", "gpar_path_normals", "gpar_lgssm_posterior_rand", "gpar_q_u", "gpar_predict", "gpar_lgssm_logpdf", "gpar_lgssm_smooth",
    "gpar_sde_predictions", "gpar_exact_logpdf", "gpar_exact_posterior",
    "gpar_ctx_set_profiling", "gpar_ctx_kernel_stats", "gpar_debug_counter", "gpar_ctx_kernel_work", "gpar_ctx_reset_stats",
    "gpar_ctx_set_lanes", "gpar_ctx_set_cu_split", "gpar_ctx_set_fit_overlap", "gpar_ctx_get_cu_split", "gpar_ctx_set_dist_cache", "gpar_ctx_set_dist_cache_keep", "gpar_ctx_dist_cache_stats",
    "gpar_pairwise_distances", "gpar_ctx_set_predict_fused", "gpar_ctx_set_input_stream", "gpar_ctx_set_schedule", "gpar_ctx_get_schedule",
    "gpar_fit_posterior", "gpar_posterior_predict", "gpar_posterior_prepare", "gpar_posterior_destroy",
    "gpar_nm_create", "gpar_nm_destroy", "gpar_nm_ask", "gpar_nm_tell", "gpar_nm_result",
)


class GparError(RuntimeError):
    """Generic failure of the native library (HIP error, OOM, ...)."""

    def __init__(self, code, msg):
        super().__init__(f"[gpar status {code}] {msg}")
        self.code = code


class PosDefException(GparError):
    """Mirrors Julia's LinearAlgebra.PosDefException thrown by `cholesky`
    (dtc.jl:119-120, gpar_scaled_inference.jl:159,188)."""


class DomainError(GparError, ValueError):
    """Mirrors Julia's DomainError / ArgumentError on malformed inputs (util.jl:112-117)."""


class Unsupported(GparError):
    pass


class GparProblem(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("m", C.c_int64), ("d", C.c_int64),
        ("t", C.c_void_p), ("v", C.c_void_p), ("ldv", C.c_int64),
        ("z", C.c_void_p), ("ldz", C.c_int64), ("y", C.c_void_p),
        ("out_kernel", C.c_int32), ("time_kernel", C.c_int32), ("kuu_noise", C.c_int32),
        ("mem", C.c_int32), ("qu_kuu_noise", C.c_int32),
    ]


class GparFitOptions(C.Structure):
    _fields_ = [("max_evals", C.c_int32), ("max_iterations", C.c_int32),
                ("g_tol", C.c_double), ("time_limit", C.c_double)]


_lib = None
_lock = threading.Lock()


def load(path: str | None = None):
    """Load libgparhip.so (raises OSError if it has not been built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("GPAR_HIP_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise OSError(f"libgparhip.so not found at {p}: run `make -C gpar-at-scale_amd` "
                          "(or __graft_entry__.build())")
        _torch_runtime_first()
        lib = C.CDLL(p)
        vp, i32, i64, dp = C.c_void_p, C.c_int32, C.c_int64, C.c_void_p
        sig = {
            "gpar_abi_version": (i32, []),
            "gpar_ctx_create": (i32, [i32, C.POINTER(vp)]),
            "gpar_ctx_destroy": (i32, [vp]),
            "gpar_ctx_set_predict_fused": (i32, [vp, i32]),
            "gpar_last_error": (C.c_char_p, [vp]),
            "gpar_ctx_workspace_bytes": (i64, [vp]),
            "gpar_ctx_trim": (i32, [vp]),
            "gpar_ctx_set_profiling": (i32, [vp, i32]),
            "gpar_ctx_kernel_stats": (i32, [vp, C.c_char_p, C.POINTER(i64), C.POINTER(C.c_double)]),
            "gpar_ctx_reset_stats": (i32, [vp]),
            "gpar_ctx_kernel_work": (i32, [vp, C.c_char_p, C.POINTER(C.c_double)]),
            "gpar_debug_counter": (i64, [C.c_char_p]),
            "gpar_ctx_set_lanes": (i32, [vp, i32]),
            "gpar_ctx_set_cu_split": (i32, [vp, i32]),
            "gpar_ctx_get_cu_split": (i32, [vp, C.POINTER(C.c_int32)]),
            "gpar_ctx_set_fit_overlap": (i32, [vp, i32]),
            "gpar_ctx_set_schedule": (i32, [vp, C.c_char_p, i32]),
            "gpar_ctx_get_schedule": (i32, [vp, C.c_char_p, C.POINTER(i32)]),
            "gpar_ctx_set_dist_cache": (i32, [vp, i64]),
            "gpar_ctx_set_dist_cache_keep": (i32, [vp, i32]),
            "gpar_ctx_dist_cache_stats": (i32, [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i64)]),
            "gpar_pairwise_distances": (i32, [vp, C.POINTER(GparProblem), dp]),
            "gpar_ctx_set_input_stream": (i32, [vp, vp, i32]),
            "gpar_dtc_objective": (i32, [vp, C.POINTER(GparProblem), i32, dp, dp]),
            "gpar_dtc_objective_A": (i32, [vp, C.POINTER(GparProblem), dp, dp, dp]),
            "gpar_fit": (i32, [vp, C.POINTER(GparProblem), i32, dp, C.POINTER(GparFitOptions),
                               dp, dp, dp]),
            "gpar_fit_predict": (i32, [vp, C.POINTER(GparProblem), i32, dp, C.POINTER(GparFitOptions),
                                       i64, vp, vp, vp, i32, i32, C.c_uint64, dp, dp, dp, vp, vp]),
            "gpar_fit_predict_chain": (i32, [vp, C.POINTER(GparProblem), i32, dp,
                                             C.POINTER(GparFitOptions), i64, vp, vp, vp, i32, i32,
                                             C.c_uint64, vp, i64, vp, dp, dp, dp, vp, vp]),
            "gpar_fit_posterior": (i32, [vp, C.POINTER(GparProblem), i32, dp, C.POINTER(GparFitOptions),
                                         dp, dp, dp, C.POINTER(vp)]),
            "gpar_posterior_predict": (i32, [vp, vp, i32, i64, vp, vp, i64, i32, i32, C.c_uint64,
                                             vp, vp]),
            "gpar_posterior_prepare": (i32, [vp, vp, i32, i64, vp]),
            "gpar_posterior_destroy": (i32, [vp]),
            "gpar_mc_normals": (i32, [vp, i32, i64, C.c_uint64, dp]),
            "gpar_path_normals": (i32, [vp, i32, i64, i32, C.c_uint64, dp]),
            "gpar_lgssm_posterior_rand": (i32, [vp, i64, dp, dp, dp, i32, dp, i32, C.c_uint64, i32, dp]),
            "gpar_q_u": (i32, [vp, C.POINTER(GparProblem), dp, dp, dp, dp]),
            "gpar_predict": (i32, [vp, C.POINTER(GparProblem), dp, i64, dp, dp, i64, i32, i32,
                                   C.c_uint64, dp, dp]),
            "gpar_lgssm_logpdf": (i32, [vp, i32, i64, dp, dp, i64, i32, dp, i32, dp]),
            "gpar_lgssm_smooth": (i32, [vp, i32, i64, dp, dp, i64, dp, i32, dp, i32, dp, dp]),
            "gpar_sde_predictions": (i32, [vp, i32, i64, dp, dp, i64, i64, dp, i32, dp,
                                           C.POINTER(GparFitOptions), i32, dp, dp, dp]),
            "gpar_exact_logpdf": (i32, [vp, i64, i64, dp, i64, dp, i32, i32, dp, i32, dp]),
            "gpar_exact_posterior": (i32, [vp, i64, i64, dp, i64, dp, i64, dp, i64, i32, i32,
                                           dp, i32, dp, dp]),
        }
        sig.update({
            "gpar_nm_create": (i32, [i32, dp, C.POINTER(GparFitOptions), C.POINTER(vp)]),
            "gpar_nm_destroy": (i32, [vp]),
            "gpar_nm_ask": (i32, [vp, dp]),
            "gpar_nm_tell": (i32, [vp, C.c_double]),
            "gpar_nm_result": (i32, [vp, dp, C.POINTER(C.c_double), C.POINTER(i32), C.POINTER(i32)]),
        })
        for name, (res, args) in sig.items():
            if name == "gpar_debug_counter" and not hasattr(lib, name):
                continue   # a diagnostic only: older builds (library A/B runs) lack it
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
        return lib


def raise_for(ctx, code):
    if code == GPAR_OK:
        return
    msg = load().gpar_last_error(ctx)
    msg = msg.decode() if msg else ""
    if code == GPAR_ERR_NOT_PD:
        raise PosDefException(code, msg)
    if code == GPAR_ERR_ARG:
        raise DomainError(code, msg)
    if code == GPAR_ERR_UNSUPPORTED:
        raise Unsupported(code, msg)
    raise GparError(code, msg)


def _torch_runtime_first():
    """PyTorch-ROCm bundles its own HIP runtime (torch/lib/libamdhip64.so, SONAME
    libamdhip64.so.7); this library links libamdhip64.so.7 too.  Imported first, torch's copy
    satisfies our dependency and the process holds ONE runtime, so torch streams / device pointers
    and our kernels share it.  Loaded first, ours comes from /opt/rocm and torch then loads its own
    by file name: two runtimes in one process, and whichever initialises second finds no GPU
    (measured on MI355X).  So torch, when installed, is imported before the CDLL."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def debug_counter(name):
    """A process-wide diagnostic counter of the library (gpar_debug_counter): "gains_fast" /
    "gains_general" = phase-3 gains launches by kernel path."""
    return int(load().gpar_debug_counter(name.encode()))


class Context:
    """One gpar_ctx (one GPU, one host thread)."""

    def __init__(self, device: int = 0):
        lib = load()
        h = C.c_void_p()
        code = lib.gpar_ctx_create(device, C.byref(h))
        if code != GPAR_OK:
            raise GparError(code, f"gpar_ctx_create(device={device}) failed (no GPU visible?)")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            load().gpar_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, code):
        raise_for(self.h, code)

    def workspace_bytes(self):
        return int(load().gpar_ctx_workspace_bytes(self.h))

    def set_profiling(self, on=True):
        self.check(load().gpar_ctx_set_profiling(self.h, 1 if on else 0))

    def kernel_stats(self, name):
        """(launches, total_ms) of a kernel family since the last reset (HIP events on the
        context stream)."""
        n = C.c_int64()
        ms = C.c_double()
        self.check(load().gpar_ctx_kernel_stats(self.h, name.encode(), C.byref(n), C.byref(ms)))
        return int(n.value), float(ms.value)

    def kernel_work(self, name):
        """Algorithmic work of the timed launches of a family since the last reset
        (gpar_ctx_kernel_work): flops for "gram", HBM bytes for "whiten"."""
        w = C.c_double()
        self.check(load().gpar_ctx_kernel_work(self.h, name.encode(), C.byref(w)))
        return float(w.value)

    def follow_stream(self, stream_ptr, enable=True):
        """Order every later call after the work queued on `stream_ptr` (a hipStream_t handle,
        e.g. torch.cuda.current_stream().cuda_stream) at the time of the call; enable=False
        forgets the stream again (the handle is not kept)."""
        self.check(load().gpar_ctx_set_input_stream(self.h, C.c_void_p(int(stream_ptr or 0)),
                                                    1 if enable else 0))

    def reset_stats(self):
        self.check(load().gpar_ctx_reset_stats(self.h))

    def set_dist_cache(self, nbytes=-1):
        """Byte budget of the fit's distance cache (gpar_ctx_set_dist_cache): -1 auto, 0 off."""
        self.check(load().gpar_ctx_set_dist_cache(self.h, int(nbytes)))

    def set_dist_cache_keep(self, keep=True):
        """Hold the distance cache past the fit call (gpar_ctx_set_dist_cache_keep); default off."""
        self.check(load().gpar_ctx_set_dist_cache_keep(self.h, 1 if keep else 0))

    def dist_cache_stats(self):
        """(outputs cached by the last fit, OOM evictions so far, cache bytes held now)."""
        o, e, b = C.c_int32(), C.c_int32(), C.c_int64()
        self.check(load().gpar_ctx_dist_cache_stats(self.h, C.byref(o), C.byref(e), C.byref(b)))
        return int(o.value), int(e.value), int(b.value)

    def trim(self):
        """Release the context's device workspace (gpar_ctx_trim)."""
        self.check(load().gpar_ctx_trim(self.h))

    def set_lanes(self, lanes):
        """1 (the default): serial batched evaluation; 2: outputs alternate over two HIP streams."""
        self.check(load().gpar_ctx_set_lanes(self.h, int(lanes)))

    def set_cu_split(self, cus_per_xcd):
        """CUs per XCD for the batched fit's whitening beside the Gram (0: whole-chip kernels)."""
        self.check(load().gpar_ctx_set_cu_split(self.h, int(cus_per_xcd)))
        self._cu_split = int(cus_per_xcd)

    def set_fit_overlap(self, on=True):
        """Round-overlapping batched fit on the CU split (gpar_ctx_set_fit_overlap; default on)."""
        self.check(load().gpar_ctx_set_fit_overlap(self.h, 1 if on else 0))

    def set_predict_fused(self, on=True):
        """Fused rows + variance kernel of the ANALYTIC prediction (gpar_ctx_set_predict_fused;
        default on, m <= 512)."""
        self.check(load().gpar_ctx_set_predict_fused(self.h, 1 if on else 0))

    def set_schedule(self, knob, value):
        """A schedule knob (gpar_ctx_set_schedule: overlap, overlap_group, qu_batch, dense_early,
        post_gram, compact_rec, predict_lanes, serialize, predict_fused, dg_rows_w, gram_group,
        fit_chunks, device_nm; the header lists their values); results are bit-identical with
        any setting except the plan knobs predict_fused, dg_rows_w and gram_group (last bits)
        and device_nm (the device's exp() in the chains fit's parameters)."""
        self.check(load().gpar_ctx_set_schedule(self.h, knob.encode(), int(value)))

    def schedule(self, knob):
        v = C.c_int32(0)
        self.check(load().gpar_ctx_get_schedule(self.h, knob.encode(), C.byref(v)))
        return int(v.value)

    def cu_split(self):
        """The CU split in effect (gpar_ctx_get_cu_split)."""
        v = C.c_int32(0)
        self.check(load().gpar_ctx_get_cu_split(self.h, C.byref(v)))
        return int(v.value)


_ctx: dict[int, Context] = {}


def context(device: int = 0) -> Context:
    c = _ctx.get(device)
    if c is None:
        c = Context(device)
        _ctx[device] = c
    return c


class NelderMead:
    """The library's Nelder-Mead (Optim.jl NelderMead restated, nelder_mead.hpp) as an
    ask/tell object; host only, usable without a GPU."""

    def __init__(self, x0, max_evals=0, max_iterations=1000, g_tol=1e-8, time_limit=0.0):
        import numpy as np
        self._np = np
        lib = load()
        self.n = len(x0)
        x = np.ascontiguousarray(np.asarray(x0, dtype=np.float64))
        opts = GparFitOptions(int(max_evals), int(max_iterations), float(g_tol), float(time_limit))
        h = C.c_void_p()
        code = lib.gpar_nm_create(self.n, x.ctypes.data_as(C.c_void_p), C.byref(opts), C.byref(h))
        if code != GPAR_OK:
            raise GparError(code, "gpar_nm_create failed")
        self.h = h

    def ask(self):
        x = self._np.zeros(self.n)
        r = load().gpar_nm_ask(self.h, x.ctypes.data_as(C.c_void_p))
        return x if r == 1 else None

    def tell(self, f):
        code = load().gpar_nm_tell(self.h, float(f))
        if code != GPAR_OK:
            raise GparError(code, "gpar_nm_tell: optimiser already finished")

    def result(self):
        x = self._np.zeros(self.n)
        f = C.c_double()
        ev = C.c_int32()
        it = C.c_int32()
        load().gpar_nm_result(self.h, x.ctypes.data_as(C.c_void_p), C.byref(f), C.byref(ev), C.byref(it))
        return x, float(f.value), int(ev.value), int(it.value)

    def __del__(self):
        try:
            if self.h:
                load().gpar_nm_destroy(self.h)
                self.h = None
        except Exception:
            pass


def nelder_mead(f, x0, **kw):
    nm = NelderMead(x0, **kw)
    while True:
        x = nm.ask()
        if x is None:
            break
        nm.tell(f(x))
    return nm.result()
