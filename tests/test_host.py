"""CPU: the C-ABI library and the host-side logic (no GPU compute).

* libgparhip.so loads and exports every entry point include/gpar_hip.h declares;
* without a GPU the product path fails loudly (no CPU fallback);
* the library's Nelder-Mead (nelder_mead.hpp, Optim.jl NelderMead restated) follows the oracle's
  trajectory exactly, on test functions and on the DTC objective (dtc.jl:11-77), including the
  max_evals budget and g_tol stopping;
* the Python mirror's host helpers match util.jl (unpack, masks, init, ColVecs).
"""
import os
import re

import numpy as np
import pytest

from oracle import gpar_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gpar_hip.h")


@pytest.fixture(scope="module")
def G():
    import gparatscale
    gparatscale.load()   # raises OSError if the library has not been built
    return gparatscale


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(gpar_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_bound_symbols(G):
    assert header_functions() == sorted(G.EXPORTED)


def test_library_exports_every_symbol(G):
    import ctypes
    lib = ctypes.CDLL(G.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name
    assert G.load().gpar_abi_version() == 1


def test_no_gpu_fails_loudly(G):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(G.GparError):
        G.Context(0)


def rosen(x):
    return float(np.sum(100.0 * (x[1:] - x[:-1] ** 2) ** 2 + (1.0 - x[:-1]) ** 2))


@pytest.mark.parametrize("f,x0,kw", [
    (rosen, [0.0, 0.0], {}),
    (rosen, [-1.2, 1.0, 0.5, 0.3], {}),
    (lambda x: float(np.sum((x - np.arange(5)) ** 2)), np.zeros(5), {"max_evals": 37}),
    (lambda x: float(np.abs(x).sum()), [0.3, -0.7, 1.1], {"g_tol": 1e-4}),
])
def test_native_nelder_mead_matches_oracle(G, f, x0, kw):
    ref = O.nelder_mead(f, np.asarray(x0, float), **{k: v for k, v in kw.items()})
    x, fmin, evals, _ = G.nelder_mead(f, x0, **kw)
    assert evals == ref.evals
    np.testing.assert_array_equal(x, ref.x_min)
    assert fmin == ref.f_min


def test_native_nelder_mead_on_dtc_golden(G):
    """The fit loop of dtc.jl:11-77 driven by the native optimiser over the oracle objective
    reproduces the golden trajectory end point (tests/golden/nm_fit.npz)."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "nm_fit.npz"), allow_pickle=False)

    def nlml(p):
        return -O.compute_gpar_dtc_objective(g["V"], g["Z"], g["t"], g["y"], O.unpack_gpar(p))[0]

    x, fmin, evals, _ = G.nelder_mead(nlml, g["x0"], max_evals=int(g["max_evals"]))
    assert evals == int(g["evals"])
    np.testing.assert_allclose(x, g["x_min"], rtol=1e-10, atol=1e-12)


def test_nm_ask_after_done(G):
    nm = G.NelderMead([0.0], max_evals=3)
    n = 0
    while (x := nm.ask()) is not None:
        nm.tell(float(x[0] ** 2))
        n += 1
    assert n == 3
    with pytest.raises(G.GparError):
        nm.tell(0.0)


def test_host_helpers_match_util_jl(G):
    p = np.array([0.1, -0.3, 0.7, 0.2, -2.0])
    np.testing.assert_allclose(G.unpack_gpar(p), O.unpack_gpar(p))
    np.testing.assert_allclose(G.unpack_gp(p[:3]), O.unpack_gp(p[:3]))
    np.testing.assert_array_equal(G.get_time_mask(5), O.get_time_mask(5))
    np.testing.assert_array_equal(G.get_output_mask(5), O.get_output_mask(5))
    with pytest.raises(ValueError):
        G.get_output_mask(1)
    x = G.parse_initial_params([0.5, None, 1.0], rng=np.random.default_rng(0))
    assert x[0] == 0.5 and x[2] == 1.0 and 0.0 <= x[1] < 1.0
    np.testing.assert_array_equal(G.to_colvecs(np.arange(6.0).reshape(3, 2)),
                                  O.to_colvecs(np.arange(6.0).reshape(3, 2)))


def test_data_generator_matches_oracle(G):
    from gparatscale import data as D
    ds = D.gpar_dataset(500, 5, seed=3, observation_noise=0.8, gaps=2, gap_len=30)
    t, Y = O.synthetic_gpar(500, 5, seed=3, noise=0.8, gaps=2, gap_len=30)
    np.testing.assert_array_equal(ds["t"], t)
    np.testing.assert_array_equal(ds["Y"], Y)
