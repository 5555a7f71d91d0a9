"""Argument validation of the Python API before anything reaches the library or the GPU (CPU).

The C side cannot see the lengths of caller buffers, so the bindings check them: mismatched
lengths raise DomainError (util.jl:112-117's error type for malformed inputs) instead of letting
a kernel read or write past a buffer."""
import numpy as np
import pytest

G = pytest.importorskip("gparatscale")


def _data(n=50, D=3, M=8):
    rng = np.random.default_rng(0)
    t = np.arange(n) / 30.0
    V = rng.normal(size=(D, n))
    Z = V[:, :M].copy()
    y = rng.normal(size=n)
    return t, V, Z, y


def test_make_problem_length_mismatch():
    t, V, Z, y = _data()
    with pytest.raises(G.DomainError):
        G.make_problem(V, Z, t[:-1], y)
    with pytest.raises(G.DomainError):
        G.make_problem(V, Z, t, y[:-2])


def test_make_problem_dimension_mismatch():
    t, V, Z, y = _data()
    with pytest.raises(G.DomainError):
        G.make_problem(V, Z[:2], t, y)


def test_predict_scaled_inference_shape():
    t, V, Z, y = _data()
    ts = t[:10] + 0.01
    theta = (1.0, 1.0, 1.0, 1.0, 0.2)
    with pytest.raises(G.DomainError):          # wrong input dimension
        G.predict_scaled(V, Z, t, y, theta, ts, V[:2, :10])
    with pytest.raises(G.DomainError):          # one point short of the inference times
        G.predict_scaled(V, Z, t, y, theta, ts, V[:, :9])


def test_fit_predict_batch_shapes():
    t, V, Z, y = _data()
    pr, keep = G.make_problem(V, Z, t, y)
    ts = t[:10] + 0.01
    x0 = np.zeros((1, 5))
    with pytest.raises(G.DomainError):          # one V_star per problem
        G.fit_predict_batch([pr], x0, ts, [])
    with pytest.raises(G.DomainError):          # V_star with N* != len(t_star)
        G.fit_predict_batch([pr], x0, ts, [V[:, :12]])
    with pytest.raises(G.DomainError):          # V_star = None needs a chain
        G.fit_predict_batch([pr], x0, ts, [None])
    chain = np.zeros((10, 4))
    with pytest.raises(G.DomainError):          # chain_cols: one per problem
        G.fit_predict_batch([pr], x0, ts, [None], chain=chain, chain_cols=[1, 2])
    with pytest.raises(G.DomainError):          # chain column out of range
        G.fit_predict_batch([pr], x0, ts, [None], chain=chain, chain_cols=[4])
    with pytest.raises(G.DomainError):          # chain narrower than the inputs
        G.fit_predict_batch([pr], x0, ts, [None], chain=np.zeros((10, 2)), chain_cols=[-1])
