"""Synthetic GPAR data (src/data/toy_data.jl) generalised to P outputs.

toy_data.jl:9-40 draws x = range(0, STEP*n), chains y1 = f1(x), y2 = f2(x, y1), y3 = f3(x, y1, y2)
with noise Normal(0, observation_noise^2) -- the *std* is the square (toy_data.jl:29), 0.8^2 = 0.64
for the big dataset -- and removes `nr_nuked_intervals` gaps (toy_data.jl:42-57).  For p > 3 the
build defines y_p = cos(y_{p-1})^2 + sin(pi t / (20 + p)) + 0.1 y_{p-2}.  Inputs of
output p are the observed (noisy) previous outputs, as in GPAR_scaled_examples.jl:132-175.
Host-side numpy: data generation is set-up, not the hot path.
"""
from __future__ import annotations

import numpy as np

START = 0.0
STEP_SIZE = 1.0 / 30.0


def f1_big(x):
    return 3.0 - np.sin(np.pi / 10.0 * (x + 1.0)) - np.power(x, 0.3)


def f2_big(x, y1):
    return np.cos(y1) ** 2 + np.sin(np.pi / 20.0 * x)


def f3_big(x, y1, y2):
    return y2 * y1 ** 2 + 0.1 * x


def f_small(p, x, ys):
    if p == 1:
        return -np.sin(10 * np.pi * (x + 1)) / (2 * x + 1) - x ** 4
    if p == 2:
        return np.cos(ys[0]) ** 2 + np.sin(3 * x)
    return ys[1] * ys[0] ** 2 + 3 * x


def f_big(p, x, ys):
    if p == 1:
        return f1_big(x)
    if p == 2:
        return f2_big(x, ys[0])
    if p == 3:
        return f3_big(x, ys[0], ys[1])
    return np.cos(ys[p - 2]) ** 2 + np.sin(np.pi * x / (20.0 + p)) + 0.1 * ys[p - 3]


def fmt_count(n: int) -> str:
    """1000000 -> '1e6' (bench metric strings)."""
    e = len(str(int(n))) - 1
    return f"{n // 10 ** e}e{e}" if n % 10 ** e == 0 else str(n)


def nuke(x, nr_intervals, per_interval):
    """toy_data.jl:42-57."""
    if nr_intervals == 0:
        return x, 0
    kept = len(x) // (nr_intervals + 1)
    parts = [x[:kept]] + [x[i * kept + per_interval:(i + 1) * kept] for i in range(1, nr_intervals + 1)]
    nx = np.concatenate(parts)
    return nx, len(x) - len(nx)


def gpar_dataset(n, P, seed=0, observation_noise=0.8, gaps=0, gap_len=300, n_star=None):
    """Returns dict(t, Y (n x P observed, noisy), t_star, F_star (n_star x P noiseless truth)).

    t_star interleaves the training grid (midpoints, plus the first point) so N* = n by default,
    the north-star predict workload."""
    rng = np.random.default_rng(seed)
    x = START + STEP_SIZE * np.arange(n, dtype=np.float64)
    x, _ = nuke(x, gaps, gap_len)
    std = observation_noise ** 2
    ys = []
    for p in range(1, P + 1):
        ys.append(f_big(p, x, ys) + rng.normal(0.0, std, size=x.shape[0]))
    Y = np.stack(ys, axis=1)
    n_star = len(x) if n_star is None else n_star
    ts = START + STEP_SIZE * (np.arange(n_star, dtype=np.float64) + 0.5) * (len(x) / n_star)
    fs = []
    for p in range(1, P + 1):
        fs.append(f_big(p, ts, fs))
    return dict(t=x, Y=Y, t_star=ts, F_star=np.stack(fs, axis=1))


def pseudo_inputs(V_rows, M, seed):
    """Z_p = M rows of V_p sampled without replacement (seed p).  V_rows: n x D."""
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(V_rows.shape[0], size=M, replace=False))
    return np.ascontiguousarray(V_rows[idx])
