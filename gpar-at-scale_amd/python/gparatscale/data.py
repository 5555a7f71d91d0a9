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


def pseudo_index(n, M, seed):
    """The rows pseudo_inputs(V_rows, M, seed) takes from an n-row V (sorted)."""
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n, size=M, replace=False))


def gpar_dataset_device(n, P, seed=0, observation_noise=0.8, device="cuda"):
    """gpar_dataset's training half generated on the GPU with torch (the stress config: N = 1e7,
    P = 256 is 20 GB of Y, minutes of numpy): t (n,) and Y (n x P, observed = f_big chain + noise
    with std observation_noise^2), both fp64 on `device`.  The same functions as gpar_dataset; the
    noise comes from torch's device generator (seeded), so the values differ from the numpy
    generator's -- synthetic inputs of the same shape and distribution."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    x = START + STEP_SIZE * torch.arange(n, dtype=torch.float64, device=device)
    Y = torch.empty((n, P), dtype=torch.float64, device=device)
    std = observation_noise ** 2
    pi = float(np.pi)
    for p in range(1, P + 1):
        if p == 1:
            f = 3.0 - torch.sin(pi / 10.0 * (x + 1.0)) - torch.pow(x, 0.3)
        elif p == 2:
            f = torch.cos(Y[:, 0]) ** 2 + torch.sin(pi / 20.0 * x)
        elif p == 3:
            f = Y[:, 1] * Y[:, 0] ** 2 + 0.1 * x
        else:
            f = torch.cos(Y[:, p - 2]) ** 2 + torch.sin(pi * x / (20.0 + p)) + 0.1 * Y[:, p - 3]
        Y[:, p - 1] = f + std * torch.randn(n, dtype=torch.float64, device=device, generator=g)
    return x, Y
