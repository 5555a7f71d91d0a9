"""EEG example driver (examples/eeg.jl), the caller on the input side of the hot path.

eeg.jl reads two CSVs and, for three channels (fz, f1, f2), fits
  * independent exact GPs on time                      (eeg.jl:29-51,  optimized.jl:76-97)
  * an exact GPAR chain with the earlier channels as inputs, evaluated at every training time
    with the *predicted* means of the earlier outputs   (eeg.jl:54-87, 177-208)
  * the scaled GPAR (DTC + LGSSM) with Z = V and the same chained inference inputs
                                                       (eeg.jl:212-281, gpar_scaled_inference.jl)
The CSVs live in examples/datasets/eeg/ upstream, which is git-ignored; `synthetic_eeg`
builds a stand-in of the same shape.  The reference casts the exact-path targets to Float32
(eeg.jl:32,...); here everything stays Float64.
"""
from __future__ import annotations

import numpy as np

from . import api

TRAIN_COLS = ("time", "f3", "f4", "f5", "f6", "fz", "f1", "f2")   # eeg.jl:12-20
TEST_COLS = ("time", "fz", "f1", "f2")                            # eeg.jl:22-25
DATA_RANGE = slice(0, 156)                                        # eeg.jl:28  1:156
TEST_RANGE = slice(156, 256)                                      # eeg.jl:29  157:256


def read_eeg(train_csv: str, test_csv: str) -> dict:
    """CSV.read of eeg_train.csv / eeg_test.csv (header row, comma separated), columns by
    position as eeg.jl:12-25 splits them."""
    def load(path, cols):
        a = np.genfromtxt(path, delimiter=",", skip_header=1, dtype=np.float64)
        a = np.atleast_2d(a)
        if a.shape[1] < len(cols):
            raise ValueError(f"{path}: expected at least {len(cols)} columns, got {a.shape[1]}")
        return {c: np.ascontiguousarray(a[:, i]) for i, c in enumerate(cols)}
    return {"train": load(train_csv, TRAIN_COLS), "test": load(test_csv, TEST_COLS)}


def write_eeg(data: dict, train_csv: str, test_csv: str) -> None:
    """Inverse of read_eeg (header + rows), for fixtures and the synthetic stand-in."""
    for part, cols, path in (("train", TRAIN_COLS, train_csv), ("test", TEST_COLS, test_csv)):
        a = np.stack([data[part][c] for c in cols], axis=1)
        np.savetxt(path, a, delimiter=",", header=",".join(cols), comments="")


def synthetic_eeg(seed: int = 0, n: int = 256) -> dict:
    """Stand-in with the dataset's shape: 256 samples of 7 correlated channels on [0, 1);
    test rows = the last 100 samples of fz, f1, f2 (eeg.jl:28-29)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n, dtype=np.float64) / n
    base = [np.sin(2 * np.pi * (3 + k) * t + rng.uniform(0, 2 * np.pi)) for k in range(4)]
    f3, f4, f5, f6 = (b + 0.3 * rng.standard_normal(n) for b in base)
    fz = 2.0 * base[0] - base[1] + 0.5 * np.cos(6 * np.pi * t) + 0.2 * rng.standard_normal(n)
    f1 = 0.8 * fz + base[2] + 0.2 * rng.standard_normal(n)
    f2 = np.tanh(f1) + 0.5 * base[3] + 0.2 * rng.standard_normal(n)
    train = dict(time=t, f3=f3, f4=f4, f5=f5, f6=f6, fz=fz, f1=f1, f2=f2)
    test = dict(time=t[TEST_RANGE].copy(), fz=fz[TEST_RANGE].copy(), f1=f1[TEST_RANGE].copy(),
                f2=f2[TEST_RANGE].copy())
    return {"train": train, "test": test}


def run_eeg(data: dict, max_evals: int = 0, time_limit: float = 3.0, mode: str = "mc",
            samples: int = 100, seed: int = 0, device: int = 0) -> dict:
    """The eeg.jl pipeline.  Returns per channel: the independent GP, the exact GPAR and the
    scaled GPAR means / stds at every training time, plus the fitted hyperparameters.

    max_evals > 0 bounds every Nelder-Mead run (reproducible); otherwise the fits stop on
    g_tol / iterations, and the scaled ones at `time_limit` seconds (eeg.jl: 3.0).  Missing
    initial log-parameters are drawn U(0,1) from `seed` (util.jl:128-134)."""
    rng = np.random.default_rng(seed)
    tr = data["train"]
    t_all = tr["time"]
    dr = DATA_RANGE
    t = t_all[dr]
    out = {"time": t_all}

    # independent exact GPs (eeg.jl:30-51): fz, f1 Matern52; f2 Matern12 with its init
    gp_cfg = {"fz": ("matern52", dict()),
              "f1": ("matern52", dict()),
              "f2": ("matern12", dict(i_log_l=-2.0, i_log_process_var=1.0, i_log_noise_sigma=-3.0))}
    for ch, (kern, init) in gp_cfg.items():
        gp, th = api.create_optim_gp(t, tr[ch][dr], kern, max_evals=max_evals, rng=rng,
                                     device=device, **init)
        m, v = gp.marginals(t_all)
        out[f"gp_{ch}"] = dict(theta=th, mean=m, std=np.sqrt(np.maximum(v, 0.0)))

    # exact GPAR chain (eeg.jl:54-87 fit, 177-208 marginals with chained means)
    inputs = [tr["f3"], tr["f4"], tr["f5"], tr["f6"]]
    means = []
    init_fz = dict(i_log_time_l=-3.0, i_log_time_var=1.0, i_log_out_l=6.0, i_log_out_var=4.0,
                   i_log_noise_sigma=-2.0)
    for ch in ("fz", "f1", "f2"):
        X = np.vstack([t] + [a[dr] for a in inputs])
        init = init_fz if ch == "fz" else {}
        gpar, th = api.create_optim_gpar(X, tr[ch][dr], "matern52", "matern52", max_evals=max_evals,
                                         rng=rng, device=device, **init)
        X_star = np.vstack([t_all] + [a for a in inputs[:4]] + means)
        m, v = gpar.marginals(X_star)
        out[f"gpar_{ch}"] = dict(theta=th, mean=m, std=np.sqrt(np.maximum(v, 0.0)))
        inputs = inputs + [tr[ch]]
        means.append(m)

    # scaled GPAR (eeg.jl:212-281): V = Z = the channels, inference at every training time with
    # the exact GPAR means of the earlier outputs
    chans = [tr["f3"], tr["f4"], tr["f5"], tr["f6"]]
    for k, ch in enumerate(("fz", "f1", "f2")):
        V = np.vstack([c[dr] for c in chans])
        V_star = np.vstack([tr[c] for c in ("f3", "f4", "f5", "f6")] + means[:k])
        m, s = api.get_gpar_scaled_predictions(
            V, V, t, tr[ch][dr], t_all, V_star, optimization_time_limit=time_limit,
            max_evals=max_evals, mode=mode, samples=samples, seed=seed + k, rng=rng, device=device)
        out[f"scaled_{ch}"] = dict(mean=m, std=s)
        chans = chans + [tr[ch]]
    return out
