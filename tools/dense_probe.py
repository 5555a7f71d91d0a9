"""The dense tail's kernels in isolation: batched DTC objectives of `--batch` outputs at a short
series (N = 2000, so the blocked Cholesky / inverse / Lambda / finish launches dominate), M
pseudo-points, `--reps` calls; run under rocprofv3 --kernel-trace --stats for their durations.
    python tools/dense_probe.py [--m 512] [--batch 8] [--reps 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import gparatscale as G
    from gparatscale import data as D
    ds = D.gpar_dataset(2000, 6, seed=1, observation_noise=0.7, n_star=10)
    t, Y = ds["t"], ds["Y"]
    probs, keep = [], []
    for i in range(a.batch):
        V = np.ascontiguousarray(Y[:, :4].T)
        Z = np.ascontiguousarray(D.pseudo_inputs(Y[:, :4], a.m, seed=i + 1).T)
        pr, k = G.make_problem(V, Z, t, np.ascontiguousarray(Y[:, 4 + i % 2]))
        probs.append(pr)
        keep.append(k)
    th = np.tile([[1.1, 0.9, 1.3, 0.8, 0.3]], (a.batch, 1))
    for _ in range(a.reps):
        v = G.dtc_objective_batch(probs, th)
    print(list(np.asarray(v)[:2]))


if __name__ == "__main__":
    main()
