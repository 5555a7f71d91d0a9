"""Bit-identity check of two library builds on a workload that runs every gains variant.

    python tools/lib_bitcheck.py run out.npz          (the library GPAR_HIP_LIB points at, or the
                                                       in-tree one)
    python tools/lib_bitcheck.py compare a.npz b.npz  (exit 1 on any differing bit)

Workload (one MI355X): a headline-schedule fit_predict_batch at N = 4e5 + 57 (the auto CU split,
the distance cache, a partial last chunk) over five outputs (the round overlap: compact gains
records with the data filter) and over three outputs (round by round: full records), predictions
on the merged grid (the noise-vector gains), the temporal-only chains' fit + smoothing (gains
without data, with the filtered covariances, with and without a noise vector).  A kernel change
that claims the same arithmetic (r05: the gains' phase 3 fast path) must reproduce every value.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))


def run(out):
    import torch
    import gparatscale as G
    from gparatscale import data as D
    dev = torch.device("cuda", 0)
    N, M, NS = 400_057, 512, 30_011
    ds = D.gpar_dataset(N, 34, seed=5, observation_noise=0.8, n_star=NS)
    Y = torch.from_numpy(ds["Y"]).to(dev)
    t = torch.from_numpy(ds["t"]).to(dev)
    ts = torch.from_numpy(ds["t_star"]).to(dev)
    Fs = torch.from_numpy(ds["F_star"]).to(dev)
    res = {}
    for tag, outs in (("ov", [2, 3, 9, 17, 33]), ("rr", [4, 12, 25])):
        probs, keep = [], []
        for p in outs:
            Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, : p - 1], M, seed=p)).to(dev)
            pr, k = G.make_problem(Y[:, : p - 1], Z, t, Y[:, p - 1].contiguous(), qu_kuu_noise=True)
            probs.append(pr)
            keep.append((k, Z))
        x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(outs), 1))
        fr, means, stds = G.fit_predict_batch(probs, x0, ts, [Fs[:, : p - 1] for p in outs],
                                              max_evals=8, g_tol=-1.0)
        res[tag + "_theta"] = fr.theta
        res[tag + "_nlml"] = fr.nlml
        res[tag + "_mean"] = np.array([m.cpu().numpy() for m in means])
        res[tag + "_std"] = np.array([s.cpu().numpy() for s in stds])
    th, m1, v1 = G.get_sde_predictions_device(t, Y[:, :3].T.contiguous(), ts, "matern32",
                                              (0.0, 0.0, -2.0), max_evals=10)
    res["sde_theta"], res["sde_mean"], res["sde_var"] = th, m1.cpu().numpy(), v1.cpu().numpy()
    th5 = np.tile([[1.3, 0.8, 0.1]], (2, 1))
    th_h, y_h = ds["t"][:20_011], ds["Y"][:20_011, :2].T.copy()
    noise = np.where(np.arange(20_011) % 3 == 0, 1e10, -1.0)
    sm, sv = G.lgssm_smooth_batch(th_h, y_h, th5, "matern52", noise=noise)
    res["smooth_noise_mean"], res["smooth_noise_var"] = sm, sv
    sm, sv = G.lgssm_smooth_batch(th_h, y_h, th5, "matern52")
    res["smooth_mean"], res["smooth_var"] = sm, sv
    res["logpdf"] = G.lgssm_logpdf_batch(th_h, y_h, th5, "matern52")
    np.savez(out, **res)
    print("saved", out, sorted(res))


def compare(a, b, tols):
    """tols: {key prefix: rtol} for outputs a change is allowed to move within rounding (a new
    summation order); every other output must be bit-identical."""
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        same = np.array_equal(A[k], B[k])
        diff = np.max(np.abs(A[k] - B[k]) / np.maximum(np.abs(A[k]), 1e-300)) if not same else 0.0
        tol = next((v for p, v in tols.items() if k.startswith(p)), None)
        ok = same or (tol is not None and diff <= tol)
        verdict = "bit-identical" if same else f"max rel {diff:.3e} (allowed {tol})"
        print(f"{k:20s} {verdict}{'' if ok else '  FAIL'}")
        bad += not ok
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        tols = dict((kv.split("=")[0], float(kv.split("=")[1])) for kv in sys.argv[4:])
        compare(sys.argv[2], sys.argv[3], tols)
