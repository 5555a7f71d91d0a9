"""Per-kernel timing of single-output analytic predictions at N = N* (default 1e6), M = 512, for a
few input widths D, under whatever GPAR_* environment (or GPAR_HIP_LIB variant library) the
process was started with.  Prints one JSON line per D with the HIP-event averages of the
prediction kernel families and a SHA-256 of the predicted means / stds, so two runs can be
compared for bit identity without shipping the arrays back.
    python tools/whiten_ab.py [--dims 32 63] [--reps 3]
(r05: A/B of a producer/consumer form of the fused whitening, 4.6 -> 5.8 ms at D = 32)"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))

import numpy as np  # noqa: E402


def run(a):
    import torch
    import gparatscale as G
    from gparatscale import data as D
    dev = torch.device("cuda", 0)
    P = max(a.dims) + 1
    ds = D.gpar_dataset(a.n, P, seed=0)
    t = torch.from_numpy(ds["t"]).to(dev)
    Y = torch.from_numpy(ds["Y"]).to(dev)
    ts = torch.from_numpy(ds["t_star"]).to(dev)
    Fs = torch.from_numpy(ds["F_star"]).to(dev)
    ctx = G.context(0)
    theta = (2.0, 2.0, 2.0, 2.0, float(np.exp(-2.0) + 1e-3))
    for d in a.dims:
        p = d + 1
        Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, :d], a.m, seed=p)).to(dev)
        y = Y[:, d].contiguous()
        args = (Y[:, :d], Z, t, y, theta, ts, Fs[:, :d], "matern52", "matern52")
        G.predict_scaled(*args, mode="analytic", qu_kuu_noise=True)   # warm-up
        torch.cuda.synchronize()
        ctx.set_profiling(True)
        ctx.reset_stats()
        for _ in range(a.reps):
            m, s = G.predict_scaled(*args, mode="analytic", qu_kuu_noise=True)
        torch.cuda.synchronize()
        out = {"D": d, "N": a.n, "M": a.m, "whiten_ws": os.environ.get("GPAR_WHITEN_WS", "1")}
        for fam in ("pred_whiten", "pred_adjoint", "pred_var", "predictions"):
            k, ms = ctx.kernel_stats(fam)
            if k:
                out[fam + "_ms"] = ms / k
        ctx.set_profiling(False)
        h = hashlib.sha256()
        for arr in (m, s):
            h.update(np.ascontiguousarray(arr.cpu().numpy()).tobytes())
        out["sha256"] = h.hexdigest()
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--dims", type=int, nargs="+", default=[16, 32, 48, 63])
    ap.add_argument("--reps", type=int, default=3)
    run(ap.parse_args())


if __name__ == "__main__":
    main()
