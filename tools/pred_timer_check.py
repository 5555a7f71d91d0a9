"""Checks the library's "predictions" span (HIP events around gpar_fit_predict's predictions)
against the host clock around the same call: 3 outputs at N = N* = 2e5, M = 256, one evaluation."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gparatscale as G  # noqa: E402
from gparatscale import data as D  # noqa: E402

ds = D.gpar_dataset(200_000, 4, seed=0)
dev = torch.device("cuda", 0)
t, Y = torch.from_numpy(ds["t"]).to(dev), torch.from_numpy(ds["Y"]).to(dev)
ts, Fs = torch.from_numpy(ds["t_star"]).to(dev), torch.from_numpy(ds["F_star"]).to(dev)
probs, keep = [], []
for p in (2, 3, 4):
    Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, : p - 1], 256, seed=p)).to(dev)
    pr, k = G.make_problem(Y[:, : p - 1], Z, t, Y[:, p - 1].contiguous(), qu_kuu_noise=True)
    probs.append(pr)
    keep.append((k, Z))
x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (3, 1))
ctx = G.context()
ctx.set_profiling(True)
for rep in range(3):
    ctx.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    G.fit_predict_batch(probs, x0, ts, [Fs[:, : p - 1] for p in (2, 3, 4)], max_evals=1, g_tol=-1.0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    n, ms = ctx.kernel_stats("predictions")
    parts = {f: ctx.kernel_stats(f) for f in ("pred_whiten", "pred_adjoint", "pred_var", "gram")}
    print(f"rep {rep}: call {wall:.1f} ms; predictions span n={n} {ms:.1f} ms; parts {parts}", flush=True)
del probs, keep
ctx.close()
