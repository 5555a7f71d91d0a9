"""Prediction-path probe: gpar_fit_predict for a few outputs at N = N* (default 1e6), M = 512,
one objective evaluation each, so the kernel profile is dominated by the prediction kernels
(variance GEMM, adjoint pass, predict rows).  Run under rocprofv3 --stats for per-kernel times."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gparatscale as G  # noqa: E402
from gparatscale import data as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--outputs", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--dmin", type=int, default=1, help="the first output's input dimension")
    a = ap.parse_args()
    P = a.dmin + a.outputs
    ds = D.gpar_dataset(a.n, P, seed=0)
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(ds["t"]).to(dev)
    Y = torch.from_numpy(ds["Y"]).to(dev)
    ts = torch.from_numpy(ds["t_star"]).to(dev)
    Fs = torch.from_numpy(ds["F_star"]).to(dev)
    problems, keep = [], []
    outs = list(range(a.dmin + 1, P + 1))
    for p in outs:
        Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, : p - 1], a.m, seed=p)).to(dev)
        pr, k = G.make_problem(Y[:, : p - 1], Z, t, Y[:, p - 1].contiguous(), qu_kuu_noise=True)
        problems.append(pr)
        keep.append((k, Z))
    x0 = np.tile([0.0, 0.0, 0.0, 0.0, -2.0], (len(problems), 1))
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        G.fit_predict_batch(problems, x0, ts, [Fs[:, : p - 1] for p in outs], max_evals=1,
                            g_tol=-1.0)
        torch.cuda.synchronize()
        print(f"rep {r}: {time.perf_counter() - t0:.3f} s for {len(problems)} outputs", flush=True)
    # release the library's context and the device tensors while the runtime (and a profiler's
    # tool library) is still up: under rocprofv3 --pmc the process otherwise faulted in a static
    # destructor after the profiler had finalised
    del problems, keep, t, Y, ts, Fs
    G.context().close()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
