"""Run a few DTC objective evaluations of one north-star output (N=1e6, M=512, D inputs) on the
GPU, for rocprofv3 counter passes and kernel timing of the Gram / whitening kernels.

    rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gram_kernel -d gpurun_out/pmc_fetch \
        -o run --output-format csv -- python3 tools/gram_probe.py --evals 3
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--evals", type=int, default=3)
    ap.add_argument("--kernel", default="matern52")
    ap.add_argument("--fit", action="store_true",
                    help="time gpar_fit (max_evals = --evals) instead of objective calls: the fit's "
                         "distance cache is used for D >= 17")
    ap.add_argument("--batch", type=int, default=1,
                    help="fit / evaluate this many copies of the output in one batched call (>= 2 "
                         "runs the batched fit's pipelined, CU-split Gram stage)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import gparatscale as G
    from gparatscale import data as D

    P = a.d + 1
    dev = torch.device("cuda", 0)
    if P <= 64:
        ds = D.gpar_dataset(a.n, P, seed=0, observation_noise=0.8)
        t = torch.from_numpy(ds["t"]).to(dev)
        Y = torch.from_numpy(ds["Y"]).to(dev)
        Z = torch.from_numpy(D.pseudo_inputs(ds["Y"][:, : P - 1], a.m, seed=P)).to(dev)
    else:
        # wide inputs (config 5, D up to 255): scaled / shifted copies of 8 observed outputs,
        # built on the device (a 256-output dataset at N = 1e7 takes minutes on the host)
        ds = D.gpar_dataset(a.n, 9, seed=0, observation_noise=0.8)
        t = torch.from_numpy(ds["t"]).to(dev)
        Yb = torch.from_numpy(ds["Y"]).to(dev)
        Y = torch.empty((a.n, P), dtype=torch.float64, device=dev)
        for q in range(P - 1):
            Y[:, q] = Yb[:, q % 8] * (1.0 + 0.013 * (q // 8)) + 0.05 * (q // 8)
        Y[:, P - 1] = Yb[:, 8]
        rows = torch.from_numpy(np.random.default_rng(P).choice(a.n, a.m, replace=False)).to(dev)
        Z = Y[rows, : P - 1].contiguous()
    y = Y[:, P - 1].contiguous()
    pr, keep = G.make_problem(Y[:, : P - 1], Z, t, y, a.kernel, "matern52")
    prs = [pr] * a.batch
    ctx = G.context(0)
    theta = np.tile(np.array([[1.0, 1.0, 1.0, 1.0, 0.2]]), (a.batch, 1))
    def ev(th):
        try:
            return G.dtc_objective_batch(prs, th)
        except G.GparError:   # timing ablations (GPAR_HIP_LIB) compute garbage on purpose
            if not os.environ.get("GPAR_HIP_LIB"):
                raise
            return [float("nan")]

    if a.fit:
        x0 = np.tile(np.array([[0.0, 0.0, 0.0, 0.0, -2.0]]), (a.batch, 1))
        G.fit_batch(prs, x0, max_evals=2, g_tol=-1.0)
        ctx.set_profiling(True)
        ctx.reset_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fr = G.fit_batch(prs, x0, max_evals=a.evals, g_tol=-1.0)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3 / a.evals
        out = [f"N={a.n} M={a.m} D={a.d} batch={a.batch} fit ms/eval={el:.3f} nlml={fr.nlml[0]:.6f}"]
        for k in ("gram", "whiten", "gains", "dense"):
            n, ms = ctx.kernel_stats(k)
            if n:
                out.append(f"{k}: {n} launches avg {ms / n:.4f} ms")
        print("; ".join(out))
        return
    ev(theta)
    ctx.set_profiling(True)
    ctx.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.evals):
        v = ev(theta * (1.0 + 0.01 * i))
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3 / a.evals
    out = [f"N={a.n} M={a.m} D={a.d} ms/eval={el:.3f} dtc={v[0]:.6f}"]
    for k in ("gram", "whiten", "gains", "dense"):
        n, ms = ctx.kernel_stats(k)
        if n:
            out.append(f"{k}: {n} launches avg {ms / n:.4f} ms")
    print("; ".join(out), flush=True)


if __name__ == "__main__":
    main()
