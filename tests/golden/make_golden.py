"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no tests or golden vectors and Julia is absent, so the
fixtures are produced by the oracle (oracle/gpar_oracle.py), after the oracle itself has passed
the reference's cross-check identities (examples/dtc_example.jl:8-64; tests/test_oracle.py).
They freeze the oracle's answers at small sizes (N <= 2000, M <= 64, P <= 6; fixed seeds) so the
GPU box compares against data files rather than re-deriving them.

    python tests/golden/make_golden.py        # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import gpar_oracle as O  # noqa: E402

# name, n, P, M, seed, gaps, out_kernel, time_kernel, theta
DTC_CASES = [
    ("dtc_m52_m52", 1200, 3, 48, 101, 0, "matern52", "matern52", (1.3, 0.9, 0.7, 1.1, 0.2)),
    ("dtc_eq_m32_gaps", 1500, 4, 64, 102, 3, "eq", "matern32", (2.0, 1.1, 2.5, 0.8, 0.15)),
    ("dtc_m32_m12", 800, 5, 32, 103, 0, "matern32", "matern12", (0.9, 0.5, 1.2, 1.4, 0.5)),
    ("dtc_m12_m52", 2000, 2, 24, 104, 1, "matern12", "matern52", (3.0, 2.0, 4.0, 0.9, 0.05)),
]


def gpar_case(n, P, M, seed, gaps):
    t, Y = O.synthetic_gpar(n, P, seed=seed, noise=0.3, gaps=gaps, gap_len=max(1, n // 20))
    V = Y[:, : P - 1].T.copy()
    y = Y[:, P - 1].copy()
    Z = O.pick_pseudo_inputs(V, M, seed + 7)
    return t, V, Z, y


def main():
    for name, n, P, M, seed, gaps, ok, tk, theta in DTC_CASES:
        t, V, Z, y = gpar_case(n, P, M, seed, gaps)
        dtc, A = O.compute_gpar_dtc_objective(V, Z, t, y, theta, ok, tk)
        out = dict(t=t, V=V, Z=Z, y=y, theta=np.array(theta), out_kernel=ok, time_kernel=tk,
                   dtc=dtc, A_head=A[:, :128].copy(), A_colsq=np.sum(A * A, axis=0))
        if name == "dtc_m52_m52":
            # q(u) (Cuu without noise, gpar_scaled_inference.jl:157) and analytic predictions
            me, cov, U, _ = O.compute_q_u(V, Z, t, y, theta, ok, tk)
            ts = t[::7] + 0.5 * (t[1] - t[0])
            Vs = V[:, ::7] + 0.01
            mean, std = O.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, theta, ok, tk)
            out.update(m_e=me, cov_e=cov, U_u=U, t_star=ts, V_star=Vs, pred_mean=mean, pred_std=std)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)

    # temporal-only path: LGSSM logpdf, smoother marginals, NM-fitted SDE predictions
    t, Y = O.synthetic_gpar(1500, 3, seed=3, noise=0.4, gaps=2, gap_len=100)
    ts = np.sort(np.concatenate([t[::11] + 0.013, [t[0] - 0.5, t[-1] + 0.7]]))
    out = dict(t=t, y=Y[:, 0], t_star=ts)
    for kind, th in (("matern12", (0.5, 1.3, 0.2)), ("matern32", (2.0, 0.7, 0.6)),
                     ("matern52", (10.0, 2.0, 0.05))):
        lg = O.create_lgssm(t, *th, kind=kind)
        out[f"logpdf_{kind}"] = O.lgssm_logpdf(lg, Y[:, 0])
        out[f"theta_{kind}"] = np.array(th)
        m, v = O.sde_predict_fixed(t, Y[:, 0], ts, th, kind)
        out[f"smooth_mean_{kind}"], out[f"smooth_var_{kind}"] = m, v
    th, m, v = O.get_sde_predictions(t, Y[:, 0], ts, "matern52", log_theta0=(0.0, 0.0, -2.0),
                                     max_evals=60)
    out.update(sde_fit_theta=np.array(th), sde_fit_mean=m, sde_fit_var=v)
    np.savez_compressed(os.path.join(HERE, "temporal.npz"), **out)

    # Nelder-Mead trajectory on the DTC objective (the fit loop, dtc.jl:11-77)
    t, V, Z, y = gpar_case(600, 3, 24, 105, 0)
    x0 = np.array([0.0, 0.0, 0.0, 0.0, -2.0])

    def nlml(p):
        return -O.compute_gpar_dtc_objective(V, Z, t, y, O.unpack_gpar(p))[0]

    nm = O.nelder_mead(nlml, x0, max_evals=40)
    np.savez_compressed(os.path.join(HERE, "nm_fit.npz"), t=t, V=V, Z=Z, y=y, x0=x0, max_evals=40,
                        x_min=nm.x_min, f_min=nm.f_min, evals=nm.evals)

    # exact GP / GPAR (optimized.jl:19-239), EQ kernels
    t, Y = O.synthetic_gpar(400, 3, seed=9, noise=0.3)
    X = np.vstack([t, Y[:, 0], Y[:, 1]])
    theta = (1.5, 1.2, 2.0, 0.7, 0.25)
    K = O.exact_gpar_kernel(X, X, theta)
    Xs = X[:, ::5] + 0.02
    Ks = O.exact_gpar_kernel(X, Xs, theta)
    kss = np.diag(O.exact_gpar_kernel(Xs, Xs, theta))
    mean, var = O.exact_posterior(K, Ks, kss, Y[:, 2], theta[4])
    # plain GP on time with a Matern-3/2 kernel (optimized.jl:28-36), theta = (l, pv, sigma)
    th1 = (0.7, 1.4, 0.3)
    K1 = O.exact_gp_kernel(t, t, th1, "matern32")
    ts = t[::3] + 0.01
    m1, v1 = O.exact_posterior(K1, O.exact_gp_kernel(t, ts, th1, "matern32"),
                               np.full(len(ts), th1[1] ** 2), Y[:, 0], th1[2])
    np.savez_compressed(os.path.join(HERE, "exact.npz"), X=X, y=Y[:, 2], X_star=Xs,
                        theta=np.array(theta), logpdf=O.exact_logpdf(K, Y[:, 2], theta[4]),
                        post_mean=mean, post_var=var, gp_t=t, gp_y=Y[:, 0], gp_t_star=ts,
                        gp_theta=np.array(th1), gp_logpdf=O.exact_logpdf(K1, Y[:, 0], th1[2]),
                        gp_mean=m1, gp_var=v1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
