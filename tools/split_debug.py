"""Batched objective on the driver test's problems (D = 1, 5, 20) in the current split mode:
prints the lml of each output at a few thetas (compare runs with GPAR_SPLIT_CUS / _DGW set)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpar-at-scale_amd", "python"))
import torch  # noqa: F401  (one HIP runtime for torch and the library)
import gparatscale as G
from oracle import gpar_oracle as O

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
t, Y = O.synthetic_gpar(n, 21, seed=31, noise=0.3)
probs, keep = [], []
for p in [2, 6, 21]:
    V = np.ascontiguousarray(Y[:, : p - 1].T)
    Z = O.pick_pseudo_inputs(V, 24, p)
    pr, k = G.make_problem(V, Z, t, Y[:, p - 1])
    probs.append(pr)
    keep.append(k)
for th in ([1.0, 1.0, 1.0, 1.0, 0.135], [1.3, 0.8, 1.1, 0.9, 0.2], [0.7, 1.2, 0.9, 1.1, 0.1]):
    lml = G.dtc_objective_batch(probs, np.tile(np.array(th), (3, 1)))
    print("theta", th, "lml", " ".join(f"{v:.12e}" for v in np.atleast_1d(lml)))
fr = G.fit_batch(probs, np.tile(np.array([0.0, 0.0, 0.0, 0.0, -2.0]), (3, 1)), max_evals=40, g_tol=-1.0)
print("fit theta", np.array2string(fr.theta, precision=10))
