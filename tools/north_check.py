"""One-off: DTC objective of one north-star output (N=1e6, M=512, D=32) on the GPU vs the numpy
oracle (minutes of CPU; not part of the test suite)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))
import numpy as np  # noqa: E402
import gparatscale as G  # noqa: E402
from gparatscale import data as D  # noqa: E402
from oracle import gpar_oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ds = D.gpar_dataset(n, 33, seed=0, observation_noise=0.8)
V = ds["Y"][:, :32].T.copy()
y = ds["Y"][:, 32].copy()
Z = D.pseudo_inputs(ds["Y"][:, :32], 512, seed=33).T.copy()
theta = (1.0, 1.0, 1.0, 1.0, 0.2)
got = G.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta)
print("gpu", repr(got), flush=True)
t0 = time.time()
ref, parts = O.compute_gpar_dtc_objective(V, Z, ds["t"], y, theta, return_parts=True)
print("oracle", repr(ref), f"{time.time() - t0:.0f}s rel {abs(got - ref) / abs(ref):.3e}", flush=True)
lam = np.linalg.eigvalsh(parts["Lam"])
print("Lambda eig range", lam.min(), lam.max(), "cond", lam.max() / lam.min())
