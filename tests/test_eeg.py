"""The eeg.jl driver (gparatscale.eeg): CSV layout (CPU) and the full pipeline on the GPU.

The EEG CSVs are git-ignored upstream (examples/datasets/eeg/), so the pipeline runs
on gparatscale.eeg.synthetic_eeg, a stand-in of the same shape; parity of its exact-GPAR stage is
checked against the oracle's exact posterior at the fitted hyperparameters (optimized.jl:201-239)."""
import numpy as np
import pytest

from oracle import gpar_oracle as O


def test_eeg_csv_roundtrip(tmp_path):
    from gparatscale import eeg
    d = eeg.synthetic_eeg(seed=3)
    tr, te = str(tmp_path / "eeg_train.csv"), str(tmp_path / "eeg_test.csv")
    eeg.write_eeg(d, tr, te)
    r = eeg.read_eeg(tr, te)
    assert open(tr).readline().strip() == ",".join(eeg.TRAIN_COLS)
    for part, cols in (("train", eeg.TRAIN_COLS), ("test", eeg.TEST_COLS)):
        for c in cols:
            np.testing.assert_allclose(r[part][c], d[part][c], rtol=1e-15)
    assert r["train"]["time"].shape == (256,) and r["test"]["fz"].shape == (100,)


@pytest.mark.gpu
def test_eeg_pipeline_gpu():
    from gparatscale import eeg
    d = eeg.synthetic_eeg(seed=1)
    out = eeg.run_eeg(d, max_evals=40, mode="analytic", seed=0)
    tr = d["train"]
    for ch in ("fz", "f1", "f2"):
        for stage in ("gp", "gpar", "scaled"):
            r = out[f"{stage}_{ch}"]
            assert r["mean"].shape == (256,) and np.all(np.isfinite(r["mean"]))
            assert np.all(np.isfinite(r["std"])) and np.all(r["std"] >= 0)
    # exact GPAR fz stage against the oracle at the fitted theta
    th = out["gpar_fz"]["theta"]
    dr = eeg.DATA_RANGE
    X = np.vstack([tr["time"][dr], tr["f3"][dr], tr["f4"][dr], tr["f5"][dr], tr["f6"][dr]])
    Xs = np.vstack([tr["time"], tr["f3"], tr["f4"], tr["f5"], tr["f6"]])
    K = O.exact_gpar_kernel(X, X, th, "matern52", "matern52")
    Ks = O.exact_gpar_kernel(X, Xs, th, "matern52", "matern52")
    kss = np.diag(O.exact_gpar_kernel(Xs, Xs, th, "matern52", "matern52"))
    m, v = O.exact_posterior(K, Ks, kss, tr["fz"][dr], th[4])
    np.testing.assert_allclose(out["gpar_fz"]["mean"], m, rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(out["gpar_fz"]["std"], np.sqrt(np.maximum(v, 0)), rtol=1e-6, atol=1e-8)
