"""-m gpu: the GPU library under a multi-rank process group (bench.py --gpus N).

World sizes 2 and 3 over gloo, every rank on cuda:0 of the one-GPU box (tests/gpu_multirank_worker.py:
broadcast of the inputs from rank 0, LPT output shards, one batched gpar_fit per rank on device
inputs, all-reduce gather of the fitted rows).  Each output's Nelder-Mead and objective are
independent of the batch it runs in, so the gathered hyperparameters must equal, bit for bit,
one single-process batched fit of all outputs (GPAR_scaled_examples.jl:132-175 fits every output
on its own).  The ranks are child processes started before they touch the GPU; the test waits
for them under a timeout.

The chained sweep across ranks: each rank fits its outputs into a
posterior (gpar_fit_posterior), then the ordered sweep of shard.chained_predictions runs the real
Posterior.predict / prepare in every rank and broadcasts each predicted mean from its owner; the
means, stds and theta must equal one single-process gpar_fit_predict_chain bit for bit.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gparatscale")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gpu_multirank_worker as W  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world(world, out, mode="given"):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "gpu_multirank_worker.py"), out, mode],
                                      env=env, cwd=ROOT))
    codes = []
    for pr in procs:
        try:
            codes.append(pr.wait(timeout=100))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * world, codes
    with open(out) as f:
        return json.load(f)


def _serial():
    from gparatscale import data as Dd
    ds = Dd.gpar_dataset(W.N, W.P, seed=3, observation_noise=0.5)
    dev = torch.device("cuda", 0)
    t_d = torch.from_numpy(ds["t"]).to(dev)
    Y_d = torch.from_numpy(ds["Y"]).to(dev)
    keep, problems = [], []
    for p in range(2, W.P + 1):
        Z = torch.from_numpy(Dd.pseudo_inputs(ds["Y"][:, : p - 1], W.M, seed=p)).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous())
        problems.append(pr)
        keep.append(k)
    fr = G.fit_batch(problems, np.tile(W.X0, (W.P - 1, 1)), max_evals=W.EV, g_tol=-1.0, device=0)
    torch.cuda.synchronize()
    return fr.theta


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gpu_fit_equals_single_process(world, tmp_path):
    got = _run_world(world, str(tmp_path / "theta.json"))
    assert got["world"] == world
    flat = sorted(p for s in got["shards"] for p in s)
    assert flat == list(range(1, W.P + 1))                       # disjoint, complete partition
    assert all(len(s) > 0 for s in got["shards"])
    th = np.array(got["theta"])
    np.testing.assert_array_equal(th[1:], _serial())
    assert np.all(th[1:] > 0)


def _serial_chain():
    from gparatscale import data as Dd
    ds = Dd.gpar_dataset(W.N, W.P, seed=3, observation_noise=0.5, n_star=W.NS)
    dev = torch.device("cuda", 0)
    t_d = torch.from_numpy(ds["t"]).to(dev)
    Y_d = torch.from_numpy(ds["Y"]).to(dev)
    ts_d = torch.from_numpy(ds["t_star"]).to(dev)
    keep, problems = [], []
    outs = list(range(2, W.P + 1))
    for p in outs:
        Z = torch.from_numpy(Dd.pseudo_inputs(ds["Y"][:, : p - 1], W.M, seed=p)).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(), qu_kuu_noise=True)
        problems.append(pr)
        keep.append((k, Z))
    chain = torch.zeros((W.NS, W.P), dtype=torch.float64, device=dev)
    chain[:, 0] = torch.from_numpy(ds["F_star"][:, 0]).to(dev)
    fr, means, stds = G.fit_predict_batch(problems, np.tile(W.X0, (len(outs), 1)), ts_d,
                                          [None] * len(outs), max_evals=W.EV, g_tol=-1.0,
                                          chain=chain, chain_cols=[p - 1 for p in outs])
    torch.cuda.synchronize()
    return (fr.theta, np.array([m.cpu().numpy() for m in means]),
            np.array([s.cpu().numpy() for s in stds]))


@pytest.mark.parametrize("world", [2, 3])
def test_cross_rank_chained_sweep_equals_fit_predict_chain(world, tmp_path):
    got = _run_world(world, str(tmp_path / "chain.json"), mode="chained")
    th, means, stds = _serial_chain()
    np.testing.assert_array_equal(np.array(got["theta"])[1:], th)
    np.testing.assert_array_equal(np.array(got["means"]), means)
    np.testing.assert_array_equal(np.array(got["stds"]), stds)
    assert np.all(np.isfinite(means)) and np.all(stds > 0)


@pytest.mark.parametrize("world", [2, 3])
def test_cross_rank_chained_blocks_equal_fit_predict_chain(world, tmp_path):
    """bench.py's staggered chained path (assign_chained blocks, chained_sweep_blocks' point-to-point
    relay and final broadcast) with the real posteriors on device tensors: bit-identical to one
    single-process gpar_fit_predict_chain."""
    got = _run_world(world, str(tmp_path / "blocks.json"), mode="chained_blocks")
    flat = [p for s in got["shards"] for p in s]
    assert sorted(flat) == list(range(1, W.P + 1))
    th, means, stds = _serial_chain()
    np.testing.assert_array_equal(np.array(got["theta"])[1:], th)
    np.testing.assert_array_equal(np.array(got["means"]), means)
    np.testing.assert_array_equal(np.array(got["stds"]), stds)
