"""bench.py --gpus N started directly (no torchrun): the parent starts N rank processes itself.

CPU only.  With --stub the ranks join a gloo group and report their output shards instead of
running the job (gparatscale.shard.assign_outputs, the partition the GPU ranks use); without it
the parent must refuse to run when fewer than N devices are visible (none here)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_launcher_spawns_ranks_with_disjoint_shards():
    r = _bench("--gpus", "2", "--stub")
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    ranks = sorted(line["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == [0, 1]
    assert [x["local_rank"] for x in ranks] == [0, 1]
    a, b = (set(x["outputs"]) for x in ranks)
    assert a and b and not (a & b)
    assert a | b == set(range(1, line["P"] + 1))


def test_launcher_four_ranks():
    r = _bench("--gpus", "4", "--stub", "--config", "dtc")
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 4
    flat = sorted(p for x in line["ranks"] for p in x["outputs"])
    assert flat == list(range(1, line["P"] + 1))


def test_launcher_refuses_missing_devices():
    # no GPU in this container: --gpus 2 must fail before any rank starts
    r = _bench("--gpus", "2")
    assert r.returncode == 2
    assert "device(s) visible" in r.stderr
