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


def test_launcher_parent_never_initialises_hip(monkeypatch, capfd):
    """the launcher parent must stay HIP-free.  Every torch entry point that
    could initialise HIP raises here; the parent still counts devices, spawns the ranks and
    forwards rank 0's line (the stub ranks are separate processes)."""
    import importlib.util
    import torch

    def boom(*a, **k):
        raise AssertionError("the launcher parent initialised HIP")

    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setattr(torch.cuda, "is_available", boom)
    monkeypatch.setattr(torch.cuda, "init", boom)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    spec = importlib.util.spec_from_file_location("bench_launch_check", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.launch_ranks(2, ["--gpus", "2", "--stub"], stub=True) == 0
    line = json.loads(capfd.readouterr().out.strip().splitlines()[-1])
    assert line["n_gpus"] == 2


def test_visible_gpu_count_reads_kfd_topology(tmp_path):
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_count_check", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for i, gid in enumerate([0, 0, 51234, 7781, 9123]):   # two CPU nodes, three GPUs
        (tmp_path / str(i)).mkdir()
        (tmp_path / str(i) / "gpu_id").write_text(f"{gid}\n")
    (tmp_path / "junk").mkdir()                           # no gpu_id file: ignored
    assert bench.visible_gpu_count(str(tmp_path), env={}) == 3
    assert bench.visible_gpu_count(str(tmp_path), env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.visible_gpu_count(str(tmp_path), env={"ROCR_VISIBLE_DEVICES": ""}) == 0
    assert bench.visible_gpu_count(str(tmp_path / "absent"), env={}) == 0


def test_launcher_fails_fast_when_a_rank_dies():
    """rank 1 exits with status 3 before its gather; rank 0 is then waiting in
    the gloo all_gather for it.  The launcher must notice, terminate rank 0 and return 3 well before
    the process group's timeout (set high here so only the launcher can end the wait)."""
    import time
    env_timeout = dict(GPAR_PG_TIMEOUT_S="600")
    t0 = time.monotonic()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_timeout)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub",
                        "--stub-fail", "1:3"], env=env, capture_output=True, text=True, timeout=90)
    dt = time.monotonic() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert dt < 30, dt
    assert "rank 1 exited with status 3" in r.stderr
    assert not r.stdout.strip()   # no JSON line from a failed job


def test_launcher_fails_fast_when_rank0_dies():
    r = _bench("--gpus", "3", "--stub", "--stub-fail", "0:5", timeout=90)
    assert r.returncode == 5, r.stderr[-2000:]
    assert "rank 0 exited with status 5" in r.stderr
