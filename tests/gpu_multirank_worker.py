"""One rank of tests/test_gpu_multirank.py (started by the test as a child process, with RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT in its environment; every rank uses cuda:0).

The multi-GPU path of bench.py with the real GPU library: rank 0 builds the GPAR data and
broadcasts it (shard.broadcast_inputs, over gloo here, RCCL in bench), each rank fits the GPAR
outputs assign_outputs() gives it with one batched gpar_fit on device inputs, and
shard.gather_thetas all-reduces the P x 5 rows.  Rank 0 writes the gathered rows to argv[1].
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

N, P, M, EV = 3000, 6, 32, 20
X0 = [0.0, 0.0, 0.0, 0.0, -2.0]


def main(out):
    from gparatscale import api as G
    from gparatscale import data as Dd
    from gparatscale import shard as S
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t_h = torch.zeros(N, dtype=torch.float64)
        Y_h = torch.zeros((N, P), dtype=torch.float64)
        if rank == 0:
            ds = Dd.gpar_dataset(N, P, seed=3, observation_noise=0.5)
            t_h.copy_(torch.from_numpy(ds["t"]))
            Y_h.copy_(torch.from_numpy(ds["Y"]))
        S.broadcast_inputs((t_h, Y_h))
        dev = torch.device("cuda", 0)
        t_d, Y_d = t_h.to(dev), Y_h.to(dev)
        mine = [p for p in S.assign_outputs(P, world)[rank] if p >= 2]
        res = {}
        if mine:
            keep, problems = [], []
            for p in mine:
                Z = torch.from_numpy(Dd.pseudo_inputs(Y_h.numpy()[:, : p - 1], M, seed=p)).to(dev)
                pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous())
                problems.append(pr)
                keep.append(k)
            fr = G.fit_batch(problems, np.tile(X0, (len(mine), 1)), max_evals=EV, g_tol=-1.0,
                             device=0)
            torch.cuda.synchronize()
            res = {p: fr.theta[i] for i, p in enumerate(mine)}
        th = S.gather_thetas(res, P)
        if rank == 0:
            with open(out, "w") as f:
                json.dump({"world": world, "shards": S.assign_outputs(P, world),
                           "theta": th.tolist()}, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
