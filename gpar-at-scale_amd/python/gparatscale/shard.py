"""Output sharding across GPUs (one process per GPU, torch.distributed over RCCL / gloo).

The reference fits GPAR outputs one after another in a serial loop
(examples/GPAR_scaled_examples.jl:132-175, gpar_scaled_inference.jl:20-136 per output).  Output p
only needs the *observed* previous outputs y_1..y_{p-1} as inputs, never a fitted model of them,
so outputs are independent work units: each rank fits and predicts its own outputs with no
data-path collective.  Shared inputs (t, Y, t*) are broadcast from rank 0 once; the fitted
hyperparameters (P x 5 doubles) are gathered with one small all-reduce per step.
"""
from __future__ import annotations

import heapq

import numpy as np

# Per-objective-evaluation cost of output p at the north config on one MI355X (bench r02x,
# profiles/rocprof_bench_r02x_north_stats.csv): the batched fit whitens every GPAR output beside
# the previous output's Gram on the CU split, with every output's distances cached (N >= 2^16,
# include/gpar_hip.h gpar_ctx_set_dist_cache), so one output-evaluation costs the Gram's span,
# ~5.1 ms, whatever the input dimension D = p - 1; the dense tail, carries and gains add ~0.1.
# The temporal-only output 1 is ~20x cheaper.  Only relative sizes matter: LPT then deals the
# GPAR outputs evenly (8 GPUs: seven ranks with 8 of them, one with 7 plus output 1).
OUTPUT_EVAL_MS = 5.2
SDE_MS = 0.4


def output_cost(p: int) -> float:
    return SDE_MS if p == 1 else OUTPUT_EVAL_MS


def assign_outputs(P: int, world: int) -> list[list[int]]:
    """Longest-processing-time-first assignment of outputs 1..P to `world` ranks.

    Deterministic (ties broken by rank), every output owned by exactly one rank."""
    heap = [(0.0, r) for r in range(world)]
    owned: list[list[int]] = [[] for _ in range(world)]
    for p in sorted(range(1, P + 1), key=lambda q: (-output_cost(q), q)):
        load, r = heapq.heappop(heap)
        owned[r].append(p)
        heapq.heappush(heap, (load + output_cost(p), r))
    return [sorted(o) for o in owned]


def broadcast_inputs(tensors, src: int = 0):
    """Broadcast already-allocated tensors from rank `src` (no-op without a process group)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    for x in tensors:
        dist.broadcast(x, src)


def gather_thetas(local: dict, P: int, device=None) -> np.ndarray:
    """All ranks' fitted hyperparameters as a P x 5 array (row p-1 = output p).

    Each output is owned by exactly one rank, so a sum all-reduce of zero-padded rows is a gather."""
    import torch
    import torch.distributed as dist
    th = np.zeros((P, 5))
    for p, v in local.items():
        v = np.asarray(v, dtype=np.float64)
        th[p - 1, : v.shape[0]] = v
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        tt = torch.from_numpy(th)
        if device is not None:
            tt = tt.to(device)
        dist.all_reduce(tt)
        th = tt.cpu().numpy()
    return th


def owners_of(shards: list[list[int]]) -> dict[int, int]:
    """Output -> owning rank, from an assign_outputs() partition."""
    return {p: r for r, owned in enumerate(shards) for p in owned}


def chained_predictions(outputs, owners: dict, predict_fn, chain, prepare_fn=None):
    """Predictions with chained inference inputs across ranks (GPAR_scaled_examples.jl:172,
    eeg.jl:249,274: output p's inference inputs include the predicted means of earlier outputs).

    `chain` (N* x K tensor, same contents on every rank) holds the inference inputs: columns the
    caller fills (observed / true inputs) and one column p - 1 per output p in `outputs`, written
    here.  Outputs are taken in the given order; the owner of p calls predict_fn(p, chain) ->
    (mean, std) and then broadcasts the mean (8 N* bytes over RCCL / gloo) from itself, and every
    rank stores it in chain[:, p - 1] before the next output starts.  The fits are independent
    and run before this on each rank; only this ordered sweep is serial across ranks.
    prepare_fn(p) (optional, e.g. Posterior.prepare) queues the part of p's prediction that does
    not read the chain; each rank calls it for its next output before predicting the current one
    (and for its first output up front), so that part runs beside the sweep.
    Returns {p: (mean, std)} for this rank's outputs."""
    import torch
    import torch.distributed as dist
    on = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    rank = dist.get_rank() if on else 0
    col = torch.empty(chain.shape[0], dtype=chain.dtype, device=chain.device)
    mine = {}
    own = [p for p in outputs if owners[p] == rank]
    nxt = {a: b for a, b in zip(own, own[1:])}
    if prepare_fn is not None and own:
        prepare_fn(own[0])
    for p in outputs:
        owner = owners[p]
        if owner == rank:
            if prepare_fn is not None and p in nxt:
                prepare_fn(nxt[p])
            mean, std = predict_fn(p, chain)
            mine[p] = (mean, std)
            col.copy_(torch.as_tensor(mean, dtype=chain.dtype).to(chain.device))
        if on:
            dist.broadcast(col, owner)
        chain[:, p - 1].copy_(col)
    return mine
