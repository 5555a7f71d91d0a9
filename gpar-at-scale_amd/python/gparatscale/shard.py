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


# fp64 MFMA peak (flop/s) and HBM bandwidth (B/s) of one MI355X: the sized cost model below
# prices memory-bound bytes in flop-equivalents at their ratio
_PEAK_FLOPS, _PEAK_BYTES = 78.6e12, 8.0e12


def output_cost_sized(p: int, n: int, m: int, evals: int) -> float:
    """Cost of output p's fit at n training points and m pseudo-points in flop-equivalents, where
    the input width D = p - 1 matters (BASELINE config 5: N = 1e7, M = 1024, D up to 255).  Per
    evaluation the Gram's N M (M + 1) flops and the cached whitening's 8 N (2 Mp + 20) bytes; once
    per fit the distance pass, 2 N Mp D flops on MFMA (the fit computes an output's distances
    once and every evaluation reads them, include/gpar_hip.h gpar_ctx_set_dist_cache), spread
    over its `evals` evaluations.  The temporal-only output 1 is O(N)."""
    mp = (m + 127) // 128 * 128
    if p == 1:
        return 400.0 * n
    d = p - 1
    gram = float(n) * m * (m + 1)
    whiten = 8.0 * n * (2 * mp + 20) * _PEAK_FLOPS / _PEAK_BYTES
    dist = 2.0 * n * mp * d / max(int(evals), 1)
    return gram + whiten + dist


def assign_outputs(P: int, world: int, cost=None) -> list[list[int]]:
    """Longest-processing-time-first assignment of outputs 1..P to `world` ranks.  cost(p): an
    output's relative cost (default output_cost, the north config's D-independent model).

    Deterministic (ties broken by rank), every output owned by exactly one rank."""
    cost = cost or output_cost
    heap = [(0.0, r) for r in range(world)]
    owned: list[list[int]] = [[] for _ in range(world)]
    for p in sorted(range(1, P + 1), key=lambda q: (-cost(q), q)):
        load, r = heapq.heappop(heap)
        owned[r].append(p)
        heapq.heappush(heap, (load + cost(p), r))
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


# ---------------------------------------------------------------------------- chained, staggered
# With chained inference inputs the fits are independent but the predictions are serial in output
# order.  chained_predictions above runs the sweep after every rank's fits: each prediction then
# runs on one GPU while the others wait (63 x 14.4 ms at north, the rank's fits 2.3 s before it).
# assign_chained instead gives every rank a contiguous block of outputs, early blocks smaller, so
# that the owner of the first block finishes its fits first and starts the sweep while the later
# ranks are still fitting; each later block is sized so its fits end about when the sweep reaches
# it.  chained_sweep_blocks then passes the means along block by block (point to point).
# Defaults: one rank's batched fit + posterior at the north config, fit_ms(n) ~ FIT_FIXED_MS +
# FIT_MS_PER_OUTPUT n, and one chained prediction SWEEP_MS_PER_OUTPUT, least-squares fitted to the
# r05s one-GPU shard lines (bench --shard R/8 --inference chained, ranks 0 / 3 / 7 with 6 / 8 / 9
# GPAR outputs: 1789, 2155, 2453 ms of fits, 13.71 ms per chained prediction;
# profiles/chained_projection_r05s.json).  assign_chained picks the same blocks as with r05l's.
FIT_FIXED_MS = 477.0
FIT_MS_PER_OUTPUT = 216.0
SWEEP_MS_PER_OUTPUT = 13.7
# a block of k means (8 N* bytes each) to the next owner: ASSUMED xGMI figures (never measured on
# this pool, whose boxes have one GPU): 50 GB/s effective and 40 us per transfer
XFER_GBS_ASSUMED = 50.0
XFER_LAT_MS_ASSUMED = 0.04


def chained_schedule(blocks, fit_ms, sweep_ms, xfer_ms):
    """Timeline of a staggered chained job: blocks[r] = number of GPAR outputs of rank r (in output
    order), fit_ms(n) its fit time, sweep_ms one prediction, xfer_ms(k) the transfer of k means to
    the next owner.  Returns (makespan_ms, [(fit_end, sweep_start, sweep_end)] per rank)."""
    t_prev, done, rows = None, 0, []
    for n in blocks:
        f = fit_ms(n) if n else 0.0
        start = f if t_prev is None else max(f, t_prev + (xfer_ms(done) if done else 0.0))
        end = start + sweep_ms * n
        rows.append((f, start, end))
        if n:
            t_prev, done = end, done + n
    return max(r[2] for r in rows), rows


def assign_chained(P: int, world: int, fit_ms=None, sweep_ms: float = SWEEP_MS_PER_OUTPUT,
                   xfer_ms=None) -> list[list[int]]:
    """Contiguous output blocks for a chained job over `world` ranks: rank r owns GPAR outputs
    a_r..b_r with a_{r+1} = b_r + 1 (output 1, the temporal-only chain whose inference inputs are
    given, goes to rank 0).  The block sizes minimise chained_schedule's makespan (dynamic program
    over ranks; every rank gets at least one output when P - 1 >= world).  Deterministic."""
    fit_ms = fit_ms or (lambda n: FIT_FIXED_MS + FIT_MS_PER_OUTPUT * n)
    xfer_ms = xfer_ms or (lambda k: 0.0)
    G = P - 1
    lo = 1 if G >= world else 0
    INF = float("inf")
    # best[r][k]: earliest end of the sweep through ranks 0..r owning the first k GPAR outputs
    best = [[INF] * (G + 1) for _ in range(world)]
    arg = [[0] * (G + 1) for _ in range(world)]
    for k in range(lo, G + 1):
        best[0][k] = (fit_ms(k) if k else 0.0) + sweep_ms * k
        arg[0][k] = k
    for r in range(1, world):
        for k in range(G + 1):
            for n in range(lo, k + 1):
                prev = best[r - 1][k - n]
                if prev == INF:
                    continue
                f = fit_ms(n) if n else 0.0
                end = max(f, prev + (xfer_ms(k - n) if k - n else 0.0)) + sweep_ms * n if n else prev
                if end < best[r][k] - 1e-9:
                    best[r][k], arg[r][k] = end, n
    sizes, k = [], G
    for r in range(world - 1, -1, -1):
        n = arg[r][k]
        sizes.append(n)
        k -= n
    sizes.reverse()
    owned, p = [], 2
    for r, n in enumerate(sizes):
        owned.append(([1] if r == 0 else []) + list(range(p, p + n)))
        p += n
    return owned


def chained_sweep_blocks(shards, predict_fn, chain, prepare_fn=None, gather=True):
    """The chained sweep over contiguous blocks (assign_chained): each rank receives the earlier
    blocks' predicted means point to point from their owners, predicts its own block in order
    (predict_fn(p, chain) -> (mean, std), its next output prepared ahead with prepare_fn), and
    sends its block's means to every later rank.  No rank waits in a collective for a rank that is
    still fitting.  gather: at the end the last rank broadcasts the whole chain, so every rank
    holds every mean (as chained_predictions leaves it).  `chain` as chained_predictions'.
    Returns {p: (mean, std)} for this rank's outputs."""
    import torch
    import torch.distributed as dist
    on = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    rank = dist.get_rank() if on else 0
    world = dist.get_world_size() if on else 1
    gp = [[p for p in s if p >= 2] for s in shards]
    for r in range(1, world):
        prev = [p for s in gp[:r] for p in s]
        if gp[r] and prev and min(gp[r]) < max(prev):
            raise ValueError("chained_sweep_blocks: blocks must be contiguous in output order")
    # gloo moves host tensors point to point; RCCL moves device tensors
    host = on and dist.get_backend() == "gloo"

    def cols(r):
        return [p - 1 for p in gp[r]]

    own = gp[rank]
    if prepare_fn is not None and own:
        prepare_fn(own[0])   # beside the wait for the earlier blocks
    for r in range(rank):     # the earlier blocks, in order
        if not gp[r]:
            continue
        buf = torch.empty((chain.shape[0], len(gp[r])), dtype=chain.dtype,
                          device="cpu" if host else chain.device)
        dist.recv(buf, src=r)
        chain[:, cols(r)] = buf.to(chain.device)
    mine = {}
    for i, p in enumerate(own):
        if prepare_fn is not None and i + 1 < len(own):
            prepare_fn(own[i + 1])
        mean, std = predict_fn(p, chain)
        mine[p] = (mean, std)
        chain[:, p - 1] = torch.as_tensor(mean, dtype=chain.dtype).to(chain.device)
    works = []
    if on and own:
        blk = chain[:, cols(rank)].contiguous()
        blk = blk.cpu() if host else blk
        for r in range(rank + 1, world):
            works.append(dist.isend(blk, dst=r))
    for w in works:
        w.wait()
    if on and gather:
        last = max((r for r in range(world) if gp[r]), default=0)
        full = chain.contiguous()
        full = full.cpu() if host else full
        dist.broadcast(full, last)
        chain.copy_(full.to(chain.device))
    return mine
