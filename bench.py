#!/usr/bin/env python3
"""bench.py -- GPAR-at-scale fit+predict throughput on MI355X (BASELINE.json metric).

One *step* = the whole GPAR job of BASELINE.json's north star (N=1e6 time points, M=512
pseudo-points, P=64 outputs), the per-output driver of examples/GPAR_scaled_examples.jl:86-175:
  * output 1: get_sde_predictions (temporal-only LGSSM: NM fit + RTS smoothing at t*),
  * outputs 2..P: get_optim_scaled_gpar_params (DTC objective, Nelder-Mead with exactly
    `--evals` objective evaluations per output, fixed init log theta = (0, 0, 0, 0, -2)) and the
    prediction half of get_gpar_scaled_predictions (analytic mode) at N* = N test times with the
    noiseless previous outputs as inference inputs (GPAR_scaled_examples.jl:139 style).
Inputs (t, Y, pseudo-inputs, test grid) are resident in HBM before the timed region.
Multi-GPU: one process per GPU (torch.distributed, RCCL); outputs are sharded by cost-balanced assignment (gparatscale.shard),
shared inputs are broadcast from rank 0 once (untimed); per step the fitted thetas are
all-gathered.  value = N * P / wall-clock per step (pts*outputs/s, whole job).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config north|eeg|dtc|small|ssm]

Launch: under torchrun (WORLD_SIZE set) every process is one rank.  Started directly with
--gpus N > 1, the parent checks that N devices are visible (KFD topology in sysfs: it never
initialises HIP, nor imports torch) and starts N rank processes itself (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment); it forwards rank 0's JSON
line and exits with the first non-zero rank status.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpar-at-scale_amd", "python"))

import numpy as np  # noqa: E402

CONFIGS = {
    # BASELINE.json metric / north star: N=1e6, M=512, P=64
    "north": dict(N=1_000_000, M=512, P=64, evals=50, out_kernel="matern52"),
    # configs[3]: EEG-shaped N~1e5, M=512, P=64
    "eeg": dict(N=100_000, M=512, P=64, evals=50, out_kernel="matern52"),
    # configs[1]: DTC sparse GPAR N=1e5, M=256, P=8, RBF (EQ) output kernel
    "dtc": dict(N=100_000, M=256, P=8, evals=50, out_kernel="eq"),
    "small": dict(N=20_000, M=128, P=4, evals=20, out_kernel="matern52"),
    # configs[2]: state-space (Matern-3/2) temporal-only chains, N=1e6, P=16 (a9, batched over
    # chains: one NM over all chains, then RTS smoothing at N* = N test times)
    "ssm": dict(N=1_000_000, M=0, P=16, evals=50, out_kernel="matern32", temporal=True),
    # configs[4] (stress): N=1e7, M=1024, P=256 DTC-GPAR, per-evaluation throughput only (SURVEY
    # §8d: "one full fit would be hours"): each step is one batched Nelder-Mead fit of `evals`
    # objective evaluations per GPAR output of the rank's shard (stress_main)
    "stress": dict(N=10_000_000, M=1024, P=256, evals=6, out_kernel="matern52", per_eval=True),
}
# MI355X dense fp64 matrix peak: 1024 SIMDs x 2048 flop per v_mfma_f64_16x16x4_f64 / 64 cycles
# (SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA = 64, profiles/) x 2.4 GHz = 78.6 TF/s (AMD spec value)
FP64_MFMA_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0
# HBM bytes per launch from the PMC passes of this round's sources (tools/pmc_passes.sh, D = 32),
# else the newest earlier round's (the line names the file it used: roofline.traffic_source)
PMC_FILE = "pmc_gram_whiten_r06.json"
PMC_FALLBACK = "pmc_gram_whiten_r05.json"
# the stress config's Gram traffic (tools/pmc_stress.sh: N = 1e7, M = 1024)
PMC_STRESS_FILE = "pmc_gram_whiten_stress_r06.json"


def pmc_traffic(names):
    """(Gram bytes, whitening bytes, file) per launch from the first profiles/ PMC summary found."""
    for name in names:
        f = os.path.join(ROOT, "profiles", name)
        if os.path.exists(f):
            with open(f) as fh:
                pj = json.load(fh)
            return pj.get("hbm_bytes_per_launch"), pj.get("whiten_hbm_bytes_per_launch"), name
    return None, None, None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="north", choices=sorted(CONFIGS))
    ap.add_argument("--evals", type=int, default=None)
    ap.add_argument("--predict", default="analytic", choices=["analytic", "mc", "path"],
                    help="prediction estimator: analytic (S -> infinity limit), mc (the reference's "
                         "100-sample estimator, gpar_scaled_inference.jl:110-130), path (tmp.jl:"
                         "119-167: q(u) draws + posterior_rand paths of the time GP)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--separate-predict", action="store_true",
                    help="gpar_fit then one gpar_predict per output (q(u) recomputes the Gram at the "
                         "fitted theta) instead of gpar_fit_predict (reuses the fit's Gram there)")
    ap.add_argument("--lanes", type=int, default=1, choices=[1, 2],
                    help="HIP streams a batched objective alternates outputs over (gpar_ctx_set_lanes); "
                         "2 overlaps one output's whitening with another's Gram (+2%% throughput, but "
                         "per-launch kernel durations then include the sharing)")
    ap.add_argument("--cu-split", type=int, default=None,
                    help="CUs per XCD that whiten beside the Gram in the batched fit "
                         "(gpar_ctx_set_cu_split; default: the library's, 8 where N Mp^2 >= 1e11); "
                         "0 = whole-chip kernels")
    ap.add_argument("--inference", default="given", choices=["given", "chained"],
                    help="test inputs of output p: 'given' = the noiseless previous outputs at t* "
                         "(GPAR_scaled_examples.jl:139); 'chained' = output 1's true values and the "
                         "PREDICTED means of outputs 2..p-1 (GPAR_scaled_examples.jl:172, eeg.jl:249)")
    ap.add_argument("--inputs", default="device", choices=["device", "host"],
                    help="'device': inputs resident in HBM before the timed region (the bench "
                         "contract's value); 'host': numpy inputs and outputs through the C-ABI's "
                         "host-memory mode (the Julia binding's case), so every step includes the "
                         "library's H2D / D2H copies over PCIe")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank rehearsal on ONE GPU: every rank uses device 0 and the gloo "
                         "backend (RCCL runs one rank per device); exercises the launcher, sharding, "
                         "broadcasts and gathers with the real kernels -- not a scaling measurement")
    ap.add_argument("--qu-noise-free", action="store_true",
                    help="q(u) with the reference's noise-free Cuu (gpar_scaled_inference.jl:157) "
                         "instead of Cuu + sigma^2 I (qu_kuu_noise, the default here: the noise-free "
                         "Cuu of M=512 pseudo-inputs drawn from the data is numerically singular)")
    ap.add_argument("--api", default="batched", choices=["batched", "per-output"],
                    help="'batched': one gpar_fit_predict call for all owned outputs (the library's "
                         "multi-output driver); 'per-output': one single-output gpar_fit_predict call "
                         "per output, as a reference caller's loop through the Julia shim's "
                         "get_gpar_scaled_predictions makes them (GPAR_scaled_examples.jl:132-175)")
    ap.add_argument("--shard", default=None,
                    help="R/W: run exactly rank R's outputs of the W-way output assignment "
                         "(gparatscale.shard.assign_outputs; assign_chained with --inference "
                         "chained) on this one GPU, the code path of one "
                         "rank of a W-GPU job, to predict the per-rank step time")
    ap.add_argument("--dist-cache", default="keep", choices=["keep", "release"],
                    help="'keep' (the bench default): the fit's distance-cache buffers stay allocated "
                         "between calls (gpar_ctx_set_dist_cache_keep; the distances themselves are "
                         "recomputed by every fit, nothing is carried across steps) -- re-allocating "
                         "258 GB per step costs ~5.8 s on MI355X (fresh VRAM is cleared); 'release': "
                         "the library default, freed when each fit call returns")
    ap.add_argument("--h2h-steps", type=int, default=2,
                    help="after the timed device-resident steps, this many host->host steps "
                         "(SURVEY §8d's unit: one pinned upload of t, Y, t*, F* and the pseudo-inputs "
                         "per step, means / stds downloaded), reported as host_to_host beside value")
    ap.add_argument("--schedule", default="",
                    help="schedule knobs as k=v,k=v (gpar_ctx_set_schedule, include/gpar_hip.h: "
                         "overlap, overlap_group, predict_fused, qu_batch, dense_early, "
                         "predict_lanes, serialize, post_gram, compact_rec, dg_rows_w, gram_group)")
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-check-file", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--stub", action="store_true",
                    help="launcher check without a GPU: ranks join a gloo group, take their output "
                         "shards and report them; no compute (tests/test_bench_launch.py)")
    ap.add_argument("--stub-fail", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], stub=args.stub or args.rehearse))
    if args.stub:
        return stub_rank(args)
    if args.cpu_baseline_child:
        return cpu_baseline_child(args)
    if CONFIGS[args.config].get("per_eval"):
        return stress_main(args)
    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    cfg0 = CONFIGS[args.config]
    # the CPU baseline runs in a child process started before anything touches the GPU, so it
    # overlaps the inputs and the warm-up steps; it is joined before the timed region
    cpu_child = None
    if (world0 == 1 and not args.no_cpu_baseline and args.shard is None and args.api == "batched"):
        cpu_child = start_cpu_baseline(args)

    import torch
    import torch.distributed as dist
    import gparatscale as G
    from gparatscale import data as D
    from gparatscale import shard as S

    cfg = dict(CONFIGS[args.config])
    if args.evals:
        cfg["evals"] = args.evals
    N, M, P, EV = cfg["N"], cfg["M"], cfg["P"], cfg["evals"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[rank {rank}] note: --gpus {args.gpus} but WORLD_SIZE={world}; n_gpus reports WORLD_SIZE")
    if args.rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a bounded collective timeout: a rank stuck waiting for a dead peer fails instead of
        # sitting out torch's 10-minute default (the launcher also ends the job on the first
        # failing rank)
        if args.rehearse:
            dist.init_process_group("gloo", timeout=pg_timeout())
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout())

    # every rank's view of the job: the next SCALE record shows the backend (nccl = RCCL) and N
    # distinct devices
    me = {"rank": rank, "local_rank": local, "device": torch.cuda.current_device(),
          "world_size": dist.get_world_size() if world > 1 else 1,
          "backend": dist.get_backend() if world > 1 else None, "host": socket.gethostname()}
    try:
        props = torch.cuda.get_device_properties(dev)
        me["device_name"] = props.name
        me["device_uuid"] = str(getattr(props, "uuid", "")) or None
        me["pci_bus_id"] = getattr(props, "pci_bus_id", None)
    except Exception:   # noqa: BLE001  telemetry only
        pass
    rank_info = [me]
    if world > 1:
        rank_info = [None] * world
        dist.all_gather_object(rank_info, me)

    # ---------------------------------------------------------------- inputs (untimed)
    t0 = time.perf_counter()
    if rank == 0:
        ds = D.gpar_dataset(N, P, seed=0, observation_noise=0.8)
        t_h, Y_h, ts_h, Fs_h = ds["t"], ds["Y"], ds["t_star"], ds["F_star"]
        n_eff, ns_eff = len(t_h), len(ts_h)
    else:
        n_eff = ns_eff = 0
    if world > 1:
        sz = torch.tensor([n_eff, ns_eff], device=dev)
        dist.broadcast(sz, 0)
        n_eff, ns_eff = int(sz[0]), int(sz[1])
    t_d = torch.empty(n_eff, dtype=torch.float64, device=dev)
    Y_d = torch.empty((n_eff, P), dtype=torch.float64, device=dev)
    ts_d = torch.empty(ns_eff, dtype=torch.float64, device=dev)
    Fs_d = torch.empty((ns_eff, P), dtype=torch.float64, device=dev)
    if rank == 0:
        t_d.copy_(torch.from_numpy(t_h)); Y_d.copy_(torch.from_numpy(Y_h))
        ts_d.copy_(torch.from_numpy(ts_h)); Fs_d.copy_(torch.from_numpy(Fs_h))
    S.broadcast_inputs((t_d, Y_d, ts_d, Fs_d))   # RCCL broadcast of the shared inputs over xGMI
    temporal = cfg.get("temporal", False)
    # chained inference inputs: contiguous output blocks, early ranks smaller, so the sweep starts
    # on the first rank while the later ones still fit (shard.assign_chained); given inputs: LPT
    chained_job = args.inference == "chained" and not temporal
    assign = S.assign_chained if chained_job else S.assign_outputs
    shards = assign(P, world) if not temporal else \
        [[p for p in range(1, P + 1) if (p - 1) % world == r] for r in range(world)]
    mine = shards[rank]
    shard_of = None
    if args.shard:
        if world > 1 or temporal:
            sys.exit("--shard R/W: one process, the GPAR configs")
        r_, w_ = (int(x) for x in args.shard.split("/"))
        shard_of = (r_, w_)
        shards = assign(P, w_)
        mine = shards[r_]
    gpar_out = [p for p in mine if p >= 2] if not temporal else []
    Yh = Y_d.cpu().numpy() if (gpar_out or args.inference == "chained") else None
    # q(u) with Kuu + sigma^2 I (qu_kuu_noise) unless --qu-noise-free: the reference's jitter-free
    # Cuu (gpar_scaled_inference.jl:157) is numerically singular for M=512 pseudo-inputs drawn
    # from the data at fitted lengthscales; the objective itself is unchanged (dtc.jl:35,119).
    qn = not args.qu_noise_free
    problems, keep, ycols, Zs = [], [], {}, {}
    for p in gpar_out:
        ycols[p] = Y_d[:, p - 1].contiguous()
        Zs[p] = torch.from_numpy(D.pseudo_inputs(Yh[:, : p - 1], M, seed=p)).to(dev)
        pr, k = G.make_problem(Y_d[:, : p - 1], Zs[p], t_d, ycols[p], cfg["out_kernel"], "matern52",
                               qu_kuu_noise=qn)
        problems.append(pr)
        keep.append(k)
    y1 = Y_d[:, 0].contiguous() if 1 in mine else None
    if temporal:   # every owned output is a temporal-only chain (rows of one contiguous block)
        y1 = Y_d[:, [p - 1 for p in mine]].T.contiguous() if mine else None
    host = args.inputs == "host"
    if args.api == "per-output" and (args.inference != "given" or temporal or args.separate_predict):
        sys.exit("--api per-output: given inference inputs, the GPAR configs only")
    if host:
        if world > 1 or args.inference != "given" or temporal or args.separate_predict:
            sys.exit("--inputs host: one rank, given inference inputs, the GPAR configs only")
        # the same problems from host (numpy) buffers: D x N ColVecs, as the Julia shim passes them
        Yh_all = Y_d.cpu().numpy()
        t_hh, ts_hh, Fs_hh = t_d.cpu().numpy(), ts_d.cpu().numpy(), Fs_d.cpu().numpy()
        problems, keep = [], []
        for p in gpar_out:
            pr, k = G.make_problem(np.ascontiguousarray(Yh_all[:, : p - 1].T), Zs[p].cpu().numpy().T,
                                   t_hh, np.ascontiguousarray(Yh_all[:, p - 1]), cfg["out_kernel"],
                                   "matern52", qu_kuu_noise=qn)
            problems.append(pr)
            keep.append(k)
        Vs_h = [np.ascontiguousarray(Fs_hh[:, : p - 1].T) for p in gpar_out]
        y1_h = np.ascontiguousarray(Yh_all[:, 0]) if y1 is not None else None
    x0 = np.tile(np.array([0.0, 0.0, 0.0, 0.0, -2.0]), (len(problems), 1))
    torch.cuda.synchronize()
    log(f"[rank {rank}] inputs ready in {time.perf_counter() - t0:.1f}s: N={n_eff} N*={ns_eff} "
        f"M={M} P={P} outputs={mine}")

    ctx = G.context(local)
    ctx.set_lanes(args.lanes)
    knobs = {}
    for kv in filter(None, args.schedule.split(",")):
        k, v = kv.split("=")
        ctx.set_schedule(k.strip(), int(v))
        knobs[k.strip()] = int(v)
    if args.cu_split is not None:
        ctx.set_cu_split(args.cu_split)
    cu_split = ctx.cu_split()
    # the default split applies only to batched fits with N Mp^2 >= 1e11 (include/gpar_hip.h)
    mp = (M + 127) // 128 * 128
    if args.cu_split is None and float(N) * mp * mp < 1e11:
        cu_split = 0
    chained = args.inference == "chained" and not temporal
    if chained:
        # inference inputs: column 0 = output 1's true values at t*, column p-1 = output p's
        # predicted mean, written as the predictions run in output order
        chain_d = Fs_d.clone()
        owners = S.owners_of(shards)
        gpar_all = list(range(2, P + 1))
        if shard_of:
            # untimed set-up of the one-rank chained measurement: every output's posterior (a short
            # fit: the sweep's cost does not depend on theta), so the timed step can run the whole
            # sweep the real job's ranks wait through
            probs_all, keep_all = [], []
            for p in gpar_all:
                if p not in Zs:
                    Zs[p] = torch.from_numpy(D.pseudo_inputs(Yh[:, : p - 1], M, seed=p)).to(dev)
                    ycols[p] = Y_d[:, p - 1].contiguous()
                pr, k = G.make_problem(Y_d[:, : p - 1], Zs[p], t_d, ycols[p], cfg["out_kernel"],
                                       "matern52", qu_kuu_noise=qn)
                probs_all.append(pr)
                keep_all.append(k)
            post_all = G.fit_posterior(probs_all, np.tile(x0[0], (len(probs_all), 1)), max_evals=6,
                                       g_tol=-1.0, device=local, keep=keep_all)

    ctx.set_dist_cache_keep(args.dist_cache == "keep")
    per_output = args.api == "per-output"
    last = {}   # the last step's FitResult per output (the self-check after the timed region)

    def fit_predict_outputs(ts, Vs):
        """get_gpar_scaled_predictions for every owned GPAR output: one batched call, or one
        single-output call per output (--api per-output)."""
        if not per_output:
            return G.fit_predict_batch(problems, x0, ts, Vs, max_evals=EV, g_tol=-1.0,
                                       mode=args.predict, samples=100, seed=gpar_out[0],
                                       device=local)
        th, nl = np.zeros((len(problems), 5)), np.zeros(len(problems))
        means, stds = [], []
        for i in range(len(problems)):
            fr, m, sd = G.fit_predict_batch(problems[i:i + 1], x0[i:i + 1], ts, Vs[i:i + 1],
                                            max_evals=EV, g_tol=-1.0, mode=args.predict, samples=100,
                                            seed=gpar_out[0] + i, device=local)
            th[i], nl[i] = fr.theta[0], fr.nlml[0]
            means.append(m[0])
            stds.append(sd[0])
        return G.FitResult(th, nl, np.full(len(problems), EV, dtype=np.int32)), means, stds

    def step():
        res = {}
        if host:
            if problems:
                fr, _, _ = fit_predict_outputs(ts_hh, Vs_h)
                last["fit"] = fr
                for i, p in enumerate(gpar_out):
                    res[p] = fr.theta[i]
            if y1_h is not None:
                th1, _, _ = G.get_sde_predictions(t_hh, y1_h, ts_hh, "matern52", i_log_time_l=0.0,
                                                  i_log_time_var=0.0, i_log_noise_sigma=-2.0,
                                                  max_evals=EV, g_tol=-1.0, device=local)
                res[1] = np.array(list(th1) + [0.0, 0.0])
            return S.gather_thetas(res, P, dev)
        if chained and world == 1 and not shard_of:
            fr, _, _ = G.fit_predict_batch(problems, x0, ts_d, [None] * len(problems),
                                           max_evals=EV, g_tol=-1.0, mode=args.predict, samples=100,
                                           seed=gpar_out[0], device=local, chain=chain_d,
                                           chain_cols=[p - 1 for p in gpar_out])
            for i, p in enumerate(gpar_out):
                res[p] = fr.theta[i]
        elif chained:
            # independent fits per rank, each keeping its outputs' q(u) on the device
            # (gpar_fit_posterior), then the ordered prediction sweep across ranks: only the
            # inference-input-dependent predictions run inside it, and each predicted mean is
            # broadcast by its owner as soon as it is ready (shard.py)
            post = None
            t_fit0 = time.perf_counter()
            if problems:
                post = G.fit_posterior(problems, x0, max_evals=EV, g_tol=-1.0, device=local,
                                       keep=keep)
                for i, p in enumerate(gpar_out):
                    res[p] = post.theta[i]
            torch.cuda.synchronize()
            t_sw = time.perf_counter()
            last.setdefault("fit_s", []).append(t_sw - t_fit0)
            if shard_of:
                # one rank of the W-way job on this GPU: its own fits above, then the whole
                # P-output sweep (the other ranks' outputs from the untimed posteriors of the
                # set-up) -- the serial part every rank of the real job waits through
                def pick(p):
                    return ((post, gpar_out.index(p)) if p in gpar_out else
                            (post_all, gpar_all.index(p)))
                S.chained_predictions(
                    gpar_all, {p: 0 for p in gpar_all},
                    lambda p, c: pick(p)[0].predict(pick(p)[1], ts_d, c[:, : p - 1],
                                                    mode=args.predict, samples=100, seed=p),
                    chain_d,
                    prepare_fn=lambda p: pick(p)[0].prepare(pick(p)[1], ts_d))
            else:
                # the staggered sweep: earlier blocks' means arrive point to point, this rank's
                # block runs as soon as its own fits and those means are in (shard.py)
                idx = {p: i for i, p in enumerate(gpar_out)}
                S.chained_sweep_blocks(
                    shards,
                    lambda p, c: post.predict(idx[p], ts_d, c[:, : p - 1], mode=args.predict,
                                              samples=100, seed=p),
                    chain_d, prepare_fn=lambda p: post.prepare(idx[p], ts_d))
            torch.cuda.synchronize()
            last.setdefault("sweep_s", []).append(time.perf_counter() - t_sw)
        elif problems and not args.separate_predict:
            # get_gpar_scaled_predictions for every owned output: batched fit, then predictions
            fr, means, stds = fit_predict_outputs(ts_d, [Fs_d[:, : p - 1] for p in gpar_out])
            last["fit"], last["means"], last["stds"] = fr, means, stds
            for i, p in enumerate(gpar_out):
                res[p] = fr.theta[i]
        elif problems:
            fr = G.fit_batch(problems, x0, max_evals=EV, g_tol=-1.0, device=local)
            for i, p in enumerate(gpar_out):
                res[p] = fr.theta[i]
        if y1 is not None:
            tk = cfg["out_kernel"] if temporal else "matern52"
            th1, m1, v1 = G.get_sde_predictions_device(t_d, y1, ts_d, tk, (0.0, 0.0, -2.0),
                                                       max_evals=EV, device=local)
            last["temporal"] = (m1, v1)
            if temporal:
                for i, p in enumerate(mine):
                    res[p] = np.array(list(np.atleast_2d(th1)[i]) + [0.0, 0.0])
            else:
                res[1] = np.array(list(th1) + [0.0, 0.0])
        for i, p in enumerate(gpar_out if args.separate_predict else []):
            G.predict_scaled(Y_d[:, : p - 1], Zs[p], t_d, ycols[p], res[p], ts_d, Fs_d[:, : p - 1],
                             cfg["out_kernel"], "matern52", mode=args.predict, samples=100,
                             seed=p, device=local, qu_kuu_noise=qn)
        return S.gather_thetas(res, P, dev)   # fitted hyperparameters, P x 5 (tiny)

    if args.qu_noise_free:
        # the reference's noise-free Cuu (gpar_scaled_inference.jl:157-159) can be numerically
        # singular for M = 512 pseudo-inputs drawn from the data: the reference then throws
        # PosDefException, and so does the library -- report that instead of a throughput
        step0 = step

        def step():
            t_fail = time.perf_counter()
            try:
                return step0()
            except G.PosDefException as e:
                torch.cuda.synchronize()
                if rank == 0:
                    print(json.dumps({"metric": "GPAR fit+predict wall-clock (ms) and pts\u00b7outputs/sec, "
                                                f"N={D.fmt_count(N)} M={M} P={P}",
                                      "value": None, "unit": "pts\u00b7outputs/s", "n_gpus": world,
                                      "error": str(e), "qu_convention": "noise-free Cuu (reference)",
                                      "seconds_until_error": time.perf_counter() - t_fail,
                                      "config": {"workload": args.config, "qu_kuu_noise": False}}),
                          flush=True)
                sys.exit(3)
    for _ in range(args.warmup):
        step()
    cpu_res = None
    if cpu_child is not None:   # joined before the timed region (untimed)
        cpu_res = join_cpu_baseline(cpu_child)
    ctx.set_profiling(True)
    ctx.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ts0 = time.perf_counter()
    for _ in range(args.steps):
        theta = step()
    torch.cuda.synchronize()
    busy = (time.perf_counter() - ts0) * 1e3 / args.steps   # this rank's own work, before the barrier
    if world > 1:
        dist.barrier()
    el = (time.perf_counter() - ts0) * 1e3 / args.steps
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e[0])
    # every rank's own times in the line (untimed gather): its step up to the closing barrier and,
    # with chained inputs, its fits + posteriors and its part of the sweep (waits included)
    mine_t = {"step_busy_ms": busy,
              "fit_ms": 1e3 * float(np.mean(last["fit_s"][-args.steps:])) if last.get("fit_s") else None,
              "sweep_ms": 1e3 * float(np.mean(last["sweep_s"][-args.steps:])) if last.get("sweep_s") else None,
              "outputs": mine}
    times_all = [mine_t]
    if world > 1:
        times_all = [None] * world
        dist.all_gather_object(times_all, mine_t)
    for ri, tt in zip(rank_info, times_all):
        ri.update(tt)
    gram_n, gram_ms = ctx.kernel_stats("gram")
    wh_n, wh_ms = ctx.kernel_stats("whiten")
    rnd_n, rnd_ms = ctx.kernel_stats("fit_round")   # round-by-round fits: entry -> values per round
    fc_n, fc_ms = ctx.kernel_stats("fit_call")      # whole batched fits (any schedule)
    # ... and along each round (split fits): entry -> first output's gains -> its whitening -> its
    # short chain -> the first Gram's start -> the last Gram's end -> the values on the host
    marks = {k: ctx.kernel_stats(k) for k in ("head_gains", "head_w0", "head_p0", "head_gram_wait",
                                               "round_grams", "round_tail")}
    rh_n = marks["head_gains"][0]
    rh_ms = sum(marks[k][1] for k in ("head_gains", "head_w0", "head_p0", "head_gram_wait"))
    rt_n, rt_ms = marks["round_tail"]
    pred = {}
    for fam, bound in (("pred_whiten", "hbm"), ("pred_adjoint", "hbm"), ("pred_rows", "hbm"),
                       ("pred_gemm", "mfma"), ("pred_var", "mfma")):
        pn, pms = ctx.kernel_stats(fam)
        if pn:
            w = ctx.kernel_work(fam) / (pms * 1e-3)
            pred[fam] = ({"bound": bound, "achieved": w / 1e9, "unit": "GB/s", "peak": HBM_PEAK_GBS,
                          "frac": w / 1e9 / HBM_PEAK_GBS} if bound == "hbm" else
                         {"bound": bound, "achieved": w / 1e12, "unit": "TFLOP/s",
                          "peak": FP64_MFMA_PEAK_TFLOPS, "frac": w / 1e12 / FP64_MFMA_PEAK_TFLOPS})
            pred[fam].update(launches=pn, avg_ms=pms / pn, ms_per_step=pms / args.steps,
                             work_per_launch=ctx.kernel_work(fam) / pn)
    pwall_n, pwall_ms = ctx.kernel_stats("predictions")   # wall span of each call's predictions
    # the temporal chains' spans, read before the untimed self-check adds launches of its own
    chain_stats = {fam: (ctx.kernel_stats(fam), ctx.kernel_work(fam))
                   for fam in ("chains_logpdf", "chains_smooth")}
    gram_work = ctx.kernel_work("gram")      # flops, N*M*(M+1) per launch
    wh_work = ctx.kernel_work("whiten")      # algorithmic HBM bytes (include/gpar_hip.h)
    try:   # telemetry only: never fails the line
        free_b, total_b = torch.cuda.mem_get_info(dev)
        cached, evictions, held = ctx.dist_cache_stats()
        memory = {"library_workspace_gb": ctx.workspace_bytes() / 1e9, "device_free_gb": free_b / 1e9,
                  "device_total_gb": total_b / 1e9,
                  "dist_cache": {"outputs_cached_last_fit": cached, "oom_evictions": evictions,
                                 "held_gb": held / 1e9, "keep": args.dist_cache == "keep"},
                  "note": "after the timed steps; the workspace includes the fit's distance cache "
                          "only with keep (else it is released when each fit call returns)"}
    except Exception as e:   # noqa: BLE001
        memory = {"error": repr(e)}
    probe = None
    if rank == 0 and cu_split and problems and not host and args.lanes == 1:
        # after the timed region: the same kernels whole-chip (gpar_ctx_set_cu_split(ctx, 0)) in
        # a batched fit of four outputs around D = 32 (pipelined, distance cache), so the line
        # also carries the kernels' own fractions next to the split job's.  (A one-output fit
        # idles the GPU between evaluations and measures ~10 % slower Grams: cold clocks.)
        i = max(0, min(len(problems) - 4, 30))
        sub = problems[i:i + 4]
        ctx.set_cu_split(0)
        ctx.reset_stats()
        G.fit_batch(sub, x0[: len(sub)], max_evals=8, g_tol=-1.0, device=local)
        ctx.set_cu_split(-1 if args.cu_split is None else args.cu_split)
        pg_n, pg_ms = ctx.kernel_stats("gram")
        pw_n, pw_ms = ctx.kernel_stats("whiten")
        if pg_n and pw_n:
            pg = ctx.kernel_work("gram") / (pg_ms * 1e-3) / 1e12
            pw = ctx.kernel_work("whiten") / (pw_ms * 1e-3) / 1e9
            probe = {"outputs": gpar_out[i:i + len(sub)], "evals": 8,
                     "gram": {"avg_ms": pg_ms / pg_n, "achieved_tflops": pg,
                              "frac": pg / FP64_MFMA_PEAK_TFLOPS},
                     "whiten": {"avg_ms": pw_ms / pw_n, "achieved_gbs": pw, "frac": pw / HBM_PEAK_GBS},
                     "note": "untimed, after the timed steps: a batched fit of these outputs with "
                             "the CU split off (whole-chip kernels), HIP events as above"}
    pred_probe = None
    if rank == 0 and problems and not host and "fit" in last and args.predict == "analytic":
        # after the timed region: two outputs' predictions one at a time (gpar_predict: one lane,
        # whole chip), so each prediction kernel's HIP-event time is its own duration, not a span
        # shared with the other lane's kernels as in the timed calls
        fr = last["fit"]
        idx = sorted({len(problems) // 2, len(problems) - 1})
        ctx.reset_stats()
        for i in idx:
            p = gpar_out[i]
            G.predict_scaled(Y_d[:, : p - 1], Zs[p], t_d, ycols[p], fr.theta[i], ts_d,
                             Fs_d[:, : p - 1], cfg["out_kernel"], "matern52", mode="analytic",
                             device=local, qu_kuu_noise=qn)
        pred_probe = {"outputs": [gpar_out[i] for i in idx]}
        for fam, bound in (("pred_whiten", "hbm"), ("pred_adjoint", "hbm"), ("pred_var", "mfma")):
            pn, pms = ctx.kernel_stats(fam)
            if pn:
                w = ctx.kernel_work(fam) / (pms * 1e-3)
                pred_probe[fam] = ({"avg_ms": pms / pn, "achieved": w / 1e9, "unit": "GB/s",
                                    "frac": w / 1e9 / HBM_PEAK_GBS} if bound == "hbm" else
                                   {"avg_ms": pms / pn, "achieved": w / 1e12, "unit": "TFLOP/s",
                                    "frac": w / 1e12 / FP64_MFMA_PEAK_TFLOPS})
        pred_probe["note"] = ("untimed, after the timed steps: single-output gpar_predict calls at "
                              "the fitted theta (one stream, whole chip), HIP events per kernel family "
                              "as roofline_predict")
    self_check = None
    if rank == 0 and problems and "fit" in last:
        # the timed steps' own outputs: each checked output's -nlml (the objective value the
        # split, cached, pipelined batched fit reached at its returned theta) against a fresh
        # single-output whole-chip evaluation at that theta (no split, no cache, no pipeline)
        fr = last["fit"]
        idx = sorted({0, len(problems) // 2, len(problems) - 1})
        saved = ctx.cu_split()
        ctx.set_cu_split(0)
        rels = []
        for i in idx:
            v = G.dtc_objective_batch([problems[i]], fr.theta[i:i + 1], device=local)[0]
            rels.append(abs(-v - fr.nlml[i]) / abs(v))
        ctx.set_cu_split(-1 if args.cu_split is None else saved)
        self_check = {"outputs": [gpar_out[i] for i in idx], "max_rel": max(rels),
                      "ok": bool(max(rels) <= 1e-9),
                      "what": "-nlml of the timed run's last step at its fitted theta vs a fresh "
                              "whole-chip single-output gpar_dtc_objective there (rel <= 1e-9)"}
    if (rank == 0 and temporal and cpu_child is not None
            and os.path.getsize(cpu_child.check_path) > 0):
        # the C port's chain logpdfs (every chain, N) and chain 1's smoothed prediction on the merged
        # grid at SSM_CHECK_THETA, computed by the CPU baseline child on this run's data, against
        # gpar_lgssm_logpdf / gpar_lgssm_smooth (untimed)
        ref = np.load(cpu_child.check_path)
        t_h, ts_h = t_d.cpu().numpy(), ts_d.cpu().numpy()
        Yc = Y_d[:, [p - 1 for p in mine]].T.contiguous().cpu().numpy()
        th = np.tile(np.array([SSM_CHECK_THETA]), (len(mine), 1))
        g_lml = np.asarray(G.lgssm_logpdf_batch(t_h, Yc, th, cfg["out_kernel"], device=local))
        tm, order, is_test, _ = merged_sde_grid(t_h, ts_h, SSM_CHECK_THETA[2])
        y0 = np.where(is_test, 0.0, np.concatenate([Yc[0], np.zeros(len(ts_h))])[order])
        gm, gv = G.lgssm_smooth_batch(tm, y0[None, :], th[:1], cfg["out_kernel"],
                                      noise=np.where(is_test, 1e10, -1.0), device=local)
        gm, gv = np.asarray(gm)[0][is_test], np.asarray(gv)[0][is_test]
        lrel = float(np.max(np.abs(g_lml - ref["lml"]) / np.abs(ref["lml"])))
        mex = float(np.max(np.abs(gm - ref["mean"]) / (1e-9 * np.abs(ref["mean"]) + 1e-10 * np.abs(ref["mean"]).max())))
        vex = float(np.max(np.abs(gv - ref["var"]) / (1e-9 * np.abs(ref["var"]) + 1e-12 * np.abs(ref["var"]).max())))
        self_check = {"cpu_port": {
            "reference": "C port (oracle/cpu_ref, pinned to the numpy oracle by tests/test_cpu_ref.py), "
                         "run by the cpu_baseline child on this data",
            "theta": list(SSM_CHECK_THETA), "chains": len(mine), "lml_max_rel": lrel,
            "mean_excess": mex, "var_excess": vex,
            "ok": bool(lrel <= 1e-10 and mex <= 1.0 and vex <= 1.0),
            "what": "every chain's logpdf at N (rel <= 1e-10) and chain 1's smoothed mean / variance at "
                    "t* on the merged grid (rtol 1e-9, atol 1e-10 / 1e-12 max|ref|; *_excess <= 1 "
                    "passes), against the port"}}
        self_check["ok"] = self_check["cpu_port"]["ok"]
    p_chk = check_output(P)
    if (rank == 0 and cpu_child is not None and p_chk in gpar_out and not host
            and os.path.getsize(cpu_child.check_path) > 0):
        # the C port's objective and analytic prediction of output p_chk at CHECK_THETA, computed
        # by the CPU baseline child on this run's own data, against the GPU's (gpar_dtc_objective,
        # gpar_predict: the prediction at N* = N takes predict_var's prefetching path, as the
        # timed predictions do)
        ref = np.load(cpu_child.check_path)
        i = gpar_out.index(p_chk)
        v = G.dtc_objective_batch([problems[i]], [CHECK_THETA], device=local)[0]
        gm, gs = G.predict_scaled(Y_d[:, : p_chk - 1], Zs[p_chk], t_d, ycols[p_chk], CHECK_THETA,
                                  ts_d, Fs_d[:, : p_chk - 1], cfg["out_kernel"], "matern52",
                                  mode="analytic", device=local, qu_kuu_noise=qn)
        gm, gs = gm.cpu().numpy(), gs.cpu().numpy()
        rm, rs = ref["mean"], ref["std"]

        def excess(a, b):   # max |a - b| / (rtol |b| + atol): <= 1 passes rtol 1e-7, atol 1e-8 max|b|
            return float(np.max(np.abs(a - b) / (1e-7 * np.abs(b) + 1e-8 * np.abs(b).max())))
        port = {"reference": "C port (oracle/cpu_ref, pinned to the numpy oracle by "
                             "tests/test_cpu_ref.py), run by the cpu_baseline child on this data",
                "output": p_chk, "theta": list(CHECK_THETA), "dtc_gpu": v, "dtc_port": float(ref["dtc"][0]),
                "dtc_rel": abs(v - float(ref["dtc"][0])) / abs(float(ref["dtc"][0])),
                "mean_max_abs": float(np.max(np.abs(gm - rm))), "std_max_abs": float(np.max(np.abs(gs - rs))),
                "mean_excess": excess(gm, rm), "std_excess": excess(gs, rs)}
        port["ok"] = bool(port["dtc_rel"] <= 1e-9 and port["mean_excess"] <= 1.0
                          and port["std_excess"] <= 1.0)
        port["what"] = ("gpar_dtc_objective (rel <= 1e-9) and gpar_predict's mean / std (rtol 1e-7, "
                        "atol 1e-8 max|ref|; *_excess <= 1 passes) at N = N*, against the port")
        self_check = dict(self_check or {}, cpu_port=port)
        self_check["ok"] = bool(self_check.get("ok", True) and port["ok"])
    h2h = None
    if (rank == 0 and world == 1 and args.h2h_steps > 0 and problems and not host and not chained
            and not temporal and not shard_of and not per_output and not args.separate_predict):
        # SURVEY §8d's host->host unit ("host->host wall-clock, excluding setup"): the
        # same job, every step starting from pinned host copies of its inputs -- t, Y (N x P), t*,
        # F* (N* x P) and the pseudo-inputs, one upload each into the buffers the problems view --
        # and ending with every output's mean / std (and output 1's smoothed marginals) in pinned
        # host memory.  Untimed set-up: the pinned buffers.
        t_pin, Y_pin = t_d.cpu().pin_memory(), Y_d.cpu().pin_memory()
        ts_pin, Fs_pin = ts_d.cpu().pin_memory(), Fs_d.cpu().pin_memory()
        Z_pin = {p: Zs[p].cpu().pin_memory() for p in gpar_out}
        res_pin = torch.empty((2 * len(gpar_out) + 2, ns_eff), dtype=torch.float64).pin_memory()
        up = 8 * (t_pin.numel() + Y_pin.numel() + ts_pin.numel() + Fs_pin.numel()
                  + sum(z.numel() for z in Z_pin.values()))
        th_dev = theta

        def h2h_step():
            for dst, src in ((t_d, t_pin), (Y_d, Y_pin), (ts_d, ts_pin), (Fs_d, Fs_pin)):
                dst.copy_(src, non_blocking=True)
            for p in gpar_out:   # the problems' views: pseudo-inputs uploaded, target columns
                Zs[p].copy_(Z_pin[p], non_blocking=True)
                ycols[p].copy_(Y_d[:, p - 1])
            if y1 is not None:
                y1.copy_(Y_d[:, 0])
            th = step()
            k = 0
            for m_, s_ in zip(last["means"], last["stds"]):
                res_pin[k].copy_(m_, non_blocking=True)
                res_pin[k + 1].copy_(s_, non_blocking=True)
                k += 2
            if "temporal" in last:
                res_pin[k].copy_(last["temporal"][0], non_blocking=True)
                res_pin[k + 1].copy_(last["temporal"][1], non_blocking=True)
                k += 2
            torch.cuda.synchronize()
            return th, k

        torch.cuda.synchronize()
        th0 = time.perf_counter()
        for _ in range(args.h2h_steps):
            th_h, nres = h2h_step()
        el_h = (time.perf_counter() - th0) * 1e3 / args.h2h_steps
        h2h = {"ms_per_step": el_h, "steps": args.h2h_steps, "value": n_eff * P / (el_h / 1e3),
               "vs_device_resident": el_h / el, "bytes_up_per_step": up,
               "bytes_down_per_step": 8 * nres * ns_eff,
               "same_thetas_as_timed_steps": bool(np.array_equal(th_h, th_dev)),
               "note": "after the timed device-resident steps: each step uploads t, Y, t*, F* and "
                       "the pseudo-inputs from pinned host memory into the buffers the problems "
                       "view, runs the job, and downloads every prediction to pinned host memory "
                       "(SURVEY §8d host->host unit; value stays the device-resident figure)"}
    if cpu_child is not None:
        try:
            os.unlink(cpu_child.check_path)
        except OSError:
            pass
    out = None
    if rank == 0:
        P_work = len(mine) if shard_of else P
        value = n_eff * P_work / (el / 1e3)
        flops = float(n_eff) * M * (M + 1)       # N*M*(M+1) per Gram launch
        avg = gram_ms / max(gram_n, 1)
        achieved = gram_work / (gram_ms * 1e-3) / 1e12 if gram_n else None
        traffic = wtraffic = tsrc = None
        if args.config == "north":   # tools/pmc_passes.sh at the north config
            traffic, wtraffic, tsrc = pmc_traffic([PMC_FILE, PMC_FALLBACK])
        out = {
            # BASELINE.json's metric string (north), the same wording at the other configs' sizes
            "metric": "GPAR fit+predict wall-clock (ms) and pts\u00b7outputs/sec, "
                      f"N={D.fmt_count(N)} M={M} P={P}",
            "value": value,
            "unit": "pts\u00b7outputs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (toy_data.jl big-set functions, P outputs, seed 0)",
            "config": {"workload": f"GPAR-DTC fit+predict ({args.config})", "N": n_eff, "N_star": ns_eff,
                       "M": M, "P": P, "evals_per_output": EV, "predict": args.predict,
                       "out_kernel": cfg["out_kernel"], "time_kernel": "matern52",
                       "parallelism": f"outputs sharded over {world} GPU(s)",
                       "outputs_per_rank": shards, "inference": args.inference,
                       "inputs": args.inputs, "cu_split": cu_split, "qu_kuu_noise": qn,
                       "api": args.api, "dist_cache": args.dist_cache,
                       **({"schedule": knobs} if knobs else {}),
                       **({"shard": f"{shard_of[0]}/{shard_of[1]}", "shard_outputs": mine}
                          if shard_of else {})},
            "qu_convention": ("q(u) and the predictions factor Cuu + sigma^2 I (qu_kuu_noise), the "
                              "objective's regularised Kuu (dtc.jl:35,119), not the reference's "
                              "noise-free Cuu (gpar_scaled_inference.jl:157)" if qn else
                              "q(u) factors the reference's noise-free Cuu "
                              "(gpar_scaled_inference.jl:157)"),
            **({"rehearsal": "all ranks on one GPU over gloo: not a scaling measurement"}
               if args.rehearse else {}),
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": (achieved / FP64_MFMA_PEAK_TFLOPS) if achieved else None,
                         "traffic": traffic, "traffic_source": tsrc,
                         "kernel": "Gram beta^T beta + beta^T alpha, fp64 MFMA (v3: gram3_off + gram3_dg + gram3_corr + gram3_reduce per launch; lanes=2: gram2)",
                         "note": "avg_ms spans one Gram launch (HIP events): gram3_off_kernel, then "
                                 "gram3_dg_kernel and gram3_reduce; gram3_corr_slim_kernel runs "
                                 "concurrently with gram3_off_kernel on a second stream (and with "
                                 "cu_split, part of gram3_dg_kernel on the whitening CUs)",
                         "launches": gram_n, "avg_ms": avg, "flops_per_launch": flops,
                         "lanes": args.lanes},
            "ranks": rank_info,
            "kernels": {"gram_ms_per_step": gram_ms / args.steps, "whiten_ms_per_step": wh_ms / args.steps,
                        "whiten_launches": wh_n},
        }
        if wh_n:
            wa = wh_work / (wh_ms * 1e-3) / 1e9
            out["roofline_whiten"] = {
                "bound": "hbm", "achieved": wa, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": wa / HBM_PEAK_GBS, "traffic": wtraffic, "launches": wh_n,
                "avg_ms": wh_ms / wh_n, "bytes_per_launch": wh_work / wh_n,
                "kernel": "Kfu assembly + Kalman whitening (whiten_kfu_d2x2 from the fit's distance "
                          "cache for D >= 17, fused whiten_kfu_mfma below)",
                "bytes": "8 N (D + M + 20) per launch (M for D when cached), include/gpar_hip.h"}
        if fc_n and gram_n:
            out["fit_calls"] = {"calls_per_step": fc_n / args.steps, "ms_per_step": fc_ms / args.steps,
                                "not_gram_ms_per_step": (fc_ms - gram_ms) / args.steps,
                                "note": "HIP events around each batched fit (after its distance cache) "
                                        "vs the sum of the Gram spans: the fit's time off the Gram's "
                                        "critical path (round boundaries, pipeline bubbles)"}
        if rnd_n and gram_n:
            # what of the fit's rounds does not overlap a Gram: the round boundaries (dense tail
            # after the last Gram, values to the host, the simplex step, the next round's gains and
            # first whitening) plus any pipeline bubble
            out["fit_rounds"] = {"rounds_per_step": rnd_n / args.steps,
                                 "ms_per_step": rnd_ms / args.steps,
                                 "gram_ms_per_step": gram_ms / args.steps,
                                 "not_gram_ms_per_step": (rnd_ms - gram_ms) / args.steps,
                                 "head_ms_per_step": rh_ms / args.steps if rh_n else None,
                                 "tail_ms_per_step": rt_ms / args.steps if rt_n else None,
                                 "between_grams_ms_per_step": ((rnd_ms - gram_ms - rh_ms - rt_ms)
                                                               / args.steps if rh_n and rt_n else None),
                                 "marks_ms_per_step": {k: v[1] / args.steps for k, v in marks.items()
                                                       if v[0]},
                                 "note": "HIP events on the context stream around each round-by-round "
                                         "objective round (eval_dtc) vs the sum of its Gram spans"}
        if gram_n:
            # the whole job against its dominant kernel's floor: every Gram launch at the fp64
            # MFMA peak, nothing else, vs the measured step
            floor_ms = gram_work / args.steps / (FP64_MFMA_PEAK_TFLOPS * 1e12) * 1e3
            out["job_vs_gram_floor"] = {"floor_ms_per_step": floor_ms, "frac": floor_ms / el,
                                        "note": "Gram launches of one step at 78.6 TF/s / measured step"}
        if cu_split and args.lanes == 1 and gram_n and wh_n:
            # CU split: the fit's Gram runs on (32 - w) of every XCD's 32 CUs, the whitening on
            # the other w, concurrently; the fractions above are against the whole chip's peaks
            share = (32 - cu_split) / 32.0
            out["roofline"]["cu_split"] = {
                "gram_cus": 8 * (32 - cu_split), "whiten_cus": 8 * cu_split,
                "frac_vs_masked_peak": out["roofline"]["frac"] / share,
                "note": f"the fit's Gram launches run on {8 * (32 - cu_split)} CUs while the next "
                        f"output's whitening runs on the other {8 * cu_split} (CU-masked streams); "
                        f"{cu_split}/32 of the Gram's diagonal-block items run on the whitening CUs "
                        "after it, so avg_ms spans the whole Gram including that share, and "
                        "frac_vs_masked_peak (peak x the Gram's CU share) is an upper bound; "
                        "the prediction's Gram-free kernels and q(u) use the whole chip"}
            out["roofline_whiten"]["note"] = (
                f"fit launches run on {8 * cu_split} of 256 CUs beside the Gram (HBM shared), "
                "so per-launch time is not the whole-chip kernel's")
        if pred:
            pred["note"] = ("the analytic prediction's kernels (HIP events per launch, one per output "
                            "per step): pred_whiten = merged-grid Cf*u assembly + whitening "
                            "(whiten_kfu_mfma + whiten_vec; bytes 8 (N+N*) (D + M + 20)), pred_adjoint "
                            "= adjoint_local_wide (bytes 8 ((N+N*)(Mp+1+21) + N* (Mp+1))), pred_rows = "
                            "predict_rows (16 N* Mp), pred_gemm = the variance GEMM |Q V^T| with V "
                            "triangular (N* M (M+1) flops); pred_var = predict_var, the rows, mean "
                            "and variance fused (M <= 512, the default; replaces pred_rows + "
                            "pred_gemm; flops as pred_gemm)")
            pred["ms_per_step_kernel_sum"] = sum(v["ms_per_step"] for k, v in pred.items()
                                                 if isinstance(v, dict))
            if pwall_n:   # the spans above overlap across the two prediction lanes; this does not
                pred["wall_ms_per_step"] = pwall_ms / args.steps
                pred["wall_note"] = ("HIP events around all of one gpar_fit_predict call's "
                                     "predictions (q(u), both lanes, to their join)")
            if pred_probe:
                pred["one_lane_probe"] = pred_probe
            out["roofline_predict"] = pred
        out["memory"] = memory
        if h2h:
            out["host_to_host_ms_per_step"] = h2h["ms_per_step"]
            out["host_to_host"] = h2h
        if last.get("sweep_s"):
            sw = 1e3 * float(np.mean(last["sweep_s"][-args.steps:]))
            out["chained_sweep"] = {
                "ms_per_step": sw, "outputs": len(gpar_all),
                "note": "wall time of the ordered chained prediction sweep inside each timed step "
                        "(gpar_posterior_predict per output: q(u) ran with the fits)"}
            if shard_of:
                # the projected W-GPU chained step of the staggered schedule (shard.assign_chained):
                # this rank's measured fits set the scale of the affine fit-time model of shard.py
                # for every block size, the measured sweep gives the time per chained prediction,
                # and each block's means reach the next owner over xGMI at ASSUMED figures (50 GB/s
                # effective + 40 us; this pool never runs RCCL), plus the final broadcast of the
                # whole chain from the last owner (assumed likewise)
                fit_meas = el - sw
                n_r = len(gpar_out)
                model = lambda n: S.FIT_FIXED_MS + S.FIT_MS_PER_OUTPUT * n   # noqa: E731
                fit_ms = lambda n: fit_meas * model(n) / model(n_r)        # noqa: E731
                per = sw / len(gpar_all)
                xfer = lambda k: 8.0 * ns_eff * k / (S.XFER_GBS_ASSUMED * 1e9) * 1e3 + \
                    S.XFER_LAT_MS_ASSUMED                                   # noqa: E731
                blocks = [len([p for p in o if p >= 2]) for o in shards]
                mk, rows = S.chained_schedule(blocks, fit_ms, per, xfer)
                final = 8.0 * ns_eff * P / (S.XFER_GBS_ASSUMED * 1e9) * 1e3 + S.XFER_LAT_MS_ASSUMED
                out["chained_sweep"].update(
                    projected_step_ms=mk + final, fit_ms_per_step=fit_meas, block_sizes=blocks,
                    sweep_ms_per_output=per, final_broadcast_ms_assumed=final,
                    schedule_ms=[[round(v, 1) for v in r] for r in rows],
                    projection_note="staggered blocks (fit end, sweep start, sweep end per rank): "
                                    "fits scaled from this rank's measured block by shard.py's "
                                    "affine model, transfers at assumed xGMI figures")
        if self_check:
            out["self_check"] = self_check
        if probe:
            out["roofline_whole_chip_probe"] = probe
        if args.lanes > 1 and out["roofline"]:
            # two streams overlap launches: event spans are not the kernel's own duration
            out["roofline"].update(achieved=None, frac=None,
                                   note="lanes=2: per-launch event time includes the overlap with "
                                        "the other lane, not a kernel duration")
        if temporal:
            out["metric"] = "temporal-only LGSSM fit+smooth (Matern-3/2 chains), pts*chains/s"
            out["unit"] = "pts*chains/s"
            out["roofline"] = None
            out.pop("roofline_whiten", None)
            for fam, key in (("chains_logpdf", "roofline"), ("chains_smooth", "roofline_smooth")):
                (fn, fms), w = chain_stats[fam]
                if fn and fam == "chains_logpdf":
                    # the device-stepped fit times batches of rounds: count NM rounds by their
                    # algorithmic bytes (8 N (1 + chains) per round)
                    fn = max(fn, int(round(w / (8.0 * t_d.numel() * (1 + len(mine))))))
                if fn:
                    ga = w / (fms * 1e-3) / 1e9
                    out[key] = {"bound": "hbm", "achieved": ga, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": ga / HBM_PEAK_GBS, "traffic": None, "launches": fn,
                                "avg_ms": fms / fn, "ms_per_step": fms / args.steps,
                                "bytes_per_launch": w / fn}
            if "roofline" in out and out["roofline"]:
                out["roofline"].update(
                    kernel="chains_logpdf: gains_phase1 + gains_phase2 + gains_phase3 (moments) + "
                           "chain_carry_lml (the carry, the value and the device Nelder-Mead step), HIP-event "
                           "spans around batches of 8 NM rounds, reported per round",
                    bytes="8 N (t) + 8 N per active chain (y) per launch; the per-chunk outputs "
                          "(~0.7 B per step and chain) not counted")
            if out.get("roofline_smooth"):
                out["roofline_smooth"].update(
                    kernel="chains_smooth: gains with covariances + whiten_vec + carries + "
                           "adjoint + smooth_mean + cov_smooth, one span on the merged grid",
                    bytes="8 n (t) + 8 n (noise) + 24 n per chain (y in, mean and variance out), "
                          "n = N + N*")
            out["config"]["workload"] = f"temporal-only chains fit+smooth ({args.config})"
            out["config"]["time_kernel"] = cfg["out_kernel"]
        if cpu_res is not None:
            out["cpu_baseline"] = cpu_res
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def stress_main(args):
    """BASELINE config 5 (stress: N = 1e7, M = 1024, P = 256, DTC-GPAR, fp64), per-evaluation
    throughput ("Per-evaluation throughput, 8 GPUs").  Outputs 2..P are
    sharded over the ranks by LPT with the D-dependent cost model (shard.output_cost_sized); one
    step = one batched Nelder-Mead fit of exactly `evals` objective evaluations (dtc.jl:83-128) per
    GPAR output this rank owns, fixed init log theta = (0, 0, 0, 0, -2).  --shard R/W runs rank R's
    outputs of a W-way job on this one GPU.  value = N x (evaluations in the step) / step time, the
    whole job's evaluation throughput (summed over ranks).  The temporal-only output 1 (O(N)) is
    not part of this per-evaluation figure."""
    import torch
    import torch.distributed as dist
    import gparatscale as G
    from gparatscale import data as D
    from gparatscale import shard as S
    cfg = dict(CONFIGS[args.config])
    if args.evals:
        cfg["evals"] = args.evals
    N, M, P, EV = cfg["N"], cfg["M"], cfg["P"], cfg["evals"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.rehearse else int(os.environ.get("LOCAL_RANK", "0"))
    cpu_child = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu_child = start_cpu_baseline(args)   # before this process touches the GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.rehearse:
            dist.init_process_group("gloo", timeout=pg_timeout())
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout())
    cost = lambda p: S.output_cost_sized(p, N, M, EV)   # noqa: E731
    gpar_all = list(range(2, P + 1))
    w_ = world
    r_ = rank
    if args.shard:
        if world > 1:
            sys.exit("--shard R/W: one process")
        r_, w_ = (int(x) for x in args.shard.split("/"))
    shards = S.assign_outputs(P, w_, cost=cost)
    mine = [p for p in shards[r_] if p >= 2]
    # inputs (untimed): generated on the device (20 GB of Y), broadcast from rank 0 over RCCL
    t0 = time.perf_counter()
    if rank == 0:
        t_d, Y_d = D.gpar_dataset_device(N, P, seed=0, observation_noise=0.8, device=dev)
    else:
        t_d = torch.empty(N, dtype=torch.float64, device=dev)
        Y_d = torch.empty((N, P), dtype=torch.float64, device=dev)
    S.broadcast_inputs((t_d, Y_d))
    problems, keep = [], []
    for p in mine:
        idx = torch.from_numpy(D.pseudo_index(N, M, seed=p)).to(dev)
        Z = Y_d[idx, : p - 1].contiguous()
        pr, k = G.make_problem(Y_d[:, : p - 1], Z, t_d, Y_d[:, p - 1].contiguous(),
                               cfg["out_kernel"], "matern52")
        problems.append(pr)
        keep.append((k, Z))
    x0 = np.tile(np.array([0.0, 0.0, 0.0, 0.0, -2.0]), (len(problems), 1))
    torch.cuda.synchronize()
    torch.cuda.empty_cache()   # the generator's temporaries back to the device for the library
    log(f"[rank {rank}] stress inputs ready in {time.perf_counter() - t0:.1f}s: N={N} M={M} "
        f"P={P} shard {r_}/{w_}: {len(mine)} outputs (D {min(mine) - 1}..{max(mine) - 1})")
    ctx = G.context(local)
    for kv in filter(None, args.schedule.split(",")):
        k, v = kv.split("=")
        ctx.set_schedule(k.strip(), int(v))
    if args.cu_split is not None:
        ctx.set_cu_split(args.cu_split)
    ctx.set_dist_cache_keep(args.dist_cache == "keep")
    last = {}

    def step():
        fr = G.fit_batch(problems, x0, max_evals=EV, g_tol=-1.0, device=local) if problems else None
        last["fit"] = fr
        return fr

    for _ in range(args.warmup):
        step()
    cpu_res = join_cpu_baseline(cpu_child, timeout=1800) if cpu_child is not None else None
    ctx.set_profiling(True)
    ctx.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ts0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    busy = (time.perf_counter() - ts0) * 1e3 / args.steps
    if world > 1:
        dist.barrier()
    el = (time.perf_counter() - ts0) * 1e3 / args.steps
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e[0])
    fams = {k: ctx.kernel_stats(k) for k in ("gram", "whiten", "dist2", "fit_call", "fit_round")}
    works = {k: ctx.kernel_work(k) for k in ("gram", "whiten", "dist2")}
    evals_rank = len(problems) * EV
    evals_all = evals_rank
    if world > 1:
        e = torch.tensor([float(evals_rank)], dtype=torch.float64, device=dev)
        dist.all_reduce(e)
        evals_all = int(e[0])
    elif args.shard:
        evals_all = evals_rank   # this rank's share of the W-way job, measured alone
    out = None
    if rank == 0:
        gn, gms = fams["gram"]
        wn, wms = fams["whiten"]
        dn, dms = fams["dist2"]
        gach = works["gram"] / (gms * 1e-3) / 1e12 if gn else None
        value = float(N) * evals_all / (el / 1e3)
        per_eval_ms = el / max(evals_rank, 1)
        # the whole stress job (every GPAR output, 50 evaluations each) projected from this rank's
        # per-evaluation time and the LPT loads of the sized cost model
        stress_traffic, _, stress_tsrc = pmc_traffic([PMC_STRESS_FILE])
        loads = [sum(cost(p) for p in sh if p >= 2) for sh in shards]
        mine_load = loads[r_]
        proj_s = (el / 1e3) * (50.0 / EV) * max(loads) / mine_load if mine_load else None
        out = {
            "metric": "GPAR-DTC objective evaluation throughput (pts\u00b7evaluations/s), "
                      f"N={D.fmt_count(N)} M={M} P={P}",
            "value": value, "unit": "pts\u00b7evaluations/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (toy_data.jl big-set functions extended to P outputs, generated on "
                    "the device with torch's seeded generator)",
            "config": {"workload": "GPAR-DTC per-evaluation (stress)", "N": N, "M": M, "P": P,
                       "evals_per_output": EV, "out_kernel": cfg["out_kernel"],
                       "time_kernel": "matern52", "outputs": mine,
                       "parallelism": f"outputs sharded over {w_} GPU(s) (LPT, D-dependent cost)",
                       **({"shard": f"{r_}/{w_}"} if args.shard else {}),
                       "cu_split": ctx.cu_split(), "dist_cache": args.dist_cache,
                       **({"schedule": args.schedule} if args.schedule else {})},
            "ms_per_evaluation": per_eval_ms,
            "evaluations_per_step": evals_rank,
            "roofline": {"bound": "mfma", "achieved": gach, "peak": FP64_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": gach / FP64_MFMA_PEAK_TFLOPS if gach else None,
                         "traffic": stress_traffic, "traffic_source": stress_tsrc,
                         "launches": gn, "avg_ms": gms / gn if gn else None,
                         "flops_per_launch": float(N) * M * (M + 1),
                         "kernel": "Gram beta^T beta + beta^T alpha, fp64 MFMA (gram3_off + gram3_dg "
                                   "+ gram3_corr + gram3_reduce), HIP events per launch"},
            "job_vs_gram_floor": {"floor_ms_per_step": works["gram"] / args.steps /
                                  (FP64_MFMA_PEAK_TFLOPS * 1e12) * 1e3,
                                  "frac": works["gram"] / args.steps /
                                  (FP64_MFMA_PEAK_TFLOPS * 1e12) * 1e3 / el},
            "projected_job": {"seconds": proj_s, "gpus": w_, "evals_per_output": 50,
                              "note": "every GPAR output's 50-evaluation fit on W GPUs: this rank's "
                                      "measured step x 50 / evals x (largest rank load / this "
                                      "rank's load) under shard.output_cost_sized"},
            "ranks": [{"rank": r, "outputs": len([p for p in sh if p >= 2]),
                       "load_rel": loads[r] / max(loads)} for r, sh in enumerate(shards)],
        }
        if wn:
            wa = works["whiten"] / (wms * 1e-3) / 1e9
            out["roofline_whiten"] = {"bound": "hbm", "achieved": wa, "peak": HBM_PEAK_GBS,
                                      "unit": "GB/s", "frac": wa / HBM_PEAK_GBS, "launches": wn,
                                      "avg_ms": wms / wn, "bytes_per_launch": works["whiten"] / wn,
                                      "kernel": "Kfu + Kalman whitening (whiten_kfu_d2x2 from cached "
                                                "or freshly computed distances)"}
        if dn:
            da = works["dist2"] / (dms * 1e-3) / 1e12
            out["roofline_dist"] = {"bound": "mfma", "achieved": da, "peak": FP64_MFMA_PEAK_TFLOPS,
                                    "unit": "TFLOP/s", "frac": da / FP64_MFMA_PEAK_TFLOPS,
                                    "launches": dn, "avg_ms": dms / dn,
                                    "flops_per_launch": works["dist2"] / dn,
                                    "kernel": "dist2_mfma_kernel: |v - z|^2 cross products 2 N Mp D "
                                              "on MFMA (cache fill or per-evaluation pass)"}
        fc_n, fc_ms = fams["fit_call"]
        if fc_n and gn:
            out["fit_calls"] = {"ms_per_step": fc_ms / args.steps,
                                "not_gram_ms_per_step": (fc_ms - gms) / args.steps}
        if cpu_res is not None:
            out["cpu_baseline"] = cpu_res
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def stress_cpu_baseline(N, M, P, out_kernel, n_sample=1_000_000, check_path=None):
    """The stress config's CPU baseline: the C/OpenMP port (oracle/cpu_ref, pinned to the numpy
    oracle by tests/test_cpu_ref.py) times ONE DTC objective evaluation of the widest output
    (D = P - 1 = 255, M pseudo-points) at n_sample = 1e6 points, scaled linearly in N (every piece
    of the evaluation is O(N): Kfu, the M + 1 filter sweeps, the N M^2 Gram; the M^3 tail is
    negligible), so value = N / (that time x N / n_sample) pts*evaluations/s."""
    sys.path.insert(0, ROOT)
    from oracle import gpar_oracle as O
    from oracle import cpu_ref as CR
    try:
        from threadpoolctl import threadpool_info
        blas = max([x.get("num_threads", 1) for x in threadpool_info() if x.get("user_api") == "blas"] + [1])
    except Exception:
        blas = 1
    cores = max(CR.threads(), blas)
    d = P - 1
    t, Y = O.synthetic_gpar(n_sample, d + 1, seed=1, noise=0.8)
    V = np.ascontiguousarray(Y[:, :d].T)
    y = np.ascontiguousarray(Y[:, d])
    Z = O.pick_pseudo_inputs(V, M, 3)
    theta = CHECK_THETA
    CR.compute_gpar_dtc_objective(V[:, :4096], Z, t[:4096], y[:4096], theta, out_kernel, "matern52")
    t0 = time.perf_counter()
    val, _ = CR.compute_gpar_dtc_objective(V, Z, t, y, theta, out_kernel, "matern52")
    t_eval = time.perf_counter() - t0
    t_scaled = t_eval * N / n_sample
    return {"value": N / t_scaled, "unit": "pts\u00b7evaluations/s", "cores": int(cores),
            "kind": "port", "host_cpu": _cpu_model(), "eval_seconds_sample": t_eval,
            "eval_seconds_at_N": t_scaled, "dtc_sample": float(val),
            "ran": "in a child process beside the GPU warm-up (joined before the timed region)",
            "sample": f"C/OpenMP + OpenBLAS restatement (oracle/cpu_ref), {int(cores)} threads: one DTC "
                      f"objective evaluation at N = {n_sample}, M = {M}, D = {d} (the widest output) = "
                      f"{t_eval:.2f}s, scaled linearly to N = {N}: {t_scaled:.1f}s per evaluation"}


LAUNCH_KILL_GRACE_S = 10.0   # SIGTERM -> SIGKILL grace for the surviving ranks of a failed job


def pg_timeout():
    """The process group's collective timeout: 120 s (GPAR_PG_TIMEOUT_S overrides).  Every
    collective of the bench waits at most one rank's step (a few seconds at 8 ranks) or the input
    set-up on rank 0."""
    return datetime.timedelta(seconds=float(os.environ.get("GPAR_PG_TIMEOUT_S", "120")))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count(root="/sys/class/kfd/kfd/topology/nodes", env=None):
    """GPUs this process could use, counted WITHOUT initialising HIP (the launcher parent must stay
    HIP-free: torch.cuda.device_count() may fall back to hipGetDeviceCount when amdsmi discovery
    fails).  KFD topology nodes with a non-zero gpu_id are GPUs (CPU nodes have 0); a
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES list narrows the count."""
    env = os.environ if env is None else env
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "gpu_id")) as f:
                    if int(f.read().strip() or "0") != 0:
                        n += 1
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(n, argv, stub=False):
    """Start one bench process per GPU (rank r on device r) and forward rank 0's JSON line.

    The parent never initialises HIP (it does not even import torch): the devices are counted from
    the KFD topology in sysfs (visible_gpu_count), and only the rank processes touch the GPU.
    Returns the exit status: 2 when fewer than n devices are visible (not checked with stub, the
    CPU-only launcher check), else the first non-zero rank status (0 when every rank succeeded)."""
    have = visible_gpu_count()
    if not stub and have < n:
        log(f"bench: --gpus {n} but only {have} device(s) visible")
        return 2
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr,
                                      text=True))
    # rank 0's stdout is drained by a thread (a full pipe must never block it) while the parent
    # polls every rank: the first rank to exit non-zero ends the job -- the others are terminated
    # (SIGTERM, then SIGKILL after a grace period) instead of waiting in a collective for a peer
    # that is gone until the process group's timeout
    lines0 = []
    reader = threading.Thread(target=lambda: lines0.extend(procs[0].stdout), daemon=True)
    reader.start()
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = bad[0]
            break
        if all(c is not None for c in codes):
            break
        time.sleep(0.1)
    if failed is not None:
        log(f"bench: rank {failed[0]} exited with status {failed[1]}; terminating the others")
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.monotonic() + LAUNCH_KILL_GRACE_S
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reader.join(timeout=5)
    for line in lines0:   # the JSON line to stdout, anything a library printed to stderr
        line = line.rstrip("\n")
        print(line, file=sys.stdout if line.startswith("{") else sys.stderr, flush=True)
    codes = [p.returncode for p in procs]
    if failed is not None:
        log(f"bench: rank exit statuses {codes}")
        return failed[1] if failed[1] > 0 else 1
    return 0


def stub_rank(args):
    """One rank of the --stub launcher check: gloo group, output shards, no GPU and no compute.
    --stub-fail R:CODE makes rank R exit with CODE before the gather (the launcher's fail-fast
    test: the other ranks then wait in the collective until the launcher ends them)."""
    import torch.distributed as dist
    from gparatscale import shard as S
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    P = CONFIGS[args.config]["P"]
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=pg_timeout())
    if args.stub_fail:
        fr, fc = (int(x) for x in args.stub_fail.split(":"))
        if fr == rank:
            log(f"[rank {rank}] --stub-fail: exiting with {fc} before the gather")
            os._exit(fc)
    mine = S.assign_outputs(P, world)[rank]
    got = [None] * world
    if world > 1:
        dist.all_gather_object(got, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                                     "outputs": mine})
        dist.destroy_process_group()
    else:
        got = [{"rank": 0, "local_rank": 0, "outputs": mine}]
    if rank == 0:
        print(json.dumps({"stub": True, "n_gpus": world, "P": P, "ranks": got}), flush=True)


def _cpu_model():
    """The host CPU's model name (/proc/cpuinfo, as lscpu reports it) and the CPUs this process
    may use (its affinity mask; os.cpu_count() shows the whole machine on a shared box)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count()
    return {"model": model, "machine_cpus": os.cpu_count(), "affinity_cpus": avail,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def _cpu_threads():
    """Threads for the CPU baseline: the box's CPU share (OMP_NUM_THREADS, else the affinity mask)
    less one, which the GPU process's host thread keeps while the baseline runs beside its
    warm-up."""
    env = os.environ.get("OMP_NUM_THREADS")
    try:
        share = int(env) if env else len(os.sched_getaffinity(0))
    except (ValueError, AttributeError, OSError):
        share = os.cpu_count() or 1
    return max(1, share - 1)


def start_cpu_baseline(args):
    """Start the CPU baseline (cpu_baseline below) in a child process, before this process touches
    the GPU: it then runs beside the inputs and the warm-up steps instead of after the timed region.
    Returns the Popen (joined by join_cpu_baseline before the timed region); its check_path is the
    .npz the child leaves its objective value and predictions in (the self-check's reference)."""
    import tempfile
    th = _cpu_threads()
    env = dict(os.environ, OMP_NUM_THREADS=str(th), OPENBLAS_NUM_THREADS=str(th))
    fd, path = tempfile.mkstemp(prefix="gpar_cpu_check_", suffix=".npz")
    os.close(fd)
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--config", args.config,
           "--cpu-check-file", path]
    if args.evals:
        cmd += ["--evals", str(args.evals)]
    if args.qu_noise_free:
        cmd += ["--qu-noise-free"]
    log(f"cpu_baseline: child process with {th} threads beside the warm-up")
    child = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    child.check_path = path
    return child


def join_cpu_baseline(child, timeout=900):
    try:
        out, _ = child.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        child.kill()
        child.communicate()
        return {"value": None, "error": f"cpu baseline child exceeded {timeout}s"}
    for line in out.splitlines()[::-1]:
        if line.startswith("{"):
            return json.loads(line)
    return {"value": None, "error": f"cpu baseline child exited {child.returncode} without a result"}


def cpu_baseline_child(args):
    cfg = dict(CONFIGS[args.config])
    if args.evals:
        cfg["evals"] = args.evals
    if cfg.get("temporal", False):
        print(json.dumps(ssm_cpu_baseline(cfg["N"], cfg["P"], cfg["evals"], cfg["out_kernel"],
                                          check_path=args.cpu_check_file)), flush=True)
        return
    if cfg.get("per_eval"):
        print(json.dumps(stress_cpu_baseline(cfg["N"], cfg["M"], cfg["P"], cfg["out_kernel"],
                                             check_path=args.cpu_check_file)), flush=True)
        return
    res = cpu_baseline(cfg["N"], cfg["N"], cfg["M"], cfg["P"], cfg["evals"], cfg["out_kernel"],
                       qu_kuu_noise=not args.qu_noise_free, check_path=args.cpu_check_file)
    print(json.dumps(res), flush=True)


def _cpu_sample(CR, O, n, ns, M, d, out_kernel, theta, qu_kuu_noise=True, data=None):
    """One DTC objective evaluation and one analytic prediction of the C port at n training /
    ns test points (D = d inputs): (seconds, seconds, objective value, (mean, std)).  data: the
    bench's own (V, Z, t, y, t_star, V_star) of one output, else a seeded synthetic problem."""
    if data is None:
        t, Y = O.synthetic_gpar(n, d + 1, seed=1, noise=0.8)
        V = Y[:, :d].T
        y = Y[:, d]
        Z = O.pick_pseudo_inputs(V, M, 3)
        ts = np.sort(np.random.default_rng(2).uniform(t[0], t[-1], ns))
        Vs = np.vstack([np.interp(ts, t, V[q]) for q in range(d)])
    else:
        V, Z, t, y, ts, Vs = data
    t0 = time.perf_counter()
    val, _ = CR.compute_gpar_dtc_objective(V, Z, t, y, theta, out_kernel, "matern52")
    t_eval = time.perf_counter() - t0
    t0 = time.perf_counter()
    pred = CR.get_gpar_scaled_predictions_fixed(V, Z, t, y, ts, Vs, theta, out_kernel, "matern52",
                                                qu_kuu_noise=qu_kuu_noise)
    return t_eval, time.perf_counter() - t0, float(val), pred


# The output whose data the CPU baseline times and the bench's self-check compares the GPU with
# (D = 32 at the north config: the job's median width).
CHECK_OUTPUT = 33
# the fixed hyperparameters of that comparison (natural units; log theta = (log 2, ..., -2))
CHECK_THETA = (2.0, 2.0, 2.0, 2.0, float(np.exp(-2.0) + 1e-3))


def check_output(P):
    return min(CHECK_OUTPUT, P)


def bench_output_data(N, P, M, p):
    """Output p's problem exactly as the bench builds it (gparatscale.data, seed 0): host
    (V D x N, Z D x M, t, y, t_star, V_star D x N*)."""
    from gparatscale import data as D
    ds = D.gpar_dataset(N, P, seed=0, observation_noise=0.8)
    Y = ds["Y"]
    V = np.ascontiguousarray(Y[:, : p - 1].T)
    Z = np.ascontiguousarray(D.pseudo_inputs(Y[:, : p - 1], M, seed=p).T)
    Vs = np.ascontiguousarray(ds["F_star"][:, : p - 1].T)
    return V, Z, ds["t"], np.ascontiguousarray(Y[:, p - 1]), ds["t_star"], Vs


def _reference_literal_cost(O, N, P, EV, t_eval, sizes=(2000, 4000, 8000)):
    """The reference as written evaluates logdet(noise_matrix) with a dense N x N LU of the time
    covariance plus noise (src/gp/dtc.jl:96-99,123), O(N^3) on top of the O(N) filter the port
    times.  Timed here (scipy lu_factor, this process's BLAS threads) at N <= 8000, fitted as
    c N^3 on the largest size and extrapolated to the job's N -- where the dense matrix alone would
    take 8 N^2 bytes (8 TB at N = 1e6), so the reference cannot run the job at all."""
    try:
        from scipy.linalg import lu_factor
        times = {}
        for n in sizes:
            t = np.sort(np.random.default_rng(5).uniform(0.0, n / 10.0, n))
            Sig = O.dense_time_cov(t, "matern52", 2.0, 4.0) + 0.02 * np.eye(n)
            lu_factor(Sig[:200, :200], check_finite=False)   # warm the BLAS threads
            t0 = time.perf_counter()
            lu_factor(Sig, overwrite_a=True, check_finite=False)
            times[n] = time.perf_counter() - t0
            del Sig
        nmax = max(sizes)
        c = times[nmax] / float(nmax) ** 3
        t_lu = c * float(N) ** 3
        t_job = (P - 1) * EV * (t_eval + t_lu)
        return {"lu_seconds": {str(k): round(v, 3) for k, v in times.items()},
                "lu_seconds_at_N_extrapolated": t_lu, "job_seconds_extrapolated": t_job,
                "value": N * P / t_job, "unit": "pts·outputs/s", "dense_bytes_at_N": 8.0 * N * N,
                "note": "dense LU of the N x N noise matrix per evaluation (dtc.jl:96-99,123), c N^3 "
                        f"from N = {nmax}, plus the port's O(N) evaluation; the predictions are left "
                        "out (they would add more)"}
    except Exception as exc:   # telemetry only
        return {"error": repr(exc)}


def cpu_baseline(N, NS, M, P, EV, out_kernel, n_ratio=100_000, qu_kuu_noise=True,
                 check_path=None):
    """Time the C/OpenMP CPU restatement of the reference path (oracle/cpu_ref.{c,py}, SURVEY §8d
    "cpu_ref": kernel assembly, Kalman gains and per-column decorrelate sweeps, RTS smoother in C;
    cholesky / trsm / gemm in OpenBLAS, as the reference leaves them to Julia's OpenBLAS; "port").

    Threaded leg (the OpenMP / OpenBLAS threads this process was given): one DTC objective
    evaluation and one analytic prediction on the bench's own data of output CHECK_OUTPUT (N
    training points, N* = NS test points, D = p - 1) at CHECK_THETA, so nothing is extrapolated in
    N: job = (P - 1) outputs x (EV evaluations + 1 prediction).  The objective value and the
    predicted mean / std go to check_path (.npz) for the bench's self-check against the GPU.
    One-thread figure (the reference's sequential column loop, dtc.jl:110-117): the same two
    pieces at N = N* = n_ratio with all threads and with one (threadpoolctl's limit of 1); the
    one-thread job is the threaded job scaled by those measured ratios (assumption: the thread
    speed-up at n_ratio holds at the job's N)."""
    sys.path.insert(0, ROOT)
    from oracle import gpar_oracle as O
    from oracle import cpu_ref as CR
    try:
        from threadpoolctl import threadpool_info
        blas = max([x.get("num_threads", 1) for x in threadpool_info() if x.get("user_api") == "blas"] + [1])
    except Exception:
        blas = 1
    cores = max(CR.threads(), blas)
    theta = CHECK_THETA
    p_chk = check_output(P)
    d_sample = p_chk - 1
    data = bench_output_data(N, P, M, p_chk)
    _cpu_sample(CR, O, 4096, 1024, M, d_sample, out_kernel, theta, qu_kuu_noise)   # warm-up, untimed
    t_eval, t_pred, val, (pm_, ps_) = _cpu_sample(CR, O, N, NS, M, d_sample, out_kernel, theta,
                                                  qu_kuu_noise, data=data)
    if check_path:
        np.savez(check_path, dtc=np.array([val]), mean=pm_, std=ps_, theta=np.array(theta),
                 output=np.array([p_chk]))
    t_job = (P - 1) * (EV * t_eval + t_pred)
    single = None
    try:
        from threadpoolctl import threadpool_limits
        n_ratio = min(n_ratio, N)
        em, pm, _, _ = _cpu_sample(CR, O, n_ratio, n_ratio, M, d_sample, out_kernel, theta,
                                   qu_kuu_noise)
        with threadpool_limits(limits=1):
            e1, p1, _, _ = _cpu_sample(CR, O, n_ratio, n_ratio, M, d_sample, out_kernel, theta,
                                       qu_kuu_noise)
        re_, rp_ = e1 / em, p1 / pm
        tj1 = (P - 1) * (EV * t_eval * re_ + t_pred * rp_)
        single = {"value": N * P / tj1, "cores": 1,
                  "sample": f"N = N* = {n_ratio}: 1 eval {em:.2f}s with {int(cores)} threads, {e1:.2f}s "
                            f"with 1 (x{re_:.2f}); 1 predict {pm:.2f}s / {p1:.2f}s (x{rp_:.2f}); the "
                            f"threaded job scaled by these ratios: est {tj1:.0f}s per job"}
    except Exception as exc:   # threadpoolctl missing: report the threaded figure only
        single = {"value": None, "error": repr(exc)}
    literal = _reference_literal_cost(O, N, P, EV, t_eval)
    return {"value": N * P / t_job, "unit": "pts·outputs/s", "cores": int(cores), "kind": "port",
            "host_cpu": _cpu_model(), "single_thread": single, "reference_literal": literal,
            "ran": "in a child process beside the GPU warm-up (joined before the timed region)",
            "sample": f"C/OpenMP + OpenBLAS restatement (oracle/cpu_ref), {int(cores)} threads, on the "
                      f"bench's own output {p_chk} (D = {d_sample}) at fixed theta: 1 DTC objective eval "
                      f"(N={N}, M={M}) = {t_eval:.2f}s + 1 analytic predict (N={N}, N*={NS}) = "
                      f"{t_pred:.2f}s; job = {P - 1} outputs x ({EV} evals + 1 predict) = {t_job:.0f}s "
                      "(no extrapolation in N)"}


# the fixed chain hyperparameters (l, process sd, noise sd) of the ssm config's CPU timing and
# self-check
SSM_CHECK_THETA = (1.5, 1.2, 0.4)


def merged_sde_grid(t, t_star, noise_sd):
    """get_sde_predictions' smoothing grid (temporal_gp_inference.jl:93-113): training and test
    times merged (stable), R = sigma^2 on training steps and 1e10 on test steps.  Returns
    (t_merged, order, is_test, R)."""
    tc = np.concatenate([t, t_star])
    order = np.argsort(tc, kind="stable")
    is_test = order >= len(t)
    R = np.where(is_test, 1e10, noise_sd * noise_sd)
    return tc[order], order, is_test, R


def ssm_cpu_baseline(N, P, EV, kind, check_path=None):
    """The ssm config's CPU baseline: the C port (oracle/cpu_ref: gains, decorrelate, RTS smoother
    mean and variance, pinned to the numpy oracle by tests/test_cpu_ref.py) on the bench's own P
    chains, one chain per pool thread (ctypes releases the GIL; each chain's recursion is
    sequential).  Timed: one NM round = every chain's logpdf at N (temporal_gp_inference.jl:78), and
    the smoothing of every chain on the merged grid of N + N* steps (:93-113); job = EV rounds +
    the smoothing, as the GPU job runs (g_tol = -1: exactly EV evaluations per chain).  The chain
    logpdfs and chain 1's predicted mean / variance at SSM_CHECK_THETA go to check_path for the
    bench's self-check."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, ROOT)
    from oracle import cpu_ref as CR
    from gparatscale import data as D
    ds = D.gpar_dataset(N, P, seed=0, observation_noise=0.8)
    t, Y, ts = ds["t"], ds["Y"], ds["t_star"]
    ys = [np.ascontiguousarray(Y[:, p]) for p in range(P)]
    l, pv, ns = SSM_CHECK_THETA
    workers = max(1, min(P, _cpu_threads()))
    tm, order, is_test, R = merged_sde_grid(t, ts, ns)
    ym = [np.where(is_test, 0.0, np.concatenate([y, np.zeros(len(ts))])[order]) for y in ys]
    CR.lgssm_logpdf(kind, t[:4096], ys[0][:4096], l, pv * pv, ns * ns)   # warm-up, untimed
    with ThreadPoolExecutor(workers) as ex:
        rounds = []
        for _ in range(3):
            t0 = time.perf_counter()
            lml = list(ex.map(lambda y: CR.lgssm_logpdf(kind, t, y, l, pv * pv, ns * ns), ys))
            rounds.append(time.perf_counter() - t0)
        t_round = float(np.median(rounds))
        t0 = time.perf_counter()
        sm = list(ex.map(lambda y: CR.lgssm_smooth(kind, tm, y, l, pv * pv, ns * ns, rvec=R), ym))
        t_smooth = time.perf_counter() - t0
    if check_path:
        m0, v0 = sm[0]
        np.savez(check_path, lml=np.array(lml), theta=np.array(SSM_CHECK_THETA),
                 mean=m0[is_test], var=v0[is_test])
    t_job = EV * t_round + t_smooth
    return {"value": N * P / t_job, "unit": "pts*chains/s", "cores": workers, "kind": "port",
            "host_cpu": _cpu_model(), "round_seconds": t_round, "smooth_seconds": t_smooth,
            "job_seconds": t_job,
            "ran": "in a child process beside the GPU warm-up (joined before the timed region)",
            "sample": f"C restatement (oracle/cpu_ref), {P} chains over {workers} threads (one chain "
                      f"per thread), the bench's own data at theta = {SSM_CHECK_THETA}: one NM round "
                      f"(every chain's logpdf, N={N}) = {t_round:.3f}s (median of 3) + the smoothing "
                      f"of every chain on the merged grid (N + N* = {len(tm)}) = {t_smooth:.2f}s; job "
                      f"= {EV} rounds + smoothing = {t_job:.2f}s (no extrapolation in N)"}


if __name__ == "__main__":
    main()
