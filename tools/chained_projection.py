"""Projected W-GPU chained step of the staggered schedule from one-GPU measurements.

Input: bench.py --shard R/W --inference chained lines for ranks covering every block size of
shard.assign_chained(P, W) (e.g. the first, a middle and the last rank).  Each line measures that
rank's own fits + posteriors (`fit_ms_per_step`) and the whole ordered sweep of the job's P - 1
predictions on one GPU (`ms_per_step` of chained_sweep).  The projection replays
shard.chained_schedule with the MEASURED fit time of each block size (interpolated affinely between
measured sizes when one is missing), the measured time per chained prediction (mean over the
lines), and transfers at the ASSUMED xGMI figures of shard.py (no RCCL on this pool).

usage: python tools/chained_projection.py W line.json [line.json ...] > projection.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gpar-at-scale_amd", "python"))
from gparatscale import shard as S  # noqa: E402


def main():
    W = int(sys.argv[1])
    lines = [json.load(open(f)) for f in sys.argv[2:]]
    fit = {}
    per, ns, P, ref = [], None, None, None
    for d in lines:
        cs = d["chained_sweep"]
        n = len([p for p in d["config"]["shard_outputs"] if p >= 2])
        fit.setdefault(n, []).append(cs["fit_ms_per_step"])
        per.append(cs["sweep_ms_per_output"])
        P = d["config"]["P"]
        ns = d["config"]["N_star"]
    fitm = {n: sum(v) / len(v) for n, v in fit.items()}
    ks = sorted(fitm)

    def fit_ms(n):
        if n in fitm:
            return fitm[n]
        a, b = (ks[0], ks[-1]) if len(ks) > 1 else (ks[0], ks[0])
        if a == b:
            return fitm[a] * (S.FIT_FIXED_MS + S.FIT_MS_PER_OUTPUT * n) / \
                (S.FIT_FIXED_MS + S.FIT_MS_PER_OUTPUT * a)
        return fitm[a] + (fitm[b] - fitm[a]) * (n - a) / (b - a)

    sweep = sum(per) / len(per)

    def xfer(k):
        return 8.0 * ns * k / (S.XFER_GBS_ASSUMED * 1e9) * 1e3 + S.XFER_LAT_MS_ASSUMED

    shards = S.assign_chained(P, W, fit_ms=fit_ms, sweep_ms=sweep, xfer_ms=xfer)
    blocks = [len([p for p in o if p >= 2]) for o in shards]
    mk, rows = S.chained_schedule(blocks, fit_ms, sweep, xfer)
    final = 8.0 * ns * P / (S.XFER_GBS_ASSUMED * 1e9) * 1e3 + S.XFER_LAT_MS_ASSUMED
    # the unstaggered schedule: every rank LPT-balanced, then the serial sweep
    flat_blocks = [len([p for p in o if p >= 2]) for o in S.assign_outputs(P, W)]
    flat = max(fit_ms(n) for n in flat_blocks) + sweep * (P - 1) + (P - 1) * xfer(1)
    print(json.dumps({
        "W": W, "P": P, "n_star": ns, "measured_fit_ms": fitm, "sweep_ms_per_output": sweep,
        "block_sizes": blocks, "schedule_ms": [[round(v, 1) for v in r] for r in rows],
        "projected_step_ms": mk + final, "final_broadcast_ms_assumed": final,
        "unstaggered_projected_step_ms": flat,
        "assumed": f"xGMI {S.XFER_GBS_ASSUMED} GB/s effective + {S.XFER_LAT_MS_ASSUMED} ms per transfer",
    }, indent=1))


if __name__ == "__main__":
    main()
