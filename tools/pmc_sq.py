"""Summarise tools/pmc_passes.sh: per-dispatch counters of the Gram and whitening kernels
(rocprofv3 --pmc, one counter group per pass) -> derived figures, JSON on stdout.

Conventions (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles
summed over waves; SQ_VALU_MFMA_BUSY_CYCLES in cycles summed over SIMDs; GRBM_GUI_ACTIVE summed
over the 8 XCDs (effective clock = GRBM_GUI_ACTIVE / 8 / kernel time); FETCH_SIZE (KiB) reports
half of wide streaming reads on gfx950 (doubled here); WRITE_SIZE (KiB) exact."""
import csv
import glob
import json
import sys
from collections import defaultdict

import os

# the probe's sizes (tools/pmc_passes.sh: the north shape; PMC_N / PMC_M / PMC_D for another, e.g.
# the stress config's N = 1e7, M = 1024, tools/pmc_stress.sh)
N = int(os.environ.get("PMC_N", 1_000_000))
M = int(os.environ.get("PMC_M", 512))
D = int(os.environ.get("PMC_D", 32))
SIMDS = 1024


def avg(x):
    return sum(x) / len(x) if x else None


def load(d):
    """-> (counters, durations, kernels): k -> counter -> per-launch value, k -> per-launch
    seconds, where a Gram "launch" is one launch_gram call (v3: gram3_off + gram3_dg (one or two
    dispatches: with the CU split a share runs on the whitening CUs) + gram3_corr + gram3_reduce;
    v2: gram2_kernel + gram2_reduce) and a whitening launch one dispatch: each kernel's counters
    summed over its dispatches, divided by the number of launches (the reduction's dispatches for
    the Gram).  Under --pmc the dispatches are serialised, so the durations add."""
    per = defaultdict(lambda: defaultdict(float))   # (k, kernel, dispatch) -> counter -> value
    dur = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "gram" in name:
                k = "gram"
            elif "whiten_kfu" in name:
                k = "whiten"
            else:
                continue
            sub = name.split("(")[0]
            key = (k, sub, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            if "Start_Timestamp" in r and r.get("End_Timestamp"):
                dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    disp = defaultdict(set)
    for (k, sub, di) in per:
        disp[(k, sub)].add(di)
    nl = {}
    for k in ("gram", "whiten"):
        red = [len(v) for (kk, sub), v in disp.items() if kk == k and "reduce" in sub]
        nl[k] = max(red) if red else sum(len(v) for (kk, _), v in disp.items() if kk == k)
    out = defaultdict(lambda: defaultdict(float))
    for (k, sub, _), cs in per.items():
        for c, v in cs.items():
            if "corr_slim" in sub and c.startswith("GRBM_"):
                continue   # elapsed-cycle counter of a kernel that overlaps gram3_off_kernel
            out[k][c] += v / nl[k]
    durs = defaultdict(float)
    for (k, sub, _), t in dur.items():
        if "corr_slim" in sub:   # runs concurrently with gram3_off_kernel outside --pmc
            continue
        durs[k] += t / nl[k]
    kernels = defaultdict(list)
    for (k, sub) in disp:
        kernels[k].append(sub)
    return out, durs, kernels, nl


def main(root):
    res = {"source": os.environ.get("PMC_SOURCE") or
                     "tools/pmc_passes.sh: rocprofv3 --pmc passes over tools/gram_probe.py "
                     f"--fit --evals 4 --batch 3 (N={N}, M={M}, D={D}; the batched fit's CU-split "
                     "Gram stage; the whitening reads the fit's distance cache: whiten_kfu_d2x2); "
                     "per-launch values: counters summed over every dispatch of the family, divided "
                     "by the launches (Gram v3: OFF + DG share(s) + correction + reduction)"}
    sq, dsq, kn, nl = load(root + "/sq1")
    fe, _, _, _ = load(root + "/fetch")
    wr, _, _, _ = load(root + "/write")
    for k in ("gram", "whiten"):
        c = dict(sq[k])                                # per launch, summed over its kernels
        t = dsq[k] or None
        e = {"kernels": sorted(kn[k]), "launches": nl[k], "counters": c, "kernel_s_under_pmc": t}
        if t and c.get("GRBM_GUI_ACTIVE"):
            clk = c["GRBM_GUI_ACTIVE"] / 8 / t
            e["effective_clock_GHz"] = clk / 1e9
            if c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                e["mfma_busy_fraction"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * clk * t)
            if c.get("SQ_INSTS_MFMA"):
                e["cycles_per_mfma"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_INSTS_MFMA"]
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            e["wave_time_fraction"] = {"active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / w,
                                       "wait_inst_any (issue stall)": c.get("SQ_WAIT_INST_ANY", 0) / w,
                                       "wait_any (waitcnt/barrier)": c.get("SQ_WAIT_ANY", 0) / w}
        f = fe[k].get("FETCH_SIZE")
        wb = wr[k].get("WRITE_SIZE")
        e["hbm_read_bytes"] = f * 1024 * 2 if f is not None else None
        e["hbm_write_bytes"] = wb * 1024 if wb is not None else None
        res[k] = e
    res["gram"]["algorithmic"] = {"flop": N * M * (M + 1), "bytes": N * M * 8,
                                  "mfma": N * M * (M + 1) // 2048}
    g = res["gram"]
    if g.get("hbm_read_bytes") is not None and g.get("hbm_write_bytes") is not None:
        res["hbm_bytes_per_launch"] = g["hbm_read_bytes"] + g["hbm_write_bytes"]   # bench.py traffic
    res["whiten"]["algorithmic"] = {"bytes": 8 * N * (M + M + 20),
                                    "note": "cached distances read, gains records + fix-up rows "
                                            "read, beta written (include/gpar_hip.h)"}
    w = res["whiten"]
    if w.get("hbm_read_bytes") is not None and w.get("hbm_write_bytes") is not None:
        res["whiten_hbm_bytes_per_launch"] = w["hbm_read_bytes"] + w["hbm_write_bytes"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
