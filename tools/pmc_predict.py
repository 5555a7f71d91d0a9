"""Summarise tools/pmc_predict.sh: per-dispatch counters of the prediction kernels (rocprofv3
--pmc passes) -> per kernel: average duration under --pmc, HBM bytes (FETCH_SIZE x 2: gfx950
reports half of wide streaming reads; WRITE_SIZE exact), effective clock, MFMA busy fraction and
wave-time split (MI355X_MICROARCH.md conventions, as tools/pmc_sq.py), against each kernel's
algorithmic bytes at N = N* = 1e6, M = 512 (Mp = 512), D = 62..63."""
import csv
import glob
import json
import sys
from collections import defaultdict

N = NS = 1_000_000
NT = N + NS
M = MP = 512
SIMDS = 1024
ALGO = {  # algorithmic HBM bytes per launch (bench.py roofline_predict)
    "whiten_kfu_mfma": 8 * NT * (62.5 + M + 20),
    "adjoint_local_wide": 8 * (NT * (MP + 1 + 21) + NS * (MP + 1)),
    "predict_rows": 16 * NS * MP,
    "gemm_nt_kernel": 8 * NS * MP,
}
FLOPS = {"predict_var": NS * M * (M + 1)}   # the variance product's triangle (bench.py pred_var)


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            sub = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gpar::", "").split("<")[0]
            key = (sub, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = defaultdict(lambda: defaultdict(list))
    for (sub, di), cs in per.items():
        for c, v in cs.items():
            out[sub][c].append(v)
        if (sub, di) in dur:
            out[sub]["_dur"].append(dur[(sub, di)])
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}


def main(root):
    sq, fe, wr = load(root + "/sq1"), load(root + "/fetch"), load(root + "/write")
    lds = load(root + "/lds")
    res = {"source": "tools/pmc_predict.sh: rocprofv3 --pmc passes over tools/predict_probe.py "
                     "--outputs 2 --dmin 62 (N = N* = 1e6, M = 512, D = 62, 63); per-dispatch averages"}
    for k in sorted(sq):
        c = sq[k]
        t = c.get("_dur")
        e = {"dispatch_s_under_pmc": t, "counters": {a: b for a, b in c.items() if a != "_dur"}}
        if t and c.get("GRBM_GUI_ACTIVE"):
            clk = c["GRBM_GUI_ACTIVE"] / 8 / t
            e["effective_clock_GHz"] = clk / 1e9
            if c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                e["mfma_busy_fraction"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * clk * t)
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            e["wave_time_fraction"] = {"active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / w,
                                       "wait_inst_any (issue stall)": c.get("SQ_WAIT_INST_ANY", 0) / w,
                                       "wait_any (waitcnt/barrier)": c.get("SQ_WAIT_ANY", 0) / w}
        if k in lds:
            e["lds_counters"] = {a: b for a, b in lds[k].items() if a != "_dur"}
        if k in FLOPS and t:
            e["tflops"] = FLOPS[k] / t / 1e12
            e["frac_of_fp64_peak"] = FLOPS[k] / t / 78.6e12
        f = fe.get(k, {}).get("FETCH_SIZE")
        wb = wr.get(k, {}).get("WRITE_SIZE")
        e["hbm_read_bytes"] = f * 1024 * 2 if f is not None else None
        e["hbm_write_bytes"] = wb * 1024 if wb is not None else None
        if k in ALGO:
            e["algorithmic_bytes"] = ALGO[k]
            if t:
                e["algorithmic_GBps"] = ALGO[k] / t / 1e9
                e["frac_of_8TBps"] = ALGO[k] / t / 8e12
        res[k] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
