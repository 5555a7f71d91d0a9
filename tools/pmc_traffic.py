"""Per-launch HBM traffic of the Gram / whitening kernels from two rocprofv3 PMC passes.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/gram_pmc_<round>.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (summed over the counter's instances); the fetch
figure is doubled per MI355X_MICROARCH.md (gfx950 FETCH_SIZE reports half of streamed reads)."""
import csv
import json
import sys

N, M, D = 1_000_000, 512, 32
NCH = (N + 255) // 256


def per_dispatch(path, needle):
    per = {}
    for r in csv.DictReader(open(path + "/run_counter_collection.csv")):
        if needle in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sum(per.values()) / max(len(per), 1), len(per)


def main(fetch_dir, write_dir):
    gf, n1 = per_dispatch(fetch_dir, "gram_kernel")
    gw, _ = per_dispatch(write_dir, "gram_kernel")
    wf, _ = per_dispatch(fetch_dir, "whiten_kfu")
    ww, _ = per_dispatch(write_dir, "whiten_kfu")
    out = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                  "tools/gram_probe.py --evals 3 (N=1e6, M=512, D=32)",
        "units": "bytes per launch; FETCH_SIZE (KiB) x 1024 x 2 (gfx950 correction), WRITE_SIZE (KiB) x 1024. "
                 "The Gram stages beta by global_load_lds_dwordx4 (16 B/lane, the calibrated width).",
        "gram_kernel": {"launches": n1, "fetch_kib_raw": gf, "write_kib_raw": gw,
                        "hbm_read_bytes": gf * 2048, "hbm_write_bytes": gw * 1024,
                        "algorithmic_bytes": N * M * 8 + N * 8 + NCH * M * 4 * 8 * 2,
                        "algorithmic_note": "beta (N x M f64) and alpha read once + the chunk correction's "
                                            "E_j, C_j (nch x M x 4 f64 each)"},
        "whiten_kfu_mfma_D32": {"fetch_kib_raw": wf, "write_kib_raw": ww, "hbm_read_bytes": wf * 2048,
                                "hbm_write_bytes": ww * 1024,
                                "algorithmic_bytes": N * D * 8 + N * 16 * 8 + N * M * 8},
    }
    out["hbm_bytes_per_launch"] = out["gram_kernel"]["hbm_read_bytes"] + out["gram_kernel"]["hbm_write_bytes"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
