"""Where a batched fit's time goes between Grams: reads a rocprofv3 --kernel-trace CSV
(run_kernel_trace.csv) of a north bench step and reports, per Nelder-Mead round, the Gram stream's
busy span and the gap from the round's last Gram reduction to the next round's first Gram, with the
kernels that run in that gap (summed durations).

usage: python tools/trace_rounds.py gpurun_out/<dir>/run_kernel_trace.csv [--top 20]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--hip", default=None, help="rocprofv3 --hip-trace CSV (run_hip_api_trace.csv): "
                    "the host's HIP calls inside the median boundary")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    name_key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    ev = []
    for r in rows:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[name_key]))
    ev.sort()
    t0 = ev[0][0]
    off = [e for e in ev if "gram3_off_kernel" in e[2]]
    red = [e for e in ev if "gram3_reduce" in e[2]]
    # a round boundary: a gap between consecutive OFF kernels much larger than a Gram
    gaps = []
    for a_, b_ in zip(off, off[1:]):
        gaps.append((b_[0] - a_[1], a_, b_))
    if not gaps:
        print("no gram3_off_kernel dispatches")
        return
    med = sorted(g for g, _, _ in gaps)[len(gaps) // 2]
    bounds = [(g, x, y) for g, x, y in gaps if g > 5 * max(med, 1000) + 1_000_000]
    print(f"{len(off)} OFF dispatches, median OFF-to-OFF gap {med / 1e3:.1f} us, "
          f"{len(bounds)} round boundaries (gap > 1 ms)")
    tot_gap = 0
    inside = collections.Counter()
    inside_n = collections.Counter()
    for g, x, y in bounds:
        # the last reduction of the round ends after x (the last OFF); the gap is counted from it
        last_red = max((e for e in red if x[0] <= e[0] <= y[0]), default=None, key=lambda e: e[1])
        start = last_red[1] if last_red else x[1]
        tot_gap += y[0] - start
        for e in ev:
            if start <= e[0] < y[0]:
                inside[e[2][:60]] += e[1] - e[0]
                inside_n[e[2][:60]] += 1
    nb = max(len(bounds), 1)
    print(f"mean gap from the round's last reduction to the next round's first OFF: "
          f"{tot_gap / nb / 1e6:.3f} ms ({tot_gap / 1e9:.3f} s over {len(bounds)} boundaries)")
    print("kernels starting inside those gaps (sum of durations per boundary, calls per boundary):")
    for k, v in inside.most_common(a.top):
        print(f"  {k:60s} {v / nb / 1e6:8.3f} ms {inside_n[k] / nb:6.1f}")
    # the typical round boundary: the median gap, as a timeline of the kernels that start in it
    if bounds:
        g_sorted = sorted(bounds, key=lambda b: b[0])
        print("boundary gaps (ms), sorted:", [round(g / 1e6, 2) for g, _, _ in g_sorted])
        g, x, y = g_sorted[len(g_sorted) // 2]
        last_red = max((e for e in red if x[0] <= e[0] <= y[0]), default=None, key=lambda e: e[1])
        start = last_red[1] if last_red else x[1]
        print(f"median boundary: {(y[0] - start) / 1e6:.3f} ms from the last reduction to the next OFF;"
              " kernels (start, end in ms from the last reduction's end):")
        for e in ev:
            if start - 2_000_000 <= e[0] < y[0] + 200_000:
                print(f"  {(e[0] - start) / 1e6:8.3f} {(e[1] - start) / 1e6:8.3f}  {e[2][:70]}")
        if a.hip:
            hrows = list(csv.DictReader(open(a.hip)))
            fn = "Function" if "Function" in hrows[0] else "Name"
            calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[fn]) for r in hrows)
            inside = [c_ for c_ in calls if start <= c_[0] < y[0]]
            print(f"HIP API calls inside the median boundary: {len(inside)}, "
                  f"{sum(c_[1] - c_[0] for c_ in inside) / 1e6:.3f} ms in calls; per function "
                  "(count, total ms):")
            agg = collections.defaultdict(lambda: [0, 0])
            for c_ in inside:
                agg[c_[2]][0] += 1
                agg[c_[2]][1] += c_[1] - c_[0]
            for k, (n_, t_) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
                print(f"  {k:40s} {n_:5d} {t_ / 1e6:8.3f}")
            print("timeline of the calls (start, duration in ms from the last reduction's end):")
            for c_ in inside:
                if c_[1] - c_[0] > 20_000:   # calls longer than 20 us
                    print(f"  {(c_[0] - start) / 1e6:8.3f} {(c_[1] - c_[0]) / 1e6:8.3f}  {c_[2]}")
    span = ev[-1][1] - t0
    print(f"trace span {span / 1e9:.3f} s")


if __name__ == "__main__":
    main()
