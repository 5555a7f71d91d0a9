"""Between-Gram time of a fit whose every Nelder-Mead round has ONE Gram launch set (a grouped
Gram of a rank's shard, bench.py --config eeg --shard R/8): reads a rocprofv3 --kernel-trace CSV
and reports, averaged over the gaps from one Gram's reduction end to the next Gram's OFF start,
the gap's wall time, the GPU-idle part of it (no kernel running) and the kernels that run in it
(summed durations, by name), plus the Gram span itself.

usage: python tools/trace_gaps.py gpurun_out/<dir>/run_kernel_trace.csv [--top 25]
"""
import argparse
import collections
import csv


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("gpar::", "")[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key]) for r in rows)
    off = [e for e in ev if "gram3_off_kernel" in e[2]]
    red = [e for e in ev if "gram3_reduce" in e[2]]
    if len(off) < 2:
        print("fewer than two gram3_off_kernel dispatches")
        return
    gaps, spans = [], []
    for o in off:
        r = next((x for x in red if x[0] >= o[0]), None)
        if r:
            spans.append(r[1] - o[0])
    for o, o2 in zip(off, off[1:]):
        r = next((x for x in red if x[0] >= o[0] and x[1] <= o2[0]), None)
        if r:
            gaps.append((r[1], o2[0]))
    by = collections.Counter()
    idle = 0
    wall = 0
    for g0, g1 in gaps:
        wall += g1 - g0
        inside = [e for e in ev if e[1] > g0 and e[0] < g1]
        for s, e, nm in inside:
            by[short(nm)] += min(e, g1) - max(s, g0)
        cur = g0
        for s, e, _ in sorted(inside):
            if s > cur:
                idle += s - cur
            cur = max(cur, e)
        if g1 > cur:
            idle += g1 - cur
    ng = max(len(gaps), 1)
    print(f"{len(off)} Gram launch sets, span {sum(spans) / len(spans) / 1e3:.1f} us avg; "
          f"{len(gaps)} gaps: wall {wall / ng / 1e3:.1f} us avg, GPU idle {idle / ng / 1e3:.1f} us avg")
    for nm, t in by.most_common(a.top):
        print(f"  {t / ng / 1e3:9.1f} us  {nm}")


if __name__ == "__main__":
    main()
