"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, grouped by kernel name and grid size
(e.g. the batched gains launches by chain count): calls, mean / min / max microseconds.

usage: python tools/trace_kernels.py run_kernel_trace.csv [--match gains] [--top 40]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    name_key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    gkeys = [k for k in rows[0] if k.lower().startswith("grid")]
    groups = collections.defaultdict(list)
    for r in rows:
        n = r[name_key]
        if a.match and a.match not in n:
            continue
        grid = tuple(r[k] for k in gkeys)
        groups[(n[:60], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("grid columns:", gkeys)
    items = sorted(groups.items(), key=lambda kv: -sum(kv[1]))[: a.top]
    for (n, g), d in items:
        print(f"{n:60s} grid={'x'.join(g):>18s} calls={len(d):5d} mean={sum(d) / len(d):9.1f} "
              f"min={min(d):9.1f} max={max(d):9.1f} us")


if __name__ == "__main__":
    main()
