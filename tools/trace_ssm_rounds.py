"""Round boundaries of the temporal-only chains fit (bench.py --config ssm): reads a rocprofv3
--kernel-trace CSV and reports, per Nelder-Mead round, the span from the round's first gains
launch (gains_phase1) to its chain_carry_lml end, and the boundary from that end to the next
round's gains_phase1 start (host simplex step, theta upload, launch latency), with the kernels
that run inside the boundary.

usage: python tools/trace_ssm_rounds.py <run_kernel_trace.csv>
"""
import collections
import csv
import statistics
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("gpar::", "")[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key]) for r in rows)
p1 = [e for e in ev if "gains_phase1<" in e[2]]
lm = [e for e in ev if "chain_carry_lml" in e[2]]
spans, gaps, idle = [], [], []
inside = collections.Counter()
for a, b in zip(lm, lm[1:]):
    nxt = [e for e in p1 if e[0] > a[1] and e[0] < b[0]]
    if not nxt:
        continue
    s = nxt[0][0]
    gaps.append((s - a[1]) / 1e3)
    busy = 0
    for e in ev:
        if e[0] >= a[1] and e[1] <= s:
            busy += e[1] - e[0]
            inside[short(e[2])] += (e[1] - e[0]) / 1e3
    idle.append((s - a[1] - busy) / 1e3)
    prev = [e for e in p1 if e[0] <= a[0]]
    if prev:
        spans.append((a[1] - prev[-1][0]) / 1e3)
n = len(gaps)
print("rounds", n)
if n:
    print("round span  median %.1f us  mean %.1f" % (statistics.median(spans), statistics.mean(spans)))
    print("boundary    median %.1f us  mean %.1f  (GPU idle mean %.1f)" % (
        statistics.median(gaps), statistics.mean(gaps), statistics.mean(idle)))
    for k, v in inside.most_common(10):
        print("  in boundary: %-60s %.1f us per round" % (k, v / n))
per = collections.defaultdict(list)
for e in ev:
    per[short(e[2])].append((e[1] - e[0]) / 1e3)
print("kernels (calls, mean us):")
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:14]:
    print("  %-60s %5d %9.1f" % (k, len(v), statistics.mean(v)))
