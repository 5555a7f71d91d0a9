"""Side-by-side kernel stats of two rocprofv3 --stats runs (tools/gpu_ab_kernels.sh)."""
import csv
import glob
import sys


def load(d):
    f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"].split("(")[0][:60]: (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6)
            for r in csv.DictReader(open(f))}


a, b = load(sys.argv[1]), load(sys.argv[2])
names = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0))[1], b.get(k, (0, 0))[1]))
print(f"{'kernel':60s} {'calls':>6s} {'base ms':>9s} {'var ms':>9s}")
for k in names[:30]:
    ca, ta = a.get(k, (0, 0.0))
    cb, tb = b.get(k, (0, 0.0))
    print(f"{k:60s} {max(ca, cb):6d} {ta:9.2f} {tb:9.2f}")
print(f"{'TOTAL':60s} {'':6s} {sum(v[1] for v in a.values()):9.2f} {sum(v[1] for v in b.values()):9.2f}")
