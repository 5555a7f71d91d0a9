"""Summarise a rocprofv3 rocpd database (<run>_results.db) as kernel-stats CSV.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/<name>.csv

Columns follow rocprofv3's --stats kernel_stats.csv: Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs."""
import csv
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, tot, f"{avg:.1f}", f"{100.0 * tot / total:.3f}", mn, mx])


if __name__ == "__main__":
    main(sys.argv[1])
