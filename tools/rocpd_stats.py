"""Kernel statistics (the rocprofv3 --stats table) from a rocprofv3 rocpd database.

    python tools/rocpd_stats.py RUN_RESULTS.db OUT.csv

Columns as rocprofv3's kernel_stats.csv: Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs (durations of every dispatch of the kernel in the database)."""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1:3]
    con = sqlite3.connect(db)
    agg = {}
    for name, dur in con.execute("select name, duration from kernels"):
        agg.setdefault(name, []).append(float(dur))
    tot = sum(sum(v) for v in agg.values()) or 1.0
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), int(sum(v)), round(sum(v) / len(v), 1), round(100 * sum(v) / tot, 3),
                        int(min(v)), int(max(v))])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print("%-60s %4d %10.1f us avg" % (name.split("(")[0][:60], len(v), sum(v) / len(v) / 1e3))


if __name__ == "__main__":
    main()
