#!/usr/bin/env python3
"""Kernel statistics (name, calls, total/avg/min/max ns, share) from a rocprofv3 rocpd SQLite database —
the same table `rocprofv3 --stats` writes as kernel_stats.csv, for runs that produced only the .db."""
import csv
import sqlite3
import sys


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                     "from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, t, a, lo, hi, 100.0 * t / tot) for n, k, t, a, lo, hi in rows]


def main():
    db, out = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None
    rows = kernel_stats(db)
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", r[4], r[5], f"{r[6]:.2f}"])


if __name__ == "__main__":
    main()
