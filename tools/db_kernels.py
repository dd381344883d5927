#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd SQLite output (--kernel-trace): launches, total / average µs, share;
optionally restricted to dispatches after the first `--skip-frac` of the trace.  Usage: db_kernels.py results.db
[--top N] [--by-grid]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--by-grid", action="store_true", help="split each kernel by grid shape")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    key = "name || ' g=' || grid_x || 'x' || grid_y || 'x' || grid_z" if a.by_grid else "name"
    rows = cur.execute(f"select {key}, count(*), sum(duration), avg(duration) from kernels group by 1 "
                       "order by 3 desc").fetchall()
    total = sum(r[2] for r in rows)
    print(f"total kernel time {total / 1e6:.3f} ms over {sum(r[1] for r in rows)} launches")
    for name, n, tot, avg in rows[: a.top]:
        print(f"{tot / 1e6:9.3f} ms {100 * tot / total:5.1f}% {n:7d} x {avg / 1e3:8.2f} us  {name[:110]}")


if __name__ == "__main__":
    main()
