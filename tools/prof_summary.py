#!/usr/bin/env python3
"""Per-kernel time per bench step from a rocprofv3 rocpd database (kernel trace of `bench.py --steps 1
--warmup 1`: the two runs are averaged)."""
import collections
import sqlite3
import sys


def main():
    db, runs = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    c = sqlite3.connect(db)
    rows = c.execute("select start, end, name from kernels order by start").fetchall()
    by, cnt = collections.Counter(), collections.Counter()
    for s, e, n in rows:
        k = n.split("(")[0][-44:]
        by[k] += e - s
        cnt[k] += 1
    span = (rows[-1][1] - rows[0][0]) / 1e6
    print(f"busy {sum(by.values()) / runs / 1e6:.1f} ms/step, span {span / runs:.1f} ms/step")
    for k, v in by.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 24):
        print(f"{v / runs / 1e6:8.2f} ms/step {cnt[k] / runs:8.0f} {v / cnt[k] / 1e3:9.2f} us  {k}")


if __name__ == "__main__":
    main()
