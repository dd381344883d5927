#!/usr/bin/env python3
"""Idle gaps on the GPU timeline of a rocprofv3 --kernel-trace rocpd database: span vs busy (union of kernel
intervals) over the last `--window` ms of the trace (one bench step), and the largest gaps with the kernels on
either side.  Usage: db_gaps.py results.db [--window MS] [--top N]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window", type=float, default=0.0, help="only the last WINDOW ms of the trace (0 = all)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).cursor().execute("select start, end, name from kernels order by start").fetchall()
    if a.window > 0:
        t_end = max(r[1] for r in rows)
        rows = [r for r in rows if r[0] >= t_end - a.window * 1e6]
    busy, gaps, cur_end, prev = 0, [], rows[0][0], None
    for s, e, n in rows:
        if s > cur_end:
            gaps.append((s - cur_end, prev, n, s))
            busy += e - s
            cur_end = e
        elif e > cur_end:
            busy += e - cur_end
            cur_end = e
        prev = n
    span = cur_end - rows[0][0]
    print(f"kernels {len(rows)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(span - busy) / 1e6:.2f} ms")
    tot = sum(g[0] for g in gaps)
    small = sum(g[0] for g in gaps if g[0] < 20e3)
    print(f"gaps {len(gaps)}: total {tot / 1e6:.2f} ms, of which gaps < 20 us {small / 1e6:.2f} ms")
    for g, p, n, s in sorted(gaps, reverse=True)[: a.top]:
        print(f"{g / 1e3:9.1f} us  at {(s - rows[0][0]) / 1e6:8.2f} ms  after {p[:60]}  before {n[:60]}")


if __name__ == "__main__":
    main()
