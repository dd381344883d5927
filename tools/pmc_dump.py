#!/usr/bin/env python3
"""Per-kernel counter averages from rocprofv3 --pmc rocpd databases: pmc_dump.py <kernel regex> <db>..."""
import collections
import re
import sqlite3
import sys


def main():
    rx = re.compile(sys.argv[1])
    for db in sys.argv[2:]:
        c = sqlite3.connect(db)
        vals = collections.defaultdict(list)
        durs = {}
        for name, cn, v, d, disp in c.execute(
                "select kernel_name, counter_name, value, duration, dispatch_id from counters_collection"):
            if rx.search(name):
                vals[cn].append(v)
                durs[disp] = d
        print(db, f"dispatches={len(durs)} avg_dur_us={sum(durs.values()) / max(len(durs), 1) / 1e3:.1f}")
        for cn in sorted(vals):
            print(f"   {cn:28s} {sum(vals[cn]) / len(vals[cn]):16.0f}")


if __name__ == "__main__":
    main()
