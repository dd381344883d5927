#!/usr/bin/env python3
"""HBM-side traffic per launch of the dominant kernel class from rocprofv3 PMC passes (MI355X_MICROARCH.md,
HBM/rocprofv3: FETCH_SIZE and WRITE_SIZE in separate passes, KB units; on gfx950 FETCH_SIZE reports half the
bytes of 16-B-per-lane streaming reads, so it is doubled; WRITE_SIZE is exact for such stores and for f32
atomics).  Inputs are the rocpd databases (run_results.db) or run_counter_collection.csv files of the two passes.
Writes the JSON that bench.py reads for roofline.traffic.

usage: pmc_traffic.py <fetch pass> <write pass> <kernel regex> <out.json> <command>"""
import csv
import json
import re
import sqlite3
import sys


def per_dispatch(path, counter, rx):
    out = {}
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection").fetchall()
    else:
        rows = [(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]))
                for r in csv.DictReader(open(path))]
    for disp, name, cn, v in rows:
        if cn == counter and re.search(rx, name):
            out[disp] = out.get(disp, 0.0) + float(v)
    return out


def main():
    fpath, wpath, rx, out, cmd = sys.argv[1:6]
    f = per_dispatch(fpath, "FETCH_SIZE", rx)
    w = per_dispatch(wpath, "WRITE_SIZE", rx)
    n = len(f)
    fetch = 2.0 * sum(f.values()) * 1024.0
    write = sum(w.values()) * 1024.0 * n / max(len(w), 1)
    res = {"kernel_regex": rx, "launches": n, "fetch_bytes_corrected": fetch, "write_bytes": write,
           "per_launch_bytes": (fetch + write) / max(n, 1), "command": cmd,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-include-regex), "
                     "FETCH_SIZE x2 (gfx950 16-B/lane read correction), KB x 1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
