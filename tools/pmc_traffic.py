#!/usr/bin/env python3
"""HBM-side traffic per launch of the dominant kernel class from rocprofv3 PMC passes (MI355X_MICROARCH.md,
HBM/rocprofv3: FETCH_SIZE and WRITE_SIZE in separate passes, KB units; on gfx950 FETCH_SIZE reports half the
bytes of 16-B-per-lane streaming reads, so it is doubled; WRITE_SIZE is exact for such stores and for f32
atomics).  Writes the JSON that bench.py reads for roofline.traffic.

usage: pmc_traffic.py <fetch run_counter_collection.csv> <write csv> <kernel regex> <out.json> <command>"""
import csv
import json
import re
import sys


def per_dispatch(path, counter, rx):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and re.search(rx, r["Kernel_Name"]):
            out[r["Dispatch_Id"]] = float(r["Counter_Value"])
    return out


def main():
    fcsv, wcsv, rx, out, cmd = sys.argv[1:6]
    f = per_dispatch(fcsv, "FETCH_SIZE", rx)
    w = per_dispatch(wcsv, "WRITE_SIZE", rx)
    n = len(f)
    fetch = 2.0 * sum(f.values()) * 1024.0
    write = sum(w.values()) * 1024.0
    res = {"kernel_regex": rx, "launches": n, "fetch_bytes_corrected": fetch, "write_bytes": write,
           "per_launch_bytes": (fetch + write) / max(n, 1), "command": cmd,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-include-regex), "
                     "FETCH_SIZE x2 (gfx950 16-B/lane read correction), KB x 1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
