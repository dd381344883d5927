#!/usr/bin/env python3
"""Per-kernel-class launch times of GRAPH-REPLAYED bench steps, from a rocprofv3 --kernel-trace of
`bench.py --no-prof` (every step replays its captured decode-step graphs; no eager instrumented step), for the bench
line's `roofline.graph_replayed` figure: the class's average launch duration as the timed steps run it, beside the
eager HIP-event figure bench.py measures live (events per launch would perturb the graphs).

Classes follow tools/pmc_classes.py (first regex match wins).  Input: the kernel-trace CSV (Kernel_Name,
Start_Timestamp, End_Timestamp) or a rocpd SQLite database (kernels table).

usage: trace_classes.py <out.json> <steps incl. warm-up> <kernel_trace.csv | run.db>
"""
import collections
import csv
import datetime
import hashlib
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_classes import klass  # noqa: E402


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        yield from c.execute("select name, start, end from kernels")
        return
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])


def main():
    out, steps, src = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    n = collections.Counter()
    ns = collections.Counter()
    for name, t0, t1 in rows(src):
        k = klass(name) or "other"   # every launch lands in a class, so the classes sum to the trace total
        n[k] += 1
        ns[k] += t1 - t0
    res = {k: {"launches": n[k], "launches_per_step": round(n[k] / steps, 1), "ms_per_step": round(ns[k] / steps / 1e6, 3),
               "avg_us": round(ns[k] / n[k] / 1e3, 3)} for k in sorted(n)}
    tot = sum(ns.values())
    res["_total"] = {"launches": sum(n.values()), "ms_per_step": round(tot / steps / 1e6, 3)}
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "light-whisper_amd", "libqasr.so")
    res["_meta"] = {"lib_sha256_16": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib)
                    else None, "steps": steps, "source": os.path.basename(src),
                    "generated_utc": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds")}
    json.dump(res, open(out, "w"), indent=1)
    for k, r in res.items():
        print(k, r)
    top = collections.Counter()
    for name, t0, t1 in rows(src):
        if klass(name) is None:
            top[name.split("(")[0][:90]] += t1 - t0
    for name, t in top.most_common(8):   # what "other" holds
        print(f"  other: {t / steps / 1e6:8.3f} ms/step  {name}")


if __name__ == "__main__":
    main()
