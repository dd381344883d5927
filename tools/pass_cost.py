#!/usr/bin/env python3
"""Verify-pass kernel cost by row bucket from rocprofv3 kernel stats of tools/verify_cost.py runs (one run per n, each
= 6 one-pass calls on the same prompt): kernel time of a run minus the n = 1 run's, per pass, plus the 1-row pass's own
kernel time (the decoder kernels that appear only in the passes).  usage: pass_cost.py <stats_n1.csv> <stats_n2.csv> …"""
import csv
import re
import sys


def total(path):
    rows = list(csv.DictReader(open(path)))
    return sum(float(r["TotalDurationNs"]) for r in rows), rows


def main():
    files = sys.argv[1:]
    t1, rows1 = total(files[0])
    # the 1-row pass: the fused GEMVs, the split decode attention, argmax / lm_head GEMV launches of the 6 calls
    one = sum(float(r["TotalDurationNs"]) for r in rows1
              if re.search(r"k_gemv_wide|k_attention<128, 2, 4, true, 64>|k_argmax", r["Name"])) / 6 / 1e6
    print(f"n=1: {one:.3f} ms of kernels per pass (1.00)")
    for f in files[1:]:
        n = int(re.search(r"_(\d+)\.csv$", f).group(1))
        t, _ = total(f)
        ms = one + (t - t1) / 6 / 1e6
        print(f"n={n}: {ms:.3f} ms of kernels per pass ({ms / one:.2f})")


if __name__ == "__main__":
    main()
