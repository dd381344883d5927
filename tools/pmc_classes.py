#!/usr/bin/env python3
"""Per-kernel-class hardware counters from rocprofv3 --pmc passes (rocpd databases), for the roofline evidence
north_star asks for ("rocprof HBM GB/s and MFMA-busy against gfx950 peak").

Counters are summed over the dispatches of each class and reported raw next to the derived figures:
  * MFMA busy   = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), 1,024 SIMDs; kernel cycles = GRBM_GUI_ACTIVE / 8
                  (summed over the 8 XCDs, MI355X_MICROARCH.md "DVFS give-back"; short dispatches read high);
  * HBM traffic = 2 x FETCH_SIZE + WRITE_SIZE (KB; FETCH_SIZE reports half the bytes of 16-B-per-lane streaming
                  reads on gfx950, MI355X_MICROARCH.md §HBM), GB/s over the class's summed dispatch time;
  * wait split  = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES.
The derived MfmaUtil / VALUBusy of ROCm 7.2 use gfx94x formulas on gfx950, so only raw counters are used here.

usage: pmc_classes.py <out.json> <pass.db>...
"""
import collections
import json
import re
import sqlite3
import sys

CLASSES = [  # (class, kernel-name regex) — first match wins
    # bench.py's ProfScope classes split the Q8 GEMM by row count (prefill / encoder M > 256, decode M <= 256); by name,
    # M > 256 is the 128x128 K-64 tile (kernels_q8.hip cfg 4) alone — the other big tiles (cfg 8 / 9 / 10, 128x128 /
    # 64x128 / 64x64 K-128) are the decode steps' vocabulary projections, which the eager step counts as decode
    ("gemm_q8_prefill", r"k_gemm_q8d<2, 2, 4, 4, 3, 64[,>]"),
    ("gemm_q8_decode", r"k_gemm_q8d<|k_gemm_q8_ks<|k_gemm_q8<"),
    ("gemv_q8", r"k_gemv_q8|k_gemv_wide"),
    ("xr_linear", r"k_xr_linear|k_xr_gu"),
    ("gemm_q8_exact", r"k_gemm_q8_exact"),
    ("gemm_mx", r"k_gemm_mx"),
    ("attention_decode", r"k_attention<"),
    ("attention_tile", r"k_attn_tile"),
    ("conv3x3", r"k_conv3x3"),
    ("rmsnorm", r"k_rmsnorm"),
    ("layernorm", r"k_layernorm"),
    ("mel", r"k_mel"),
    ("argmax", r"k_argmax"),
]
SIMDS = 1024
GRBM_UNITS = 8


def klass(name):
    for c, rx in CLASSES:
        if re.search(rx, name):
            return c
    return None


def main():
    out = sys.argv[1]
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    passes = collections.defaultdict(lambda: collections.defaultdict(set))   # class → counter → pass dbs seen
    disp = collections.defaultdict(dict)   # class → dispatch id → duration ns (per pass db)
    for db in sys.argv[2:]:
        c = sqlite3.connect(db)
        seen = set()
        for name, cn, v, d, di in c.execute(
                "select kernel_name, counter_name, value, duration, dispatch_id from counters_collection"):
            k = klass(name)
            if k is None:
                continue
            sums[k][cn] += float(v)
            passes[k][cn].add(db)
            if (db, di) not in seen:
                seen.add((db, di))
                disp[k][(db, di)] = float(d)
    for k in sums:   # a counter collected in several passes (GRBM_GUI_ACTIVE rides along in each): per-pass mean
        for cn in sums[k]:
            sums[k][cn] /= max(1, len(passes[k][cn]))
    res = {}
    for k in sorted(sums):
        s = sums[k]
        n_db = len({db for db, _ in disp[k]})
        dur_ns = sum(disp[k].values()) / max(n_db, 1)          # per pass
        launches = len(disp[k]) / max(n_db, 1)
        r = {"launches_per_pass": round(launches), "avg_us": round(dur_ns / max(launches, 1) / 1e3, 2),
             "raw": {cn: v for cn, v in sorted(s.items())}}
        if s.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in s:
            r["mfma_busy"] = round(s["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * s["GRBM_GUI_ACTIVE"] / GRBM_UNITS), 4)
        if s.get("GRBM_GUI_ACTIVE") and dur_ns:
            r["clock_ghz"] = round(s["GRBM_GUI_ACTIVE"] / GRBM_UNITS / dur_ns, 3)
        if "FETCH_SIZE" in s and "WRITE_SIZE" in s and dur_ns:
            b = (2 * s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024
            r["hbm_bytes_per_launch"] = round(b / max(launches, 1))
            r["hbm_gbps"] = round(b / dur_ns, 1)
        if s.get("SQ_WAVE_CYCLES"):
            r["wait_any_frac"] = round(s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"], 3)
            r["wait_inst_frac"] = round(s.get("SQ_WAIT_INST_ANY", 0) / s["SQ_WAVE_CYCLES"], 3)
            r["active_inst_frac"] = round(s.get("SQ_ACTIVE_INST_ANY", 0) / s["SQ_WAVE_CYCLES"], 3)
        res[k] = r
    # provenance: the library build the passes profiled (bench.py uses the counters only for the same build)
    import datetime
    import hashlib
    import os

    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "light-whisper_amd", "libqasr.so")
    res["_meta"] = {"lib_sha256_16": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib)
                    else None, "generated_utc": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds")}
    json.dump(res, open(out, "w"), indent=1)
    for k, r in res.items():
        if k != "_meta":
            print(k, {x: y for x, y in r.items() if x != "raw"})


if __name__ == "__main__":
    main()
