"""CPU tests of the measurement plumbing: the per-class kernel-trace summary (tools/trace_classes.py) and the bench
line's graph-replayed roofline figure read from it (bench.py graph_replayed), on synthetic trace rows."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for name, t0, t1 in rows:
            w.writerow([name, t0, t1])


def test_trace_classes_per_step_times(tmp_path):
    """dispatches are classed by pmc_classes' regexes (prefill tile before the decode catch-all; the decode steps'
    big-tile vocabulary projection counts as decode, like the eager step's row-count split), per-step counts and times
    divide by the step count, unknown kernels land in "other", and the classes sum to the trace total"""
    rows = []
    t = 0
    for step in range(4):
        for _ in range(3):   # decode GEMM: 3 × 20 µs per step
            rows.append(("void qasr::k_gemm_q8d<4, 1, 1, 4, 3, 128, 1, true>(signed char const*)", t, t + 20_000))
            t += 25_000
        rows.append(("void qasr::k_gemm_q8d<2, 2, 4, 4, 3, 64, 1, false>(signed char const*)", t, t + 500_000))
        t += 600_000
        rows.append(("qasr::k_something_else(int)", t, t + 1000))
        t += 2000
        rows.append(("void qasr::k_gemm_q8d<2, 2, 4, 4, 2, 128, 1, true>(signed char const*)", t, t + 20_000))
        t += 25_000
    src, out = tmp_path / "run_kernel_trace.csv", tmp_path / "x_trace_classes.json"
    _trace(src, rows)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_classes.py"), str(out), "4", str(src)],
                   check=True, capture_output=True)
    d = json.loads(out.read_text())
    assert d["gemm_q8_decode"]["launches"] == 16 and d["gemm_q8_decode"]["launches_per_step"] == 4.0
    assert d["gemm_q8_decode"]["avg_us"] == 20.0 and d["gemm_q8_decode"]["ms_per_step"] == 0.08
    assert d["gemm_q8_prefill"]["launches_per_step"] == 1.0 and d["gemm_q8_prefill"]["avg_us"] == 500.0
    assert d["other"]["launches"] == 4 and d["other"]["avg_us"] == 1.0
    assert set(d) == {"gemm_q8_decode", "gemm_q8_prefill", "other", "_total", "_meta"} and d["_meta"]["steps"] == 4
    parts = sum(v["ms_per_step"] for k, v in d.items() if not k.startswith("_"))
    assert parts == pytest.approx(d["_total"]["ms_per_step"], rel=1e-6) and d["_total"]["launches"] == 24


def test_bench_graph_replayed_roofline(tmp_path, monkeypatch):
    """bench.graph_replayed prices the committed graph-replayed launch time with this run's algorithmic bytes (HBM
    classes) or flops (MFMA classes), prefers the file recorded for the loaded library, and is None without one"""
    import bench

    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    p = {"ms": 100.0, "count": 1000, "bytes": 20e6 * 1000, "flops": 1e12}
    assert bench.graph_replayed("gemm_q8_decode", p) is None
    (tmp_path / "profiles").mkdir()
    old = {"gemm_q8_decode": {"launches": 40, "launches_per_step": 10.0, "ms_per_step": 1.0, "avg_us": 40.0},
           "_meta": {"lib_sha256_16": "aaaa", "generated_utc": "2026-01-02T00:00:00+00:00"}}
    new = {"gemm_q8_decode": {"launches": 40, "launches_per_step": 10.0, "ms_per_step": 0.2, "avg_us": 20.0},
           "gemm_q8_prefill": {"launches": 4, "launches_per_step": 1.0, "ms_per_step": 0.5, "avg_us": 500.0},
           "_meta": {"lib_sha256_16": "bbbb", "generated_utc": "2026-01-01T00:00:00+00:00"}}
    (tmp_path / "profiles" / "old_trace_classes.json").write_text(json.dumps(old))
    (tmp_path / "profiles" / "new_trace_classes.json").write_text(json.dumps(new))
    monkeypatch.setattr(bench, "lib_sha16", lambda: "bbbb")
    r = bench.graph_replayed("gemm_q8_decode", p)
    assert r["matches_build"] and r["source"].endswith("new_trace_classes.json")
    assert r["avg_launch_us"] == 20.0 and r["unit"] == "GB/s"
    assert r["achieved"] == pytest.approx(20e6 / 20e-6 / 1e9, rel=1e-3)            # 1,000 GB/s
    assert r["frac"] == pytest.approx(1000.0 / 8000.0, rel=1e-3)
    q = bench.graph_replayed("gemm_q8_prefill", {"ms": 1.0, "count": 1, "bytes": 1.0, "flops": 2.5e11})
    assert q["unit"] == "TFLOP/s" and q["achieved"] == pytest.approx(2.5e11 / 500e-6 / 1e12, rel=1e-3)
    monkeypatch.setattr(bench, "lib_sha16", lambda: "cccc")   # no file for this build: the newest, flagged
    r = bench.graph_replayed("gemm_q8_decode", p)
    assert not r["matches_build"] and r["source"].endswith("old_trace_classes.json")


def test_bench_roofline_headline_is_graph_replayed(tmp_path, monkeypatch):
    """with a trace recorded for the loaded library the line's headline achieved / frac / avg_launch_us are the
    graph-replayed figures (reproducible from profiles/ as algorithmic bytes per launch / trace avg / 8 TB/s),
    the eager HIP-event figure kept under "eager"; without one the eager figure stays the headline"""
    import bench

    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "pmc_evidence", lambda k: None)
    p = {"ms": 25.0, "count": 1000, "bytes": 20e6 * 1000, "flops": 1e12}   # eager: 25 µs per launch
    r = bench.class_roofline("gemm_q8_decode", p)
    assert "eager" not in r and r["avg_launch_us"] == 25.0
    (tmp_path / "profiles").mkdir()
    tr = {"gemm_q8_decode": {"launches": 40, "launches_per_step": 10.0, "ms_per_step": 0.2, "avg_us": 20.0},
          "_meta": {"lib_sha256_16": "bbbb", "generated_utc": "2026-01-01T00:00:00+00:00"}}
    (tmp_path / "profiles" / "x_trace_classes.json").write_text(json.dumps(tr))
    monkeypatch.setattr(bench, "lib_sha16", lambda: "bbbb")
    r = bench.class_roofline("gemm_q8_decode", p)
    assert r["avg_launch_us"] == 20.0 and r["frac"] == pytest.approx(20e6 / 20e-6 / 8e12, rel=1e-3)
    assert r["eager"]["avg_launch_us"] == 25.0 and r["eager"]["frac"] == pytest.approx(20e6 / 25e-6 / 8e12, rel=1e-3)
    assert r["frac"] == r["graph_replayed"]["frac"]
