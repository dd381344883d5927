#!/usr/bin/env python3
"""Cost of batch-invariant C4 decode GEMMs: every batched decode row computed with the single-row
decode's arithmetic (qasr_op_gemm_exact_rows: the GEMV's block fma chains and wave-sum tree, 32-row chunks)
instead of the deterministic batched GEMM table (qasr_op_linear_q8 path 2 / qasr_op_gemm_swiglu_q8).  Times both per
decoder matrix and row count with COLD weights (a ring of copies larger than the Infinity Cache, as in a decode step
streaming 28 layers), then prices one C4 bench step: Σ over its decode steps of 28 × (exact − table) at that step's
live rows (bench.py's 256-segment workload, FORCE_TPS tokens per audio-s + 1).  GPU.
usage: python tools/exact_cost.py [out.json]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

# (tag, N, K, epi): 0 store, 1 residual, 3 gate/up + SwiGLU (table: fused epilogue; exact: store + swiglu op)
SHAPES = [("qkv", 4096, 2048, 0), ("o", 2048, 2048, 1), ("gu", 12288, 2048, 3), ("down", 2048, 6144, 1),
          ("lm", 151936, 2048, 0)]
MS = list(range(16, 257, 16))
LAYERS = 28


def c4_rows(total=256, seed=1, tps=8):
    """live rows of each decode step of bench.py's C4 workload (make_workload's durations, n_new = round(tps·s) + 1)"""
    secs = np.random.default_rng(seed).uniform(2.0, 12.0, size=total)
    n_new = np.array([int(round(tps * int(s * 16000) / 16000)) + 1 for s in secs])
    return [int((n_new > t).sum()) for t in range(int(n_new.max()))]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    part = torch.empty(256 * 12288 * 8, dtype=torch.float32, device=dev)
    cnt = torch.zeros(8192, dtype=torch.int32, device=dev)
    _lib.check(lib.qasr_op_set_gemm_fixup(part.data_ptr(), part.numel() * 4, cnt.data_ptr(), cnt.numel()))
    table, exact = {}, {}
    for tag, N, K, epi in SHAPES:
        copies = max(2, int(768e6 // (N * K * 1.0625)) + 1)
        wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
        ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
        s4 = []
        for w in ws:   # the decoder matrices carry their regrouped stage scales (model.cpp ensure_stage_scales)
            o = torch.empty_like(w)
            _lib.check(lib.qasr_op_stage_scales(w.data_ptr(), N, K, o.data_ptr(), None))
            _lib.check(lib.qasr_op_register_stage_scales(w.data_ptr(), N, K, o.data_ptr()))
            s4.append(o)
        for M in MS:
            xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            xd = torch.rand(M, K // 32, device=dev) * 0.01
            y = torch.zeros(M, N, device=dev)
            hq = torch.empty(M, max(N // 2, 1), dtype=torch.int8, device=dev)
            hd = torch.empty(M, max(N // 64, 1), device=dev)

            def run_table(i):
                if epi == 3:
                    _lib.check(lib.qasr_op_gemm_swiglu_q8(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                          ws[i].data_ptr(), N, K, hq.data_ptr(), hd.data_ptr(), None))
                    return
                _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(), ws[i].data_ptr(),
                                                 N, K, None, y.data_ptr() if epi == 1 else None, y.data_ptr(), N,
                                                 epi, 2, None))

            def run_exact(i):   # one launch: 32-row chunks along grid.y
                _lib.check(lib.qasr_op_gemm_exact_rows(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                       ws[i].data_ptr(), N, K, y.data_ptr() if epi == 1 else None,
                                                       y.data_ptr(), N, 1 if epi == 1 else 0, None))
                if epi == 3:
                    _lib.check(lib.qasr_op_swiglu_q8_interleaved(y.data_ptr(), M, N // 2, hq.data_ptr(),
                                                                 hd.data_ptr(), None))

            for name, fn, out in (("table", run_table, table), ("exact", run_exact, exact)):
                fn(0)
                torch.cuda.synchronize()
                n = copies * max(1, 16 // copies)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(n):
                    fn(i % copies)
                e1.record()
                torch.cuda.synchronize()
                out[(tag, M)] = e0.elapsed_time(e1) / n * 1e3
            print(f"{tag:5s} M={M:4d} table {table[(tag, M)]:8.1f}us exact {exact[(tag, M)]:8.1f}us "
                  f"x{exact[(tag, M)] / table[(tag, M)]:.2f}", flush=True)
        for w in ws:
            _lib.check(lib.qasr_op_register_stage_scales(w.data_ptr(), N, K, None))
        del wq, ws, s4
        torch.cuda.empty_cache()

    def at(d, tag, m):   # piecewise-linear in rows between the measured row counts
        ms = np.array(MS, dtype=float)
        return float(np.interp(m, ms, [d[(tag, x)] for x in MS]))

    rows = c4_rows()
    res = {"rows_per_step": rows, "per_shape_us": {f"{t}:{m}": [round(table[(t, m)], 2), round(exact[(t, m)], 2)]
                                                     for t, *_ in SHAPES for m in MS}}
    for name, d in (("table", table), ("exact", exact)):
        layer = sum(LAYERS * at(d, t, m) for m in rows for t, *_ in SHAPES if t != "lm")
        lm = sum(at(d, "lm", m) for m in rows)
        res[f"{name}_ms_per_c4_step"] = round((layer + lm) / 1e3, 2)
    res["delta_ms_per_c4_step"] = round(res["exact_ms_per_c4_step"] - res["table_ms_per_c4_step"], 2)
    print(json.dumps({k: v for k, v in res.items() if k != "per_shape_us" and k != "rows_per_step"}), flush=True)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
