#!/usr/bin/env python3
"""The decode steps' vocabulary projection (1.7B: N 151,936 × K 2,048) at few rows, COLD weights (a ring of copies
larger than the Infinity Cache): the exact-row paths — the MFMA exact kernel (qasr_op_gemm_exact_rows) and the
weight-streaming GEMV in row groups (qasr_op_gemv_fused, GV_NONE) — against the table GEMM (qasr_op_linear_q8).
Both exact paths give the 1-row GEMV's bits per row (tests/test_ops_gpu.py); this times them.  GPU.
usage: python tools/lmhead_cost.py [rows,...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

N, K = 151936, 2048


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    rows = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4,5,8,12,16,20,24,32").split(",")]
    copies = max(2, int(768e6 // (N * K * 1.0625)) + 1)
    wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
    ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
    p = lambda t: t.data_ptr()  # noqa: E731
    for M in rows:
        xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        xd = torch.rand(M, K // 32, device=dev) * 0.01
        y = torch.zeros(M, N, device=dev)
        y2 = torch.zeros(M, N, device=dev)
        y3 = torch.zeros(M, N, device=dev)
        paths = {
            "table": lambda i: lib.qasr_op_linear_q8(p(xq), p(xd), M, p(wq[i]), p(ws[i]), N, K, None, None, p(y), N,
                                                     0, 2, None),
            "exact_mfma": lambda i: lib.qasr_op_gemm_exact_rows(p(xq), p(xd), M, p(wq[i]), p(ws[i]), N, K, None,
                                                                p(y), N, 0, None),
            "gemv_rows": lambda i: lib.qasr_op_gemv_fused(0, None, 0, None, 0.0, M, p(xq), p(xd), p(wq[i]), p(ws[i]),
                                                          N, K, None, p(y2), N, 0, None, None, None),
            "xr_vocab": lambda i: lib.qasr_op_xr_vocab(p(xq), p(xd), M, p(wq[i]), p(ws[i]), N, K, p(y3), N, None),
        }
        res = {}
        for name, fn in paths.items():
            if fn(0) != 0:
                res[name] = None
                continue
            torch.cuda.synchronize()
            n = copies * 4
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(n):
                _lib.check(fn(i % copies))
            e1.record()
            torch.cuda.synchronize()
            res[name] = e0.elapsed_time(e1) / n * 1e3
        # the last call of each path used weight copy (n - 1) % copies: recompute all three on copy 0, then compare
        for name in ("exact_mfma", "gemv_rows", "xr_vocab"):
            if res.get(name):
                _lib.check(paths[name](0))
        torch.cuda.synchronize()
        same = bool(torch.equal(y, y2)) if res.get("exact_mfma") and res.get("gemv_rows") else None
        same3 = bool(torch.equal(y3, y2)) if res.get("xr_vocab") and res.get("gemv_rows") else None
        print(f"lm_head M={M:3d} " + "  ".join(f"{k} {v:7.1f}us" if v else f"{k} n/a" for k, v in res.items()) +
              f"  exact==gemv bits: {same}  xr_vocab==gemv bits: {same3}", flush=True)


if __name__ == "__main__":
    main()
