#!/usr/bin/env python3
"""Decode-GEMM timing on the automatic path with and without the weight-streaming kernel (k_gemm_q8_ws), cold
weights (a ring of copies beyond the Infinity Cache), the 1.7B decoder shapes at 8–64 rows.  GPU.
usage: python tools/ws_probe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
from qasr import _lib  # noqa: E402

SHAPES = [("qkv", 4096, 2048, 0), ("o", 2048, 2048, 1), ("down", 2048, 6144, 1), ("gu", 12288, 2048, 3),
          ("lm", 151936, 2048, 0)]


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    for tag, N, K, epi in SHAPES:
        copies = max(2, int(768e6 // (N * K * 1.0625)) + 1)
        wq = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(copies)]
        ws = [(torch.rand(N, K // 32, device=dev) * 0.01).half() for _ in range(copies)]
        for M in (8, 16, 32, 48, 64, 96):
            xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
            xd = torch.rand(M, K // 32, device=dev) * 0.01
            y = torch.zeros(M, N, device=dev)
            hq = torch.empty(M, N // 2, dtype=torch.int8, device=dev)
            hd = torch.empty(M, N // 64, device=dev)
            rec = {"shape": tag, "M": M}
            for rows in (0, 64):
                _lib.check(lib.qasr_op_set_gemm_ws_rows(rows, 1))

                def run(i):
                    if epi == 3:
                        _lib.check(lib.qasr_op_gemm_swiglu_q8_cfg(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                                  ws[i].data_ptr(), N, K, hq.data_ptr(), hd.data_ptr(),
                                                                  -1, None))
                    else:
                        _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq[i].data_ptr(),
                                                         ws[i].data_ptr(), N, K, None,
                                                         y.data_ptr() if epi == 1 else None, y.data_ptr(), N, epi, 2,
                                                         None))
                run(0)
                torch.cuda.synchronize()
                n = copies * max(1, 24 // copies)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(n):
                    run(i % copies)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / n * 1e3
                rec["ws" if rows else "gemm"] = round(us, 2)
            rec["ws_TBps"] = round(N * K * 1.0625 / rec["ws"] / 1e6, 2)
            print(json.dumps(rec), flush=True)
        del wq, ws
        torch.cuda.empty_cache()
    _lib.check(lib.qasr_op_set_gemm_ws_rows(16, 0))


if __name__ == "__main__":
    main()
