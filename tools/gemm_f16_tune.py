#!/usr/bin/env python3
"""A/B of the Q8 GEMM on int8 operands (i8 MFMA, qasr_op_linear_q8) against f16-carried operands
(f16 MFMA, qasr_op_linear_q8h): agreement and time on the engine's shapes (GPU)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-whisper_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from qasr import _lib  # noqa: E402
from gemm_tune import SHAPES  # noqa: E402


def timeit(fn, flops):
    fn()
    torch.cuda.synchronize()
    iters = max(3, min(50, int(2e12 / flops * 20)))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    only = sys.argv[1:]
    for tag, M, N, K, epi in SHAPES:
        if only and not any(o in tag for o in only):
            continue
        xq = torch.randint(-127, 128, (M, K), dtype=torch.int8, device=dev)
        xd = torch.rand(M, K // 32, device=dev) * 0.01
        wq = torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev)
        ws = (torch.rand(N, K // 32, device=dev) * 0.01).half()
        xh, wh = xq.half(), wq.half()
        y1 = torch.zeros(M, N, device=dev)
        y2 = torch.zeros(M, N, device=dev)
        flops = 2.0 * M * N * K
        r = {}

        def i8():
            _lib.check(lib.qasr_op_linear_q8(xq.data_ptr(), xd.data_ptr(), M, wq.data_ptr(), ws.data_ptr(), N, K, None,
                                             None, y1.data_ptr(), N, 0, 2, None))
        r["i8"] = timeit(i8, flops)
        for cfg in range(4):
            def f16():
                _lib.check(lib.qasr_op_linear_q8h(xh.data_ptr(), xd.data_ptr(), M, wh.data_ptr(), ws.data_ptr(), N, K,
                                                  None, None, y2.data_ptr(), N, 0, cfg, None))
            r[f"h{cfg}"] = timeit(f16, flops)
            if cfg == 0:   # the i8 and f16-carried kernels compute the same values (exact block sums, same rescale)
                err = (y1 - y2).abs().max().item() / (y1.abs().max().item() + 1e-9)
        out = " ".join(f"{k}:{v:8.1f}us {flops / v / 1e6:5.0f}TF" for k, v in r.items())
        print(f"{tag:14s} M={M:6d} N={N:6d} K={K:5d} relerr={err:.1e} | {out}", flush=True)


if __name__ == "__main__":
    main()
